/*
 * rr_kv.c — batched store I/O around the GPU path (include/rr_kv.h):
 * one store call per batch, one upload and one download per batch, encode / decode and the
 * optional snappy step back to back on the device.
 */
#include <stdlib.h>
#include <string.h>

#include "rr_internal.h"
#include "../../include/rr_kv.h"
#include "../../include/rr_snappy.h"

#define fail rr_fail

typedef struct { void *p[8]; int n; } dbufs;
static void *dalloc(dbufs *b, size_t bytes) {
    void *p = NULL;
    if (b->n >= 8 || hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return NULL;
    b->p[b->n++] = p;
    return p;
}
static void dfree_all(dbufs *b) {
    for (int i = 0; i < b->n; i++) hipFree(b->p[i]);
    b->n = 0;
}

/* blob bytes rr_encode_batch may write for this flat batch (rr_serdes.h encode bound):
 * 13 per value + 24 per descriptor + every STR / ZLRAW payload */
static uint64_t encode_bound(size_t k, const rr_elem *elems, uint64_t n_elems) {
    uint64_t b = 13 * (uint64_t)k + 24 * n_elems + 16;
    for (uint64_t i = 0; i < n_elems; i++) b += elems[i].len;
    return (b + 15) & ~15ull;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { rc = fail(RR_API_EHIP, "%s: %s", #x, hipGetErrorString(e_)); goto out; } } while (0)
#define NEED(p) do { if (!(p)) { rc = fail(RR_API_ENOMEM, "allocation failed"); goto out; } } while (0)

int rr_kv_dump_batch(rr_ctx *c, const rr_kv_ops *kv, int dbi, size_t k, const char *const *keys,
                     const size_t *key_lens, const rr_value *values, const rr_elem *elems, uint64_t n_elems,
                     const uint8_t *arena, uint64_t arena_bytes, int flags) {
    if (!c || !kv || !kv->write_batch || (k && (!keys || !key_lens || !values)) || (n_elems && !elems) ||
        (arena_bytes && !arena))
        return fail(RR_API_EINVAL, "rr_kv_dump_batch: NULL argument");
    if (k == 0) return RR_API_OK;
    dbufs d = {{0}, 0};
    int rc = RR_API_OK;
    uint8_t *host = NULL;
    uint64_t *hoffs = NULL;
    const void **vals = NULL;
    size_t *vlens = NULL;
    hipStream_t s = c->stream;
    const uint64_t cap = encode_bound(k, elems, n_elems);
    CK(hipSetDevice(c->device));
    rr_value *dv = dalloc(&d, k * sizeof(rr_value));
    rr_elem *de = dalloc(&d, (n_elems ? n_elems : 1) * sizeof(rr_elem));
    uint8_t *da = dalloc(&d, arena_bytes + 16);
    uint8_t *dout = dalloc(&d, cap + 16);
    uint64_t *doffs = dalloc(&d, (k + 1) * sizeof(uint64_t));
    NEED(dv && de && da && dout && doffs);
    CK(hipMemcpyAsync(dv, values, k * sizeof(rr_value), hipMemcpyHostToDevice, s));
    if (n_elems) CK(hipMemcpyAsync(de, elems, n_elems * sizeof(rr_elem), hipMemcpyHostToDevice, s));
    if (arena_bytes) CK(hipMemcpyAsync(da, arena, arena_bytes, hipMemcpyHostToDevice, s));
    rr_flat_batch fin = {dv, de, da, k, n_elems, arena_bytes};
    rr_blob_batch blobs = {dout, doffs, k, cap};
    if ((rc = rr_encode_batch(c, &fin, &blobs, c->d_totals, s))) goto out;
    rr_totals t;
    CK(hipMemcpyAsync(&t, c->d_totals, sizeof t, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    if (t.bytes == ~0ull) { rc = fail(RR_API_EDEVICE, "encode: device-side failure"); goto out; }
    if (t.n_bad) { rc = fail(RR_API_EINVAL, "rr_kv_dump_batch: %llu values cannot be encoded", (unsigned long long)t.n_bad); goto out; }
    const uint8_t *src = dout;
    const uint64_t *soffs = doffs;
    if (flags & RR_KV_SNAPPY) {
        const uint64_t zcap = rr_snappy_compress_bound(k, cap);
        uint8_t *dz = dalloc(&d, zcap + 16);
        uint64_t *dzo = dalloc(&d, (k + 1) * sizeof(uint64_t));
        NEED(dz && dzo);
        rr_blob_batch z = {dz, dzo, k, zcap};
        if ((rc = rr_snappy_compress_batch(c, &blobs, &z, s))) goto out;
        src = dz;
        soffs = dzo;
    }
    NEED(hoffs = (uint64_t *)malloc((k + 1) * sizeof(uint64_t)));
    CK(hipMemcpyAsync(hoffs, soffs, (k + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    NEED(host = (uint8_t *)malloc(hoffs[k] ? hoffs[k] : 1));
    if (hoffs[k]) CK(hipMemcpyAsync(host, src, hoffs[k], hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    NEED(vals = (const void **)malloc(k * sizeof(void *)));
    NEED(vlens = (size_t *)malloc(k * sizeof(size_t)));
    for (size_t i = 0; i < k; i++) {
        vals[i] = host + hoffs[i];
        vlens[i] = (size_t)(hoffs[i + 1] - hoffs[i]);
    }
    if (kv->write_batch(kv->user, dbi, k, keys, key_lens, vals, vlens)) rc = fail(RR_API_EINVAL, "write_batch failed");
out:
    dfree_all(&d);
    free(host); free(hoffs); free(vals); free(vlens);
    return rc;
}

/* varint32 length preamble of a snappy stream (snappy.cc:779-800); 0 on success */
static int snappy_len(const uint8_t *p, size_t n, uint64_t *len) {
    uint32_t v = 0, shift = 0;
    for (size_t i = 0; i < n && shift < 32; i++, shift += 7) {
        const uint32_t b = p[i], val = b & 0x7F;
        if (shift == 28 && val >= 16) return -1;
        v |= val << shift;
        if (b < 128) { *len = v; return 0; }
    }
    return -1;
}

int rr_kv_restore_batch(rr_ctx *c, const rr_kv_ops *kv, int dbi, size_t k, const char *const *keys,
                        const size_t *key_lens, int flags, rr_rdb_flat *out) {
    if (!c || !kv || !kv->multi_get || !out || (k && (!keys || !key_lens))) return fail(RR_API_EINVAL, "rr_kv_restore_batch: NULL argument");
    memset(out, 0, sizeof *out);
    if (k == 0) return RR_API_OK;
    dbufs d = {{0}, 0};
    int rc = RR_API_OK;
    hipStream_t s = c->stream;
    void **vals = (void **)calloc(k, sizeof(void *));
    size_t *vlens = (size_t *)calloc(k, sizeof(size_t));
    uint64_t *soffs = (uint64_t *)calloc(k + 1, sizeof(uint64_t)), *boffs = NULL;
    uint8_t *host = NULL;
    NEED(vals && vlens && soffs);
    if (kv->multi_get(kv->user, dbi, k, keys, key_lens, vals, vlens)) { rc = fail(RR_API_EINVAL, "multi_get failed"); goto out; }
    for (size_t i = 0; i < k; i++) {
        if (!vals[i]) { rc = fail(RR_API_EINVAL, "key %zu not found", i); goto out; }
        soffs[i + 1] = soffs[i] + vlens[i];
    }
    const uint64_t sbytes = soffs[k], spad = (sbytes + 15) & ~15ull;
    NEED(host = (uint8_t *)calloc(spad + 16, 1));
    for (size_t i = 0; i < k; i++) memcpy(host + soffs[i], vals[i], vlens[i]);
    uint64_t bbytes = sbytes;
    if (flags & RR_KV_SNAPPY) {   /* the blob sizes come from the streams' preambles */
        bbytes = 0;
        for (size_t i = 0; i < k; i++) {
            uint64_t l;
            if (snappy_len(host + soffs[i], vlens[i], &l)) { rc = fail(RR_API_EINVAL, "value %zu: bad snappy preamble", i); goto out; }
            bbytes += l;
        }
    }
    const uint64_t bpad = (bbytes + 15) & ~15ull, ecap = rr_decode_elem_bound(k, bbytes);
    CK(hipSetDevice(c->device));
    uint8_t *ds = dalloc(&d, spad + 16);
    uint64_t *dso = dalloc(&d, (k + 1) * sizeof(uint64_t));
    NEED(ds && dso);
    CK(hipMemcpyAsync(ds, host, spad, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(dso, soffs, (k + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    rr_blob_batch blobs = {ds, dso, k, spad};
    if (flags & RR_KV_SNAPPY) {
        uint8_t *db = dalloc(&d, bpad + 16), *dst = dalloc(&d, k);
        uint64_t *dbo = dalloc(&d, (k + 1) * sizeof(uint64_t));
        NEED(db && dst && dbo);
        CK(hipMemsetAsync(db, 0, bpad + 16, s));   /* (the decode reads the padding as zeros) */
        rr_blob_batch z = {ds, dso, k, spad}, b = {db, dbo, k, bpad};
        if ((rc = rr_snappy_decompress_batch(c, &z, &b, dst, s))) goto out;
        uint8_t *hst = (uint8_t *)malloc(k);
        NEED(hst);
        hipError_t e = hipMemcpyAsync(hst, dst, k, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        size_t bad = k;
        for (size_t i = 0; e == hipSuccess && i < k && bad == k; i++)
            if (hst[i]) bad = i;
        const uint8_t code = bad < k ? hst[bad] : 0;
        free(hst);
        CK(e);
        if (bad < k) { rc = fail(RR_API_EINVAL, "value %zu does not decompress (snappy status %u)", bad, code); goto out; }
        blobs = b;
    }
    rr_value *dv = dalloc(&d, k * sizeof(rr_value));
    rr_elem *de = dalloc(&d, (ecap ? ecap : 1) * sizeof(rr_elem));
    uint8_t *da = dalloc(&d, bpad + 16);
    NEED(dv && de && da);
    rr_flat_batch flat = {dv, de, da, k, ecap, bpad};
    if ((rc = rr_decode_batch(c, &blobs, &flat, c->d_totals, s))) goto out;
    rr_totals t;
    CK(hipMemcpyAsync(&t, c->d_totals, sizeof t, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    if (t.bytes == ~0ull) { rc = fail(RR_API_EDEVICE, "decode: device-side failure"); goto out; }
    out->n = k;
    out->n_elems = t.n_elems < ecap ? t.n_elems : ecap;
    out->bytes = bbytes;
    out->values = (rr_value *)malloc(k * sizeof(rr_value));
    out->elems = (rr_elem *)malloc((out->n_elems ? out->n_elems : 1) * sizeof(rr_elem));
    out->arena = (uint8_t *)malloc(bbytes + 16);
    NEED(out->values && out->elems && out->arena);
    CK(hipMemcpyAsync(out->values, dv, k * sizeof(rr_value), hipMemcpyDeviceToHost, s));
    if (out->n_elems) CK(hipMemcpyAsync(out->elems, de, out->n_elems * sizeof(rr_elem), hipMemcpyDeviceToHost, s));
    if (bbytes) CK(hipMemcpyAsync(out->arena, da, bbytes, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
out:
    if (rc != RR_API_OK) rr_rdb_flat_free(out);
    dfree_all(&d);
    if (vals && kv->free_val)
        for (size_t i = 0; i < k; i++)
            if (vals[i]) kv->free_val(kv->user, vals[i]);
    free(vals); free(vlens); free(soffs); free(boffs); free(host);
    return rc;
}
