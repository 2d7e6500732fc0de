/*
 * rr_snappy_api.c — host layer of the GPU block compression (include/rr_snappy.h, SURVEY.md
 * §8f row f3): argument checks, the context's scratch, and host-pointer forms that stage
 * through the context's device buffers.
 */
#include <stdlib.h>
#include <string.h>

#include "rr_internal.h"
#include "../../include/rr_snappy.h"

#define fail rr_fail

uint64_t rr_snappy_max_compressed_length(uint64_t n) { return 32 + n + n / 6; }

uint64_t rr_snappy_compress_bound(uint64_t n, uint64_t data_bytes) {
    return ((32 * n + data_bytes + data_bytes / 6) + 15 + 16) & ~15ull;
}

static int aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

int rr_snappy_compress_batch(rr_ctx *c, const rr_blob_batch *in, rr_blob_batch *out, void *stream) {
    if (!c || !in || !out || !in->offsets || !out->offsets) return fail(RR_API_EINVAL, "NULL argument");
    if (out->n != in->n) return fail(RR_API_EINVAL, "out->n != in->n");
    if (in->n >= RR_MAX_VALUES) return fail(RR_API_EINVAL, "batch too large");
    if (in->n && (!in->data || !out->data)) return fail(RR_API_EINVAL, "NULL buffer");
    if (in->n && !aligned16(in->data)) return fail(RR_API_EINVAL, "in->data not 16-byte aligned");
    if (in->data_cap & 15) return fail(RR_API_EINVAL, "in->data_cap must be a multiple of 16");
    const uint64_t slot_bytes = rr_snappy_compress_bound(in->n, in->data_cap);
    if (out->data_cap < slot_bytes) return fail(RR_API_EINVAL, "out->data_cap < rr_snappy_compress_bound(n, in->data_cap)");
    HIPCHK(hipSetDevice(c->device));
    int rc = rr_ensure_scratch(c, rr_snappy_scratch_words(in->n, slot_bytes), (hipStream_t)stream);
    if (rc) return rc;
    HIPCHK(rr_launch_snappy_compress(in->data, in->data_cap, in->offsets, in->n, out->data, out->offsets, c->scratch, slot_bytes,
                                     (hipStream_t)stream));
    return rr_mark_scratch(c, (hipStream_t)stream);
}

int rr_snappy_decompress_batch(rr_ctx *c, const rr_blob_batch *in, rr_blob_batch *out, uint8_t *status,
                               void *stream) {
    if (!c || !in || !out || !in->offsets || !out->offsets) return fail(RR_API_EINVAL, "NULL argument");
    if (out->n != in->n) return fail(RR_API_EINVAL, "out->n != in->n");
    if (in->n >= RR_MAX_VALUES) return fail(RR_API_EINVAL, "batch too large");
    if (in->n && (!in->data || !status)) return fail(RR_API_EINVAL, "NULL buffer");
    if (in->n && !aligned16(in->data)) return fail(RR_API_EINVAL, "in->data not 16-byte aligned");
    if (in->data_cap & 15) return fail(RR_API_EINVAL, "in->data_cap must be a multiple of 16");
    HIPCHK(hipSetDevice(c->device));
    int rc = rr_ensure_scratch(c, rr_snappy_scratch_words(in->n, 0), (hipStream_t)stream);
    if (rc) return rc;
    HIPCHK(rr_launch_snappy_decompress(in->data, in->data_cap, in->offsets, in->n, out->data, out->data_cap, out->offsets, status,
                                       c->scratch, (hipStream_t)stream));
    return rr_mark_scratch(c, (hipStream_t)stream);
}

#define GROW(P, C, N) do { int r_ = rr_dgrow((void **)&(P), &(C), (N)); if (r_) return r_; } while (0)

int rr_snappy_compress_batch_host(rr_ctx *c, const uint8_t *data, const uint64_t *offsets, uint64_t n, uint8_t *out,
                                  uint64_t out_cap, uint64_t *out_offsets) {
    if (!c || !offsets || !out_offsets || (n && (!data || !out))) return fail(RR_API_EINVAL, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    const uint64_t bytes = offsets[n], pbytes = (bytes + 15) & ~15ull;
    const uint64_t cap = rr_snappy_compress_bound(n, pbytes);
    if (out_cap < rr_snappy_compress_bound(n, bytes)) return fail(RR_API_EINVAL, "out_cap too small");
    GROW(c->d_in, c->c_in, pbytes + 16);
    GROW(c->d_off, c->c_off, (n + 1) * sizeof(uint64_t));
    GROW(c->d_out, c->c_out, cap + 16);
    GROW(c->d_ooff, c->c_ooff, (n + 1) * sizeof(uint64_t));
    if (bytes) HIPCHK(hipMemcpyAsync(c->d_in, data, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_off, offsets, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    rr_blob_batch in = {(uint8_t *)c->d_in, (uint64_t *)c->d_off, n, pbytes};
    rr_blob_batch o = {(uint8_t *)c->d_out, (uint64_t *)c->d_ooff, n, cap};
    int rc = rr_snappy_compress_batch(c, &in, &o, c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(out_offsets, c->d_ooff, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (out_offsets[n] > out_cap) return fail(RR_API_EDEVICE, "compressed output larger than its bound");
    if (out_offsets[n]) HIPCHK(hipMemcpyAsync(out, c->d_out, out_offsets[n], hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return RR_API_OK;
}

int rr_snappy_decompress_batch_host(rr_ctx *c, const uint8_t *data, const uint64_t *offsets, uint64_t n, uint8_t *out,
                                    uint64_t out_cap, uint64_t *out_offsets, uint8_t *status) {
    if (!c || !offsets || !out_offsets || (n && (!data || !status))) return fail(RR_API_EINVAL, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    const uint64_t bytes = offsets[n], pbytes = (bytes + 15) & ~15ull;
    GROW(c->d_in, c->c_in, pbytes + 16);
    GROW(c->d_off, c->c_off, (n + 1) * sizeof(uint64_t));
    GROW(c->d_ooff, c->c_ooff, (n + 1) * sizeof(uint64_t));
    GROW(c->d_vals, c->c_vals, n + 16);   /* per-block status */
    GROW(c->d_out, c->c_out, out_cap + 16);
    if (bytes) HIPCHK(hipMemcpyAsync(c->d_in, data, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_off, offsets, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    rr_blob_batch in = {(uint8_t *)c->d_in, (uint64_t *)c->d_off, n, pbytes};
    rr_blob_batch o = {(uint8_t *)c->d_out, (uint64_t *)c->d_ooff, n, out_cap};
    int rc = rr_snappy_decompress_batch(c, &in, &o, (uint8_t *)c->d_vals, c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(out_offsets, c->d_ooff, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    if (n) HIPCHK(hipMemcpyAsync(status, c->d_vals, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (out_offsets[n] > out_cap) return fail(RR_API_EINVAL, "out_cap %llu < announced output %llu",
                                              (unsigned long long)out_cap, (unsigned long long)out_offsets[n]);
    if (out_offsets[n]) HIPCHK(hipMemcpyAsync(out, c->d_out, out_offsets[n], hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return RR_API_OK;
}
