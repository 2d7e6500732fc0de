/*
 * test_kv.c — batched store I/O around the GPU path (include/rr_kv.h, row f2) against an
 * in-memory store with MultiGet / WriteBatch semantics (RocksDB is not part of this build).
 *
 * The golden fixtures' valid blobs, repeated to K values, are decoded (rr_decode_batch_host),
 * dumped under K keys with one rr_kv_dump_batch, and restored with one rr_kv_restore_batch:
 *   - plain: every stored value is the bytes serObject writes for the fixture's object (the
 *     fixture's re-encoded form, lru masked to 24 bits); the restored flat batch equals the
 *     decode of those bytes record for record, descriptor for descriptor, arena byte for byte;
 *   - RR_KV_SNAPPY: every stored value is a snappy stream that decompresses (GPU,
 *     rr_snappy_decompress_batch_host) to those bytes; the restore is the same flat batch;
 *   - a missing key fails the restore; a write_batch sees all K puts in one call.
 * Needs the GPU.  Exit status 0 when every check passes.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rr_kv.h"
#include "rr_snappy.h"
#include "fixtures.h"

static int fails;
#define CHECK(c, ...) do { if (!(c)) { fails++; printf("FAIL: "); printf(__VA_ARGS__); printf("\n"); } } while (0)

/* ---- the store: open addressing over (dbi, key) ---- */
typedef struct { int dbi; char *key; size_t klen; void *val; size_t vlen; } slot_t;
typedef struct { slot_t *s; size_t cap, n, batches, puts; } store_t;
static uint64_t h64(int dbi, const char *k, size_t n) {
    uint64_t h = 1469598103934665603ull ^ (uint64_t)dbi;
    for (size_t i = 0; i < n; i++) h = (h ^ (uint8_t)k[i]) * 1099511628211ull;
    return h;
}
static slot_t *find(store_t *st, int dbi, const char *k, size_t n, int make) {
    for (uint64_t i = h64(dbi, k, n) & (st->cap - 1);; i = (i + 1) & (st->cap - 1)) {
        slot_t *e = &st->s[i];
        if (!e->key) {
            if (!make) return NULL;
            e->dbi = dbi; e->key = malloc(n ? n : 1); memcpy(e->key, k, n); e->klen = n; st->n++;
            return e;
        }
        if (e->dbi == dbi && e->klen == n && !memcmp(e->key, k, n)) return e;
    }
}
static int st_get(void *u, int dbi, size_t k, const char *const *keys, const size_t *kl, void **vals, size_t *vl) {
    store_t *st = u;
    for (size_t i = 0; i < k; i++) {
        slot_t *e = find(st, dbi, keys[i], kl[i], 0);
        vals[i] = NULL;
        if (!e) continue;
        vals[i] = malloc(e->vlen ? e->vlen : 1);
        memcpy(vals[i], e->val, e->vlen);
        vl[i] = e->vlen;
    }
    return 0;
}
static int st_put(void *u, int dbi, size_t k, const char *const *keys, const size_t *kl, const void *const *vals,
                  const size_t *vl) {
    store_t *st = u;
    st->batches++;
    for (size_t i = 0; i < k; i++) {
        slot_t *e = find(st, dbi, keys[i], kl[i], 1);
        free(e->val);
        e->val = malloc(vl[i] ? vl[i] : 1);
        memcpy(e->val, vals[i], vl[i]);
        e->vlen = vl[i];
        st->puts++;
    }
    return 0;
}
static void st_free_val(void *u, void *v) { (void)u; free(v); }

static void decode(rr_ctx *ctx, const uint8_t *const *b, const size_t *l, size_t k, rr_rdb_flat *f, uint8_t **data_out,
                   uint64_t **offs_out) {
    uint64_t *offs = calloc(k + 1, sizeof(uint64_t));
    for (size_t i = 0; i < k; i++) offs[i + 1] = offs[i] + l[i];
    uint8_t *data = calloc(((offs[k] + 15) & ~15ull) + 16, 1);
    for (size_t i = 0; i < k; i++) memcpy(data + offs[i], b[i], l[i]);
    const uint64_t cap = rr_decode_elem_bound(k, offs[k]);
    f->values = malloc(k * sizeof(rr_value));
    f->elems = malloc((cap ? cap : 1) * sizeof(rr_elem));
    f->arena = calloc(((offs[k] + 15) & ~15ull) + 16, 1);
    rr_totals t;
    if (rr_decode_batch_host(ctx, data, offs, k, f->values, f->elems, cap, f->arena, &t) != RR_API_OK) {
        printf("decode failed: %s\n", rr_last_error());
        exit(2);
    }
    f->n = k;
    f->n_elems = t.n_elems;
    f->bytes = offs[k];
    *data_out = data;
    *offs_out = offs;
}

static void same_flat(const rr_rdb_flat *a, const rr_rdb_flat *b, const char *what) {
    CHECK(a->n == b->n && a->n_elems == b->n_elems && a->bytes == b->bytes, "%s: sizes differ", what);
    if (a->n != b->n || a->n_elems != b->n_elems || a->bytes != b->bytes) return;
    CHECK(!memcmp(a->values, b->values, a->n * sizeof(rr_value)), "%s: records differ", what);
    CHECK(!memcmp(a->elems, b->elems, a->n_elems * sizeof(rr_elem)), "%s: descriptors differ", what);
    /* the arena: every STR / ZLRAW payload (the mirror's other bytes are not part of the form) */
    for (uint64_t i = 0; i < a->n_elems; i++) {
        const rr_elem *e = &a->elems[i];
        if ((e->kind == RR_K_STR || e->kind == RR_K_ZLRAW) && memcmp(a->arena + e->data, b->arena + e->data, e->len)) {
            CHECK(0, "%s: payload of descriptor %llu differs", what, (unsigned long long)i);
            break;
        }
    }
}

int main(void) {
    rr_ctx *ctx = NULL;
    if (rr_ctx_create(0, &ctx) != RR_API_OK) { printf("no GPU: %s\n", rr_last_error()); return 2; }
    const fixture_t *valid[N_FIXTURES];
    int nvalid = 0;
    for (int i = 0; i < N_FIXTURES; i++)
        if (FIXTURES[i].status == 0) valid[nvalid++] = &FIXTURES[i];
    enum { K = 3000 };
    static const uint8_t *blob[K], *canon[K];
    static size_t blen[K], clen[K], klen[K];
    static char *keys[K];
    for (size_t i = 0; i < K; i++) {
        const fixture_t *f = valid[i % nvalid];
        blob[i] = f->blob; blen[i] = f->len;
        canon[i] = f->out; clen[i] = f->out_len;
        keys[i] = malloc(24);
        klen[i] = (size_t)snprintf(keys[i], 24, "key:%zu", i);
    }
    rr_rdb_flat src, want;
    uint8_t *d1, *d2;
    uint64_t *o1, *o2;
    decode(ctx, blob, blen, K, &src, &d1, &o1);     /* what the evictor holds */
    decode(ctx, canon, clen, K, &want, &d2, &o2);   /* what a restore must return */
    for (int mode = 0; mode < 2; mode++) {
        const int flags = mode ? RR_KV_SNAPPY : 0;
        const char *what = mode ? "snappy" : "plain";
        store_t st = {calloc(8192, sizeof(slot_t)), 8192, 0, 0, 0};
        rr_kv_ops ops = {&st, st_get, st_put, st_free_val};
        int rc = rr_kv_dump_batch(ctx, &ops, 5, K, (const char *const *)keys, klen, src.values, src.elems, src.n_elems,
                                  src.arena, src.bytes, flags);
        CHECK(rc == RR_API_OK, "%s dump: %s", what, rr_last_error());
        CHECK(st.batches == 1 && st.puts == K, "%s: %zu write batches, %zu puts", what, st.batches, st.puts);
        /* the stored bytes */
        size_t bad = 0;
        for (size_t i = 0; i < K && rc == RR_API_OK; i++) {
            slot_t *e = find(&st, 5, keys[i], klen[i], 0);
            if (!e) { bad++; continue; }
            if (!mode) {
                if (e->vlen != clen[i] || memcmp(e->val, canon[i], clen[i])) bad++;
            } else {
                uint64_t zo[2] = {0, e->vlen}, oo[2];
                uint8_t stt, *back = malloc(clen[i] + 16);
                if (rr_snappy_decompress_batch_host(ctx, e->val, zo, 1, back, clen[i] + 16, oo, &stt) != RR_API_OK ||
                    stt || oo[1] != clen[i] || memcmp(back, canon[i], clen[i]))
                    bad++;
                free(back);
                if (i > 200) break;   /* (one call per value: a sample is enough) */
            }
        }
        CHECK(bad == 0, "%s: %zu stored values differ", what, bad);
        rr_rdb_flat got;
        rc = rr_kv_restore_batch(ctx, &ops, 5, K, (const char *const *)keys, klen, flags, &got);
        CHECK(rc == RR_API_OK, "%s restore: %s", what, rr_last_error());
        if (rc == RR_API_OK) { same_flat(&got, &want, what); rr_rdb_flat_free(&got); }
        const char *missing[2] = {keys[0], "no-such-key"};
        size_t ml[2] = {klen[0], 11};
        rc = rr_kv_restore_batch(ctx, &ops, 5, 2, missing, ml, flags, &got);
        CHECK(rc != RR_API_OK, "%s: a missing key was restored", what);
        for (size_t i = 0; i < st.cap; i++) { free(st.s[i].key); free(st.s[i].val); }
        free(st.s);
    }
    for (size_t i = 0; i < K; i++) free(keys[i]);
    rr_rdb_flat_free(&src); rr_rdb_flat_free(&want);
    free(d1); free(d2); free(o1); free(o2);
    rr_ctx_destroy(ctx);
    printf("%d failures (%d values, plain and snappy)\n", fails, K);
    return fails ? 1 : 0;
}
