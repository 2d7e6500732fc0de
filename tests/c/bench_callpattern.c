/*
 * bench_callpattern.c — the compat shim inside the call patterns of the unchanged reference
 * callers (diagnostics; GPU box; prints one JSON line):
 *
 *   evictor  up to 64 keys picked per eviction cycle on the main thread, each dumped with
 *            serObject (rock_hotkey.c:348-437 -> rock.c:682-697, serObject at :691);
 *   restore  one desObject per rock-thread job (rock.c:552-575 -> :468), a wave of k jobs.
 *
 * Per cycle / wave of k = 1, 16, 64, 1024 keys (config-4 values), wall time of:
 *   shim_each   k calls of the one-value signature through the shim (serObject / desObject);
 *   shim_batch  one rr_compat_ser_batch / rr_compat_des_batch of the k keys;
 *   cpu         the faithful CPU restatement of the reference (oracle/rro_faithful.c: robj,
 *               sds, dict, skiplist building; test infrastructure linked only into this bench)
 *               over the same k values.
 * Medians over many cycles.  The answer it gives: at which k the GPU route beats the CPU path.
 *
 * usage: bench_callpattern [config]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "server.h"
#include "rock_serdes_compat.h"
#include "rr_oracle.h"

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}
static int cmpd(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}
static double median(double *t, int r) {
    qsort(t, (size_t)r, sizeof(double), cmpd);
    return t[r / 2];
}

int main(int argc, char **argv) {
    const int cfg = argc > 1 ? atoi(argv[1]) : 4;
    enum { NK = 4, POOL = 8192 };
    const size_t ks[NK] = {1, 16, 64, 1024};
    rr_host_batch hb;
    if (rr_gen_batch(cfg, POOL, rr_gen_default_seed(cfg), &hb) != RR_API_OK) return 2;
    robj **objs = malloc(sizeof(robj *) * POOL), **tmp = malloc(sizeof(robj *) * 1024);
    sds *outs = malloc(sizeof(sds) * 1024);
    void **bufs = malloc(sizeof(void *) * 1024);
    size_t *lens = malloc(sizeof(size_t) * 1024);
    uint64_t *offs = malloc(sizeof(uint64_t) * 1025);
    uint8_t *cpu_out = malloc(64u << 20);
    double *t = malloc(sizeof(double) * 4096);
    int bad = 0;
    /* the objects the evictor would hold (decoded once; warms the context and pinned buffers) */
    for (size_t i = 0; i < POOL; i++) objs[i] = desObject(hb.data + hb.offsets[i], hb.offsets[i + 1] - hb.offsets[i]);
    printf("{\"config\": %d, \"pool_values\": %d, \"unit\": \"us per cycle (median)\", \"rows\": [", cfg, POOL);
    for (int ki = 0; ki < NK; ki++) {
        const size_t k = ks[ki];
        const int R = k >= 1024 ? 40 : k >= 64 ? 200 : 800;
        double res[6];
        /* evictor: k serObject per cycle */
        for (int pass = 0; pass < 3; pass++) {
            for (int r = -5; r < R; r++) {
                const size_t v0 = ((size_t)(r + 5) * k) % (POOL - k + 1);
                const double t0 = now_us();
                if (pass == 0) {
                    for (size_t i = 0; i < k; i++) outs[i] = serObject(objs[v0 + i]);
                } else if (pass == 1) {
                    rr_compat_ser_batch(objs + v0, k, outs);
                } else {
                    for (size_t i = 0; i <= k; i++) offs[i] = hb.offsets[v0 + i] - hb.offsets[v0];
                    const double td = now_us();
                    rro_store *st = rro_faithful_decode(hb.data + hb.offsets[v0], offs, k, NULL);
                    const double te = now_us();
                    uint64_t oo[1025];
                    rro_faithful_encode(st, cpu_out, 64u << 20, oo);
                    const double tf = now_us();
                    rro_store_free(st);
                    if (r >= 0) t[r] = tf - te;   /* (serObject's share: the encode) */
                    (void)td;
                    continue;
                }
                const double t1 = now_us() - t0;
                if (r >= 0) t[r] = t1;
                for (size_t i = 0; i < k; i++) {
                    const size_t len = hb.offsets[v0 + i + 1] - hb.offsets[v0 + i];
                    if (sdslen(outs[i]) != len || memcmp(outs[i], hb.data + hb.offsets[v0 + i], len)) bad++;
                    sdsfree(outs[i]);
                }
            }
            res[pass] = median(t, R);
        }
        /* restore: k desObject (one per job) */
        for (int pass = 0; pass < 3; pass++) {
            for (int r = -5; r < R; r++) {
                const size_t v0 = ((size_t)(r + 5) * k * 7) % (POOL - k + 1);
                for (size_t i = 0; i < k; i++) {
                    bufs[i] = hb.data + hb.offsets[v0 + i];
                    lens[i] = hb.offsets[v0 + i + 1] - hb.offsets[v0 + i];
                }
                const double t0 = now_us();
                if (pass == 0) {
                    for (size_t i = 0; i < k; i++) tmp[i] = desObject(bufs[i], lens[i]);
                } else if (pass == 1) {
                    rr_compat_des_batch(bufs, lens, k, tmp);
                } else {
                    for (size_t i = 0; i <= k; i++) offs[i] = hb.offsets[v0 + i] - hb.offsets[v0];
                    rro_store *st = rro_faithful_decode(hb.data + hb.offsets[v0], offs, k, NULL);
                    const double t1 = now_us() - t0;
                    rro_store_free(st);
                    if (r >= 0) t[r] = t1;
                    continue;
                }
                const double t1 = now_us() - t0;
                if (r >= 0) t[r] = t1;
                for (size_t i = 0; i < k; i++) {   /* the restored object serializes back to the blob */
                    sds s = serObject(tmp[i]);
                    if (sdslen(s) != lens[i] || memcmp(s, bufs[i], lens[i])) bad++;
                    sdsfree(s);
                    decrRefCount(tmp[i]);
                }
            }
            res[3 + pass] = median(t, R);
        }
        printf("%s{\"k\": %zu, \"evictor_serObject\": {\"shim_each\": %.2f, \"shim_batch\": %.2f, \"cpu\": %.2f}, "
               "\"restore_desObject\": {\"shim_each\": %.2f, \"shim_batch\": %.2f, \"cpu\": %.2f}}",
               ki ? ", " : "", k, res[0], res[1], res[2], res[3], res[4], res[5]);
        fflush(stdout);
    }
    printf("], \"roundtrip_bad\": %d}\n", bad);
    for (size_t i = 0; i < POOL; i++) decrRefCount(objs[i]);
    rr_host_batch_free(&hb);
    return bad ? 1 : 0;
}
