/*
 * bench_callpattern.c — the compat shim inside the call patterns of the unchanged reference
 * callers (diagnostics; prints one JSON line):
 *
 *   evictor  keys picked per eviction cycle on the main thread, each dumped with serObject
 *            (rock_hotkey.c:348-437 -> rock.c:682-697, serObject at :691);
 *   restore  one desObject per rock-thread job (rock.c:552-575 -> :468), a wave of k jobs.
 *
 * Per cycle / wave of k keys (config-4 values), wall time of:
 *   shim_each    k calls of the one-value signature through the shim, default routing (the host
 *                codec: what rock.c gets unchanged);
 *   batch_host   one rr_compat_ser_batch / rr_compat_des_batch of the k keys on the host route;
 *   batch_gpu    the same on the GPU route (omitted without a GPU);
 *   cpu          the faithful CPU restatement of the reference (oracle/rro_faithful.c: robj,
 *                sds, dict, skiplist building; test infrastructure linked only into this bench)
 *                over the same k values.
 * Medians over many cycles.  The answers: what the per-key calls cost against the reference's own
 * C, and from which k the GPU route wins (the shim's RR_COMPAT_GPU_MIN crossover).
 *
 * usage: bench_callpattern [config] [max_k]
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
static volatile unsigned sink_all;
static double median(double *t, int r) {
    qsort(t, (size_t)r, sizeof(double), cmpd);
    return t[r / 2];
}

enum { NK = 7, POOL = 1 << 17, KMAX = 1 << 16 };
static const size_t ks[NK] = {1, 16, 64, 1024, 4096, 16384, 65536};

int main(int argc, char **argv) {
    const int cfg = argc > 1 ? atoi(argv[1]) : 4;
    const size_t kmax = argc > 2 ? (size_t)atol(argv[2]) : KMAX;
    rr_host_batch hb;
    if (rr_gen_batch(cfg, POOL, rr_gen_default_seed(cfg), &hb) != RR_API_OK) return 2;
    rr_ctx *probe = NULL;
    const int gpu = rr_ctx_create(0, &probe) == RR_API_OK;
    if (gpu) rr_ctx_destroy(probe);
    robj **objs = malloc(sizeof(robj *) * POOL), **tmp = malloc(sizeof(robj *) * KMAX);
    sds *outs = malloc(sizeof(sds) * KMAX);
    void **bufs = malloc(sizeof(void *) * KMAX);
    size_t *lens = malloc(sizeof(size_t) * KMAX);
    uint64_t *offs = malloc(sizeof(uint64_t) * (KMAX + 1)), *oo = malloc(sizeof(uint64_t) * (KMAX + 1));
    uint8_t *cpu_out = malloc(256u << 20);
    double *t = malloc(sizeof(double) * 4096);
    int bad = 0;
    /* the objects the evictor would hold */
    for (size_t i = 0; i < POOL; i++) objs[i] = desObject(hb.data + hb.offsets[i], hb.offsets[i + 1] - hb.offsets[i]);
    if (gpu) {   /* warm the GPU route (context, pinned buffers) */
        rr_compat_set_route(RR_COMPAT_ROUTE_GPU);
        rr_compat_ser_batch(objs, 1024, outs);
        for (size_t i = 0; i < 1024; i++) sdsfree(outs[i]);
    }
    printf("{\"config\": %d, \"pool_values\": %d, \"gpu\": %s, \"unit\": \"us per cycle (median)\", \"rows\": [", cfg,
           POOL, gpu ? "true" : "false");
    for (int ki = 0; ki < NK && ks[ki] <= kmax; ki++) {
        const size_t k = ks[ki];
        const int R = k >= 16384 ? 7 : k >= 1024 ? 40 : k >= 64 ? 200 : 800;
        double res[8];
        for (int i = 0; i < 8; i++) res[i] = -1;
        /* evictor: k serObject per cycle */
        for (int pass = 0; pass < 4; pass++) {
            if (pass == 2 && !gpu) continue;
            rr_compat_set_route(pass == 0 ? RR_COMPAT_ROUTE_AUTO : pass == 1 ? RR_COMPAT_ROUTE_HOST : RR_COMPAT_ROUTE_GPU);
            for (int r = -3; r < R; r++) {
                const size_t v0 = ((size_t)(r + 3) * k) % (POOL - k + 1);
                const double t0 = now_us();
                if (pass == 0) {
                    for (size_t i = 0; i < k; i++) outs[i] = serObject(objs[v0 + i]);
                } else if (pass < 3) {
                    rr_compat_ser_batch(objs + v0, k, outs);
                } else {
                    for (size_t i = 0; i <= k; i++) offs[i] = hb.offsets[v0 + i] - hb.offsets[v0];
                    rro_store *st = rro_faithful_decode(hb.data + hb.offsets[v0], offs, k, NULL);
                    const double te = now_us();
                    rro_faithful_encode(st, cpu_out, 256u << 20, oo);
                    const double tf = now_us();
                    rro_store_free(st);
                    if (r >= 0) t[r] = tf - te;   /* (serObject's share: the encode) */
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
        for (int pass = 0; pass < 4; pass++) {
            if (pass == 2 && !gpu) continue;
            rr_compat_set_route(pass == 0 ? RR_COMPAT_ROUTE_AUTO : pass == 1 ? RR_COMPAT_ROUTE_HOST : RR_COMPAT_ROUTE_GPU);
            for (int r = -3; r < R; r++) {
                const size_t v0 = ((size_t)(r + 3) * k * 7) % (POOL - k + 1);
                unsigned sink = 0;
                for (size_t i = 0; i < k; i++) {   /* (a blob just read from RocksDB is in cache: touch it) */
                    bufs[i] = hb.data + hb.offsets[v0 + i];
                    lens[i] = hb.offsets[v0 + i + 1] - hb.offsets[v0 + i];
                    for (size_t j = 0; j < lens[i]; j += 64) sink += ((const uint8_t *)bufs[i])[j];
                }
                sink_all += sink;
                const double t0 = now_us();
                if (pass == 0) {
                    for (size_t i = 0; i < k; i++) tmp[i] = desObject(bufs[i], lens[i]);
                } else if (pass < 3) {
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
                rr_compat_set_route(RR_COMPAT_ROUTE_HOST);
                for (size_t i = 0; i < k; i++) {   /* the restored object serializes back to the blob */
                    sds s = serObject(tmp[i]);
                    if (sdslen(s) != lens[i] || memcmp(s, bufs[i], lens[i])) bad++;
                    sdsfree(s);
                    decrRefCount(tmp[i]);
                }
                rr_compat_set_route(pass == 0 ? RR_COMPAT_ROUTE_AUTO : pass == 1 ? RR_COMPAT_ROUTE_HOST : RR_COMPAT_ROUTE_GPU);
            }
            res[4 + pass] = median(t, R);
        }
        printf("%s{\"k\": %zu, \"evictor_serObject\": {\"shim_each\": %.2f, \"batch_host\": %.2f, \"batch_gpu\": %.2f, "
               "\"cpu\": %.2f}, \"restore_desObject\": {\"shim_each\": %.2f, \"batch_host\": %.2f, \"batch_gpu\": %.2f, "
               "\"cpu\": %.2f}}",
               ki ? ", " : "", k, res[0], res[1], res[2], res[3], res[4], res[5], res[6], res[7]);
        fflush(stdout);
    }
    printf("], \"roundtrip_bad\": %d}\n", bad);
    for (size_t i = 0; i < POOL; i++) decrRefCount(objs[i]);
    rr_host_batch_free(&hb);
    return bad ? 1 : 0;
}
