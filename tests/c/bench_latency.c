/*
 * bench_latency.c — per-call latency of the legacy one-value signatures (rock_serdes.h:47-49)
 * the unchanged rock.c / rock_hotkey.c call: desObject per restored key (rock.c:468) and
 * serObject per evicted key on the main thread (rock.c:691, from the <= 64-pick loop at
 * rock_hotkey.c:347).  The shim (redrock_old_amd/compat) runs them on its host codec by default
 * (what rock.c gets) and, forced, on the GPU route; beside them (GPU only) the batch C-ABI with
 * one value per call, with and without the one-launch small-batch kernels (RR_CTX_NO_SMALL), and
 * the faithful CPU restatement of the reference (oracle/rro_faithful.c, test infrastructure) per
 * value.  Prints one JSON line (diagnostics).
 *
 * usage: bench_latency [config] [values]
 */
#include <math.h>
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
/* median and mean of the per-call times */
static void stats(double *t, size_t k, double *med, double *mean) {
    double s = 0;
    for (size_t i = 0; i < k; i++) s += t[i];
    qsort(t, k, sizeof(double), cmpd);
    *med = t[k / 2];
    *mean = s / (double)k;
}

/* the shim's one-value signatures over k values on the current route: desObject, then serObject
 * of what it built (which must give the blob back) */
static int shim_calls(const rr_host_batch *hb, size_t k, double *t, robj **objs, double *med, double *mean) {
    for (size_t i = 0; i < 50 && i < k; i++)   /* warm-up (a GPU route's context, its pinned buffer) */
        decrRefCount(desObject(hb->data + hb->offsets[i], hb->offsets[i + 1] - hb->offsets[i]));
    for (size_t i = 0; i < k; i++) {
        const double t0 = now_us();
        objs[i] = desObject(hb->data + hb->offsets[i], hb->offsets[i + 1] - hb->offsets[i]);
        t[i] = now_us() - t0;
    }
    stats(t, k, &med[0], &mean[0]);
    int bad = 0;
    for (size_t i = 0; i < k; i++) {
        const double t0 = now_us();
        sds s = serObject(objs[i]);
        t[i] = now_us() - t0;
        const size_t len = hb->offsets[i + 1] - hb->offsets[i];
        if (sdslen(s) != len || memcmp(s, hb->data + hb->offsets[i], len)) bad++;   /* (generated lru: 24 bits) */
        sdsfree(s);
    }
    stats(t, k, &med[1], &mean[1]);
    for (size_t i = 0; i < k; i++) decrRefCount(objs[i]);
    return bad;
}

int main(int argc, char **argv) {
    const int cfg = argc > 1 ? atoi(argv[1]) : 4;
    const size_t k = argc > 2 ? (size_t)atol(argv[2]) : 2000;
    rr_host_batch hb;
    if (rr_gen_batch(cfg, k, rr_gen_default_seed(cfg), &hb) != RR_API_OK) return 2;
    double *t = malloc(sizeof(double) * k), *t2 = malloc(sizeof(double) * k);
    robj **objs = malloc(sizeof(robj *) * k);
    double med[8], mean[8];
    for (int i = 0; i < 8; i++) med[i] = mean[i] = -1;

    /* the shim as rock.c calls it (default routing: the host codec), then forced onto the GPU */
    int bad = shim_calls(&hb, k, t, objs, &med[0], &mean[0]);
    rr_ctx *ctx = NULL;
    const int gpu = rr_ctx_create(0, &ctx) == RR_API_OK;
    if (gpu) {
        rr_compat_set_route(RR_COMPAT_ROUTE_GPU);
        bad += shim_calls(&hb, k, t, objs, &med[6], &mean[6]);
        rr_compat_set_route(RR_COMPAT_ROUTE_AUTO);

        /* the batch C-ABI, one value per call: one-launch kernels, then the pipeline */
        rr_value v;
        rr_elem *el = malloc(sizeof(rr_elem) * 70000);
        uint8_t *arena = malloc(1 << 20);
        for (int mode = 0; mode < 2; mode++) {
            rr_ctx_set_options(ctx, mode ? RR_CTX_NO_SMALL : 0);
            for (size_t i = 0; i < k + 50; i++) {
                const size_t j = i % k, len = hb.offsets[j + 1] - hb.offsets[j];
                const uint64_t o[2] = {0, len};
                rr_totals tt;
                const double t0 = now_us();
                if (rr_decode_batch_host(ctx, hb.data + hb.offsets[j], o, 1, &v, el, rr_decode_elem_bound(1, len), arena,
                                         &tt))
                    return 4;
                if (i >= 50) t[i - 50] = now_us() - t0;
            }
            stats(t, k, &med[2 + mode], &mean[2 + mode]);
        }
        rr_ctx_destroy(ctx);
    }

    /* the faithful CPU restatement (the reference's allocation pattern), one value per call */
    uint8_t *out = malloc(1 << 20);
    for (size_t i = 0; i < k; i++) {
        const uint64_t o[2] = {0, hb.offsets[i + 1] - hb.offsets[i]};
        uint64_t nb = 0;
        const double t0 = now_us();
        rro_store *st = rro_faithful_decode(hb.data + hb.offsets[i], o, 1, &nb);
        t[i] = now_us() - t0;
        uint64_t oo[2];
        const double t1 = now_us();
        rro_faithful_encode(st, out, 1 << 20, oo);
        t2[i] = now_us() - t1;
        rro_store_free(st);
    }
    stats(t, k, &med[4], &mean[4]);
    stats(t2, k, &med[5], &mean[5]);
    printf("{\"config\": %d, \"values\": %zu, \"bytes\": %llu, \"roundtrip_bad\": %d, \"gpu\": %s, "
           "\"shim_desObject_us\": {\"median\": %.3f, \"mean\": %.3f}, "
           "\"shim_serObject_us\": {\"median\": %.3f, \"mean\": %.3f}, "
           "\"shim_gpu_route_desObject_us\": {\"median\": %.2f, \"mean\": %.2f}, "
           "\"shim_gpu_route_serObject_us\": {\"median\": %.2f, \"mean\": %.2f}, "
           "\"decode_host_n1_small_us\": {\"median\": %.2f, \"mean\": %.2f}, "
           "\"decode_host_n1_pipeline_us\": {\"median\": %.2f, \"mean\": %.2f}, "
           "\"cpu_faithful_desObject_us\": {\"median\": %.3f, \"mean\": %.3f}, "
           "\"cpu_faithful_serObject_us\": {\"median\": %.3f, \"mean\": %.3f}}\n",
           cfg, k, (unsigned long long)hb.bytes, bad, gpu ? "true" : "false", med[0], mean[0], med[1], mean[1], med[6],
           mean[6], med[7], mean[7], med[2], mean[2], med[3], mean[3], med[4], mean[4], med[5], mean[5]);
    rr_host_batch_free(&hb);
    return bad ? 1 : 0;
}
