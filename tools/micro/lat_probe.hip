// Latency probe for the per-value path (diagnostics, GPU box): what one small call costs, piece
// by piece.  Build: hipcc --offload-arch=gfx950 -O2 -I include tools/micro/lat_probe.hip
//   -L redrock_old_amd -lrr_serdes -Wl,-rpath,$PWD/redrock_old_amd -o tools/micro/lat_probe
// Prints one JSON line of medians in microseconds.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/rr_serdes.h"
#include "../../redrock_old_amd/csrc/rr_kernels.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}
static int cmpd(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}
static double med(double *t, int k) {
    qsort(t, k, sizeof(double), cmpd);
    return t[k / 2];
}

__global__ void empty_kernel() {}
__global__ __launch_bounds__(1024) void big_empty_kernel(uint32_t *p) {
    __shared__ uint32_t big[35000];
    big[threadIdx.x * 34] = threadIdx.x;
    __syncthreads();
    if (p && threadIdx.x == 0) p[0] = big[5];
}
__global__ void flag_kernel(volatile uint32_t *flag, uint32_t seq) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        *flag = seq;
    }
}

int main() {
    const int K = 2000;
    double *t = (double *)malloc(sizeof(double) * K);
    hipStream_t s;
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // 1. empty launch + stream sync
    for (int i = 0; i < 50; ++i) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s); CK(hipStreamSynchronize(s)); }
    for (int i = 0; i < K; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        CK(hipStreamSynchronize(s));
        t[i] = now_us() - t0;
    }
    const double launch_sync = med(t, K);
    // 2. the launch call alone (then a sync outside the timing)
    for (int i = 0; i < K; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        t[i] = now_us() - t0;
        CK(hipStreamSynchronize(s));
    }
    const double launch_only = med(t, K);
    // 3. launch + spin on a host-mapped flag the kernel writes
    uint32_t *hf, *df;
    CK(hipHostMalloc((void **)&hf, 64, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void **)&df, hf, 0));
    *(volatile uint32_t *)hf = 0;
    for (int i = 0; i < K; ++i) {
        const uint32_t seq = (uint32_t)i + 1;
        const double t0 = now_us();
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, df, seq);
        while (*(volatile uint32_t *)hf != seq) {}
        t[i] = now_us() - t0;
    }
    CK(hipStreamSynchronize(s));
    const double launch_spin = med(t, K);
    // 4. the one-launch decode kernel on a config-4 value, device buffers (kernel + sync)
    rr_host_batch hb;
    if (rr_gen_batch(4, 64, rr_gen_default_seed(4), &hb) != RR_API_OK) return 3;
    const uint64_t len = hb.offsets[1] - hb.offsets[0];
    uint8_t *dblob;
    uint64_t *doff;
    rr_value *dval;
    rr_elem *del;
    rr_totals *dtot;
    CK(hipMalloc((void **)&dblob, 1 << 16));
    CK(hipMalloc((void **)&doff, 16));
    CK(hipMalloc((void **)&dval, 16));
    CK(hipMalloc((void **)&del, 1 << 16));
    CK(hipMalloc((void **)&dtot, 64));
    const uint64_t o[2] = {0, len};
    CK(hipMemcpy(dblob, hb.data + hb.offsets[0], len, hipMemcpyHostToDevice));
    CK(hipMemcpy(doff, o, 16, hipMemcpyHostToDevice));
    for (int i = 0; i < K; ++i) {
        const double t0 = now_us();
        CK(rr_launch_decode_small(dblob, doff, 1, dval, del, 4096, NULL, (len + 15) & ~15ull, dtot, NULL, 0, s));
        CK(hipStreamSynchronize(s));
        t[i] = now_us() - t0;
    }
    const double small_dev = med(t, K);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // kernel time alone (events)
    for (int i = 0; i < K; ++i) {
        CK(hipEventRecord(e0, s));
        CK(rr_launch_decode_small(dblob, doff, 1, dval, del, 4096, NULL, (len + 15) & ~15ull, dtot, NULL, 0, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[i] = ms * 1e3;
    }
    const double small_kernel = med(t, K);
    // 4a. event time of empty kernels: one wave, and 1024 threads with 140 KB of LDS
    double ev_empty[2];
    for (int kk = 0; kk < 2; ++kk) {
        for (int i = 0; i < K; ++i) {
            CK(hipEventRecord(e0, s));
            if (kk == 0) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
            else hipLaunchKernelGGL(big_empty_kernel, dim3(1), dim3(1024), 0, s, (uint32_t *)NULL);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[i] = ms * 1e3;
        }
        ev_empty[kk] = med(t, K);
    }
    // 4b. the kernel alone per config (values 0..7 of each, device buffers)
    double per_cfg[3];
    const int cfgs[3] = {1, 3, 4};
    for (int ci = 0; ci < 3; ++ci) {
        rr_host_batch hc;
        if (rr_gen_batch(cfgs[ci], 8, rr_gen_default_seed(cfgs[ci]), &hc) != RR_API_OK) return 3;
        int m = 0;
        for (int vi = 0; vi < 8; ++vi) {
            const uint64_t l = hc.offsets[vi + 1] - hc.offsets[vi];
            if (l > 60000) continue;
            const uint64_t oo[2] = {0, l};
            CK(hipMemcpy(dblob, hc.data + hc.offsets[vi], l, hipMemcpyHostToDevice));
            CK(hipMemcpy(doff, oo, 16, hipMemcpyHostToDevice));
            for (int i = 0; i < 200; ++i) {
                CK(hipEventRecord(e0, s));
                CK(rr_launch_decode_small(dblob, doff, 1, dval, del, 4096, NULL, (l + 15) & ~15ull, dtot, NULL, 0, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                t[m++] = ms * 1e3;
            }
        }
        per_cfg[ci] = med(t, m);
        rr_host_batch_free(&hc);
    }
    CK(hipMemcpy(dblob, hb.data + hb.offsets[0], len, hipMemcpyHostToDevice));
    CK(hipMemcpy(doff, o, 16, hipMemcpyHostToDevice));
    // 4c. the one-launch encode kernel of the same value (its flat form from the decode above),
    //     device buffers, HIP events; and a host-mapped completion word instead (launch + spin)
    CK(rr_launch_decode_small(dblob, doff, 1, dval, del, 4096, NULL, (len + 15) & ~15ull, dtot, NULL, 0, s));
    CK(hipStreamSynchronize(s));
    rr_totals dt;
    CK(hipMemcpy(&dt, dtot, sizeof dt, hipMemcpyDeviceToHost));
    uint8_t *dout;
    uint64_t *dooff;
    CK(hipMalloc((void **)&dout, 1 << 16));
    CK(hipMalloc((void **)&dooff, 16));
    for (int i = 0; i < K; ++i) {
        CK(hipEventRecord(e0, s));
        CK(rr_launch_encode_small(dval, del, dt.n_elems, dblob, len, 1, dout, (len + 15) & ~15ull, dooff, dtot, NULL, 0, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[i] = ms * 1e3;
    }
    const double enc_kernel = med(t, K);
    for (int i = 0; i < K; ++i) {
        const uint32_t seq = (uint32_t)(K + i) + 1;
        const double t0 = now_us();
        CK(rr_launch_encode_small(dval, del, dt.n_elems, dblob, len, 1, dout, (len + 15) & ~15ull, dooff, dtot, df, seq, s));
        while (*(volatile uint32_t *)hf != seq) {}
        t[i] = now_us() - t0;
    }
    CK(hipStreamSynchronize(s));
    const double enc_spin = med(t, K);
    for (int i = 0; i < K; ++i) {
        const uint32_t seq = (uint32_t)(2 * K + i) + 1;
        const double t0 = now_us();
        CK(rr_launch_decode_small(dblob, doff, 1, dval, del, 4096, NULL, (len + 15) & ~15ull, dtot, df, seq, s));
        while (*(volatile uint32_t *)hf != seq) {}
        t[i] = now_us() - t0;
    }
    CK(hipStreamSynchronize(s));
    const double dec_spin = med(t, K);
    // 5. the same through the host entry point (pinned mapped staging)
    rr_ctx *ctx;
    if (rr_ctx_create(0, &ctx) != RR_API_OK) return 4;
    rr_value v;
    rr_elem *el = (rr_elem *)malloc(1 << 16);
    rr_totals tt;
    for (int i = 0; i < 50; ++i) rr_decode_batch_host(ctx, hb.data + hb.offsets[0], o, 1, &v, el, 4096, NULL, &tt);
    for (int i = 0; i < K; ++i) {
        const double t0 = now_us();
        rr_decode_batch_host(ctx, hb.data + hb.offsets[0], o, 1, &v, el, 4096, NULL, &tt);
        t[i] = now_us() - t0;
    }
    const double host_small = med(t, K);
    printf("{\"empty_launch_sync_us\": %.2f, \"launch_call_us\": %.2f, \"empty_launch_spin_us\": %.2f, "
           "\"decode_small_device_us\": %.2f, \"decode_small_kernel_event_us\": %.2f, \"decode_host_n1_us\": %.2f, "
           "\"value_bytes\": %llu, \"kernel_us_cfg1\": %.2f, \"kernel_us_cfg3\": %.2f, \"kernel_us_cfg4\": %.2f, "
           "\"empty_event_us\": %.2f, \"empty1024_lds_event_us\": %.2f, \"encode_small_kernel_event_us\": %.2f, "
           "\"encode_small_device_spin_us\": %.2f, \"decode_small_device_spin_us\": %.2f}\n",
           launch_sync, launch_only, launch_spin, small_dev, small_kernel, host_small, (unsigned long long)len,
           per_cfg[0], per_cfg[1], per_cfg[2], ev_empty[0], ev_empty[1], enc_kernel, enc_spin, dec_spin);
    return 0;
}
