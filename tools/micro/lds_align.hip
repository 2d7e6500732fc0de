// Microbenchmark: LDS store throughput for aligned vs misaligned 16/8/4-byte stores and byte
// stores (diagnostics for the encode window image).  Usage: ./lds_align
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t *out, int iters, int mis) {
    __shared__ uint4 img4[2048];
    uint8_t *img = reinterpret_cast<uint8_t *>(img4);
    const uint32_t t = threadIdx.x;
    uint4 v = make_uint4(t, t * 3, t * 5, t * 7);
    for (int i = 0; i < iters; ++i) {
        const uint32_t base = ((t * 97 + i * 61) & 1023) * 16 + mis;   // scattered 16-B slots
        if (MODE == 0) __builtin_memcpy(img + base, &v, 16);
        else if (MODE == 1) __builtin_memcpy(img + base, &v.x, 8);
        else if (MODE == 2) __builtin_memcpy(img + base, &v.x, 4);
        else {
#pragma unroll
            for (int b = 0; b < 16; ++b) img[base + b] = (uint8_t)(v.x >> b);
        }
        v.x += 1;
        __builtin_amdgcn_s_waitcnt(0xc07f);
    }
    __syncthreads();
    out[blockIdx.x * 256 + t] = img4[t].x;
}

template <int MODE>
static float run(int mis) {
    uint32_t *d;
    hipMalloc(&d, 4096 * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k<MODE>, dim3(4096), dim3(256), 0, 0, d, 256, mis);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<MODE>, dim3(4096), dim3(256), 0, 0, d, 256, mis);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipFree(d);
    return ms;
}

int main() {
    const char *names[] = {"b128 (16 B)", "b64 (8 B)", "b32 (4 B)", "16 x b8"};
    for (int mis : {0, 1, 4, 8}) {
        printf("offset %d: %s %.3f ms  %s %.3f ms  %s %.3f ms  %s %.3f ms\n", mis, names[0], run<0>(mis), names[1],
               run<1>(mis), names[2], run<2>(mis), names[3], run<3>(mis));
    }
    return 0;
}
