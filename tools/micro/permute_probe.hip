// ds_permute_b32 semantics probe (diagnostics, GPU box): which value does a lane no other lane
// writes to receive?  Build: hipcc --offload-arch=gfx950 -O2 tools/micro/permute_probe.hip -o tools/micro/permute_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(int *out) {
    const int lane = threadIdx.x;
    // lanes 0..15 send 1 to lane (lane + 3) % 16 only when lane is even; everyone else sends nothing
    const int dst = (lane < 16 && (lane & 1) == 0) ? ((lane + 3) & 15) : lane;
    const int val = (lane < 16 && (lane & 1) == 0) ? 100 + lane : 7;
    int r;
    if (lane < 16 && (lane & 1) == 0) r = __builtin_amdgcn_ds_permute(dst * 4, val);
    else r = __builtin_amdgcn_ds_permute(dst * 4, val);
    out[lane] = r;
    // the same with inactive senders (exec off): only even lanes of row 0 execute the permute
    int s = -1;
    if (lane < 16 && (lane & 1) == 0) s = __builtin_amdgcn_ds_permute(((lane + 3) & 15) * 4, 200 + lane);
    out[64 + lane] = s;
    int t = 0x5a5a;
    t = (lane < 16 && (lane & 1) == 0) ? __builtin_amdgcn_ds_permute(((lane + 3) & 15) * 4, 300 + lane) : t;
    out[128 + lane] = t;
}
int main() {
    int *d, h[192];
    hipMalloc(&d, sizeof(h));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int j = 0; j < 3; ++j) {
        for (int i = 0; i < 20; ++i) printf("%d ", h[64 * j + i]);
        printf("\n");
    }
    return 0;
}
