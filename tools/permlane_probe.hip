// Lane mapping of v_permlane16_swap / v_permlane32_swap (gfx950): a = lane, b = 100 + lane; prints
// which source value each lane of both results holds.
//   hipcc --offload-arch=gfx950 -O2 tools/permlane_probe.hip -o build/permlane_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k(unsigned* o) {
    const unsigned x = threadIdx.x, y = 100 + threadIdx.x;
    auto r16 = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    auto r32 = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    o[threadIdx.x] = r16[0];
    o[64 + threadIdx.x] = r16[1];
    o[128 + threadIdx.x] = r32[0];
    o[192 + threadIdx.x] = r32[1];
}

int main() {
    unsigned* d;
    unsigned h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[4] = {"p16 vdst", "p16 src", "p32 vdst", "p32 src"};
    for (int t = 0; t < 4; ++t) {
        printf("%s:", names[t]);
        for (int l = 0; l < 64; l += 4) printf(" %u", h[64 * t + l]);
        printf("\n");
    }
    return 0;
}
