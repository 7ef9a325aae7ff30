// Cost of wave-uniform skipped blocks (s_cbranch taken) on gfx950: 16 unrolled `if (uniform) {work}` with
// the condition false, vs. true, one wave.  Build: hipcc --offload-arch=gfx950 -O3 -o build/probe/branch_probe tools/probe/branch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(long long* cyc, double* sink, int mask, int reps) {
    const int lane = threadIdx.x;
    double v[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) v[s] = lane + s;
    const int m = __builtin_amdgcn_readfirstlane(mask);
    long long t0 = clock64();
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            if ((m >> s) & 1) {
                v[s] = __builtin_fma(v[s], 1.0000001, 1e-9);
                asm volatile("" : "+v"(v[s]));
            }
        }
        asm volatile("" ::: "memory");
    }
    long long t1 = clock64();
    double acc = 0;
#pragma unroll
    for (int s = 0; s < 16; ++s) acc += v[s];
    sink[lane] = acc;
    if (lane == 0) cyc[0] = t1 - t0;
}
int main() {
    long long* d; double* s; long long h;
    (void)hipMalloc(&d, 8); (void)hipMalloc(&s, 64 * 8);
    int masks[] = {0, 0xFFFF, 0x5555, 0x0001};
    for (int mi = 0; mi < 4; ++mi) {
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k, 1, 64, 0, 0, d, s, masks[mi], 1000);
        (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
        printf("mask %04x: %.1f cycles per 16-slot pass\n", masks[mi], h / 1000.0);
    }
    return 0;
}
