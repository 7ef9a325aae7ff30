// Latency probe (debug): the PoseOptimization trial solve (solve6 + se3_oplus_r of orb_pose.hip) on one
// thread, timed with clock64, inputs from global memory.  hipcc --offload-arch=gfx950 -O3 ...
#include "../../orb-slam3_byzyh_amd/csrc/orb_pose.hip"
#include <cstdio>
namespace {
__global__ void k_solve_probe(const double* U, const double* bb, const double* T0, double lambda, double* out, long long* cyc) {
    if (threadIdx.x != 0) return;
    double Uv[21], b[6], T[7], x[6];
    for (int k = 0; k < 21; ++k) Uv[k] = U[k];
    for (int k = 0; k < 6; ++k) b[k] = bb[k];
    for (int k = 0; k < 7; ++k) T[k] = T0[k];
    const long long c0 = clock64();
    for (int k = 0; k < 21; ++k) asm volatile("" : "+v"(Uv[k]));
    for (int k = 0; k < 6; ++k) asm volatile("" : "+v"(b[k]));
    for (int k = 0; k < 7; ++k) asm volatile("" : "+v"(T[k]));
    const bool ok = solve6(Uv, lambda, b, x);
    for (int k = 0; k < 6; ++k) asm volatile("" : "+v"(x[k]));
    const long long c1 = clock64();
    for (int k = 0; k < 6; ++k) x[k] *= 1e-3;
    for (int k = 0; k < 6; ++k) asm volatile("" : "+v"(x[k]));
    const long long c2 = clock64();
    for (int k = 0; k < 6; ++k) asm volatile("" : "+v"(x[k]));
    se3_oplus_r(T, x);
    for (int k = 0; k < 7; ++k) asm volatile("" : "+v"(T[k]));
    const long long c3 = clock64();
    for (int k = 0; k < 7; ++k) out[k] = T[k];
    out[7] = ok;
    cyc[0] = c1 - c0;
    cyc[1] = c3 - c2;
}
}
int main() {
    double hU[21], hb[6], hT[7] = {0.1, -0.2, 0.3, 0.01, 0.02, 0.03, 0.999};
    int k = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j) hU[k++] = (i == j ? 10.0 + i : 0.1 * (i + j));
    for (int i = 0; i < 6; ++i) hb[i] = 0.5 + i;
    double *U, *b, *T, *o;
    long long* c;
    hipMalloc(&U, sizeof hU); hipMalloc(&b, sizeof hb); hipMalloc(&T, sizeof hT); hipMalloc(&o, 8 * 8); hipMalloc(&c, 16);
    hipMemcpy(U, hU, sizeof hU, hipMemcpyHostToDevice);
    hipMemcpy(b, hb, sizeof hb, hipMemcpyHostToDevice);
    hipMemcpy(T, hT, sizeof hT, hipMemcpyHostToDevice);
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_solve_probe, dim3(1), dim3(64), 0, 0, U, b, T, 0.01, o, c);
        long long hc[2];
        hipMemcpy(hc, c, 16, hipMemcpyDeviceToHost);
        printf("solve6 %lld cycles, oplus %lld cycles\n", hc[0], hc[1]);
    }
    return 0;
}
int orbgpu_fail(int code, const char*) { return code; }
extern "C" int orb_device_count() { return 1; }
