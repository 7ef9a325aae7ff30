// FP64 instruction latencies / issue costs on gfx950, one wave on one SIMD (s_memtime cycles):
// dependent chains and independent streams of v_fma_f64, v_mul_f64, v_rsq_f64, v_rcp_f64, DPP64
// row broadcasts, v_mfma_f64_16x16x4, and one wave of the LocalBA Cholesky's 16x16 diagonal factor.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/f64_lat_probe tools/probe/f64_lat_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kIt = 256;

#define REP8(X) X X X X X X X X

__global__ void k_lat(long long* cyc, double* sink, double seed) {
    const int lane = threadIdx.x;
    double a = seed + lane * 1e-3, b = 1.0000001, c = 1e-9;
    double a1 = a + 1, a2 = a + 2, a3 = a + 3, a4 = a + 4, a5 = a + 5, a6 = a + 6, a7 = a + 7;
    long long t0, t1;
    int slot = 0;
    auto rec = [&](long long d) { if (lane == 0) cyc[slot] = d; ++slot; };
    // 0: dependent v_fma_f64
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) asm volatile(REP8("v_fma_f64 %0, %0, %1, %2\n\t") : "+v"(a) : "v"(b), "v"(c));
    t1 = clock64(); rec(t1 - t0);
    // 1: independent v_fma_f64 (8 chains)
    t0 = clock64();
    for (int i = 0; i < kIt; ++i)
        asm volatile("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\tv_fma_f64 %3, %3, %8, %9\n\t"
                     "v_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\tv_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9"
                     : "+v"(a), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
    t1 = clock64(); rec(t1 - t0);
    // 2: dependent v_mul_f64
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) asm volatile(REP8("v_mul_f64 %0, %0, %1\n\t") : "+v"(a) : "v"(b));
    t1 = clock64(); rec(t1 - t0);
    // 3: dependent v_rsq_f64
    double r = a * a + 1.0;
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) asm volatile(REP8("v_rsq_f64 %0, %0\n\t") : "+v"(r));
    t1 = clock64(); rec(t1 - t0);
    // 4: independent v_rsq_f64
    double r1 = r + 1, r2 = r + 2, r3 = r + 3;
    t0 = clock64();
    for (int i = 0; i < kIt; ++i)
        asm volatile("v_rsq_f64 %0, %0\n\tv_rsq_f64 %1, %1\n\tv_rsq_f64 %2, %2\n\tv_rsq_f64 %3, %3\n\t"
                     "v_rsq_f64 %0, %0\n\tv_rsq_f64 %1, %1\n\tv_rsq_f64 %2, %2\n\tv_rsq_f64 %3, %3"
                     : "+v"(r), "+v"(r1), "+v"(r2), "+v"(r3));
    t1 = clock64(); rec(t1 - t0);
    // 5: dependent v_rcp_f64
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) asm volatile(REP8("v_rcp_f64 %0, %0\n\t") : "+v"(r));
    t1 = clock64(); rec(t1 - t0);
    // 6: dependent v_mov_b64_dpp row_newbcast (+ s_nop 1 each)
    t0 = clock64();
    for (int i = 0; i < kIt; ++i)
        asm volatile(REP8("s_nop 1\n\tv_mov_b64_dpp %0, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t") : "+v"(a));
    t1 = clock64(); rec(t1 - t0);
    // 7: dependent v_fmac_f64_dpp (accumulator chain, + s_nop 1)
    t0 = clock64();
    for (int i = 0; i < kIt; ++i)
        asm volatile(REP8("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t")
                     : "+v"(a) : "v"(b), "v"(c));
    t1 = clock64(); rec(t1 - t0);
    // 8: independent v_fmac_f64_dpp, broadcast source written before the block (one s_nop)
    t0 = clock64();
    for (int i = 0; i < kIt; ++i)
        asm volatile("s_nop 1\n\t"
                     "v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf"
                     : "+v"(a), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
    t1 = clock64(); rec(t1 - t0);
    // 9: dependent MFMA f64 16x16x4 (one accumulator)
    f64x4 acc = {a, a1, a2, a3}, acc2 = {a4, a5, a6, a7}, acc3 = acc2 + 1.0, acc4 = acc2 + 2.0;
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, acc, 0, 0, 0);
    }
    t1 = clock64(); rec(t1 - t0);
    // 10: independent MFMA f64 (4 accumulators)
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, acc2, 0, 0, 0);
            acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, acc3, 0, 0, 0);
            acc4 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, acc4, 0, 0, 0);
        }
    }
    t1 = clock64(); rec(t1 - t0);
    // 11: dependent v_add_f64
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) asm volatile(REP8("v_add_f64 %0, %0, %1\n\t") : "+v"(a) : "v"(c));
    t1 = clock64(); rec(t1 - t0);
    // 12: dependent v_fma_f32 (reference point)
    float fa = (float)a, fb = 1.0000001f, fc = 1e-9f;
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) asm volatile(REP8("v_fma_f32 %0, %0, %1, %2\n\t") : "+v"(fa) : "v"(fb), "v"(fc));
    t1 = clock64(); rec(t1 - t0);
    // 13: dependent ds_bpermute + readback chain (cross-row broadcast)
    int iv = lane;
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) iv = __builtin_amdgcn_ds_bpermute((iv & 63) << 2, iv);
    }
    t1 = clock64(); rec(t1 - t0);
    // 14: dependent v_permlane16_swap (pairs, 64-bit value as in group4_sum) + add
    double pv = a;
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int2 q = __builtin_bit_cast(int2, pv);
            const auto x = __builtin_amdgcn_permlane16_swap(q.x, q.x, false, false);
            const auto y = __builtin_amdgcn_permlane16_swap(q.y, q.y, false, false);
            pv = __builtin_bit_cast(double, int2{(int)x[0], (int)y[0]}) + __builtin_bit_cast(double, int2{(int)x[1], (int)y[1]});
        }
    }
    t1 = clock64(); rec(t1 - t0);
    // 15: the same with v_permlane32_swap
    t0 = clock64();
    for (int i = 0; i < kIt; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int2 q = __builtin_bit_cast(int2, pv);
            const auto x = __builtin_amdgcn_permlane32_swap(q.x, q.x, false, false);
            const auto y = __builtin_amdgcn_permlane32_swap(q.y, q.y, false, false);
            pv = __builtin_bit_cast(double, int2{(int)x[0], (int)y[0]}) + __builtin_bit_cast(double, int2{(int)x[1], (int)y[1]});
        }
    }
    t1 = clock64(); rec(t1 - t0);
    // 16: LDS read-modify-write of one double + release fence + LDS atomic add (the contribution tail)
    __shared__ double sh[64];
    __shared__ int cnt;
    sh[lane] = 0.0;
    if (lane == 0) cnt = 0;
    __syncthreads();
    t0 = clock64();
    for (int i = 0; i < kIt * 8; ++i) {
        sh[lane] -= pv;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_fetch_add(&cnt, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    t1 = clock64(); rec(t1 - t0);
    sink[lane] = sh[lane] + pv + cnt + a + a1 + a2 + a3 + a4 + a5 + a6 + a7 + r + r1 + r2 + r3 + acc[0] + acc2[1] + acc3[2] + acc4[3] + fa + iv;
}

int main() {
    long long* d;
    double* s;
    hipMalloc(&d, 64 * sizeof(long long));
    hipMalloc(&s, 64 * sizeof(double));
    const char* names[] = {"v_fma_f64 dependent", "v_fma_f64 independent (8)", "v_mul_f64 dependent",
                           "v_rsq_f64 dependent", "v_rsq_f64 independent (4)", "v_rcp_f64 dependent",
                           "v_mov_b64_dpp bcast dep (+s_nop 1)", "v_fmac_f64_dpp dep (+s_nop 1)",
                           "v_fmac_f64_dpp independent (8, one s_nop)", "mfma_f64_16x16x4 dependent",
                           "mfma_f64_16x16x4 independent (4 acc)", "v_add_f64 dependent", "v_fma_f32 dependent",
                           "ds_bpermute dependent", "permlane16_swap pair + add_f64 (dep)",
                           "permlane32_swap pair + add_f64 (dep)", "LDS RMW f64 + release fence + LDS atomic"};
    const int n = sizeof(names) / sizeof(names[0]);
    long long h[64];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, d, s, 1.5);
        hipMemcpy(h, d, n * sizeof(long long), hipMemcpyDeviceToHost);
    }
    for (int i = 0; i < n; ++i) printf("%-45s %7.2f cycles/instr\n", names[i], (double)h[i] / (kIt * 8));
    return 0;
}
