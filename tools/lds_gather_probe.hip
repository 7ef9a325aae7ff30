// LDS gather cost of k_describe's per-sample reads (4 row-pair words of one column) in three layouts:
//   A  row-major pairs (word = pair * 40 + col): 2 x ds_read2_b32 per sample (the current layout)
//   B  column-major pairs (word = col * 24 + pair): 2 x ds_read_b64 at any dword (4-byte aligned only)
//   C  as B with the address rounded down to 8 bytes (aligned reference for B's timing)
//   D  one ds_read_u8 per sample (a fully blurred byte patch, 40 B rows)
// 8 half-wave regions of 880 words per 256-thread block (k_describe's 28 KB), random samples in
// [0, 37)^2 per lane; every variant checks its first samples against plain dword reads.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/lds_gather_probe.hip -o build/lds_gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kWords = 880, kIters = 256;

__device__ __forceinline__ unsigned lcg(unsigned& s) { s = s * 1664525u + 1013904223u; return s >> 8; }

template <int V>
__global__ __launch_bounds__(256) void k_gather(unsigned* out, unsigned* bad) {
    __shared__ __attribute__((aligned(16))) unsigned lds[8 * kWords];
    for (int i = threadIdx.x; i < 8 * kWords; i += 256) lds[i] = i * 2654435761u;
    __syncthreads();
    const int half = threadIdx.x >> 5;
    const unsigned base = half * kWords * 4;  // bytes
    unsigned st = blockIdx.x * 256 + threadIdx.x + 12345u, acc = 0, err = 0;
    for (int it = 0; it < kIters; it += 4) {
        unsigned ad[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned r = lcg(st) % 37u, c = lcg(st) % 37u;
            if (V == 0) ad[k] = base + 4 * ((r >> 1) * 40 + c);
            else if (V == 1) ad[k] = base + 4 * (c * 24 + (r >> 1));
            else if (V == 2) ad[k] = base + 4 * ((c * 24 + (r >> 1)) & ~1u);
            else ad[k] = base + r * 40 + c;
        }
        if (V == 0) {
            uint2 a[4], b[4];
            asm volatile(
                "ds_read2_b32 %0, %8 offset1:40\n ds_read2_b32 %1, %8 offset0:80 offset1:120\n"
                "ds_read2_b32 %2, %9 offset1:40\n ds_read2_b32 %3, %9 offset0:80 offset1:120\n"
                "ds_read2_b32 %4, %10 offset1:40\n ds_read2_b32 %5, %10 offset0:80 offset1:120\n"
                "ds_read2_b32 %6, %11 offset1:40\n ds_read2_b32 %7, %11 offset0:80 offset1:120\n"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(a[0]), "=&v"(b[0]), "=&v"(a[1]), "=&v"(b[1]), "=&v"(a[2]), "=&v"(b[2]), "=&v"(a[3]), "=&v"(b[3])
                : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]));
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc += a[k].x ^ a[k].y ^ b[k].x ^ b[k].y;
                const unsigned w = ad[k] >> 2;
                if (it == 0) err |= (a[k].x != lds[w]) | (a[k].y != lds[w + 40]) | (b[k].x != lds[w + 80]) | (b[k].y != lds[w + 120]);
            }
        } else if (V == 1 || V == 2) {
            uint2 a[4], b[4];
            asm volatile(
                "ds_read_b64 %0, %8\n ds_read_b64 %1, %8 offset:8\n"
                "ds_read_b64 %2, %9\n ds_read_b64 %3, %9 offset:8\n"
                "ds_read_b64 %4, %10\n ds_read_b64 %5, %10 offset:8\n"
                "ds_read_b64 %6, %11\n ds_read_b64 %7, %11 offset:8\n"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(a[0]), "=&v"(b[0]), "=&v"(a[1]), "=&v"(b[1]), "=&v"(a[2]), "=&v"(b[2]), "=&v"(a[3]), "=&v"(b[3])
                : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]));
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc += a[k].x ^ a[k].y ^ b[k].x ^ b[k].y;
                const unsigned w = ad[k] >> 2;
                if (it == 0) err |= (a[k].x != lds[w]) | (a[k].y != lds[w + 1]) | (b[k].x != lds[w + 2]) | (b[k].y != lds[w + 3]);
            }
        } else {
            unsigned a[4];
            asm volatile(
                "ds_read_u8 %0, %4\n ds_read_u8 %1, %5\n ds_read_u8 %2, %6\n ds_read_u8 %3, %7\n"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3])
                : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]));
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc += a[k];
                if (it == 0) err |= a[k] != ((lds[ad[k] >> 2] >> (8 * (ad[k] & 3))) & 0xffu);
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (err) bad[0] = 1;
}

int main() {
    const int blocks = 4096;
    unsigned *out, *bad;
    hipMalloc(&out, blocks * 256 * 4);
    hipMalloc(&bad, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[4] = {"A row-major 2x ds_read2_b32", "B col-major 2x ds_read_b64 (4-B aligned)",
                            "C col-major 2x ds_read_b64 (8-B aligned)", "D 1x ds_read_u8"};
    for (int v = 0; v < 4; ++v) {
        hipMemset(bad, 0, 4);
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(e0, 0);
            if (v == 0) hipLaunchKernelGGL(k_gather<0>, dim3(blocks), dim3(256), 0, 0, out, bad);
            if (v == 1) hipLaunchKernelGGL(k_gather<1>, dim3(blocks), dim3(256), 0, 0, out, bad);
            if (v == 2) hipLaunchKernelGGL(k_gather<2>, dim3(blocks), dim3(256), 0, 0, out, bad);
            if (v == 3) hipLaunchKernelGGL(k_gather<3>, dim3(blocks), dim3(256), 0, 0, out, bad);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        unsigned hb = 0;
        hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
        const double samples = (double)blocks * 256 * kIters;
        printf("%-44s %8.3f ms  %6.3f ns/sample/CU-equiv  mismatch=%u\n", names[v], best, best * 1e6 / samples * 256, hb);
    }
    return 0;
}
