// Cost of a dependent kernel boundary on the device: a HIP graph of N back-to-back launches of an
// (almost) empty kernel, timed with events, for a few grid sizes; and a persistent kernel that
// crosses N grid-wide barriers (atomic counter + spin) instead.  Build:
//   hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o build/launch_cost
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_empty(const int* __restrict__ gate, int* out) {
    if (*gate) return;
    if (threadIdx.x == 0 && blockIdx.x == 0xFFFFFF) out[0] = 1;
}

// grid barrier: every block arrives on a monotonically increasing counter and waits for the
// generation to complete (vector atomics, global scope)
__global__ void k_barriers(unsigned* counter, int n, int* out) {
    const unsigned nb = gridDim.x;
    for (int i = 1; i <= n; ++i) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            atomicAdd(counter, 1u);
            for (int spin = 0; spin < (1 << 22) &&  // bounded: a non-resident grid ends instead of hanging
                               __hip_atomic_load(counter, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < nb * (unsigned)i;
                 ++spin)
                __builtin_amdgcn_s_sleep(1);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && blockIdx.x == 0xFFFFFF) out[0] = 1;
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int *gate, *out;
    unsigned* counter;
    hipMalloc(&gate, 4);
    hipMalloc(&out, 4);
    hipMalloc(&counter, 4);
    hipMemset(gate, 0, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int N = 200;
    for (int blocks : {1, 64, 256, 1024}) {
        for (int gated : {0, 1}) {
            hipMemsetAsync(gate, gated, 4, s);
            hipGraph_t g;
            hipGraphExec_t ge;
            hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
            for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, s, gate, out);
            hipStreamEndCapture(s, &g);
            hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            float best = 1e9f;
            for (int rep = 0; rep < 5; ++rep) {
                hipEventRecord(a, s);
                hipGraphLaunch(ge, s);
                hipEventRecord(b, s);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            printf("graph of %d launches, %4d blocks x 256, %s: %.2f us per launch\n", N, blocks,
                   gated ? "gated off" : "empty    ", best * 1e3f / N);
            hipGraphExecDestroy(ge);
            hipGraphDestroy(g);
        }
    }
    for (int blocks : {64, 256}) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
            hipMemsetAsync(counter, 0, 4, s);
            hipEventRecord(a, s);
            hipLaunchKernelGGL(k_barriers, dim3(blocks), dim3(256), 0, s, counter, N, out);
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        printf("persistent kernel, %d blocks, %d grid barriers: %.2f us per barrier\n", blocks, N, best * 1e3f / N);
    }
    return 0;
}
