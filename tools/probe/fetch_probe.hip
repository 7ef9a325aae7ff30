// FETCH_SIZE calibration: read the same 256 MiB buffer with 16-, 4- and 1-byte loads per lane
// (fully coalesced, each byte once) so rocprofv3 --pmc FETCH_SIZE can be compared with the bytes
// actually read.  Usage under rocprofv3: fetch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ void k_read(const T* __restrict__ p, size_t n, unsigned* __restrict__ out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = p[i];
        if constexpr (sizeof(T) == 16) acc += v.x ^ v.y ^ v.z ^ v.w;
        else acc += (unsigned)v;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keeps the loads
}

int main() {
    const size_t bytes = 256ull << 20;
    unsigned char* d;
    unsigned* o;
    if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&o, 1 << 20) != hipSuccess) return 1;
    hipMemset(d, 1, bytes);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_read<uint4>, dim3(4096), dim3(256), 0, 0, (const uint4*)d, bytes / 16, o);
        hipLaunchKernelGGL(k_read<unsigned>, dim3(4096), dim3(256), 0, 0, (const unsigned*)d, bytes / 4, o);
        hipLaunchKernelGGL(k_read<unsigned char>, dim3(4096), dim3(256), 0, 0, (const unsigned char*)d, bytes, o);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("probe done: %zu bytes per kernel\n", bytes);
    return 0;
}
