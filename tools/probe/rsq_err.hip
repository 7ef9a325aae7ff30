// Accuracy of v_rsq_f64 alone and with one / two Newton steps, against 1/sqrt in long double on the host.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
__global__ void k(const double* x, double* o, int n) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double v = x[i], y = __builtin_amdgcn_rsq(v), h = 0.5 * v;
    double y1 = y * __builtin_fma(-h, y * y, 1.5);
    double y2 = y1 * __builtin_fma(-h, y1 * y1, 1.5);
    o[3 * i] = y; o[3 * i + 1] = y1; o[3 * i + 2] = y2;
}
int main() {
    const int n = 1 << 20;
    std::vector<double> x(n), o(3 * n);
    std::mt19937_64 r(1);
    std::uniform_real_distribution<double> u(-30, 30);
    for (auto& v : x) v = std::exp(u(r));
    double *dx, *dout;
    hipMalloc(&dx, n * 8); hipMalloc(&dout, 3 * n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
    hipMemcpy(o.data(), dout, 3 * n * 8, hipMemcpyDeviceToHost);
    double e[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
        long double ref = 1.0L / std::sqrt((long double)x[i]);
        for (int k2 = 0; k2 < 3; ++k2) e[k2] = std::fmax(e[k2], (double)std::fabs((o[3 * i + k2] - ref) / ref));
    }
    std::printf("max rel err: rsq %.3g (2^%.1f), 1 NR %.3g (2^%.1f), 2 NR %.3g (2^%.1f)\n", e[0], std::log2(e[0]), e[1],
                std::log2(e[1]), e[2], std::log2(e[2]));
    return 0;
}
