// Accuracy of v_rsq_f64 and of one / two Newton steps against the host's correctly rounded 1/sqrt.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
__global__ void k(const double* x, double* r0, double* r1, double* r2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    double y = __builtin_amdgcn_rsq(v);
    r0[i] = y;
    const double h = 0.5 * v;
    y = y * __builtin_fma(-h, y * y, 1.5);
    r1[i] = y;
    y = y * __builtin_fma(-h, y * y, 1.5);
    r2[i] = y;
}
int main() {
    const int n = 1 << 22;
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> e(-30.0, 30.0), m(1.0, 2.0);
    std::vector<double> x(n), a(n), b(n), c(n);
    for (auto& v : x) v = std::ldexp(m(g), (int)e(g));
    double *dx, *da, *db, *dc;
    hipMalloc(&dx, n * 8); hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dc, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, da, db, dc, n);
    hipMemcpy(a.data(), da, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), db, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, n * 8, hipMemcpyDeviceToHost);
    double m0 = 0, m1 = 0, m2 = 0;
    for (int i = 0; i < n; ++i) {
        const long double ref = 1.0L / sqrtl((long double)x[i]);
        m0 = std::fmax(m0, (double)fabsl((a[i] - ref) / ref));
        m1 = std::fmax(m1, (double)fabsl((b[i] - ref) / ref));
        m2 = std::fmax(m2, (double)fabsl((c[i] - ref) / ref));
    }
    printf("max rel err: rsq %.3g  1 newton %.3g  2 newton %.3g  (ulp 1.1e-16)\n", m0, m1, m2);
    return 0;
}
