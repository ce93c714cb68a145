// v_rcp_f64 accuracy probe: max relative error of the raw reciprocal and after one / two
// Newton steps against correctly rounded 1/x (host long double), over log-uniform x.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__global__ void k_rcp(const double* x, double* r0, double* r1, double* r2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = x[i];
    double y = __builtin_amdgcn_rcp(d);
    r0[i] = y;
    y = fma(y, fma(-d, y, 1.0), y);
    r1[i] = y;
    y = fma(y, fma(-d, y, 1.0), y);
    r2[i] = y;
}

int main() {
    const int n = 1 << 22;
    std::vector<double> x(n), r0(n), r1(n), r2(n);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-40.0, 40.0);
    for (int i = 0; i < n; ++i) x[i] = std::exp2(u(g)) * (1.0 + 1e-3 * (i % 7));
    double *dx, *d0, *d1, *d2;
    hipMalloc(&dx, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d2, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k_rcp<<<n / 256, 256>>>(dx, d0, d1, d2, n);
    hipMemcpy(r0.data(), d0, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(r1.data(), d1, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(r2.data(), d2, n * 8, hipMemcpyDeviceToHost);
    double e[3] = {0, 0, 0};
    long exact[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
        const double t = (double)(1.0L / (long double)x[i]);
        const double* r[3] = {&r0[i], &r1[i], &r2[i]};
        for (int k = 0; k < 3; ++k) {
            e[k] = std::fmax(e[k], std::fabs(*r[k] - t) / t);
            exact[k] += *r[k] == t;
        }
    }
    printf("rcp_f64 max rel err: raw %.3e (2^%.1f), 1 Newton %.3e, 2 Newton %.3e; correctly rounded: %ld %ld %ld of %d\n",
           e[0], std::log2(e[0]), e[1], e[2], exact[0], exact[1], exact[2], n);
    return 0;
}
