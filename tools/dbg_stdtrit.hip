// Debug probe for cvq::stdtrit on the device (prints CF / log-CDF internals).
#include <cstdio>
#include <vector>
#include "../copula-msm-and-copula-garch-var_amd/csrc/cvq_common.h"
using namespace cvq;
namespace cvq { void set_error(const std::string&) {} }
__global__ void probe(TConst k, double t, double* out) {
    double lnF, lpdf;
    t_lower_logs(k, t, &lnF, &lpdf);
    const double x = k.nu / (k.nu + t * t);
    out[0] = lnF; out[1] = lpdf; out[2] = x; out[3] = ibeta_cf(k.cf_dir, k.cf_terms, x);
    out[4] = stdtrit(k, 0.019223896451809); out[5] = stdtrit(k, 9.80776103548191003e-01); out[6] = ndtri(1.0 - 9.80776103548191003e-01); out[7] = 1.0 - 9.80776103548191003e-01;
}
int main() {
    double nu = 30.0;
    TConst k{}; k.nu = nu; k.a = nu / 2; k.ln_nu = log(nu);
    k.lbeta = lgamma(nu / 2) + lgamma(0.5) - lgamma(nu / 2 + 0.5);
    k.ln_k = lgamma((nu + 1) / 2) - lgamma(nu / 2) - 0.5 * log(nu * M_PI);
    k.ln_tail = k.ln_k + (nu - 1) / 2 * k.ln_nu - k.ln_nu; k.split = (k.a + 1.0) / (k.a + 2.5);
    std::vector<double> c(2 * kCfTerms);
    ibeta_cf_coeffs(k.a, 0.5, c.data(), kCfTerms); ibeta_cf_coeffs(0.5, k.a, c.data() + kCfTerms, kCfTerms);
    double* d; hipMalloc(&d, c.size() * 8); hipMemcpy(d, c.data(), c.size() * 8, hipMemcpyHostToDevice);
    k.cf_dir = d; k.cf_cmp = d + kCfTerms; k.cf_terms = kCfTerms;
    double* o; hipMalloc(&o, 8 * 8);
    for (double t : {-2.1652612935653512, -2.1652642750356055}) {
        probe<<<1, 1>>>(k, t, o); double h[8]; hipMemcpy(h, o, 8 * 8, hipMemcpyDeviceToHost);
        printf("t=%.17g lnF=%.17g stdtrit_lo=%.17g stdtrit_hi=%.17g ndtri(pp)=%.17g pp=%.17g\n", t, h[0], h[4], h[5], h[6], h[7]);
    }
    return 0;
}
