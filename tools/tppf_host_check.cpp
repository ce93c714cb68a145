// Host check of the stdtrit guess tables + refinement (no GPU): prints
// t.ppf(p, nu) for p read from stdin, one per line, after building the tables
// exactly as make_tconst does.  usage: tppf_host_check NU < p.txt
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../copula-msm-and-copula-garch-var_amd/csrc/cvq_tppf_tables.h"
using namespace cvq;
int main(int argc, char** argv) {
    const double nu = atof(argv[1]);
    const int terms = 400;
    TConst k{};
    k.nu = nu; k.a = nu / 2; k.ln_nu = std::log(nu);
    k.lbeta = std::lgamma(nu / 2) + std::lgamma(0.5) - std::lgamma(nu / 2 + 0.5);
    k.ln_k = std::lgamma((nu + 1) / 2) - std::lgamma(nu / 2) - 0.5 * std::log(nu * M_PI);
    k.ln_tail = k.ln_k + (nu - 1) / 2 * k.ln_nu;
    k.split = (k.a + 1.0) / (k.a + 2.5); k.ln_a = std::log(k.a); k.inv_nu = 1.0 / nu; k.p_split = 0.05;
    std::vector<double> c(2 * terms);
    ibeta_cf_coeffs(k.a, 0.5, c.data(), terms);
    ibeta_cf_coeffs(0.5, k.a, c.data() + terms, terms);
    k.cf_dir = c.data(); k.cf_cmp = c.data() + terms; k.cf_terms = terms;
    std::vector<double> tab;
    bool ok = false;
    int nc = 256, nv = 64;
    for (; nc <= 4096 && !ok; nc *= 2, nv *= 2) ok = build_tppf_tables(k, nc, nv, tab);
    if (!ok) k.tab_c = nullptr;
    std::vector<double> quint;
    bool qok = false;
    if (ok)
        for (int qc = 256; qc <= 4096 && !qok; qc *= 2) qok = build_tppf_quintic(k, qc, qc < 1024 ? 128 : qc / 4, quint);
    fprintf(stderr, "tables ok=%d n_c=%d n_v=%d quintic ok=%d n_qc=%d n_qv=%d\n", ok, k.n_c, k.n_v, qok, k.n_qc, k.n_qv);
    TConst kq = k;
    if (qok) { kq.q_c = quint.data(); kq.q_v = quint.data() + 6 * k.n_qc; }
    double p;
    while (scanf("%lf", &p) == 1) {
        TConst plain = k; plain.tab_c = nullptr;
        printf("%.17g %.17g %.17g\n", stdtrit(kq, p), tppf_table_guess(k, p < 0.5 ? p : 1 - p), stdtrit(plain, p));
    }
}
