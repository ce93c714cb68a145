/*
 * cvq.h -- C ABI of the MI355X copula-VaR quadrature engine (libcvq.so).
 *
 * Drop-in boundary for the hot path of Nassim-cha/copula-MSM-and-copula-Garch-VaR
 * (reference @ 2024-11-25).  Each entry point names the reference interface it
 * replaces.  Plain C: no C++ or torch types, int32 status (0 = ok, < 0 = error,
 * text in cvq_last_error(), thread-local), caller-owned buffers.
 *
 * Memory flags: every buffer argument documented "host|device" is interpreted
 * according to the call's `mem` argument (CVQ_MEM_HOST: the library copies it
 * and returns only when the result is back on the host; CVQ_MEM_DEVICE: a
 * pointer into device memory of the plan's device, used in stream order on the
 * plan's stream, no host synchronisation).
 */
#ifndef CVQ_H
#define CVQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ----------------------------------------------------------------- status */
#define CVQ_OK               0
#define CVQ_ERR_INVALID     -1   /* bad argument (reference: ValueError)            */
#define CVQ_ERR_UNSUPPORTED -2   /* e.g. Plackett with dim != 2, dim not in {2,3}   */
#define CVQ_ERR_HIP         -3   /* HIP runtime error                               */
#define CVQ_ERR_OOM         -4   /* device allocation failed                        */
#define CVQ_ERR_STATE       -5   /* call order (e.g. solve before set_dates)        */
#define CVQ_ERR_RANGE       -6   /* a bound above the plan's v_cap                  */
#define CVQ_ERR_NUMERIC     -7   /* MSM normaliser 0 (calc_prob.py:64), UKF Z<1e-10
                                    (estimate.py:219), bisection budget exceeded    */

#define CVQ_MEM_HOST   0
#define CVQ_MEM_DEVICE 1

/* copula kinds: copulas/{gaussian,student,plackett} */
#define CVQ_GAUSSIAN 0
#define CVQ_STUDENT  1
#define CVQ_PLACKETT 2
/* model kinds: utils/model_estimation/model/{msm,garch,mean_reverting}_estimation.py */
#define CVQ_MSM   0
#define CVQ_GARCH 1
#define CVQ_UKF   2

/* quadrature strategy (all reproduce the reference) */
#define CVQ_STRATEGY_PREFIX 0    /* materialise per-date row-prefix joint mass, then solve */
#define CVQ_STRATEGY_DIRECT 1    /* evaluate each slab's nodes inside the solve kernel     */
#define CVQ_STRATEGY_COMPACT 2   /* DIRECT control flow, one barrier per level, one-wave tail */
#define CVQ_STRATEGY_SORTED 3    /* reachable nodes sorted by membership threshold: a slab is
                                    one contiguous range (2-D, and 3-D with n <= 255)       */
#define CVQ_STRATEGY_SWEEP 4     /* SORTED's node order, each bisection cell summed in one pass
                                    with prefix sums at its subtree's mids (2-D)            */

typedef struct cvq_plan cvq_plan;

/* Static quadrature inputs = the reference's grids_generations_params
 * (densities, x_values, step_size, vol_combinations) + integrations_params_static
 * (MSM unique_vol_states) + packed copula params + portfolio weights.
 * Replaces: msm_estimation.py:123-137 / garch_estimation.py:133-145 outputs as
 * consumed by calc_integral.py:8-119. */
typedef struct cvq_static {
    int32_t model;              /* CVQ_MSM | CVQ_GARCH | CVQ_UKF                        */
    int32_t copula;             /* CVQ_GAUSSIAN | CVQ_STUDENT | CVQ_PLACKETT            */
    int32_t dim;                /* assets: 2 or 3                                        */
    int32_t n;                  /* num_points                                            */
    int32_t q;                  /* unique vol states per asset (GARCH/UKF: 1)            */
    int32_t n_combos;           /* q**dim                                                */
    const double*  x_values;    /* [n]         host                                      */
    const double*  step;        /* [n]         host                                      */
    const double*  densities;   /* [dim][q][n] host (GARCH/UKF: ones)                    */
    const int32_t* combos;      /* [n_combos][dim] host, ij-meshgrid order               */
    const double*  weights;     /* [dim]       host, weights[0] > 0                      */
    const double*  vol_states;  /* [dim][q]    host, MSM unique_vol_states; else NULL    */
    const double*  copula_params; /* packed as copula_integrations_params              */
    int32_t n_copula_params;    /* Student 1+d(d-1)/2, Gaussian d(d-1)/2, Plackett 1     */
    int32_t strategy;           /* CVQ_STRATEGY_*                                        */
    double  v_cap;              /* largest portfolio level any query may use (e.g. 0)    */
} cvq_static;

/* calc_var arguments: utils/calc_var_class.py:95 (obj_var, first_guess,
 * second_guess) + the constants of :111-114 and :257. */
typedef struct cvq_solve_args {
    double obj_var;             /* 0.05   */
    double first_guess;         /* -3     */
    double second_guess_lo;     /* -3.5   */
    double second_guess_hi;     /* -2     */
    double min_var;             /* -7.5   */
    double max_var;             /* 0      */
    double lower;               /* -100   */
    double tolerance;           /* 1e-6   */
    double ptf_mean;            /* load_data.py:113, added at calc_var_class.py:171 */
} cvq_solve_args;

const char* cvq_last_error(void);
int32_t     cvq_version(void);
int32_t     cvq_device_count(int32_t* count);

/* Plan = one device + one stream + device copies of the static tables. */
int32_t cvq_plan_create(const cvq_static* s, int32_t device, cvq_plan** out);
int32_t cvq_plan_destroy(cvq_plan* plan);
/* Run every later launch of the plan on hip_stream (a hipStream_t, e.g.
 * torch.cuda.current_stream().cuda_stream).  NULL is the HIP null stream (torch's
 * default stream), so the plan's work is ordered with the caller's; a new plan
 * runs on a private non-blocking stream until this is called. */
int32_t cvq_plan_set_stream(cvq_plan* plan, void* hip_stream);
/* Reachable quadrature nodes per date (nodes with level <= v_cap in the box). */
int32_t cvq_plan_info(const cvq_plan* plan, int64_t* reach_nodes, int32_t* rows);

/* Per-kernel timing with HIP events recorded on the plan's stream (bench.py's
 * live roofline).  kind: 0 tables, 1 joint-mass/prefix, 2 solve, 3 finalize,
 * 4 slab.  cvq_plan_timing(mask) times the kinds whose bit (1 << kind) is set
 * (0 = off, 0x1F = all) and clears previous records. */
int32_t cvq_plan_timing(cvq_plan* plan, int32_t enable);
int32_t cvq_plan_kernel_time(cvq_plan* plan, int32_t kind, double* total_ms, int32_t* launches);
/* Diagnostic build aid: per-date phase timestamps (s_memtime) of the last DIRECT
 * solve, recorded only when the process runs with CVQ_STAMPS=1 (never in a timed
 * run).  host receives count uint64 values, 32 per date. */
int32_t cvq_plan_debug_stamps(cvq_plan* plan, uint64_t* host, int64_t count);
/* Diagnostic: the SORTED plan's node words in solve order (first `count` of its reachable
   nodes; the LDS byte offsets of their records, cvq_sorted_kernels.h sorted_pack) and, when
   fix != NULL, the sorted positions of the six fixed levels of the last solve's arguments. */
int32_t cvq_plan_debug_nodes(cvq_plan* plan, uint32_t* host, int64_t count, int32_t* fix);
/* Diagnostics: the ends of the solve-order segments (positions the solve's range sums start or
 * end at; inside one the node order is free).  Writes min(cap, *count) of them. */
int32_t cvq_plan_debug_cuts(cvq_plan* plan, int32_t* host, int64_t cap, int32_t* count);
/* Measurement aid (bench.py's FP64 roofline basis): with cvq_plan_count_nodes(plan, 1)
 * the following COMPACT / SORTED / SWEEP solves record how many quadrature nodes each
 * date evaluated (the phase-stamp buffer: slower, never in a timed run);
 * cvq_plan_nodes_evaluated returns the last such solve's total over its dates. */
int32_t cvq_plan_count_nodes(cvq_plan* plan, int32_t enable);
int32_t cvq_plan_nodes_evaluated(cvq_plan* plan, int64_t* total);

/* Per-date inputs = integrations_params_t (calc_integral.py:158):
 *   MSM:       a = forecasts_by_states [T][dim][q], b = forecasts [T][n_combos]
 *   GARCH/UKF: a = sigma forecasts [T][dim],        b = NULL
 * CVQ_MEM_HOST: copied.  CVQ_MEM_DEVICE: read in place by the following launches
 * (no copy); the caller keeps a and b alive and unchanged until the next call. */
int32_t cvq_set_dates(cvq_plan* plan, int64_t T, const double* a, const double* b, int32_t mem);

/* COMPACT: the caller asserts that every date of the current cvq_set_dates batch takes
 * the fast node path -- MSM: b[t] is the outer product of the per-asset rows of a[t]
 * bit for bit (compute_forecast_combinations, msm_estimation.py:392-418, and
 * cvq_msm_tables build it so); GARCH / UKF: every marginal table entry is finite.  The
 * solve then skips its deferred-date (generic path) kernel.  A date that violates the
 * assertion fails the solve with CVQ_ERR_NUMERIC.  cvq_set_dates with CVQ_MEM_HOST sets
 * the hint itself when it can prove it; CVQ_MEM_DEVICE clears it.  No reference
 * counterpart (a launch-count optimisation of the device-resident path). */
int32_t cvq_set_fast_hint(cvq_plan* plan, int32_t on);

/* Drop-in for ValueAtRiskCalcualtion.compute_integral (calc_var_class.py:179-212)
 * == calc_grids_and_integrals_results (calc_integral.py:8-119):
 * out[t] = integral of the joint copula density over the nested grid of
 * (bounds[t][0], bounds[t][1]] for date t.  bounds [T][2], out [T]. */
int32_t cvq_slab(cvq_plan* plan, const double* bounds, double* out, int32_t mem);

/* Drop-in for ValueAtRiskCalcualtion.calc_var (calc_var_class.py:95-177 +
 * bisection_algorithm :250-309), quirks Q1-Q4 reproduced.  var_out [T];
 * iters_out = bisection iterations the reference would run (may be NULL). */
int32_t cvq_solve(cvq_plan* plan, const cvq_solve_args* args, double* var_out,
                  int32_t* iters_out, int32_t mem);

/* Status of the plan's last device-mode solve or finalize (cvq_solve with
 * CVQ_MEM_DEVICE and iters_out == NULL, cvq_solve_finalize): synchronises the
 * plan's stream and returns CVQ_ERR_NUMERIC if a date did not converge within the
 * bisection budget K (only possible for non-dyadic guesses, whose K carries a
 * 2-iteration margin); iters_out = bisection iterations the reference runs (Q2/Q4).
 * Device mode never synchronises by itself: call this to check.  cvq_solve with a
 * non-NULL iters_out checks and widens K itself. */
int32_t cvq_solve_status(cvq_plan* plan, int32_t* iters_out);

/* Sharded solve, for one process per GPU (date blocks).
 * Phase 1 (local):  per-date bisection snapshots + a 16-byte header
 *   d_header: 16 bytes device, d_snaps: [T_local][cvq_snap_stride(args)] device.
 * Exchange: the caller all-gathers headers and snaps (RCCL) -- or, packed, one buffer.
 * Phase 2: finalise every date from the gathered blocks; d_var [T_total] device. */
int32_t cvq_snap_stride(const cvq_solve_args* args, int32_t* stride);
int32_t cvq_solve_local(cvq_plan* plan, const cvq_solve_args* args, void* d_header, double* d_snaps);
int32_t cvq_solve_finalize(cvq_plan* plan, const cvq_solve_args* args, const void* d_headers,
                           int32_t n_ranks, const double* d_snaps, int64_t dates_per_rank,
                           int64_t T_total, double* d_var);
/* Packed variant for ONE all-gather per solve: each rank's block is its snapshots
 * [dates_per_rank][stride] followed by its 16-byte header at header_offset (doubles;
 * cvq_solve_local's d_snaps = block, d_header = block + header_offset), block length
 * len doubles (even, so blocks stay 16-byte aligned).  d_blocks = [n_ranks][len],
 * 16-byte aligned. */
int32_t cvq_packed_block_len(const cvq_solve_args* args, int64_t dates_per_rank, int64_t* len,
                             int64_t* header_offset);
int32_t cvq_solve_finalize_packed(cvq_plan* plan, const cvq_solve_args* args, const double* d_blocks,
                                  int32_t n_ranks, int64_t dates_per_rank, int64_t T_total,
                                  double* d_var);

/* ------------------------------------------------ per-date forecast stage */
/* MSM forecasts_array (msm_estimation.py:140-202 -> calc_marginals.py:33-38 ->
 * calc_prob.py:8-69): filtered state probabilities at the end of each rolling
 * window.  returns_c: centred returns [n_in + T - 1] of ONE asset; out [T][2**k]. */
int32_t cvq_msm_filter(int32_t device, int32_t k, double m0, double sigma, double b, double gamma,
                       const double* returns_c, int64_t n_in, int64_t T, double* out, int32_t mem);
/* Device-resident MSM forecast stage for all assets in one pass (no host round trip):
 * forecasts_array (msm_estimation.py:140-202 -> calc_prob.py:8-69, filtered
 * probabilities at each window's end, Q12) + sum_forecast_by_state (:205-248, Q14)
 * + compute_forecast_combinations (:392-418, Q7), i.e. integrations_params_t ready for
 * cvq_set_dates(..., CVQ_MEM_DEVICE).  Stream-ordered on `stream` (NULL = null stream),
 * no synchronisation.  params (host) [dim][4] = (m0, sigma, b, gamma); state_map (host)
 * [dim][2**k] = index of state s's 1e-6-rounded vol among the asset's q unique vols;
 * returns_c (device) [dim][n_in + T - 1] centred returns; scratch (device) of
 * cvq_msm_tables_scratch doubles; fbs_out (device) [T][dim][q]; pi_out (device)
 * [T][q**dim].  cvq_msm_tables_status synchronises and reports a zero Bayes
 * normaliser (calc_prob.py:64-65) of the last cvq_msm_tables run on that scratch as
 * CVQ_ERR_NUMERIC. */
int32_t cvq_msm_tables_scratch(int32_t dim, int32_t k, int64_t n_in, int64_t T, int64_t* doubles);
int32_t cvq_msm_tables(int32_t device, void* stream, int32_t dim, int32_t k, const double* params,
                       const int32_t* state_map, int32_t q, const double* returns_c, int64_t n_in,
                       int64_t T, double* scratch, double* fbs_out, double* pi_out);
int32_t cvq_msm_tables_status(double* scratch, int32_t dim, int32_t k, int64_t n_in, int64_t T, void* stream);
/* In-sample MSM marginals and densities of ONE asset's return series (calc_marginals.py:7-30,
 * used by MsmEstimation.calculate_marginals_and_densities_in_sample, msm_estimation.py:90-104):
 * marg_out / dens_out [N - 1] = sum over states of the filtered probabilities of step i
 * (calc_prob.py:51-69) times norm.cdf / norm.pdf of return i - 1 (calc_prob.py:110-132).
 * CVQ_ERR_NUMERIC on a zero Bayes normaliser (calc_prob.py:64-65). */
int32_t cvq_msm_marginals(int32_t device, int32_t k, double m0, double sigma, double b, double gamma,
                          const double* returns, int64_t N, double* marg_out, double* dens_out, int32_t mem);
/* GARCH(1,1) compute_forecast (garch_estimation.py:190-231 -> garch/forecast.py:5-19).
 * out [T] = sigma forecast per window. */
int32_t cvq_garch_forecast(int32_t device, double omega, double alpha, double beta,
                           const double* returns_c, int64_t n_in, int64_t T, double* out, int32_t mem);
/* GARCH(p, q) compute_forecast, 1 <= p, q <= 4 (garch/forecast.py:5-19):
 * params (host) [1 + p + q] = (omega, alpha_1..p, beta_1..q); out [T]. */
int32_t cvq_garch_forecast_pq(int32_t device, int32_t p, int32_t q, const double* params, const double* returns_c,
                              int64_t n_in, int64_t T, double* out, int32_t mem);
/* UKF compute_forecast (mean_reverting_estimation.py:192-232 -> forecast.py:5-12 ->
 * estimate.py:230-281); Q19 semantics.  out [T]. */
int32_t cvq_ukf_forecast(int32_t device, double a, double l, double q,
                         const double* returns_c, int64_t n_in, int64_t T, double* out, int32_t mem);

/* Device-resident GARCH / UKF forecast stage for all assets (no host round trip):
 * Garch/MeanRevertingEstimation.integration_params_retrieval's sigma forecasts
 * (garch_estimation.py:133-145 -> :190-231 -> garch/forecast.py:5-19;
 * mean_reverting_estimation.py:135-147 -> :192-232 -> kalman_mean_reverting/forecast.py:5-12),
 * written as integrations_params_t [T][dim] for cvq_set_dates(..., CVQ_MEM_DEVICE).
 * Stream-ordered on `stream`, no synchronisation.  model CVQ_GARCH: orders (host)
 * [dim][2] = (p, q) per asset, 1 <= p, q <= 4 (NULL = all (1, 1)), params (host) the
 * assets' (omega, alpha_1..p, beta_1..q) rows back to back; CVQ_UKF: params (host)
 * [dim][3] = (a, l, q), orders ignored.  returns_c (device) [dim][n_in + T - 1];
 * d_err (device) one int32; sig_out (device) [T][dim].  cvq_sigma_tables_status
 * synchronises and reports a UKF failure (Z < 1e-10 / NaN, estimate.py:219-220,
 * :270-271; NaN sigma) as CVQ_ERR_NUMERIC. */
int32_t cvq_sigma_tables(int32_t device, void* stream, int32_t model, int32_t dim, const int32_t* orders,
                         const double* params, const double* returns_c, int64_t n_in, int64_t T,
                         int32_t* d_err, double* sig_out);
int32_t cvq_sigma_tables_status(const int32_t* d_err, void* stream);

/* --------------------------------------- batched in-sample likelihoods */
/* One log-likelihood per parameter candidate over the same return series
 * (optimiser inner loops).  params: MSM [B][4] = (m0, sigma, b, gamma);
 * GARCH [B][3] = (omega, alpha, beta); UKF [B][3] = (a, l, q).  out [B].
 * MSM: calc_prob.py:36-47; GARCH: garch/estimation.py:91-125; UKF: estimate.py:276. */
int32_t cvq_msm_loglik(int32_t device, int32_t k, const double* params, int64_t B,
                       const double* returns, int64_t N, double* out, int32_t mem);
int32_t cvq_garch_loglik(int32_t device, const double* params, int64_t B,
                         const double* returns, int64_t N, double* out, int32_t mem);
int32_t cvq_ukf_loglik(int32_t device, const double* params, int64_t B,
                       const double* returns, int64_t N, double* out, int32_t mem);
/* GARCH(p, q), 1 <= p, q <= 4, for the (p, q) search of GarchOptimizer.optimize
 * (garch/opti.py:89-137): params [B][1 + p + q] = (omega, alpha_1..p, beta_1..q);
 * garch/estimation.py:91-125 incl. the max(p, q) chopped prefix. */
/* UKF E-step of VolOptimizer (kalman_mean_reverting/optimize.py:28-32 ->
 * estimate.py:7-51, 230-281): per candidate (a, l, q) [B][3] the log-likelihood
 * ll_out [B] (-1e10 on the Z / NaN failure) and the filtered state path
 * states_out [N][B] (time-major; NaN column on failure).  returns: one series [N]
 * shared by all candidates (per_candidate = 0) or one per candidate [B][N]
 * (per_candidate = 1: several assets' EM chains in one launch). */
int32_t cvq_ukf_filter(int32_t device, const double* params, int64_t B, const double* returns, int32_t per_candidate,
                       int64_t N, double* ll_out, double* states_out, int32_t mem);
int32_t cvq_garch_loglik_pq(int32_t device, int32_t p, int32_t q, const double* params, int64_t B,
                            const double* returns, int64_t N, double* out, int32_t mem);

/* Special functions on the device (known-answer tests against scipy):
 * fn 0 = t.ppf(u, nu) (student.py:102), 1 = norm.ppf (gaussian.py:44),
 * 2 = erf (utils/utils.py:20), 3 = t.ppf as the solve kernels' tables evaluate it for
 * nu = 6 (integer-nu root, nu must be 6). */
int32_t cvq_special(int32_t device, int32_t fn, double nu, const double* x, int64_t n,
                    double* out, int32_t mem);

#ifdef __cplusplus
}
#endif
#endif /* CVQ_H */
