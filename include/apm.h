/*
 * apm.h — C-ABI of the MI355X-native auxiliary-pseudo-marginal GP-classification hot path
 * (libapm.so, built from auxiliary-pm-mcmc_amd/csrc/). Plain pointers and sizes only.
 *
 * Every entry point replaces a reference interface on the per-step log-pseudo-marginal path
 * (matt-graham/auxiliary-pm-mcmc, paths relative to the reference root):
 *
 *   apm_gram           <- gpdemo/kernels.pyx:12-49  isotropic_squared_exponential_kernel(K, X, theta, epsilon)
 *                         gpdemo/kernels.pyx:52-90  diagonal_squared_exponential_kernel(K, X, theta, epsilon)
 *   apm_laplace        <- gpdemo/latent_posterior_approximations.py:22-124  laplace_approximation(K, y, ...)
 *   apm_theta_eval     <- gpdemo/estimators.py:201-217 (+ :221-241)  ApproxPosteriorIS.__call__(ns, theta)
 *                         gpdemo/estimators.py:317-325               PriorMC.__call__(ns, theta)
 *                         gpdemo/estimators.py:65-82                 Laplace.__call__(theta)
 *   apm_u_eval         <- gpdemo/estimators.py:218-241  ApproxPosteriorIS.__call__(ns, cached_results=...)
 *                         gpdemo/estimators.py:323-325  PriorMC.__call__(ns, K_chol=...)
 *   apm_u_*            <- the u_sampler / elliptical-slice proposal of auxpm/samplers.py:780-788 and
 *                         auxpm/mcmc_updates.py:382 kept on the device (batched driver)
 *
 * The estimator's cached_results tuple (K_chol, C_chol, f_post) (estimators.py:166-176) becomes an
 * opaque, context-owned cache SLOT; draws u become context-owned device U BUFFERS.
 * Batched entry points evaluate `count` independent chains per call (one chain per index).
 *
 * All calls are synchronous with respect to the host (results are in host memory on return).
 * Return value: 0 on success, a negative APM_E_* code on an API/HIP failure (message via
 * apm_last_error / apm_global_error). Per-chain numerical failures are reported in status[]
 * (APM_STATUS_*), which the Python layer maps onto the reference's exceptions.
 */
#ifndef APM_H
#define APM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define APM_SUCCESS 0
#define APM_E_INVALID (-1)
#define APM_E_HIP (-2)
#define APM_E_NOMEM (-3)

/* per-chain status */
#define APM_STATUS_OK 0
#define APM_STATUS_CHOL_K 1   /* chol(K) not PD        -> numpy.linalg.LinAlgError (estimators.py:321) */
#define APM_STATUS_CHOL_B 2   /* chol(B) not PD        -> numpy.linalg.LinAlgError (lpa.py:92) */
#define APM_STATUS_CHOL_C 3   /* chol(C) not PD        -> InvalidCovarianceMatrixError (estimators.py:208-215) */
#define APM_STATUS_MAXITER 4  /* Newton not converged  -> MaximumIterationsExceededError (lpa.py:100-102) */
#define APM_STATUS_GUARD 5    /* a device-side invariant of the theta-call failed (apm_guard_read;
                                 DESIGN.md §11): the value is withheld -> DeviceInvariantError
                                 (no reference counterpart: the reference has no device) */

/* covariance kernels */
#define APM_KERNEL_ISO 0         /* kernels.pyx:12-49, theta = (log sigma, log tau) */
#define APM_KERNEL_ARD 1         /* kernels.pyx:52-90, theta = (log sigma, log tau_1..tau_D) */
#define APM_KERNEL_PRECOMPUTED 2 /* K supplied by the caller (apm_theta_eval_K) */

/* estimators */
#define APM_EST_IS 0       /* LogMarginalLikelihoodApproxPosteriorISEstimator */
#define APM_EST_PRIORMC 1  /* LogMarginalLikelihoodPriorMCEstimator */
#define APM_EST_LAPLACE 2  /* LogMarginalLikelihoodLaplaceEstimator */

typedef struct apm_ctx apm_ctx;

int apm_version(void);
int apm_device_count(void);
const char *apm_global_error(void);

/* ---- context: data (X, y) resident on `device`, workspaces for max_batch chains ------------- */
apm_ctx *apm_create(int device, int kernel_kind, const double *X, int64_t n, int64_t d,
                    int64_t ldx, const double *y, double epsilon, int64_t n_imp,
                    int64_t max_batch, int64_t n_slots, int64_t n_ubufs);
void apm_destroy(apm_ctx *ctx);
const char *apm_last_error(const apm_ctx *ctx);
int64_t apm_padded_n(const apm_ctx *ctx);
int64_t apm_theta_len(const apm_ctx *ctx);
/* Newton settings of laplace_approximation (diff_f_tol, max_iters); defaults 1e-4, 1000 */
int apm_set_newton(apm_ctx *ctx, double diff_f_tol, int64_t max_iters);
/* hipStream_t the context launches on (for device-side timing by the caller) */
void *apm_stream(apm_ctx *ctx);

/* ---- U buffers (n x n_imp standard-normal draws, fp32 on device) ----------------------------- */
int apm_u_upload(apm_ctx *ctx, int64_t ubuf, const double *U, int64_t ldu);
int apm_u_download(apm_ctx *ctx, int64_t ubuf, double *U, int64_t ldu);
/* Philox4x32-10 normals: buffer ubufs[i] <- N(0,1) stream (seeds[i], counters[i]) */
int apm_u_normal(apm_ctx *ctx, int64_t count, const int64_t *ubufs, const uint64_t *seeds,
                 const uint64_t *counters);
/* dst[i] <- ca[i] * a[i] + cb[i] * b[i]  (elliptical-slice proposal u cos(phi) + nu sin(phi)) */
int apm_u_combine(apm_ctx *ctx, int64_t count, const int64_t *dst, const int64_t *a,
                  const int64_t *b, const double *ca, const double *cb);

/* ---- estimator calls ------------------------------------------------------------------------- */
/* theta-call for `count` chains: thetas row i (ldt stride) -> log-estimate out_logf[i]; the
 * per-theta state is written to cache slot slots[i]. ubufs/slots are ignored for APM_EST_LAPLACE.
 * n_cubic_ops[i] follows the reference's accounting (estimators.py:81,217,322). */
int apm_theta_eval(apm_ctx *ctx, int estimator, int64_t count, const double *thetas, int64_t ldt,
                   const int64_t *ubufs, const int64_t *slots, double *out_logf, int *status,
                   int64_t *n_cubic_ops);
/* the same for one chain with K (n x n, ldk) computed by the caller (any kernel_func) */
int apm_theta_eval_K(apm_ctx *ctx, int estimator, const double *K, int64_t ldk, int64_t ubuf,
                     int64_t slot, double *out_logf, int *status, int64_t *n_cubic_ops);
/* cached u-call: reuse slots[i]'s per-theta state with draws ubufs[i] */
int apm_u_eval(apm_ctx *ctx, int64_t count, const int64_t *slots, const int64_t *ubufs,
               double *out_logf, int *status);
/* cache-slot lifetimes (samplers.py:563-584: an MH sampler keeps the current state's cache and the
 * proposal's alive at once). acquire: a free slot, one owner (APM_E_NOMEM when all are owned);
 * copy: one more owner of the same (immutable) state - the handle copy of the reference's tuple;
 * release: one owner fewer, the slot is free again at zero (APM_E_INVALID if not acquired);
 * refcount: owners of a slot (negative on a bad argument). Host bookkeeping, no device work.
 * apm_theta_eval / apm_u_eval take any slot index; the Python layer allocates through these. */
int apm_cache_acquire(apm_ctx *ctx, int64_t *slot);
int apm_cache_copy(apm_ctx *ctx, int64_t slot);
int apm_cache_release(apm_ctx *ctx, int64_t slot);
int64_t apm_cache_refcount(const apm_ctx *ctx, int64_t slot);
/* read a slot back (any pointer may be NULL): factor (n x n lower, fp32 rounded), f_post, g, cst */
int apm_slot_read(apm_ctx *ctx, int64_t slot, double *L, int64_t ldl, double *f_post, double *g,
                  double *cst);

/* ---- stand-alone building blocks (host in / host out) ---------------------------------------- */
int apm_gram(int device, int kernel_kind, const double *X, int64_t n, int64_t d, int64_t ldx,
             const double *theta, int64_t n_theta, double epsilon, double *K, int64_t ldk);
/* laplace_approximation(K, y, calc_cov, calc_lml, diff_f_tol, max_iters): f_out (n), C_out
 * (n x n, ldc; if calc_cov), lml_out (if calc_lml), n_iter_out = Newton iterations */
int apm_laplace(int device, const double *K, int64_t n, int64_t ldk, const double *y,
                int calc_cov, int calc_lml, double diff_f_tol, int64_t max_iters, double *f_out,
                double *C_out, int64_t ldc, double *lml_out, int64_t *n_iter_out, int *status);

/* ---- device-time accounting of the hot kernels (HIP events on the context stream) ------------ */
#define APM_PROF_GRAM 0
#define APM_PROF_CHOL_UPDATE 1
#define APM_PROF_UGEMM 2
#define APM_PROF_CHOL_UPDATE32 3
#define APM_PROF_STATS 4 /* not a kernel: launches = chains whose mixed-precision Newton solve was
                            rerun in fp64, work = refinement steps launched, total_ms = 0 */
#define APM_PROF_CHOL_UPDATE32_OUTER 5 /* the rank-64*OUTER launches among CHOL_UPDATE32 */
#define APM_PROF_CHOL_UPDATE_OUTER 6   /* the rank-64*OUTER launches among CHOL_UPDATE */
#define APM_PROF_DF_TIMEOUTS 7 /* not a kernel: launches = bounded-spin timeouts of the Newton
                                 factorisation's dataflow panel launches (each fails its chain,
                                 which the Newton loop reruns in fp64; apart from breakdowns of
                                 the fp32 factor, which are not counted here) */
#define APM_PROF_POST32_OUTER 8 /* the rank-64*OUTER trailing updates of the posterior factor's
                                   bottom block in fp32 (postcov.hip, APM_POST32) */
#define APM_PROF_POST64_RERUNS 9 /* not a kernel: launches = chains whose posterior bottom block was
                                    recomputed in fp64 (trace of C above the fp32 bound) */
#define APM_PROF_TRSV_TIMEOUTS 10 /* not a kernel: launches = bounded-spin timeouts of the Newton
                                    solves' multi-workgroup TRSV (each fails its chain, which the
                                    Newton loop reruns in fp64) */
#define APM_PROF_ICM_CHECKS 11 /* not a kernel: launches = chains whose chol(C) was also formed the
                                 reference's way (the InvalidCovarianceMatrixError check) */
#define APM_PROF_GUARD 12 /* not a kernel: launches = chains failed by the guard (APM_STATUS_GUARD) */
#define APM_PROF_NKINDS 13
/* on = 0 off; 1 the roofline kinds (GRAM, UGEMM and the two *_OUTER kinds: one event pair per
 * launch of those kernels only, so that the timing adds little to a timed region); 2 every kind
 * (CHOL_UPDATE / CHOL_UPDATE32 add an event pair around every in-panel update launch) */
int apm_prof_enable(apm_ctx *ctx, int on);
/* total device milliseconds and launch count per tracked kernel since the last reset; also the
 * algorithmic work: bytes (GRAM) or flops (CHOL_UPDATE, CHOL_UPDATE32 = the fp32 Newton
 * factorisation, UGEMM) those launches performed */
int apm_prof_read(apm_ctx *ctx, int kind, double *total_ms, int64_t *launches, double *work,
                  int reset);
/* launches the empty kernel k_apm_marker<id> (id 0..3) on the context stream: brackets a region
 * in a rocprofv3 kernel trace (tools/prof_window.py); no reference counterpart */
int apm_prof_marker(apm_ctx *ctx, int id);

/* The guard of the last IS theta-call: per chain i < count, r[4i..4i+3] =
 * |1/2 log|B| of the last Newton factor - 1/2 log|M| of the posterior factor| (the same
 * eigenvalues), | |g|^2 - f_post^T z | / max(1, |f_post^T z|) (g = chol(C)^-1 f_post from the
 * posterior factors, z = a + W f_post from the Newton vectors), |sum log diag chol(C) -
 * (1/2 log|K| - 1/2 log|M|)| (C_chol's diagonal from the slot) and max_r |(C_chol g)_r -
 * f_post_r| / max(1, max |f_post|) (every row of the slot's fp32 factor). A chain past a bound
 * fails with APM_STATUS_GUARD. */
int apm_guard_read(apm_ctx *ctx, int64_t count, double *r);

/* ---- self-test ------------------------------------------------------------------------------- */
/* C = C + A * B^T for 64x64 row-major fp64 host matrices through the f64 MFMA tile routine that
 * every Cholesky panel / trailing update uses (pins the v_mfma_f64_16x16x4 operand maps) */
int apm_selftest_tile(int device, const double *A, const double *B, double *C);
/* out[4i..4i+3] = Philox4x32-10(counter in[6i..6i+3], key in[6i+4..6i+5]) for i < n, through
 * the device round function of apm_u_normal (Salmon et al., SC'11; checked against the
 * published known-answer vectors in tests/test_gpu_kernels.py) */
int apm_selftest_philox(int device, int64_t n, const uint32_t *in, uint32_t *out);

#ifdef __cplusplus
}
#endif
#endif /* APM_H */
