// Internal launcher interface between the kernel translation units and capi.cpp.
// Nothing here is part of the public C-ABI (include/apm.h).
#pragma once
#include "apm_common.h"

// A batched fp64 matrix: chain b's element (r, c) lives at base[b*cstride + r*ld + c].
struct MatB {
    double* base;
    int64_t ld;
    int64_t cstride;
};

// The same for fp32 (mixed-precision Newton factorisation, chol32.hip).
struct MatF {
    float* base;
    int64_t ld;
    int64_t cstride;
};

// Per-chain liveness: a kernel does work for chain b iff active[b] != 0 && status[b] == 0.
struct Live {
    const int* active;
    int* status;
};

// ---- chol.hip -------------------------------------------------------------------------------
// Blocked right-looking Cholesky building blocks over TB x TB tiles (lower triangle).
// diag:   factor tile (k,k) in place, write its inverse to Dinv[b][k] and sum(log diag) to
//         ldet[b][k]; a non-positive pivot sets status[b] = fail_code.
// panel:  tiles (i,k), i in [i0, R):  A_ik <- A_ik * inv(L_kk)^T     (f64 MFMA)
// update: tiles (i,j), i in [i0, R), j0 <= j <= min(i, jend-1):
//         A_ij -= sum_{q<kc} A_{i,k0+q} A_{j,k0+q}^T  (f64 MFMA, rank 64*kc)
void launch_chol_diag(MatB A, int k, double* Dinv, int64_t dstride, double* ldet, int64_t lstride,
                      Live live, int fail_code, int nchains, hipStream_t s);
// panel rows [i0, R) minus the row tiles [glo, ghi) (pass glo = ghi = R for none)
void launch_chol_panel(MatB A, int k, int i0, int R, int glo, int ghi, const double* Dinv,
                       int64_t dstride, Live live, int nchains, hipStream_t s);
// Optional diag step fused into an update launch (the launch's tiles[0] is the diagonal tile
// (d, d); Dinv / ldet / status are written as by launch_chol_diag for k = d).
template <class TS>
struct FusedDiag {
    int enabled;
    TS* Dinv;
    int64_t dstride;
    double* ldet;
    int64_t lstride;
    int fail_code;
};
// tiles: device list of packed (i << 16) | j built by build_update_tiles (super-tile order)
// plus = true adds instead of subtracting (SYRK of the UL factorisation, postcov.hip)
void launch_chol_update(MatB A, int k0, int kc, const unsigned* tiles, int ntiles, bool plus,
                        Live live, int nchains, hipStream_t s,
                        FusedDiag<double> fd = FusedDiag<double>{0, nullptr, 0, nullptr, 0, 0});
// the same with one 128x128 super-tile per workgroup (tiles from build_update_supertiles)
// plus: 0 A -= ..., 1 A += ..., 2 A = I + Y Y^T for lower-triangular Y (depth per tile column
// truncated to the nonzero blocks; the old tile is not read). S.base: the old tiles are read from
// S (same tile coordinates, own ld / chain stride) instead of A - an out-of-place update
void launch_chol_update_t128(MatB A, int k0, int kc, const unsigned* tiles, int ntiles, int plus,
                             Live live, int nchains, hipStream_t s,
                             FusedDiag<double> fd = FusedDiag<double>{0, nullptr, 0, nullptr, 0, 0},
                             MatB S = MatB{nullptr, 0, 0});
long update_tile_count(int i0, int R, int j0, int jend);
#include <vector>
std::vector<unsigned> build_update_tiles(int i0, int R, int j0, int jend, int glo = 0, int ghi = 0);
// one step (block J) of the backward solve L^T z = r, r stored in row `rrow` of A (in place),
// z written to z[b*zstride + ...]
void launch_trsv_lt_step(MatB A, int J, int64_t rrow, const double* Dinv, int64_t dstride,
                         double* z, int64_t zstride, Live live, int nchains, hipStream_t s);
// empty kernel k_apm_marker<id> (trace bracketing, apm_prof_marker)
void launch_marker(int id, hipStream_t s);
// test hook: C(64x64) = A(64x64) * B(64x64)^T through the MFMA tile path
void launch_tile_nt_test(const double* A, const double* B, double* C, hipStream_t s);
void launch_philox_test(const uint32_t* in, uint32_t* out, int64_t n, hipStream_t s);

// ---- chol32.hip: mixed-precision Newton solve (fp32 factor of B + fp64 refinement) -----------
void launch_chol_diag32(MatF A, int k, float* Dinv, int64_t dstride, double* ldet,
                        int64_t lstride, Live live, int fail_code, int nchains, hipStream_t s);
void launch_chol_panel32(MatF A, int k, int i0, int R, int glo, int ghi, const float* Dinv,
                         int64_t dstride, Live live, int nchains, hipStream_t s);
// Bounded in-launch hand-overs of the Newton solve (k_chol_panel_df32, k_trsv32_mw). HIP promises
// no dispatch order, so a workgroup's logical index is the ticket it draws from a monotonic
// arrival counter when it starts (a ticket exists only for a workgroup that is running): a
// dataflow row then waits only on rows that have arrived, and of the TRSV's chains only the one
// holding the newest ticket can wait on a workgroup that has not. Every wait is bounded by
// `limit` polls; a bounded exit is counted in *timeouts and fails its chain (the Newton loop
// reruns it in fp64), so it can cost time but never a value.
struct SpinCtl {
    unsigned long long* ticket;    // arrival counter, shared by the launches of one stream
    unsigned long long base;       // its value before this launch (host-side running total)
    unsigned long long* timeouts;  // bounded-spin exits (APM_PROF_DF / _TRSV_TIMEOUTS)
    int limit;                     // polls before a wait gives up
};
// fp16x3 operand planes of one outer panel of the Newton matrix (chol32.hip): for each 32-column
// slice s of the panel and row r < rows, hi = fp16(x) and lo = fp16(x - hi) of the row's 32
// entries (64 bytes each), hi at base + b * cstride + (s * rows + r) * 32 and lo at + lo (fp16
// bit patterns). Written by the dataflow panel kernel for the rows below the panel's diagonal
// block; the trailing update then stages them into LDS with DMA instead of splitting fp32
// operands in registers. base == nullptr: no planes.
struct Planes16 {
    unsigned short* base;
    int64_t cstride;
    int64_t lo;
    int rows;
};
// tile columns [K, K+ncols) of an outer panel (diagonal tile (K, K) already factored) in one
// dataflow launch (chol32.hip: per-(chain, row) progress words prog[b * pstride + row], monotonic
// base per factorisation and panel); returns the launch's workgroup count (its tickets), 0 when
// nothing was launched, -1 for a panel wider than the progress word allows. pl.base != nullptr:
// the rows below the diagonal block (row tiles < pl.rows / 64) also write the panel's planes.
// inv_skip (per chain): that chain's rows below the diagonal block return at once (its
// explicit-inverse panel follows)
long launch_chol_panel_df32(MatF A, int K, int ncols, int R, FusedDiag<float> fd, Live live,
                            int nchains, int hlim, const int* h3ok, unsigned long long* prog,
                            int64_t pstride, unsigned long long base, SpinCtl sc, hipStream_t s,
                            Planes16 pl = Planes16{nullptr, 0, 0, 0}, int rhs_as = -1,
                            const int* inv_skip = nullptr);
// explicit-inverse panel of the Newton factorisation (chol32.hip), after a dataflow launch over
// the diagonal block [K, K+8) and the right-hand-side row (rhs_as): Z = inv(L_D) of the 512x512
// diagonal block as fp16x3 planes (zpl, 512 rows), by recursive doubling over fp32 scratch (zt:
// 3 x 512 x 512 per chain, zstride floats apart); then every row tile i in [K+8, nb) becomes
// X_i = A_i Z^T in one fp16x3 GEMM (in place, plus the panel's planes pl). Only the chains
// flagged in `ok` (the host's invok: 1 + K_ii < 2^15, so the split Schur-complement entries fit
// fp16's range).
void launch_panel_inv32(MatF A, int K, int nb, const float* Dinv, int64_t dstride, float* zt,
                        int64_t zstride, Planes16 zpl, Planes16 pl, Live live, int nchains,
                        const int* h3ok, hipStream_t s);
// rows [row0, R) of an outer panel [K, K+ncols) whose diagonal block is final (fd.Dinv: its
// inverses), each row a left-looking walk over the panel's columns with no waits; zrow > 0: row
// tile i is zero in the tile columns < zrow - 1 - i (postcov.hip's fp32 bottom block)
void launch_chol_panel_bulk32(MatF A, int K, int ncols, int row0, int R, int zrow,
                              FusedDiag<float> fd, Live live, int nchains, int hlim,
                              const int* h3ok, hipStream_t s,
                              Planes16 pl = Planes16{nullptr, 0, 0, 0});
void launch_chol_update32(MatF A, int k0, int kc, const unsigned* tiles, int ntiles, Live live,
                          int nchains, hipStream_t s,
                          FusedDiag<float> fd = FusedDiag<float>{0, nullptr, 0, nullptr, 0, 0},
                          int hlim = 0, const int* h3ok = nullptr);
// the same update with one 128x128 super-tile per workgroup (tiles from build_update_supertiles);
// hlim > 0: fp16x3 operands (chol32.hip) for super-tiles whose rows lie below row tile hlim, in
// the chains b with h3ok[b] != 0 (h3ok == nullptr: every chain); the others take fp32 operands.
// rhs >= 0: row tile rhs is the appended right-hand side whose first row alone is data (its
// super-tiles must hold it alone: build_update_supertiles(..., solo = rhs)); it is updated as a
// row-vector product (fp64 accumulation) instead of a 64-row tile product
void launch_chol_update32_t128(MatF A, int k0, int kc, const unsigned* tiles, int ntiles,
                               Live live, int nchains, hipStream_t s,
                               FusedDiag<float> fd = FusedDiag<float>{0, nullptr, 0, nullptr, 0, 0},
                               int hlim = 0, const int* h3ok = nullptr, int rhs = -1,
                               int role = 0,  // 1: the posterior bottom block, 3: the rhs row
                                              // alone (names only)
                               Planes16 pl = Planes16{nullptr, 0, 0, 0});  // k0's panel's planes
// the far trailing updates of the Newton factorisation on 256x256 quad tiles (chol32.hip): fp16x3
// operands from the planes only, rows below the appended right-hand side, chains with h3ok set
void launch_chol_update32_q256(MatF A, int k0, int kc, const unsigned* quads, int nq, Live live,
                               int nchains, hipStream_t s, const int* h3ok, Planes16 pl,
                               int role = 0);
std::vector<unsigned> build_update_quads(int i0, int R, int j0, int jend);
// solo >= 0: row tile solo gets super-tile rows of its own (never paired with another row tile)
std::vector<unsigned> build_update_supertiles(int i0, int R, int j0, int jend, int glo, int ghi,
                                              int solo = -1);
// y = K x from K's lower tiles (part: nb*nb*64 doubles per chain of partials); Bf.base != null
// also forms the fp32 Newton matrix I + W^1/2 K W^1/2 and its right-hand-side block (x = b)
void launch_symv(MatB K, const double* x, int64_t xstride, double* y, int64_t ystride,
                 double* part, int64_t pstride, int np, MatF Bf, const double* Ws,
                 int64_t wstride, Live live, int nchains, hipStream_t s, int symv_tpw = 1);
void launch_row32(MatF Bf, int64_t row, int np, double* out, int64_t ostride, Live live,
                  int nchains, hipStream_t s);
// blocked TRSV steps with fp32 tiles / inverses and fp64 vectors (r updated in place)
void launch_trsv_fwd32(MatF A, int J, int nb, const float* Dinv, int64_t dstride, double* r,
                       double* y, int64_t vstride, Live live, int nchains, hipStream_t s);
void launch_trsv_bwd32(MatF A, int J, const float* Dinv, int64_t dstride, double* r, double* z,
                       int64_t vstride, Live live, int nchains, hipStream_t s);
// the whole solve in one launch over TRM_G workgroups per chain (k_trsv32_mw; NaN-fills `out`
// first; fp64 r -> out, r kept); needs np <= 8192 (trsv32_mw_ok), else the per-block steps above
bool trsv32_mw_ok(int np);
void trsv32_mw_init();  // per device, once the device is current (apm_create)
// returns the launch's workgroup count (its tickets)
long launch_trsv32_mw(bool fwd, MatF A, int nb, const float* Dinv, int64_t dstride,
                      const double* r, double* out, int64_t vstride, Live live, int nchains,
                      int fail_code, SpinCtl sc, hipStream_t s);
// refinement vector ops (mode 0: out = Ws x; 1: out = Ws Kb - x - Ws Kt; 2: x += out)
// acceptance of refinement step `step` on the chains with refining[b] != 0 && status[b] == 0:
// accepted chains leave the mask; with last = true the others get status = fail_code
void launch_refine_check(const double* x, const double* d, int64_t vstride, int np, double tol,
                         int fail_code, int step, bool last, double* prev, int* refining,
                         const int* status, int nchains, hipStream_t s);
// refining[b] = chain b live
void launch_refine_mask(Live live, int* refining, int nchains, hipStream_t s);
void launch_refine(int mode, const double* Ws, const double* Kb, double* x, const double* Kt,
                   double* out, int64_t vstride, int np, Live live, int nchains, hipStream_t s);

// ---- gram.hip -------------------------------------------------------------------------------
// K[b] (np x np, identity-padded beyond n) from X (n x d, row-major, ldx) and theta[b]
// kind 0 = isotropic SE (kernels.pyx:12-49), 1 = ARD SE (kernels.pyx:52-90)
// both: write both triangles (else K's lower tiles only); K2.base: the lower tiles of tile
// columns < k2cols also to K2 (direct-form distances on the fp64 VALU, k_gram)
void launch_gram(MatB K, const double* X, int64_t ldx, int n, int d, const double* theta,
                 int64_t tstride, int kind, double eps, int np, Live live, int nchains,
                 hipStream_t s, bool both, MatB K2 = MatB{nullptr, 0, 0}, int k2cols = 1 << 30);

// ---- newton.hip -----------------------------------------------------------------------------
struct NewtonVecs {     // all per chain, stride vstride (>= np)
    double* f;          // current mode estimate
    double* fnew;
    double* W;          // W_diag
    double* Ws;         // W_diag^1/2
    double* b;          // W f + grad
    double* Kb;         // K b, later reused
    double* a;          // b - W^1/2 z
    double* z;          // TRSV result
    int64_t vstride;
};
void launch_newton_prep(NewtonVecs v, const double* y, int n, int np, Live live, int nchains,
                        hipStream_t s);
void launch_gemv(MatB M, const double* x, int64_t xstride, double* out, int64_t ostride, int np,
                 Live live, int nchains, hipStream_t s);
void launch_form_B(MatB K, MatB A, NewtonVecs v, int np, Live live, int nchains, hipStream_t s);
void launch_newton_update(NewtonVecs v, int np, Live live, int nchains, hipStream_t s);
void launch_newton_check(NewtonVecs v, int n, int np, double tol, int* active, const int* status,
                         int* n_iter, int nchains, hipStream_t s);
void launch_copy_lower(MatB src, MatB dst, int np, Live live, int nchains, hipStream_t s);
void launch_form_aug(MatB K, MatB A, NewtonVecs v, int np, Live live, int nchains,
                     hipStream_t s, bool lower_only = false);
// per chain: out[b] = -0.5 a.f + sum_n log_ndtr(y f) - 0.5*sum(ldet[0..nb))*2
void launch_laplace_lml(NewtonVecs v, const double* y, int n, const double* ldet,
                        int64_t lstride, int nb, double* out, Live live, int nchains,
                        hipStream_t s);

// cache slot: fp32 factor with an extra TB-row block (row np holds g^T for apm_slot_read; the
// estimate does not use it), plus fp64 vectors of the self-consistent epilogue (ugemm.hip)
struct SlotSet {
    float* L;           // (np + TB) x np, ld = np
    double* fpost64;    // np: f_post
    double* W64;        // np: W of the last Newton iteration (0 for PriorMC)
    double* z64;        // np: z = C^-1 f_post = a + W f_post (0 for PriorMC)
    double* cst;        // 1 per slot: 1/2 f_post^T z - 1/2 log|B|  (0 for PriorMC)
    int64_t lstride, vstride;
    // wide slots (trace of the factor's Gram L L^T above APM_WIDE_Q, ugemm.hip): the factor is
    // also kept in fp64 and their u-path runs on f64 MFMA
    double* const* L64; // per slot: np x np, ld = np, or null - buffers are attached by the host
                        // to the slots that become wide (rare), not allocated per slot
    double* rowq;       // np per slot: squared row norms of the factor (k_slot_write_L)
    int* wide;          // 1 per slot
    int* chain_wide;    // 1 per chain of the call (read back with the theta-call's results)
    double wide_q;      // the threshold (APM_WIDE_Q, overridable by the environment variable)
    double post_q;      // trace(C) above which an fp32 bottom block is recomputed in fp64
                        // (APM_POST32_Q; postcov.hip)
    const double* icm_thr;  // per chain: trace(C) below which bit 3 of chain_wide asks the host
                            // for the reference-route check of chol(C) (capi.cpp icm_check)
};
// trace(L L^T) above which a slot's u-path runs in fp64: the fp32 L.U moves
// log f by ~1e-10 x trace (11 nats at trace 1.15e11, sigma = e^18.5; < 1e-6 nats at the trace
// ~1e3 of typical thetas), so this keeps the fp32 rounding of L and U below ~1e-4 nats
#define APM_WIDE_Q 1.0e6
// trace(C) above which the posterior factor's bottom block is recomputed in fp64 (postcov.hip):
// its fp32 TRSM moves log f by ~1e-9 x trace(C) (tools/postcov_precision_study.py)
#define APM_POST32_Q 1.0e5
// write slot slots[b] from the factored work matrix. mode 1 = PriorMC (K_chol at (0,0), g = 0),
// mode 2 = IS via chol(K) (postcov.hip: chol(C) J at rows [np, 2np) cols [0, np), g in v.Kb),
// mode 3 = the same with chol(C) J in the fp32 bottom block of S32 (rows [np, 2np)); its chains
// with trace(C) > S.post_q get bit 1 of S.chain_wide (the host recomputes them in fp64, mode 2).
// Only chains with live.active[b] && !live.status[b] are written.
void launch_slot_write(MatB A, NewtonVecs v, const double* ldet, int64_t lstride, int nb,
                       SlotSet S, const int64_t* slots, int mode, int n, int np, Live live,
                       int nchains, hipStream_t s, MatF S32 = MatF{nullptr, 0, 0},
                       double* rowe = nullptr);
// the fp64 factor alone, for the call's wide slots that have a buffer attached (mode 1 or 2)
void launch_slot_write_L64(MatB A, SlotSet S, const int64_t* slots, int mode, int np, Live live,
                           int nchains, hipStream_t s);

// ---- postcov.hip ----------------------------------------------------------------------------
void launch_set_rhs(MatB A, int64_t row0, int ncols, const double* vec, int64_t vstride,
                    Live live, int nchains, hipStream_t s);
void launch_get_row(MatB A, int64_t row, int n, double* out, int64_t ostride, Live live,
                    int nchains, hipStream_t s);
// dst (from column dcol0) <- Y2 = J (W^1/2 L)^T J, and L <- L J in place, in one pass. Upper
// tiles of Y2 are zeroed: all of them (zero_all), or only the first super-diagonal, the only
// ones the single-launch SYRK (k_chol_update_t128, plus == 2) reads
void launch_form_y2_rev(MatB L, MatB dst, int64_t dcol0, const double* Ws, int64_t vstride,
                        int np, Live live, int nchains, hipStream_t s, bool zero_all);
void launch_identity_lower(MatB M, int np, Live live, int nchains, hipStream_t s);
// out = L^T x (L lower), or with rev g = J L^T J h; tile-parallel through nb*nb*64 partials per chain
void launch_trmv_tiles(bool rev, MatB L, const double* x, double* out, int64_t vstride, int np,
                       double* part, int64_t pstride, Live live, int nchains, hipStream_t s);
// fp32 working copy of the posterior factor for its bottom block (postcov.hip): S32's top rows
// <- the lower tiles of the fp64 top factor L' (rows [0, np) of A) in tile columns [k0, k1), its
// diagonal-tile inverses D32 <- D64 for those columns; bottom: S32's rows [np, 2np) <- L_K J
// (rows [np, 2np) of A) from the outer panel of each row's first nonzero tile on (the zero
// tiles the bottom's updates read included)
void launch_post32_convert(MatB A, MatF S32, const double* D64, int64_t d64stride, float* D32,
                           int64_t d32stride, int nb, int outer, int k0, int k1, bool bottom,
                           Live live, int nchains, hipStream_t s,
                           Planes16 pl = Planes16{nullptr, 0, 0, 0});
// status[b] = code where other[b] != 0 (chol(K) failure of the concurrent factorisation wins)
void launch_merge_status(int* status, const int* other, int code, int nchains, hipStream_t s);

// ---- newton.hip: read-back of up to three small device arrays (4-byte words) into mapped
// pinned host memory, back to back at dst (device address of the host buffer)
struct Export {
    const unsigned* src[4];
    int words[4];
    unsigned* dst;
};
void launch_export(const Export& e, hipStream_t s);

// ---- ugemm.hip ------------------------------------------------------------------------------
struct UPool {
    double* base;       // each buffer: np x sp fp64, ld = sp, zero padded (device normals are
                        // fp32 values; host uploads keep their fp64 values for the wide path)
    int64_t stride;
    int sp;
    float* base32;      // the same buffers rounded to fp32 (same layout), written with them: the
                        // operand k_ugemm reads (half the bytes of converting the fp64 ones there)
};
void launch_u_convert(const double* U64, int64_t ldu, int n, int S, UPool P, int64_t ubuf,
                      hipStream_t s);
void launch_u_normal(UPool P, const int64_t* ubufs, const uint64_t* seeds,
                     const uint64_t* counters, int n, int S, int nchains, hipStream_t s);
void launch_u_combine(UPool P, const int64_t* dst, const int64_t* a, const int64_t* b,
                      const double* ca, const double* cb, int n, int S, int nchains,
                      hipStream_t s);
// partial[b][i][s] = sum over rows of row-block i of t(n,s) (i < nb), partial[b][nb][s] = g^T u_s
// wide: also launch the f64 MFMA twin for the call's wide slots (k_ugemm64)
void launch_ugemm(SlotSet S, const int64_t* slots, UPool P, const int64_t* ubufs,
                  const double* y, int n, int np, double* partial, int64_t pstride,
                  const int* status, int nchains, bool wide, hipStream_t s);
void launch_lme(const double* partial, int64_t pstride, int nb, int S, int sp, SlotSet Sl,
                const int64_t* slots, double* out, const int* status, int nchains,
                hipStream_t s);

// chol(K) retry of the chains with fail[b] == code, unblocked in LAPACK's dpotf2 order (chol.hip,
// DESIGN.md §3.4): K's lower triangle into A, L in place, per-tile log-diagonal sums into ldet;
// success clears fail[b]. Returns false (nothing launched) for np > 512.
bool launch_chol_unblocked(MatB K, MatB A, int np, int* fail, int code, double* ldet,
                           int64_t lstride, int nchains, hipStream_t s);

// ---- the guard (newton.hip) --------------------------------------------------
// G[k * B + b]: 0: 1/2 log|B| of the last Newton factor, 1: 1/2 log|K|, 2..5: residuals r1..r4
// (rowe: the slot writer's per-row residuals of C_chol g = f_post, B x np)
void launch_guard_save(const double* ldet, int64_t lstride, int off, int nb, double* G, int B,
                       int k, Live live, int nchains, hipStream_t s);
void launch_guard_check(const double* ldet, int64_t lstride, int nb, const double* gvec,
                        int64_t gstride, SlotSet S, const int64_t* slots, double* G, int B,
                        double t1, double t2, double t3, double t4, const double* rowe,
                        const double* fvec, int fail_code, Live live, int nchains,
                        hipStream_t s);

// ---- stream skew (tests only; capi.cpp skew_point, APM_SKEW) ------------------------------
// Every launch goes through APM_LAUNCH, which first lets skew_point enqueue a delay kernel on the
// launch's stream when the calling thread's context asked for it: a cross-stream edge without
// its wait then reads stale data deterministically instead of by chance.
#ifdef APM_TOOL_NO_SKEW  // stand-alone development benches that include a .hip file directly
inline void skew_point(hipStream_t) {}
#else
void skew_point(hipStream_t s);
#endif
void launch_delay(int us, hipStream_t s);
#define APM_LAUNCH(kern, grid, block, lds, st, ...)                      \
    do {                                                                 \
        skew_point(st);                                                  \
        hipLaunchKernelGGL(kern, grid, block, lds, st, __VA_ARGS__);     \
    } while (0)
