// C-ABI (include/apm.h) and host orchestration of the theta-call / u-call pipelines.
//
// theta-call (ApproxPosteriorIS, gpdemo/estimators.py:203-241), per batch of chains, one stream:
//   Gram -> Newton loop { prep, K b, form B|rhs, chol(B) (+ forward solve), L^T solve, a, K a,
//   check } -> augmented chol [[B,.],[K W^1/2, K],[0, f_post^T]] -> slot -> L.U + probit -> LME
// The only host syncs are one per Newton iteration (convergence flags) and one at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <functional>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/apm.h"
#include "apm_internal.h"

#define APM_VERSION 1

static thread_local std::string g_err;

struct ProfRec {
    hipEvent_t a, b;
    int kind;
    double work;
};

// per chain: the trace(C) below which the reference's route to chol(C) is checked (icm_check):
// C's mean diagonal below APM_ICM_Q^-1 of K's largest diagonal entry, i.e. K - V^T V cancels
// ~log10(APM_ICM_Q) digits or more (1e-7 of K_ii at the golden ICM theta icm_a, 1e-5 at icm_b;
// ~1/4 at configs[2]'s sigma = e^18.5, and no chain of the bench's stationary states: unchecked)
#define APM_ICM_Q 1.0e3
// the guard's bounds (k_guard_check): r1 nats of 1/2 log-determinant between the
// last Newton factor (fp32 with fp16x3 updates) and the fp64 posterior factor, r2 relative, r3
// nats between the fp32 slot's log-diagonal and the fp64 log-determinants, r4 max |C_chol g -
// f_post| over the rows relative to max(1, max |f_post|); measured maxima in
// DESIGN.md §11 (tests/test_gpu_errors.py::test_guard_residuals_are_rounding_sized)
#define GUARD_T1 1.0
#define GUARD_T2 1.0e-6
#define GUARD_T3 5.0e-2
#define GUARD_T4 1.0e-4

// The cross-stream edges of a theta-call, one event each (DESIGN.md §11 names the producer and
// the consumer of every one). No event is recorded again before the wait that names its previous
// record has been enqueued: the per-panel edges are indexed by panel; the Newton lookahead's
// per-panel pair is recorded once per factorisation, and a factorisation starts only after the
// previous one's last far update was joined into the main stream.
struct Edges {
    hipEvent_t gram_k = nullptr;       // main -> s2: the Gram wrote K (and BL's first panel)
    hipEvent_t cholk_done = nullptr;   // s2 -> main: L_K final in BL, its log-det in ldet + nb
    hipEvent_t y2 = nullptr;           // main -> s2: L_K J formed in BL (k_form_y2_rev)
    hipEvent_t bottom_done = nullptr;  // s2 -> main: the fp32 bottom block (S32) final
    std::vector<hipEvent_t> cholk_rel; // main -> s2, per chol(K) panel: its release (no data)
    std::vector<hipEvent_t> lp_panel;  // main -> s2, per panel of L': tiles and inverses final
    std::vector<hipEvent_t> df;        // main -> s3, per Newton panel: its columns + planes final
    std::vector<hipEvent_t> far;       // s3 -> main, per Newton panel: its far update done
    std::vector<hipEvent_t*> all() {
        std::vector<hipEvent_t*> v{&gram_k, &cholk_done, &y2, &bottom_done};
        for (auto* w : {&cholk_rel, &lp_panel, &df, &far})
            for (hipEvent_t& e : *w) v.push_back(&e);
        return v;
    }
};

struct apm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int kind = 0, n = 0, d = 0, np = 0, nb = 0, P = 0, S = 0, sp = 0;
    int max_batch = 0, n_slots = 0, n_ubufs = 0;
    // tiles per outer panel of the fp64 factorisations and of the Newton matrix (<= 14: the
    // dataflow panel's progress word packs the column step in 4 bits, 15 = failed;
    // rhs_row_update32 covers a depth of 16 tiles; the explicit-inverse panels need 8)
    static constexpr int outer = 8, outer32 = 8;
    std::vector<int> slot_refs;  // owners of each cache slot (apm_cache_*; 0 = free)
    std::vector<int> slot_wide;  // host mirror of Sl.wide (read back with each theta-call)
    // fp64 factors of the wide slots: one np x np buffer attached per wide slot (Sl.L64 is the
    // device copy of l64_h), returned to l64_free when its slot is rewritten narrow
    std::vector<double*> l64_h, l64_free;
    double** l64_d = nullptr;
    double eps = 1e-8, tol = 1e-4;
    int64_t max_iters = 1000;
    std::string err;
    // device data
    double *X = nullptr, *y = nullptr, *theta = nullptr;
    MatB K{}, A{};
    double *Dinv = nullptr, *ldet = nullptr, *out = nullptr, *partial = nullptr;
    int64_t dstride = 0, lstride = 0, pstride = 0;
    NewtonVecs v{};
    double* vecbase = nullptr;
    double* rvec = nullptr;   // 3 refinement vectors per chain (mixed-precision Newton)
    double* sympart = nullptr;  // symmetric K x partials: nb*nb*64 per chain (launch_symv)
    int64_t sstride = 0;
    bool mixed = true;        // APM_MIXED=0: fp64 Newton factorisation (development knob)
    int n_refine = 3;         // maximum refinement steps per solve (APM_REFINE overrides)
    double refine_tol = 1e-3; // acceptance of a refinement step (k_refine_check)
    int *active = nullptr, *status = nullptr, *n_iter = nullptr;
    int* refining = nullptr;  // chains still refining their Newton solve
    double* refine_prev = nullptr;  // max|d| of the previous refinement step per chain
    int64_t n_refine_steps = 0, n_fp64_rerun = 0;  // statistics (apm_prof_read APM_PROF_STATS)
    int64_t n_icm_check = 0;  // chains whose C was formed the reference's way (icm_check)
    int64_t n_guard = 0;      // chains failed by the guard (APM_STATUS_GUARD)
    // APM_ICM_Q: the threshold of the check of the reference's chol(C) (icm_check; test knob: a
    // huge value checks every chain, 0 checks none)
    double icm_q = APM_ICM_Q;
    int64_t *d_slots = nullptr, *d_ubufs = nullptr, *d_i3 = nullptr;  // d_ubufs = d_slots + B
    // pinned host staging of the per-call uploads (one H2D of slots + ubufs; the per-chain
    // fp16x3 flags): [B slots][B ubufs][B h3ok]
    char* hpin = nullptr;
    int64_t* hblk = nullptr;  // pinned mirror of the d_i3 .. d_ctrs block (apm_u_normal/combine)
    double* hth = nullptr;    // pinned theta staging (B x P)
    // read-back buffer: mapped, coherent pinned host memory (4B words) written by k_export
    // (APM_EXPORT=0: filled by hipMemcpyAsync instead), dx its device address
    unsigned* hx = nullptr;
    unsigned* dx = nullptr;
    double *d_ca = nullptr, *d_cb = nullptr;
    uint64_t *d_seeds = nullptr, *d_ctrs = nullptr;
    double* U64 = nullptr;
    SlotSet Sl{};
    UPool Up{};
    std::vector<void*> allocs;
    // K's upper triangle holds valid data (host-uploaded K, or the Gram wrote both triangles);
    // otherwise every K x product uses the symmetric lower-tile kernel (launch_symv)
    bool k_full = false;
    // profiling
    int prof = 0;  // apm_prof_enable level
    std::vector<hipEvent_t> evpool;
    size_t evnext = 0;
    std::vector<ProfRec> recs;
    // update-tile lists per launch shape (i0, R, j0, jend), built once, kept on the device
    std::map<std::tuple<int, int, int, int, int, int>, std::pair<unsigned*, int>> tile_lists;
    std::map<std::tuple<int, int, int, int, int, int>, std::pair<unsigned*, int>> super_lists;
    std::map<std::tuple<int, int, int, int, int, int>, std::pair<unsigned*, int>> super_lists_solo;
    std::map<std::tuple<int, int, int, int>, std::pair<unsigned*, int>> quad_lists;
    std::map<std::tuple<int, int, int, int, int, int>, std::pair<unsigned*, int>> super_lists_ext;
    // 128x128 super-tile kernels for the outer updates: bit 0 fp32, bit 1 fp64 (APM_T128)
    bool h3 = true;       // APM_H3=0: fp32 operands in the fp32 factorisations' outer updates
    bool h3_now = false;  // some chain of the current theta-call may use fp16x3 updates
    bool h3_all = false;  // ... and every chain may (the quad-tile far updates need that)
    bool h3post_all = false;  // every chain takes fp16x3 operands in the posterior bottom block
    int* h3ok = nullptr;  // per chain: fp16x3 allowed (range check on theta_0, chol32.hip)
    int* h3post = nullptr;  // the same for the posterior factor's fp32 bottom block (h3ok + B)
    // per chain: explicit-inverse Newton panels allowed (h3ok + 2B): their fp16x3 operands are
    // Schur-complement entries of B, bounded by max B_ii <= 1 + K_ii (not by sqrt(B_ii) as the
    // walk's solved entries are), so the range check is on 1 + K_ii itself (chol32.hip)
    int* invok = nullptr;
    bool inv_any = false, inv_all = false;
    double* icm_thr = nullptr;  // per chain: SlotSet::icm_thr
    // the bottom block of the posterior factor [[J M J],[L_K J]] (the TRSM that yields chol(C) J)
    // in fp32 panel by panel beside the fp64 factorisation of J M J (postcov.hip); chains whose
    // trace(C) exceeds Sl.post_q are recomputed in fp64 (n_post64 counts them)
    int* hmask = nullptr;  // pinned: the chains of such a recomputation
    int64_t n_post64 = 0;
    // the Newton factorisation's dataflow launches also write the panel's fp16x3 operand planes
    // (Planes16), which the trailing updates stage with LDS-DMA (two buffers by panel parity: the
    // lookahead's far update reads panel K's while the dataflow launch of K + 1 writes its own)
    unsigned short* planes = nullptr;
    int64_t plane_cs = 0;  // halves per chain and buffer
    // explicit-inverse panels (chol32.hip k_zinv_* / k_panel_inv_gemm32): the dataflow launch
    // walks the diagonal block and the right-hand-side row only; Z = inv(L_D) per chain (fp32
    // scratch zt: Z, Z^T, T^T; fp16x3 planes zplanes) and one GEMM per row tile below
    static constexpr int symv_tpw = 2;  // K x: lower tiles per workgroup
    float* zt = nullptr;
    unsigned short* zplanes = nullptr;
    // per (chain, row tile) progress words, then [dataflow timeouts][TRSV timeouts][ticket]
    unsigned long long* dfprog = nullptr;
    unsigned long long df_fact = 0;        // factorisations so far (the words' monotonic base)
    // the arrival-ticket counter of the main stream's hand-over kernels (SpinCtl): reset at the
    // start of every theta-call, ticket_base = the tickets the call's launches have drawn so far
    unsigned long long ticket_base = 0;
    int spin_df = 1 << 22, spin_trsv = 1 << 20;  // poll bounds (APM_SPIN_LIMIT: tests only)
    // chains whose work the roofline accounting credits (Newton: the unconverged ones after the
    // previous convergence read; update_flops x live_n instead of x count)
    int live_n = 0;
    // chol(K) of the mixed-precision IS theta-call on a low-priority second stream, concurrent
    // with the Newton iterations, and the fp32 bottom block of the posterior factor on the same
    // stream; the far part of each Newton trailing update on stream3 beside the next panel's
    // dataflow launch (one-panel lookahead, chol_range32)
    hipStream_t stream2 = nullptr;
    hipStream_t stream3 = nullptr;
    // pacing of the concurrent chol(K) (feed_chol_k): panels it may still release in this Newton
    // iteration, from the previous theta-call's iteration count (newton_last; 0: no pacing)
    int cholk_quota = 1 << 30, newton_last = 0;
    Edges ev;  // one event per cross-stream edge
    int skew = 0;  // APM_SKEW (tests only): delay kernels in front of launches (skew_point), bit 2
                   // drops the bottom_done wait
    // per-chain guard data (k_guard_*): [1/2 log|B| of the last Newton factor][1/2 log|K|]
    // [residuals r1 .. r4 of the last theta-call]
    double* guard = nullptr;
    double* guard_rows = nullptr;  // the slot writer's row residuals of C_chol g = f_post (B x np)
    int *active2 = nullptr, *status2 = nullptr;
    // chol(K) is enqueued one outer panel at a time, each released when the main stream enters a
    // single-workgroup-per-chain TRSV (3/4 of the CUs idle) - see feed_chol_k
    int cholk_next = -1, cholk_count = 0;
    // the Gram wrote only the first outer panel's tile columns into chol(K)'s working copy: the
    // first trailing update then reads its old tiles from K (out of place, k_chol_update_t128 S)
    bool cholk_partial = false;
};

// ------------------------------------------------------------------------------- APM_SKEW
// (tests only) the calling thread's context selects delay kernels in front of every launch on
// its secondary streams (bit 0: chol(K), the posterior's bottom block, the Newton far updates)
// and/or its main stream (bit 1). Every cross-stream edge is an event (Edges); with one side of
// an edge held back by the delays, a missing or misplaced wait shows as a changed result, which
// tests/test_gpu_errors.py::test_stream_skew_is_bitwise_neutral compares bitwise.
namespace {
struct SkewState {
    int mode = 0;
    hipStream_t main = nullptr, s2 = nullptr, s3 = nullptr;
};
thread_local SkewState t_skew;
constexpr int SKEW_US_SECONDARY = 1000, SKEW_US_MAIN = 40;
struct SkewScope {  // an API entry point's launches belong to context c
    SkewState prev;
    explicit SkewScope(const apm_ctx* c) : prev(t_skew) {
        t_skew = SkewState{c->skew & 3, c->stream, c->stream2, c->stream3};
    }
    ~SkewScope() { t_skew = prev; }
};
}  // namespace

void skew_point(hipStream_t s) {
    if (!t_skew.mode || !s) return;
    if ((t_skew.mode & 1) && (s == t_skew.s2 || s == t_skew.s3))
        launch_delay(SKEW_US_SECONDARY, s);
    else if ((t_skew.mode & 2) && s == t_skew.main)
        launch_delay(SKEW_US_MAIN, s);
}

namespace {

struct HipError {
    std::string msg;
};

#define HIPC(x)                                                                              \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess)                                                                \
            throw HipError{std::string(#x) + ": " + hipGetErrorString(e_)};                  \
    } while (0)

template <class T>
T* dalloc(apm_ctx* c, size_t count) {
    void* p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(&p, count * sizeof(T));
    if (e != hipSuccess)
        throw HipError{"hipMalloc(" + std::to_string(count * sizeof(T)) +
                       " bytes): " + hipGetErrorString(e)};
    c->allocs.push_back(p);
    return static_cast<T*>(p);
}

int fail(apm_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    g_err = m;
    return code;
}

void check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw HipError{std::string("kernel launch: ") + hipGetErrorString(e)};
}

// ------------------------------------------------------------------------------- profiling
hipEvent_t next_event(apm_ctx* c) {
    if (c->evnext == c->evpool.size()) {
        hipEvent_t e;
        HIPC(hipEventCreate(&e));
        c->evpool.push_back(e);
    }
    return c->evpool[c->evnext++];
}

struct ProfScope {
    apm_ctx* c;
    int kind;
    double work;
    hipStream_t s;
    hipEvent_t a{}, b{};
    bool on = false;
    ProfScope(apm_ctx* c_, int k, double w, hipStream_t s_ = nullptr)
        : c(c_), kind(k), work(w), s(s_ ? s_ : c_->stream) {
        // the all-updates kinds time every in-panel launch: detailed level (2) only
        const bool all_upd = kind == APM_PROF_CHOL_UPDATE || kind == APM_PROF_CHOL_UPDATE32;
        if (kind >= 0 && c->prof >= (all_upd ? 2 : 1)) {
            on = true;
            a = next_event(c);
            b = next_event(c);
            HIPC(hipEventRecord(a, s));
        }
    }
    ~ProfScope() {
        if (on && hipEventRecord(b, s) == hipSuccess)
            c->recs.push_back(ProfRec{a, b, kind, work});
    }
};

// ------------------------------------------------------------------------------- building blocks
Live live_of(apm_ctx* c) { return Live{c->active, c->status}; }

// Where a factorisation runs: stream, liveness, diagonal-inverse / log-det arrays. The main path
// uses the context stream; chol(K) of the IS theta-call runs concurrently on the low-priority
// second stream with its own liveness and the upper halves of Dinv / ldet (theta_eval_impl).
struct Exec {
    hipStream_t s;
    Live lv;
    double* Dinv;
    double* ldet;
    int live_n;  // chains credited by the roofline accounting
};
Exec main_exec(apm_ctx* c) { return Exec{c->stream, live_of(c), c->Dinv, c->ldet, c->live_n}; }

// Two-level right-looking Cholesky over tile columns [k0, k1) of rows < R (tile units), the
// trailing matrix spanning columns < Cb. Outer panels of OUTER tiles (256 columns) are factored
// with the 64-wide diag / panel / inner-update steps; the rest of the matrix then receives one
// rank-256 update per outer panel (4x less read-modify-write traffic than rank-64 steps).
// row_start > 0 restricts every panel solve and update to rows >= row_start (the top-left of the
// augmented matrix is already factored); factor_diag = false reuses L_kk and inv(L_kk).

// Row tiles [lo, hi) known to be zero in panel column k (skipped by panel and update).
struct Gap {
    int lo, hi;
};
typedef Gap (*GapFn)(int k, int nb);
Gap no_gap(int, int) { return Gap{0, 0}; }
// [[J M J],[L_K J]] factorisation (postcov.hip): row tile nb+I of L_K J is zero in every column
// tile k < nb-1-I, so at column k only bottom rows >= 2nb-1-k are nonzero.
Gap y_gap(int k, int nb) { return Gap{nb, std::max(nb, 2 * nb - 1 - k)}; }

double update_flops(int i0, int R, int j0, int jend, int kc, Gap g, bool syrk_lower = false) {
    double f = 0.0;
    for (int i = i0; i < R; ++i) {
        if (i >= g.lo && i < g.hi) continue;
        const int jmax = std::min(i, jend - 1);
        for (int j = j0; j <= jmax; ++j) {
            const int k = syrk_lower ? std::min(kc, j + 1) : kc;  // plus == 2: k <= j only
            f += (i == j) ? 64.0 * 65.0 * 64.0 * k : 2.0 * 64.0 * 64.0 * 64.0 * k;
        }
    }
    return f;
}

std::pair<unsigned*, int> tile_list(apm_ctx* c, int i0, int R, int j0, int jend, Gap g) {
    auto key = std::make_tuple(i0, R, j0, jend, g.lo, g.hi);
    auto it = c->tile_lists.find(key);
    if (it != c->tile_lists.end()) return it->second;
    std::vector<unsigned> v = build_update_tiles(i0, R, j0, jend, g.lo, g.hi);
    unsigned* d = dalloc<unsigned>(c, v.size());
    HIPC(hipMemcpy(d, v.data(), sizeof(unsigned) * v.size(), hipMemcpyHostToDevice));
    auto val = std::make_pair(d, (int)v.size());
    c->tile_lists[key] = val;
    return val;
}

// Trailing update of tiles (i, j), i in [i0, R) minus the gap, j in [j0, min(i, jend-1)], by
// columns [k0, k0+kc). fuse_k >= 0: the launch also factors diagonal tile (fuse_k, fuse_k), which
// must be its first tile (i0 == j0 == fuse_k; the super-tile order starts there).
std::pair<unsigned*, int> super_list(apm_ctx* c, int i0, int R, int j0, int jend, Gap g,
                                     int solo = -1);

void tracked_update(apm_ctx* c, MatB M, int k0, int kc, int i0, int R, int j0, int jend, Gap g,
                    int plus, int count, int fuse_k = -1, int fail_code = 0,
                    const Exec* ex = nullptr, const MatB* src = nullptr) {
    const Exec E = ex ? *ex : main_exec(c);
    if (i0 < j0) i0 = j0;
    if (update_tile_count(i0, R, j0, jend) <= 0) return;
    const bool t128 = kc >= 2 && jend - j0 >= 2 && (fuse_k < 0 || (i0 == fuse_k && j0 == fuse_k));
    if (src && (!t128 || plus == 2))  // (theta_eval_impl enables it only where it holds)
        throw HipError{"out-of-place update needs the fp64 t128 path"};
    const auto tl = tile_list(c, i0, R, j0, jend, g);
    if (tl.second <= 0) return;
    FusedDiag<double> fd{0, nullptr, 0, nullptr, 0, 0};
    if (fuse_k >= 0) fd = FusedDiag<double>{1, E.Dinv, c->dstride, E.ldet, c->lstride, fail_code};
    const double fl = c->prof ? update_flops(i0, R, j0, jend, kc, g, plus == 2) * E.live_n : 0.0;
    ProfScope ps(c, APM_PROF_CHOL_UPDATE, fl, E.s);
    ProfScope ps_outer(c, kc >= 2 && jend - j0 >= 2 ? APM_PROF_CHOL_UPDATE_OUTER : -1, fl, E.s);
    if (t128) {
        const auto sl = super_list(c, i0, R, j0, jend, g);
        launch_chol_update_t128(M, k0, kc, sl.first, sl.second, plus, E.lv, count, E.s, fd,
                                src ? *src : MatB{nullptr, 0, 0});
    } else {
        if (plus == 2) throw HipError{"identity-initialised update needs the t128 path"};
        launch_chol_update(M, k0, kc, tl.first, tl.second, plus != 0, E.lv, count, E.s, fd);
    }
    check_launch();
}

// Two-level right-looking Cholesky over tile columns [k0, k1) of rows < R (tile units), the
// trailing matrix spanning columns < Cb. Outer panels of OUTER tiles (256 columns) are factored
// with 64-wide diag / panel / inner-update steps; the rest of the matrix then receives one
// rank-256 update per outer panel (4x less read-modify-write traffic than rank-64 steps). Every
// diagonal tile after the first is factored inside the update launch that completes it (fused
// diag: its one-wave latency hides under that launch instead of idling the GPU between launches).
// row_start > 0 restricts every panel solve and update to rows >= row_start (the top-left of the
// augmented matrix is already factored); factor_diag = false reuses L_kk and inv(L_kk).
// after_panel(K, Kend): called (host side) once the panel's columns are final, before its outer
// update is enqueued (the posterior factor's fp32 bottom block follows the panels on stream2).
void chol_range(apm_ctx* c, MatB M, int k0, int k1, int R, int Cb, int fail_code, int count,
                bool factor_diag = true, int row_start = 0, GapFn gap = no_gap,
                const Exec* ex = nullptr, const MatB* first_src = nullptr,
                const std::function<void(int, int)>& after_panel = nullptr) {
    const Exec E = ex ? *ex : main_exec(c);
    const Live lv = E.lv;
    const bool fuse = factor_diag && row_start <= k0;
    bool have_diag = false;  // tile (k, k) already factored by the previous update launch
    for (int K = k0; K < k1; K += c->outer) {
        const int Kend = std::min(K + c->outer, k1);
        if (fuse) {
            // left-looking inside the outer panel: column k receives all of the panel's earlier
            // columns in ONE update (depth (k-K)*64, one read-modify-write of its tiles instead
            // of k-K), whose first tile is the diagonal tile it then factors (fused diag)
            for (int k = K; k < Kend; ++k) {
                const Gap g = gap(k, c->nb);
                if (k > K)
                    tracked_update(c, M, K, k - K, k, R, k, k + 1, g, false, count, k, fail_code, &E);
                else if (!have_diag) {
                    launch_chol_diag(M, k, E.Dinv, c->dstride, E.ldet, c->lstride, lv,
                                     fail_code, count, E.s);
                    check_launch();
                }
                launch_chol_panel(M, k, k + 1, R, g.lo, g.hi, E.Dinv, c->dstride, lv, count,
                                  E.s);
                check_launch();
            }
            if (after_panel) after_panel(K, Kend);
            have_diag = Kend < k1;
            tracked_update(c, M, K, Kend - K, Kend, R, Kend, Cb, gap(Kend - 1, c->nb), false,
                           count, have_diag ? Kend : -1, fail_code, &E, K == k0 ? first_src : nullptr);
            continue;
        }
        for (int k = K; k < Kend; ++k) {
            if (factor_diag && !have_diag) {
                launch_chol_diag(M, k, E.Dinv, c->dstride, E.ldet, c->lstride, lv, fail_code,
                                 count, E.s);
                check_launch();
            }
            const Gap g = gap(k, c->nb);
            launch_chol_panel(M, k, std::max(k + 1, row_start), R, g.lo, g.hi, E.Dinv,
                              c->dstride, lv, count, E.s);
            check_launch();
            have_diag = fuse && k + 1 < Kend;
            tracked_update(c, M, k, 1, std::max(k + 1, row_start), R, k + 1, Kend, g, false,
                           count, have_diag ? k + 1 : -1, fail_code, &E);
        }
        have_diag = fuse && Kend < k1;
        tracked_update(c, M, K, Kend - K, std::max(Kend, row_start), R, Kend, Cb,
                       gap(Kend - 1, c->nb), false, count, have_diag ? Kend : -1, fail_code, &E,
                       K == k0 ? first_src : nullptr);
    }
}

// ---- fp32 factorisation of the Newton matrix (chol32.hip), in the memory of the work matrix
unsigned long long* spin_words(apm_ctx* c) {  // [dataflow timeouts][TRSV timeouts][ticket]
    return c->dfprog + (size_t)c->max_batch * (c->nb + 1);
}
SpinCtl spin_ctl(apm_ctx* c, bool trsv) {
    unsigned long long* w = spin_words(c);
    return SpinCtl{w + 2, c->ticket_base, trsv ? w + 1 : w, trsv ? c->spin_trsv : c->spin_df};
}
void reset_tickets(apm_ctx* c) {
    HIPC(hipMemsetAsync(spin_words(c) + 2, 0, sizeof(unsigned long long), c->stream));
    c->ticket_base = 0;
}
void trsv32(apm_ctx* c, bool fwd, MatF F, const float* D, int64_t ds, const double* r,
            double* out, Live lv, int count) {
    c->ticket_base += (unsigned long long)launch_trsv32_mw(
        fwd, F, c->nb, D, ds, r, out, c->v.vstride, lv, count, APM_STATUS_CHOL_B,
        spin_ctl(c, true), c->stream);
    check_launch();
}
Planes16 planes_of(apm_ctx* c, int K) {
    if (!c->planes || !c->h3_now) return Planes16{nullptr, 0, 0, 0};
    return Planes16{c->planes + ((K / c->outer32) & 1) * c->max_batch * c->plane_cs, c->plane_cs,
                    c->plane_cs / 2, c->np};
}
MatF b32_of(apm_ctx* c) {
    return MatF{reinterpret_cast<float*>(c->A.base), c->np, 2 * c->A.cstride};
}
float* dinv32_of(apm_ctx* c) { return reinterpret_cast<float*>(c->Dinv); }

std::pair<unsigned*, int> super_list(apm_ctx* c, int i0, int R, int j0, int jend, Gap g,
                                     int solo) {
    auto& lists = solo >= 0 ? c->super_lists_solo : c->super_lists;
    auto key = std::make_tuple(i0, R, j0, jend, g.lo, g.hi);
    auto it = lists.find(key);
    if (it != lists.end()) return it->second;
    std::vector<unsigned> v = build_update_supertiles(i0, R, j0, jend, g.lo, g.hi, solo);
    unsigned* d = dalloc<unsigned>(c, v.size());
    HIPC(hipMemcpy(d, v.data(), sizeof(unsigned) * v.size(), hipMemcpyHostToDevice));
    auto val = std::make_pair(d, (int)v.size());
    lists[key] = val;
    return val;
}

// the super-tiles of (i0, R, j0, jend) with row tile rhs alone, followed by that row's super-tiles
// of the columns [jend, jext): the next panel's columns of a lookahead update and the right-hand
// side row's far columns in one launch
std::pair<unsigned*, int> super_list_ext(apm_ctx* c, int i0, int R, int j0, int jend, int rhs,
                                         int jext) {
    auto key = std::make_tuple(i0, R, j0, jend, rhs, jext);
    auto it = c->super_lists_ext.find(key);
    if (it != c->super_lists_ext.end()) return it->second;
    std::vector<unsigned> v = build_update_supertiles(i0, R, j0, jend, 0, 0, rhs);
    const std::vector<unsigned> e = build_update_supertiles(rhs, rhs + 1, jend, jext, 0, 0, rhs);
    v.insert(v.end(), e.begin(), e.end());
    unsigned* d = dalloc<unsigned>(c, v.size());
    HIPC(hipMemcpy(d, v.data(), sizeof(unsigned) * v.size(), hipMemcpyHostToDevice));
    auto val = std::make_pair(d, (int)v.size());
    c->super_lists_ext[key] = val;
    return val;
}

std::pair<unsigned*, int> quad_list(apm_ctx* c, int i0, int R, int j0, int jend) {
    auto key = std::make_tuple(i0, R, j0, jend);
    auto it = c->quad_lists.find(key);
    if (it != c->quad_lists.end()) return it->second;
    std::vector<unsigned> v = build_update_quads(i0, R, j0, jend);
    unsigned* d = dalloc<unsigned>(c, std::max<size_t>(1, v.size()));
    if (!v.empty())
        HIPC(hipMemcpy(d, v.data(), sizeof(unsigned) * v.size(), hipMemcpyHostToDevice));
    auto val = std::make_pair(d, (int)v.size());
    c->quad_lists[key] = val;
    return val;
}

void tracked_update32(apm_ctx* c, MatF M, int k0, int kc, int i0, int R, int j0, int jend,
                      int count, int fuse_k = -1, int fail_code = 0, hipStream_t st = nullptr,
                      Planes16 pl = Planes16{nullptr, 0, 0, 0}, int jext = -1) {
    if (!st) st = c->stream;
    if (i0 < j0) i0 = j0;
    if (update_tile_count(i0, R, j0, jend) <= 0) return;
    const auto tl = tile_list(c, i0, R, j0, jend, Gap{0, 0});
    if (tl.second <= 0) return;
    FusedDiag<float> fd{0, nullptr, 0, nullptr, 0, 0};
    if (fuse_k >= 0)
        fd = FusedDiag<float>{1, dinv32_of(c), 2 * c->dstride, c->ldet, c->lstride, fail_code};
    const bool outer = kc >= 2 && jend - j0 >= 2 && (fuse_k < 0 || (i0 == fuse_k && j0 == fuse_k));
    // the Newton matrix's appended right-hand-side row tile (nb, rows < R) is updated as a row
    // vector (rhs_row_update32); with the quad tiles that row is a launch of its own (role 3,
    // outside the profiled scope: the roofline's launches are the quad and 128-row GEMMs)
    const int rhs = R > c->nb || jext > 0 ? c->nb : -1;
    const bool quad =
        outer && pl.base && fuse_k < 0 && c->h3_all && i0 < c->nb && jext <= 0;
    {
        const int Rg = quad ? std::min(R, c->nb) : R;
        const double fl = c->prof ? update_flops(i0, Rg, j0, jend, kc, Gap{0, 0}) * c->live_n : 0.0;
        ProfScope ps(c, APM_PROF_CHOL_UPDATE32, fl, st);
        ProfScope ps_outer(c, outer ? APM_PROF_CHOL_UPDATE32_OUTER : -1, fl, st);
        if (quad) {
            const auto ql = quad_list(c, i0, Rg, j0, jend);
            launch_chol_update32_q256(M, k0, kc, ql.first, ql.second, live_of(c), count, st,
                                      c->h3ok, pl);
        } else if (outer) {
            // jext > jend: also the right-hand-side row's columns [jend, jext)
            const auto sl = jext > jend ? super_list_ext(c, i0, R, j0, jend, rhs, jext)
                                                    : super_list(c, i0, R, j0, jend, Gap{0, 0}, rhs);
            launch_chol_update32_t128(M, k0, kc, sl.first, sl.second, live_of(c), count, st, fd,
                                      c->h3_now ? c->nb : 0, c->h3ok, rhs, 0, pl);
        } else {
            launch_chol_update32(M, k0, kc, tl.first, tl.second, live_of(c), count, st, fd,
                                 c->h3_now ? c->nb : 0, c->h3ok);
        }
        check_launch();
    }
    if (quad && R > c->nb) {
        const auto sl = super_list(c, c->nb, R, j0, jend, Gap{0, 0}, rhs);
        launch_chol_update32_t128(M, k0, kc, sl.first, sl.second, live_of(c), count, st, fd,
                                  c->nb, c->h3ok, rhs, 3, pl);
        check_launch();
    }
}

// chol_range's twin for the fp32 Newton matrix: one dataflow launch per outer panel
// (k_chol_panel_df32: the in-panel steps, fused diagonal tiles), the explicit-inverse panel for
// the chains invok allows, and the trailing update with a one-panel lookahead (the far part on
// stream3 beside the next panel's dataflow launch)
void chol_range32(apm_ctx* c, MatF M, int k0, int k1, int R, int Cb, int fail_code, int count) {
    const Live lv = live_of(c);
    float* D = dinv32_of(c);
    const int64_t ds = 2 * c->dstride;
    bool have_diag = false;
    const unsigned long long fact = ++c->df_fact;
    int far_pending = -1;  // the panel whose far update on stream3 is not yet joined
    for (int K = k0; K < k1; K += c->outer32) {
        const int Kend = std::min(K + c->outer32, k1);
        const int p = K / c->outer32;
        if (!have_diag) {
            launch_chol_diag32(M, K, D, ds, c->ldet, c->lstride, lv, fail_code, count, c->stream);
            check_launch();
        }
        // explicit-inverse panel for the invok chains; with every chain invok the dataflow
        // launch covers the diagonal block and the right-hand-side row only, else all rows, those
        // of the invok chains below the diagonal block returning at once
        const bool inv = c->inv_any && c->zt && Kend - K == 8 && Kend < c->nb &&
                         R <= c->nb + 1 && planes_of(c, K).base;
        const bool compact = inv && c->inv_all;
        const long tickets = launch_chol_panel_df32(
            M, K, Kend - K, compact ? Kend + (R > c->nb ? 1 : 0) : R,
            FusedDiag<float>{1, D, ds, c->ldet, c->lstride, fail_code}, lv, count,
            c->h3_now ? c->nb : 0, c->h3ok, c->dfprog, c->nb + 1,
            (fact << 16) | ((unsigned long long)p << 4), spin_ctl(c, false), c->stream,
            planes_of(c, K), compact && R > c->nb ? c->nb : -1, inv && !compact ? c->invok : nullptr);
        if (tickets < 0) throw HipError{"dataflow Newton panel wider than 14 tiles"};
        check_launch();
        c->ticket_base += (unsigned long long)tickets;
        if (inv) {  // the rows below the diagonal block: X_i = A_i inv(L_D)^T
            const int64_t zcs = 2 * 16 * 512 * 32;
            launch_panel_inv32(M, K, c->nb, D, ds, c->zt, 3 * 512 * 512,
                               Planes16{c->zplanes, zcs, zcs / 2, 512}, planes_of(c, K), lv,
                               count, c->invok, c->stream);
            check_launch();
        }
        have_diag = Kend < k1;
        const int Knext = std::min(Kend + c->outer32, Cb);
        if (Knext < Cb) {
            // the next panel's columns first (narrow, with the fused diagonal tile), its dataflow
            // launch next on this stream, and the rest of the trailing update (far: columns >=
            // Knext) on stream3 beside it. Edge df[p] (main -> s3): panel p's columns, planes and
            // the previous narrow update are final. The narrow update shares its tiles with the
            // previous panel's far update: edge far[p-1] (s3 -> main) orders it behind that.
            HIPC(hipEventRecord(c->ev.df[p], c->stream));
            if (far_pending >= 0) HIPC(hipStreamWaitEvent(c->stream, c->ev.far[far_pending], 0));
            // (the right-hand-side row's far columns go with the narrow update on this stream)
            tracked_update32(c, M, K, Kend - K, Kend, R, Kend, Knext, count,
                             have_diag ? Kend : -1, fail_code, nullptr, planes_of(c, K),
                             R > c->nb ? Cb : -1);
            HIPC(hipStreamWaitEvent(c->stream3, c->ev.df[p], 0));
            tracked_update32(c, M, K, Kend - K, Knext, std::min(R, c->nb), Knext, Cb, count, -1,
                             fail_code, c->stream3, planes_of(c, K));
            HIPC(hipEventRecord(c->ev.far[p], c->stream3));
            far_pending = p;
            continue;
        }
        if (far_pending >= 0) {  // (the previous far update shares these tiles)
            HIPC(hipStreamWaitEvent(c->stream, c->ev.far[far_pending], 0));
            far_pending = -1;
        }
        tracked_update32(c, M, K, Kend - K, Kend, R, Kend, Cb, count, have_diag ? Kend : -1,
                         fail_code, nullptr, planes_of(c, K));
    }
    if (far_pending >= 0) HIPC(hipStreamWaitEvent(c->stream, c->ev.far[far_pending], 0));
}

void sync(apm_ctx* c) { HIPC(hipStreamSynchronize(c->stream)); }

// Read back up to four small per-chain device arrays (after the work enqueued so far on the
// main stream) and wait: one k_export launch into the mapped host buffer, a stream
// synchronisation, host copies.
struct RB {
    const void* src;
    int bytes;
    void* host;
};
void read_back(apm_ctx* c, std::initializer_list<RB> l) {
    Export e{};
    int k = 0;
    for (const RB& r : l) {
        e.src[k] = static_cast<const unsigned*>(r.src);
        e.words[k] = r.bytes / 4;
        ++k;
    }
    e.dst = c->dx;
    launch_export(e, c->stream);
    check_launch();
    sync(c);
    int off = 0;
    for (const RB& r : l) {
        std::memcpy(r.host, reinterpret_cast<const char*>(c->hx) + off, r.bytes);
        off += r.bytes;
    }
}

// slots / ubufs of a call -> device in one copy from pinned memory
void upload_idx(apm_ctx* c, int count, const int64_t* slots, const int64_t* ubufs) {
    int64_t* h = reinterpret_cast<int64_t*>(c->hpin);
    const int B = c->max_batch;
    if (slots) std::memcpy(h, slots, sizeof(int64_t) * count);
    if (ubufs) std::memcpy(h + B, ubufs, sizeof(int64_t) * count);
    if (ubufs)
        HIPC(hipMemcpyAsync(c->d_slots, h, sizeof(int64_t) * (B + count), hipMemcpyHostToDevice,
                            c->stream));
    else if (slots)
        HIPC(hipMemcpyAsync(c->d_slots, h, sizeof(int64_t) * count, hipMemcpyHostToDevice,
                            c->stream));
}
// pinned staging of a call's per-chain flags, [16B, 28B) of hpin: fp16x3 allowed (h3ok), for
// the posterior bottom block (h3post), explicit-inverse panels (invok) - the layout of the
// device block h3ok .. h3ok + 3B, uploaded with one copy - then the icm thresholds [32B, 40B)
int* pin_h3(apm_ctx* c) { return reinterpret_cast<int*>(c->hpin + 16 * c->max_batch); }
int* pin_h3post(apm_ctx* c) { return reinterpret_cast<int*>(c->hpin + 20 * c->max_batch); }
int* pin_inv(apm_ctx* c) { return reinterpret_cast<int*>(c->hpin + 24 * c->max_batch); }
double* pin_icm(apm_ctx* c) { return reinterpret_cast<double*>(c->hpin + 32 * c->max_batch); }

// per-chain range flags of a theta-call -> device. fp16x3 operands (chol32.hip): the walk's and
// the trailing updates' operands are solved entries of L, |L_ij| <= sqrt(B_ii) <= sqrt(1 + K_ii)
// (probit W < 1); the explicit-inverse panel also splits Schur-complement entries of B itself,
// |A_ij| <= max B_ii <= 1 + K_ii, so its flag asks 1 + K_ii < 2^15 (fp16 overflows at 65504).
// h3_now = any chain flagged (else the fp32-operand kernels launch), inv_any / inv_all likewise.
void upload_h3(apm_ctx* c, int count) {
    int* h = pin_h3(c);
    int* v = pin_inv(c);
    c->h3_now = c->inv_any = false;
    c->h3_all = c->inv_all = c->h3post_all = count > 0;
    for (int b = 0; b < count; ++b) {
        c->h3post_all &= pin_h3post(c)[b] != 0;
        v[b] = v[b] && h[b];
        c->h3_now |= h[b] != 0;
        c->h3_all &= h[b] != 0;
        c->inv_any |= v[b] != 0;
        c->inv_all &= v[b] != 0;
    }
    const int B = c->max_batch;
    HIPC(hipMemcpyAsync(c->h3ok, h, sizeof(int) * (2 * B + count), hipMemcpyHostToDevice,
                        c->stream));
    double* t = pin_icm(c);
    for (int b = 0; b < count; ++b) t[b] = c->icm_q > 0.0 ? t[b] : -1.0;
    HIPC(hipMemcpyAsync(c->icm_thr, t, sizeof(double) * count, hipMemcpyHostToDevice, c->stream));
}

// wide: some slot of the call may be wide (theta-calls: unknown until the read-back; u-calls:
// the host mirror) - the f64 MFMA twin is launched as well
void u_eval_device(apm_ctx* c, int count, bool wide) {
    {
        ProfScope ps(c, APM_PROF_UGEMM, (double)c->n * (c->n + 1) * c->S * count);
        launch_ugemm(c->Sl, c->d_slots, c->Up, c->d_ubufs, c->y, c->n, c->np, c->partial,
                     c->pstride, c->status, count, wide, c->stream);
        check_launch();
    }
    launch_lme(c->partial, c->pstride, c->nb, c->S, c->sp, c->Sl, c->d_slots, c->out, c->status,
               count, c->stream);
    check_launch();
}

// Newton loop of laplace_approximation over the live chains; returns host n_iter per chain.
// B x = W^1/2 K b with the fp32 factor (its forward solve is the appended row np) and n_refine
// steps of fp64 iterative refinement; x -> v.z (chol32.hip)
void feed_chol_k(apm_ctx* c);

void newton_solve32(apm_ctx* c, int count) {
    const Live lv = live_of(c);
    hipStream_t s = c->stream;
    const int nb = c->nb, np = c->np;
    const int64_t vs = c->v.vstride, ds = 2 * c->dstride;
    MatF F = b32_of(c);
    float* D = dinv32_of(c);
    double *r1 = c->rvec, *r2 = c->rvec + c->max_batch * vs, *r3 = c->rvec + 2 * c->max_batch * vs;
    chol_range32(c, F, 0, nb, nb + 1, nb, APM_STATUS_CHOL_B, count);  // B32 formed with K b
    launch_row32(F, np, np, r1, vs, lv, count, s);  // y0 = L^-1 rhs (fp32)
    check_launch();
    const bool mw_trsv = trsv32_mw_ok(np);
    if (mw_trsv) {
        feed_chol_k(c);
        trsv32(c, false, F, D, ds, r1, c->v.z, lv, count);
    } else {
        for (int J = nb - 1; J >= 0; --J) {
            launch_trsv_bwd32(F, J, D, ds, r1, c->v.z, vs, lv, count, s);
            check_launch();
        }
    }
    // fp64 iterative refinement against B = I + W^1/2 K W^1/2, adaptive per chain: a chain
    // leaves after the step its correction passes k_refine_check; one host read of the mask per
    // step decides whether another step is launched (usually one step suffices at N=4096)
    if (c->n_refine > 0) {
        launch_refine_mask(lv, c->refining, count, s);
        check_launch();
    }
    const Live lr{c->refining, c->status};
    std::vector<int> ref_h(count);
    for (int it = 0; it < c->n_refine; ++it) {
        launch_refine(0, c->v.Ws, c->v.Kb, c->v.z, nullptr, r2, vs, np, lr, count, s);  // t
        check_launch();
        launch_symv(c->K, r2, vs, r3, vs, c->sympart, c->sstride, np, MatF{}, nullptr, 0, lr,
                    count, s, c->symv_tpw);  // K t
        check_launch();
        launch_refine(1, c->v.Ws, c->v.Kb, c->v.z, r3, r1, vs, np, lr, count, s);       // res
        check_launch();
        if (mw_trsv) {
            feed_chol_k(c);
            trsv32(c, true, F, D, ds, r1, r2, lr, count);
            feed_chol_k(c);
            trsv32(c, false, F, D, ds, r2, r3, lr, count);
        } else {
            for (int J = 0; J < nb; ++J) {
                launch_trsv_fwd32(F, J, nb, D, ds, r1, r2, vs, lr, count, s);
                check_launch();
            }
            for (int J = nb - 1; J >= 0; --J) {
                launch_trsv_bwd32(F, J, D, ds, r2, r3, vs, lr, count, s);
                check_launch();
            }
        }
        launch_refine(2, nullptr, nullptr, c->v.z, nullptr, r3, vs, np, lr, count, s);  // x += d
        check_launch();
        const bool last = it + 1 == c->n_refine;
        launch_refine_check(c->v.z, r3, vs, np, c->refine_tol, APM_STATUS_CHOL_B, it, last,
                            c->refine_prev, c->refining, c->status, count, s);
        check_launch();
        ++c->n_refine_steps;
        if (last) break;
        read_back(c, {RB{c->refining, (int)sizeof(int) * count, ref_h.data()}});
        bool any = false;
        for (int b = 0; b < count; ++b) any |= ref_h[b] != 0;
        if (!any) break;
    }
}

void newton(apm_ctx* c, int count, std::vector<int>& st_h, bool mixed, int live0) {
    const Live lv = live_of(c);
    c->live_n = live0;
    // f = 0 for the live chains only (a fallback rerun must keep the other chains' modes)
    launch_refine(3, nullptr, nullptr, nullptr, nullptr, c->v.f, c->v.vstride, c->np, lv, count,
                  c->stream);
    check_launch();
    std::vector<int> act(count, 1);  // max_iters == 0: every chain is unconverged
    const int64_t rrow = c->np;  // Newton rhs row (extra row block below B)
    int64_t it = 0;
    for (; it < c->max_iters; ++it) {
        // the concurrent chol(K)'s panels spread over the iterations the previous call took (one
        // per iteration at the stationary states): released all at once they ran beside the first
        // two iterations and slowed them more than they gained (-2.5 ms per theta-call)
        c->cholk_quota = 1 << 30;
        if (c->newton_last > 0 && c->cholk_next >= 0 && c->cholk_next < c->nb) {
            const int left = (c->nb - c->cholk_next + c->outer - 1) / c->outer;
            const int its = std::max<int>(1, c->newton_last - (int)it);
            c->cholk_quota = (left + its - 1) / its;
        }
        launch_newton_prep(c->v, c->y, c->n, c->np, lv, count, c->stream);
        check_launch();
        if (mixed) {  // K b and the fp32 B (+ its right-hand side) in one pass over K's lower half
            launch_symv(c->K, c->v.b, c->v.vstride, c->v.Kb, c->v.vstride, c->sympart, c->sstride,
                        c->np, b32_of(c), c->v.Ws, c->v.vstride, lv, count, c->stream,
                        c->symv_tpw);
        } else if (c->k_full) {
            launch_gemv(c->K, c->v.b, c->v.vstride, c->v.Kb, c->v.vstride, c->np, lv, count,
                        c->stream);
        } else {
            launch_symv(c->K, c->v.b, c->v.vstride, c->v.Kb, c->v.vstride, c->sympart, c->sstride,
                        c->np, MatF{}, nullptr, 0, lv, count, c->stream, c->symv_tpw);
        }
        check_launch();
        if (mixed) {
            newton_solve32(c, count);
        } else {
            launch_form_B(c->K, c->A, c->v, c->np, lv, count, c->stream);
            check_launch();
            chol_range(c, c->A, 0, c->nb, c->nb + 1, c->nb, APM_STATUS_CHOL_B, count);
            for (int J = c->nb - 1; J >= 0; --J) {
                launch_trsv_lt_step(c->A, J, rrow, c->Dinv, c->dstride, c->v.z, c->v.vstride, lv,
                                    count, c->stream);
                check_launch();
            }
        }
        launch_newton_update(c->v, c->np, lv, count, c->stream);
        check_launch();
        if (mixed || !c->k_full)
            launch_symv(c->K, c->v.a, c->v.vstride, c->v.fnew, c->v.vstride, c->sympart,
                        c->sstride, c->np, MatF{}, nullptr, 0, lv, count, c->stream, c->symv_tpw);
        else
            launch_gemv(c->K, c->v.a, c->v.vstride, c->v.fnew, c->v.vstride, c->np, lv, count,
                        c->stream);
        check_launch();
        launch_newton_check(c->v, c->n, c->np, c->tol, c->active, c->status, c->n_iter, count,
                            c->stream);
        check_launch();
        read_back(c, {RB{c->active, (int)sizeof(int) * count, act.data()},
                      RB{c->status, (int)sizeof(int) * count, st_h.data()}});
        int live = 0;
        for (int b = 0; b < count; ++b) live += (act[b] != 0 && st_h[b] == 0);
        if (!live) break;
        c->live_n = live;
    }
    if (mixed) c->newton_last = (int)std::min<int64_t>(it + 1, c->max_iters);
    c->cholk_quota = 1 << 30;
    bool changed = false;
    for (int b = 0; b < count; ++b)
        if (act[b] != 0 && st_h[b] == 0) {
            st_h[b] = APM_STATUS_MAXITER;
            changed = true;
        }
    if (changed)
        HIPC(hipMemcpyAsync(c->status, st_h.data(), sizeof(int) * count, hipMemcpyHostToDevice,
                            c->stream));
}

// Newton for the IS estimator: mixed precision, with an fp64 rerun for any chain whose fp32
// factorisation broke down (B is SPD with eigenvalues >= 1, so only for extreme theta)
void drain_chol_k(apm_ctx* c);

void newton_is(apm_ctx* c, int count, std::vector<int>& st_h) {
    newton(c, count, st_h, c->mixed, count);
    if (!c->mixed) return;
    std::vector<int> redo;
    for (int b = 0; b < count; ++b)
        if (st_h[b] == APM_STATUS_CHOL_B) redo.push_back(b);
    if (redo.empty()) return;
    c->n_fp64_rerun += (int64_t)redo.size();
    std::vector<int> nit(count);
    HIPC(hipMemcpyAsync(nit.data(), c->n_iter, sizeof(int) * count, hipMemcpyDeviceToHost,
                        c->stream));
    sync(c);
    for (int b : redo) {
        st_h[b] = 0;
        nit[b] = 0;
    }
    HIPC(hipMemcpyAsync(c->status, st_h.data(), sizeof(int) * count, hipMemcpyHostToDevice,
                        c->stream));
    HIPC(hipMemcpyAsync(c->n_iter, nit.data(), sizeof(int) * count, hipMemcpyHostToDevice,
                        c->stream));
    // The fp64 rerun forms B and its right-hand-side row in A's rows [0, np]; row block np is
    // the first row block of BL, which the concurrent chol(K) on stream2 may still be writing:
    // let chol(K) finish first (L_K is recomputed after the rerun anyway, theta_eval_impl)
    drain_chol_k(c);
    // only the redo chains are live now: converged chains have active = 0, failed ones status != 0
    newton(c, count, st_h, false, (int)redo.size());
}

// apm_laplace's covariance C = K - V^T V (lpa.py:111-112) in the bottom-right of A: the
// augmented matrix [[B,.],[K W^1/2, K]] with the last fp64 Newton factor in its top-left
void augmented(apm_ctx* c, int count) {
    const Live lv = live_of(c);
    HIPC(hipMemsetD32Async(c->active, 1, count, c->stream));
    launch_form_aug(c->K, c->A, c->v, c->np, lv, count, c->stream);
    check_launch();
    const int nb = c->nb, R = 2 * nb + 1, Cb = 2 * nb;
    chol_range(c, c->A, 0, nb, R, Cb, APM_STATUS_CHOL_B, count, /*factor_diag=*/false, /*rows>=*/nb);
}

// Posterior-covariance factor through chol(K) (postcov.hip): 4N^3/3 flops instead of the
// augmented 7N^3/3. Leaves chol(C) J in rows [np, 2np) x cols [0, np) of A, g in v.Kb and
// log|B| = log|M| in ldet[0..nb).
MatB bl_of(apm_ctx* c) { return MatB{c->A.base + (int64_t)c->np * c->A.ld, c->A.ld, c->A.cstride}; }

// chol(K) into the bottom-left block BL of the work matrix for the concurrent path: own stream
// (ex.s), liveness (active2 / status2, so that Newton convergence does not mask it) and the upper
// halves of Dinv / ldet (the Newton factorisation uses the lower halves and the top rows of A).
// chol_k_begin copies K and factors the first outer panel; each feed_chol_k call releases the
// next outer panel (panel + its trailing update) behind an event of the main stream, at most
// cholk_quota per Newton iteration (newton(): the panels left spread over the iterations the
// previous call took).
Exec k_exec(apm_ctx* c, hipStream_t s);
void chol_k_panel(apm_ctx* c, const Exec& ex) {
    const int K = c->cholk_next;
    if (K < 0 || K >= c->nb) return;
    // first panel after a partial Gram copy: the trailing update reads K's tiles (out of place)
    const MatB* src = (K == 0 && c->cholk_partial) ? &c->K : nullptr;
    chol_range(c, bl_of(c), K, std::min(K + c->outer, c->nb), c->nb, c->nb, APM_STATUS_CHOL_K,
               c->cholk_count, true, 0, no_gap, &ex, src);
    c->cholk_next = K + c->outer;
}
void chol_k_begin(apm_ctx* c, int count, const Exec& ex, bool copy = true, bool partial = false) {
    HIPC(hipMemsetD32Async(c->active2, 1, count, ex.s));
    HIPC(hipMemsetAsync(c->status2, 0, sizeof(int) * count, ex.s));
    if (copy) {  // (else the Gram wrote K's lower tiles into BL as well, or those of the first
                 // outer panel's tile columns: partial)
        launch_copy_lower(c->K, bl_of(c), c->np, ex.lv, count, ex.s);
        check_launch();
    }
    c->cholk_partial = !copy && partial;
    c->cholk_next = 0;
    c->cholk_count = count;
    chol_k_panel(c, ex);
}
// edge cholk_rel[p] (main -> s2) carries no data: chol(K) works in BL, ldet + nb and the upper
// half of Dinv, which nothing on the main stream touches while it runs (the fp64 Newton rerun,
// which writes BL's first row block, drains it first); it only releases the panel behind the
// main stream's TRSVs, whose single-workgroup-per-chain launches leave most CUs idle
void feed_chol_k(apm_ctx* c) {
    if (c->cholk_next < 0 || c->cholk_next >= c->nb) return;
    if (c->cholk_quota <= 0) return;
    --c->cholk_quota;
    hipEvent_t e = c->ev.cholk_rel[c->cholk_next / c->outer];
    HIPC(hipEventRecord(e, c->stream));
    HIPC(hipStreamWaitEvent(c->stream2, e, 0));
    chol_k_panel(c, k_exec(c, c->stream2));
}
// all of chol(K) on one stream (the rerun after an fp64 Newton fallback)
void chol_k_into_bl(apm_ctx* c, int count, const Exec& ex) {
    chol_k_begin(c, count, ex);
    while (c->cholk_next >= 0 && c->cholk_next < c->nb) chol_k_panel(c, ex);
    c->cholk_next = -1;
}

// enqueue what is left of the concurrent chol(K) and order the main stream behind it (edge
// cholk_done, s2 -> main: L_K in BL, the log-dets in ldet + nb, status2)
void drain_chol_k(apm_ctx* c) {
    if (c->cholk_next < 0) return;
    while (c->cholk_next < c->nb) chol_k_panel(c, k_exec(c, c->stream2));
    c->cholk_next = -1;
    HIPC(hipEventRecord(c->ev.cholk_done, c->stream2));
    HIPC(hipStreamWaitEvent(c->stream, c->ev.cholk_done, 0));
}

Exec k_exec(apm_ctx* c, hipStream_t s) {
    return Exec{s, Live{c->active2, c->status2}, c->Dinv + (int64_t)c->nb * 4096, c->ldet + c->nb,
                c->cholk_count};
}

// The bottom block of [[J M J],[L_K J]] after the fp64 factorisation of J M J = L' L'^T: the TRSM
// (L_K J) L'^-T = chol(C) J as a blocked right-looking solve in fp32 on a working copy S32 in
// the free right half of A (postcov.hip): per outer panel of L', the rows' left-looking walks over
// the panel's columns (the dataflow kernel's no-wait twin, k_chol_panel_df32<true>, against the
// fp32 inverses of L''s diagonal tiles), then the rank-64*outer update of the rows' remaining
// columns on the 128x128 super-tile kernel (fp16x3 operands where h3post allows). Row tile nb + I
// of L_K J is zero before tile column nb - 1 - I (chol(C) J keeps that pattern), so a panel
// touches only the rows whose first nonzero tile lies in or before it. The fp64 route costs N^3/3
// flops per chain on the f64 MFMA; chol(C) enters the estimate only through the fp32 slot and
// L.U, and moves log f by ~1e-9 x trace(C) in fp32 (tools/postcov_precision_study.py), so chains
// with trace(C) > Sl.post_q are recomputed in fp64 after the slot write (bottom64_rerun).
MatF s32_of(apm_ctx* c) {
    return MatF{reinterpret_cast<float*>(c->A.base + c->np), 2 * c->A.ld, 2 * c->A.cstride};
}
float* d32post_of(apm_ctx* c) { return reinterpret_cast<float*>(c->Dinv + (int64_t)c->nb * 4096); }
// fp16x3 operand planes of the bottom block's trailing updates: the Newton planes' memory (free
// once the Newton loop is done: both parity buffers of a chain hold the 2 np rows of [top;
// bottom]), written per outer panel by the conversion (the top's rows below the diagonal block)
// and the bottom rows' walks, read by the quad-tile update on the same stream (stream2), so one
// buffer serves every panel. Only when every chain of the call takes fp16x3 operands there.
Planes16 post_planes_of(apm_ctx* c) {
    if (!c->planes || !c->h3post_all) return Planes16{nullptr, 0, 0, 0};
    return Planes16{c->planes, 2 * c->plane_cs, c->plane_cs, 2 * c->np};
}

// one outer panel [K, Kend) of the bottom block on stream s: the rows' walks, then the update of
// their remaining columns
void post_bottom32_steps(apm_ctx* c, int count, int K, int Kend, hipStream_t s) {
    const Live lv = live_of(c);
    const int nb = c->nb;
    MatF S = s32_of(c);
    const int64_t ds32 = 2 * c->dstride;
    const int hlim = c->h3 ? 2 * nb : 0;
    const int row0 = std::max(nb, 2 * nb - Kend);  // rows with a nonzero tile in the panel
    const Planes16 pl = Kend < nb ? post_planes_of(c) : Planes16{nullptr, 0, 0, 0};
    launch_chol_panel_bulk32(S, K, Kend - K, row0, 2 * nb, 2 * nb,
                             FusedDiag<float>{0, d32post_of(c), ds32, nullptr, 0, 0}, lv, count,
                             hlim, c->h3post, s, pl);
    check_launch();
    if (Kend >= nb) return;
    const double fl =
        c->prof ? update_flops(row0, 2 * nb, Kend, nb, Kend - K, Gap{0, 0}) * c->live_n : 0.0;
    ProfScope ps(c, APM_PROF_POST32_OUTER, fl, s);
    if (pl.base) {  // 256x256 quad tiles from the planes (bitwise the split-while-staged kernel)
        const auto ql = quad_list(c, row0, 2 * nb, Kend, nb);
        launch_chol_update32_q256(S, K, Kend - K, ql.first, ql.second, lv, count, s, c->h3post,
                                  pl, /*role: the posterior bottom block*/ 1);
    } else {
        const auto sl = super_list(c, row0, 2 * nb, Kend, nb, Gap{0, 0});
        launch_chol_update32_t128(S, K, Kend - K, sl.first, sl.second, lv, count, s,
                                  FusedDiag<float>{0, nullptr, 0, nullptr, 0, 0}, hlim, c->h3post,
                                  -1, /*role: the posterior bottom block*/ 1);
    }
    check_launch();
}

// The bottom block's copy once L_K J is formed, then each outer panel of the bottom on the
// low-priority stream2 as soon as the fp64 factorisation has finished that panel of L'
// (post_bottom32_panel, chol_range's after_panel): the bottom's fp32 work fills the CUs the fp64
// in-panel steps leave idle instead of following the factorisation. Edge y2 (main -> s2): L_K J
// in BL's fp64 rows, the chains' liveness (active reset by post_cov_lk).
void post_bottom32_begin(apm_ctx* c, int count) {
    HIPC(hipEventRecord(c->ev.y2, c->stream));
    HIPC(hipStreamWaitEvent(c->stream2, c->ev.y2, 0));
    launch_post32_convert(c->A, s32_of(c), c->Dinv, c->dstride, d32post_of(c), 2 * c->dstride,
                          c->nb, c->outer, 0, 0, true, live_of(c), count, c->stream2);
    check_launch();
}
// edge lp_panel[p] (main -> s2): the columns [K, Kend) of L' (rows K .. nb) and their diagonal
// inverses (Dinv, first half) are final; the main stream's trailing update that follows writes
// only columns >= Kend and Dinv[Kend]
void post_bottom32_panel(apm_ctx* c, int count, int K, int Kend) {
    hipEvent_t e = c->ev.lp_panel[K / c->outer];
    HIPC(hipEventRecord(e, c->stream));
    HIPC(hipStreamWaitEvent(c->stream2, e, 0));
    launch_post32_convert(c->A, s32_of(c), c->Dinv, c->dstride, d32post_of(c), 2 * c->dstride,
                          c->nb, c->outer, K, Kend, false, live_of(c), count, c->stream2,
                          Kend < c->nb ? post_planes_of(c) : Planes16{nullptr, 0, 0, 0});
    check_launch();
    post_bottom32_steps(c, count, K, Kend, c->stream2);
}

// the guard (newton.hip k_guard_check) of the chains `lv` admits, after their slot write
void guard_check(apm_ctx* c, Live lv, int count) {
    launch_guard_check(c->ldet, c->lstride, c->nb, c->v.Kb, c->v.vstride, c->Sl, c->d_slots,
                       c->guard, c->max_batch, GUARD_T1, GUARD_T2, GUARD_T3, GUARD_T4,
                       c->guard_rows, c->v.f, APM_STATUS_GUARD, lv, count, c->stream);
    check_launch();
}

// The fp64 bottom block for the chains flagged by the slot writer (bit 1 of Sl.chain_wide):
// (L_K J) L'^-T on the still intact fp64 rows [np, 2np) of A and L' (chol_range restricted to
// those rows, the chains masked through active2), then their slots again in mode 2 and the u-path
// of the call again (the other chains' values are recomputed unchanged).
void bottom64_rerun(apm_ctx* c, int count, const std::vector<int>& redo) {
    const int nb = c->nb;
    for (int b = 0; b < count; ++b) c->hmask[b] = 0;
    for (int b : redo) c->hmask[b] = 1;
    HIPC(hipMemcpyAsync(c->active2, c->hmask, sizeof(int) * count, hipMemcpyHostToDevice,
                        c->stream));
    const Live lr{c->active2, c->status};
    const Exec ex{c->stream, lr, c->Dinv, c->ldet, (int)redo.size()};
    chol_range(c, c->A, 0, nb, 2 * nb, nb, APM_STATUS_CHOL_C, count, /*factor_diag=*/false,
               /*row_start=*/nb, y_gap, &ex);
    launch_slot_write(c->A, c->v, c->ldet, c->lstride, nb, c->Sl, c->d_slots, 2, c->n, c->np, lr,
                      count, c->stream, MatF{nullptr, 0, 0}, c->guard_rows);
    check_launch();
    guard_check(c, lr, count);  // (the fp64 bottom's rows now: r3, r4 were skipped before)
    c->n_post64 += (int64_t)redo.size();
}

// The reference's own route to chol(C) (estimators.py:206-215, lpa.py:107-112) for the chains
// whose C is small against K (bit 3 of Sl.chain_wide, APM_ICM_Q): C = K - V^T V with
// V = L^-1 W^1/2 K and L = chol(B) of the last Newton iteration, all fp64, as the bottom-right
// block of the factorisation of the augmented matrix [[B, .], [K W^1/2, K]] (k_form_B +
// k_form_aug, then one blocked Cholesky of 2N columns). The push-through factor the estimate uses
// cannot fail (M is SPD for any W >= 0); the reference's explicitly formed C can be numerically
// indefinite (a property of the route: it fails under 1-ulp perturbations of B at the golden ICM
// thetas and passes under them at configs[2]'s sigma = e^18.5, tools/icm_route_study.py). A chain
// whose C fails here gets APM_STATUS_CHOL_C, raised as InvalidCovarianceMatrixError (masked in
// batched calls) as the reference does. Only flagged chains pay (8N^3/3 flops each); A is free
// by now. (At the golden ICM thetas the device's chol(K) fails first: K's definiteness there is
// below its rounding)
void icm_check(apm_ctx* c, int count, const std::vector<int>& chk) {
    const int nb = c->nb;
    for (int b = 0; b < count; ++b) c->hmask[b] = 0;
    for (int b : chk) c->hmask[b] = 1;
    HIPC(hipMemcpyAsync(c->active2, c->hmask, sizeof(int) * count, hipMemcpyHostToDevice,
                        c->stream));
    const Live lr{c->active2, c->status};
    launch_form_B(c->K, c->A, c->v, c->np, lr, count, c->stream);
    check_launch();
    launch_form_aug(c->K, c->A, c->v, c->np, lr, count, c->stream, !c->k_full);
    check_launch();
    const Exec ex{c->stream, lr, c->Dinv, c->ldet, (int)chk.size()};
    chol_range(c, c->A, 0, 2 * nb, 2 * nb, 2 * nb, APM_STATUS_CHOL_C, count, true, 0, no_gap,
               &ex);
    c->n_icm_check += (int64_t)chk.size();
}

// fp64 factor buffers of wide slots (Sl.L64): attached on demand, recycled through l64_free
void attach_l64(apm_ctx* c, int64_t slot) {
    if (c->l64_h[slot]) return;
    if (!c->l64_free.empty()) {
        c->l64_h[slot] = c->l64_free.back();
        c->l64_free.pop_back();
    } else {
        c->l64_h[slot] = dalloc<double>(c, c->np * c->np);
    }
}
void detach_l64(apm_ctx* c, int64_t slot) {
    if (!c->l64_h[slot]) return;
    c->l64_free.push_back(c->l64_h[slot]);
    c->l64_h[slot] = nullptr;
}
void upload_l64(apm_ctx* c) {  // pageable source: the copy has read it when the call returns
    HIPC(hipMemcpyAsync(c->l64_d, c->l64_h.data(), sizeof(double*) * c->n_slots,
                        hipMemcpyHostToDevice, c->stream));
}

// L_K ready in BL (chol_k_into_bl); h = L_K^-1 f_post = L_K^T a because f_post = K a
void post_cov_lk(apm_ctx* c, int count, bool have_lk = false) {
    const Live lv = live_of(c);
    hipStream_t s = c->stream;
    HIPC(hipMemsetD32Async(c->active, 1, count, s));
    const int nb = c->nb, np = c->np;
    const int64_t vs = c->v.vstride;
    MatB TL = c->A;
    MatB BL = bl_of(c);
    if (have_lk) {
        launch_trmv_tiles(false, BL, c->v.a, c->v.z, vs, np, c->sympart, c->sstride, lv, count,
                          s);                                                 // h = L_K^T a -> z
        check_launch();
    } else {
        launch_copy_lower(c->K, BL, np, lv, count, s);
        check_launch();
        launch_set_rhs(c->A, 2 * (int64_t)np, np, c->v.f, vs, lv, count, s);  // f_post under K
        check_launch();
        chol_range(c, BL, 0, nb, nb + 1, nb, APM_STATUS_CHOL_K, count);       // L_K, h = L_K^-1 f
        launch_get_row(c->A, 2 * (int64_t)np, np, c->v.z, vs, lv, count, s);  // h -> z
        check_launch();
        launch_guard_save(c->ldet, c->lstride, 0, nb, c->guard, c->max_batch, 1, lv, count, s);
        check_launch();  // (1/2 log|K| before M's factorisation overwrites ldet[0, nb))
    }
    // J M J = I + Y2 Y2^T: on the 128x128 super-tile path one launch writes it without reading TL
    // (tile column j takes Y2's column blocks k <= j); otherwise TL starts as I and receives
    // panel-wide updates (Y2 lower: j >= K suffices)
    const bool syrk1 = nb >= 2;
    launch_form_y2_rev(BL, TL, np, c->v.Ws, vs, np, lv, count, s, !syrk1);  // Y2, Y = L_K J
    check_launch();
    // the bottom block's fp32 copy of L_K J (stream2, HBM-bound) beside the SYRK (MFMA-bound)
    // rather than beside the first panel's latency-bound in-panel steps (-1.4 ms per stationary
    // theta-call, profiles/r05_conv_early_ab.txt)
    post_bottom32_begin(c, count);
    if (syrk1) {
        tracked_update(c, TL, nb, nb, 0, nb, 0, nb, Gap{0, 0}, 2, count);
    } else {
        launch_identity_lower(TL, np, lv, count, s);
        check_launch();
        for (int K = 0; K < nb; K += c->outer) {
            const int Kend = std::min(K + c->outer, nb);
            tracked_update(c, TL, nb + K, Kend - K, K, nb, K, nb, Gap{0, 0}, 1, count);
        }
    }
    // J M J alone in fp64 (its log-determinant is log|B|), the fp32 bottom block following its
    // panels on stream2
    chol_range(c, TL, 0, nb, nb, nb, APM_STATUS_CHOL_C, count, true, 0, no_gap, nullptr, nullptr,
               [c, count](int K, int Kend) { post_bottom32_panel(c, count, K, Kend); });
    launch_trmv_tiles(true, TL, c->v.z, c->v.Kb, vs, np, c->sympart, c->sstride, lv, count,
                      s);                                                     // g = J L'^T J h
    check_launch();
    // edge bottom_done (s2 -> main): the slot writer reads the bottom block (S32). APM_SKEW bit 2
    // (tests only) drops this one wait, so that the skew test can show a missing edge being caught
    HIPC(hipEventRecord(c->ev.bottom_done, c->stream2));
    if (!(c->skew & 4)) HIPC(hipStreamWaitEvent(c->stream, c->ev.bottom_done, 0));
}

void theta_eval_impl(apm_ctx* c, int est, int count, bool gram, double* out_logf, int* status,
                     int64_t* nops) {
    const Live lv = live_of(c);
    c->live_n = count;
    HIPC(hipMemsetD32Async(c->active, 1, count, c->stream));
    HIPC(hipMemsetAsync(c->status, 0, sizeof(int) * count, c->stream));
    HIPC(hipMemsetAsync(c->n_iter, 0, sizeof(int) * count, c->stream));
    reset_tickets(c);
    // IS: chol(K) runs on the second stream while the Newton iterations run on the main one
    const bool ov = est == APM_EST_IS && c->mixed;
    // the matrix a factorisation of K starts from (chol(K)'s working copy BL, or PriorMC's A):
    // the Gram writes K's lower tiles there too instead of a later copy pass
    MatB k2{nullptr, 0, 0};
    int k2cols = 1 << 30;
    if (gram) {
        if (est == APM_EST_PRIORMC) {
            k2 = c->A;
        } else if (ov) {
            k2 = bl_of(c);
            // chol(K)'s first trailing update can read its old tiles from K (out of place): the
            // Gram then copies only the first outer panel's tile columns (~1/4 of the lower tiles
            // at N = 4096 instead of all of them)
            if (c->outer >= 2 && c->nb - c->outer >= 2) k2cols = c->outer;
        }
    }
    if (gram) {
        // every consumer on this path reads K's lower tiles: the Gram writes N(N+1)/2 entries
        // 
        c->k_full = false;
        const double nk = c->k_full ? (double)c->n * c->n : 0.5 * (double)c->n * (c->n + 1);
        ProfScope ps(c, APM_PROF_GRAM, 8.0 * ((double)c->n * c->d + nk) * count + 8.0 * c->P);
        launch_gram(c->K, c->X, c->d, c->n, c->d, c->theta, c->P, c->kind, c->eps, c->np, lv,
                    count, c->stream, c->k_full, k2, k2cols);
        check_launch();
    }
    std::vector<int> st_h(count, 0), it_h(count, 0);
    if (est == APM_EST_PRIORMC) {
        if (!k2.base) {
            launch_copy_lower(c->K, c->A, c->np, lv, count, c->stream);
            check_launch();
        }
        chol_range(c, c->A, 0, c->nb, c->nb, c->nb, APM_STATUS_CHOL_K, count);
        launch_slot_write(c->A, c->v, c->ldet, c->lstride, c->nb, c->Sl, c->d_slots, 1, c->n,
                          c->np, lv, count, c->stream);
        check_launch();
        u_eval_device(c, count, true);
    } else {
        if (ov) {
            // edge gram_k (main -> s2): K and BL's first outer panel written by the Gram, the
            // chains' theta (the statuses chol(K) keeps apart: status2 / active2)
            HIPC(hipEventRecord(c->ev.gram_k, c->stream));
            HIPC(hipStreamWaitEvent(c->stream2, c->ev.gram_k, 0));
            chol_k_begin(c, count, k_exec(c, c->stream2), /*copy=*/k2.base == nullptr,
                         /*partial=*/k2cols < c->nb);
        }
        const int64_t reruns = c->n_fp64_rerun;
        if (est == APM_EST_LAPLACE) {  // log|B| of the Newton factor itself: fp64 (lpa.py:116)
            newton(c, count, st_h, false, count);
        } else {
            newton_is(c, count, st_h);
            // the guard's 1/2 log|B| of the last Newton factor (k_guard_check)
            launch_guard_save(c->ldet, c->lstride, 0, c->nb, c->guard, c->max_batch, 0, lv,
                              count, c->stream);
            check_launch();
        }
        c->live_n = 0;
        for (int b = 0; b < count; ++b) c->live_n += st_h[b] == 0;
        if (ov) {
            drain_chol_k(c);  // what the TRSVs did not take (a no-op after an fp64 rerun)
            if (c->n_fp64_rerun != reruns)  // the fp64 Newton rerun used rows of BL: redo L_K
                chol_k_into_bl(c, count, k_exec(c, c->stream));
            // a chain whose blocked chol(K) failed is factored once more in LAPACK's dpotf2
            // order (chol.hip k_chol_unblocked, n <= 512) before LinAlgError is raised: at the
            // reference's InvalidCovarianceMatrixError thetas K's definiteness is decided by the
            // rounding order
            if (launch_chol_unblocked(c->K, bl_of(c), c->np, c->status2, APM_STATUS_CHOL_K,
                                      c->ldet + c->nb, c->lstride, count, c->stream))
                check_launch();
            launch_merge_status(c->status, c->status2, APM_STATUS_CHOL_K, count, c->stream);
            check_launch();
            launch_guard_save(c->ldet, c->lstride, c->nb, c->nb, c->guard, c->max_batch, 1, lv,
                              count, c->stream);  // 1/2 log|K| (chol(K) on stream2: ldet + nb)
            check_launch();
        }
        if (est == APM_EST_LAPLACE) {
            launch_laplace_lml(c->v, c->y, c->n, c->ldet, c->lstride, c->nb, c->out, lv, count,
                               c->stream);
            check_launch();
        } else {
            post_cov_lk(c, count, ov);
            launch_slot_write(c->A, c->v, c->ldet, c->lstride, c->nb, c->Sl, c->d_slots,
                              3, c->n, c->np, lv, count, c->stream, s32_of(c), c->guard_rows);
            check_launch();
            guard_check(c, lv, count);
            u_eval_device(c, count, true);
        }
    }
    std::vector<int> wide_h(count, 0);
    if (est == APM_EST_LAPLACE) {
        read_back(c, {RB{c->out, (int)sizeof(double) * count, out_logf},
                      RB{c->status, (int)sizeof(int) * count, st_h.data()},
                      RB{c->n_iter, (int)sizeof(int) * count, it_h.data()}});
    } else {
        read_back(c, {RB{c->out, (int)sizeof(double) * count, out_logf},
                      RB{c->status, (int)sizeof(int) * count, st_h.data()},
                      RB{c->n_iter, (int)sizeof(int) * count, it_h.data()},
                      RB{c->Sl.chain_wide, (int)sizeof(int) * count, wide_h.data()}});
        const int64_t* hs = reinterpret_cast<const int64_t*>(c->hpin);  // the call's slots
        std::vector<int> chk;  // bit 3: the reference's route to chol(C) is checked (icm_check)
        for (int b = 0; b < count; ++b)
            if (st_h[b] == 0 && (wide_h[b] & 8) && est == APM_EST_IS) chk.push_back(b);
        std::vector<int> redo, rewrite;  // fp32 bottom blocks above the trace bound (bit 1);
        bool attached = false;           // wide slots whose fp64 factor was not written (bit 2)
        for (int b = 0; b < count; ++b) {  // (a guard-failed chain's slot was written too)
            if (st_h[b] != 0 && st_h[b] != APM_STATUS_GUARD) continue;
            const bool rd = (wide_h[b] & 2) && est == APM_EST_IS && st_h[b] == 0;
            if (rd) redo.push_back(b);
            if ((wide_h[b] & 4) && !c->l64_h[hs[b]]) {
                attach_l64(c, hs[b]);
                attached = true;
                if (!rd) rewrite.push_back(b);
            }
        }
        if (attached) upload_l64(c);
        if (!redo.empty()) bottom64_rerun(c, count, redo);  // (writes the wide ones' fp64 factor)
        if (!rewrite.empty()) {
            if (!redo.empty()) sync(c);  // (hmask feeds bottom64_rerun's pending copy)
            for (int b = 0; b < count; ++b) c->hmask[b] = 0;
            for (int b : rewrite) c->hmask[b] = 1;
            HIPC(hipMemcpyAsync(c->active2, c->hmask, sizeof(int) * count, hipMemcpyHostToDevice,
                                c->stream));
            launch_slot_write_L64(c->A, c->Sl, c->d_slots, est == APM_EST_PRIORMC ? 1 : 2, c->np,
                                  Live{c->active2, c->status}, count, c->stream);
            check_launch();
        }
        if (!redo.empty() || !rewrite.empty()) {
            u_eval_device(c, count, true);
            read_back(c, {RB{c->out, (int)sizeof(double) * count, out_logf},
                          RB{c->status, (int)sizeof(int) * count, st_h.data()},
                          RB{c->Sl.chain_wide, (int)sizeof(int) * count, wide_h.data()}});
        }
        // the slots as the slot writer left them: the host mirror (slot_wide, the fp64 factor
        // attachments) follows every slot written this call, also of a chain the reference-route
        // check fails below (its slot holds a complete state that no caller reads)
        const std::vector<int> st_slot = st_h;
        if (!chk.empty()) {  // (after everything that reads A)
            icm_check(c, count, chk);
            read_back(c, {RB{c->status, (int)sizeof(int) * count, st_h.data()}});
        }
        for (int b = 0; b < count; ++b) c->n_guard += st_h[b] == APM_STATUS_GUARD;
        bool detached = false;
        for (int b = 0; b < count; ++b) {
            if (st_slot[b] != 0 && st_slot[b] != APM_STATUS_GUARD) continue;
            c->slot_wide[hs[b]] = wide_h[b] & 1;
            if (!(wide_h[b] & 1) && c->l64_h[hs[b]]) {
                detach_l64(c, hs[b]);
                detached = true;
            }
        }
        if (detached) upload_l64(c);
    }
    for (int b = 0; b < count; ++b) {
        status[b] = st_h[b];
        if (nops) {
            if (est == APM_EST_PRIORMC) nops[b] = 1;                   // estimators.py:322
            else if (est == APM_EST_LAPLACE) nops[b] = it_h[b];        // lpa.py:441-443 (i)
            else nops[b] = (int64_t)it_h[b] + 1 + 2;                   // estimators.py:217
        }
    }
}

bool check_idx(apm_ctx* c, int64_t count, const int64_t* idx, int64_t lim, const char* what) {
    for (int64_t i = 0; i < count; ++i)
        if (idx[i] < 0 || idx[i] >= lim) {
            fail(c, APM_E_INVALID, std::string(what) + " index out of range");
            return false;
        }
    return true;
}

void init_ctx(apm_ctx* c, int device, int kind, const double* X, int64_t n, int64_t d,
              int64_t ldx, const double* y, double eps, int64_t S, int64_t max_batch,
              int64_t n_slots, int64_t n_ubufs) {
    c->device = device;
    // the library's environment knobs, read here once per context: two
    // correctness fallbacks (APM_MIXED=0: fp64 Newton factorisation; APM_H3=0: fp32 operands in
    // the fp32 factorisations' outer updates) and test thresholds / test modes that the GPU
    // tests use to reach rare paths. The defaults are the product.
    HIPC(hipSetDevice(device));
    trsv32_mw_init();
    if (const char* e = getenv("APM_MIXED")) c->mixed = atoi(e) != 0;
    if (const char* e = getenv("APM_H3")) c->h3 = atoi(e) != 0;
    // acceptance of a refinement step (test threshold: 0 sends every chain to the fp64 rerun)
    if (const char* e = getenv("APM_REFINE_TOL")) c->refine_tol = atof(e);
    // the reference-route check of chol(C) (icm_check): trace(C) below n K_ii / APM_ICM_Q
    // (test threshold: 1 checks every chain, 0 none)
    if (const char* e = getenv("APM_ICM_Q")) c->icm_q = std::max(0.0, atof(e));
    // poll bound of every in-launch hand-over wait (tests/test_gpu_errors.py forces the
    // bounded-spin exits with 1 and checks that no chain returns a wrong value with status 0)
    if (const char* e = getenv("APM_SPIN_LIMIT")) c->spin_df = c->spin_trsv = std::max(1, atoi(e));
    // delay kernels in front of every launch on the secondary streams (bit 0) and/or on the main
    // stream (bit 1): a cross-stream edge without its wait then gives a wrong result
    // deterministically (tests/test_gpu_errors.py::test_stream_skew_is_bitwise_neutral); bit 2
    // removes one edge's wait (bottom_done) to show that such a result is caught
    if (const char* e = getenv("APM_SKEW")) c->skew = std::max(0, std::min(7, atoi(e)));
    {  // main stream at the highest priority: the concurrent chol(K) only fills idle CUs
        int least = 0, greatest = 0;
        HIPC(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIPC(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest));
        HIPC(hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, least));
        HIPC(hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, least));
    }
    c->kind = kind;
    c->n = (int)n;
    c->d = (int)d;
    c->np = (int)((n + 63) / 64 * 64);
    c->nb = c->np / 64;
    {  // one event per cross-stream edge (Edges): the per-panel ones indexed by panel
        const int np64 = (c->nb + c->outer - 1) / c->outer, np32 = (c->nb + c->outer32 - 1) / c->outer32;
        c->ev.cholk_rel.assign(np64, nullptr);
        c->ev.lp_panel.assign(np64, nullptr);
        c->ev.df.assign(np32, nullptr);
        c->ev.far.assign(np32, nullptr);
        for (hipEvent_t* e : c->ev.all()) HIPC(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    c->P = kind == APM_KERNEL_ISO ? 2 : (kind == APM_KERNEL_ARD ? (int)d + 1 : 0);
    c->S = (int)S;
    c->sp = (int)((S + 63) / 64 * 64);
    c->max_batch = (int)max_batch;
    c->n_slots = (int)n_slots;
    c->slot_refs.assign((size_t)n_slots, 0);
    c->n_ubufs = (int)n_ubufs;
    c->eps = eps;
    const int64_t np = c->np, B = max_batch;
    if (kind != APM_KERNEL_PRECOMPUTED && d > 0) {
        c->X = dalloc<double>(c, n * d);
        std::vector<double> Xc((size_t)(n * d));
        for (int64_t i = 0; i < n; ++i)
            for (int64_t k = 0; k < d; ++k) Xc[i * d + k] = X[i * ldx + k];
        HIPC(hipMemcpy(c->X, Xc.data(), sizeof(double) * n * d, hipMemcpyHostToDevice));
    }
    c->y = dalloc<double>(c, np);
    std::vector<double> yp((size_t)np, 0.0);
    if (y)
        for (int64_t i = 0; i < n; ++i) yp[i] = y[i];
    HIPC(hipMemcpy(c->y, yp.data(), sizeof(double) * np, hipMemcpyHostToDevice));
    c->theta = dalloc<double>(c, B * std::max(c->P, 1));
    c->K = MatB{dalloc<double>(c, B * np * np), np, np * np};
    const int64_t arows = 2 * np + 64, acols = 2 * np;
    c->A = MatB{dalloc<double>(c, B * arows * acols), acols, arows * acols};
    c->dstride = 2 * c->nb * 4096;
    c->Dinv = dalloc<double>(c, B * c->dstride);
    c->lstride = 2 * c->nb;
    c->ldet = dalloc<double>(c, B * c->lstride);
    c->out = dalloc<double>(c, B);
    c->pstride = (int64_t)c->nb * c->sp;
    c->partial = dalloc<double>(c, B * c->pstride);
    const int64_t vs = np;
    c->vecbase = dalloc<double>(c, 8 * B * vs);
    c->rvec = dalloc<double>(c, 3 * B * vs);
    c->sstride = (int64_t)c->nb * c->nb * 64;
    c->sympart = dalloc<double>(c, B * c->sstride);
    c->v = NewtonVecs{c->vecbase,          c->vecbase + 1 * B * vs, c->vecbase + 2 * B * vs,
                      c->vecbase + 3 * B * vs, c->vecbase + 4 * B * vs, c->vecbase + 5 * B * vs,
                      c->vecbase + 6 * B * vs, c->vecbase + 7 * B * vs, vs};
    HIPC(hipMemset(c->vecbase, 0, sizeof(double) * 8 * B * vs));
    c->active = dalloc<int>(c, B);
    c->status = dalloc<int>(c, B);
    c->n_iter = dalloc<int>(c, B);
    c->refining = dalloc<int>(c, B);
    c->active2 = dalloc<int>(c, B);
    c->status2 = dalloc<int>(c, B);
    c->refine_prev = dalloc<double>(c, B);
    c->d_slots = dalloc<int64_t>(c, 2 * B);
    c->d_ubufs = c->d_slots + B;
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&c->hpin), (size_t)B * 40, hipHostMallocDefault));
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&c->hmask), sizeof(int) * (size_t)B,
                       hipHostMallocDefault));
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&c->hx), (size_t)B * 20,
                       hipHostMallocMapped | hipHostMallocCoherent));
    HIPC(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->dx), c->hx, 0));
    c->h3ok = dalloc<int>(c, 3 * B);
    c->h3post = c->h3ok + B;
    c->invok = c->h3ok + 2 * B;
    c->guard = dalloc<double>(c, 6 * B);
    HIPC(hipMemset(c->guard, 0, sizeof(double) * 6 * B));
    c->guard_rows = dalloc<double>(c, B * np);
    c->icm_thr = dalloc<double>(c, B);
    // + 3: the bounded-spin timeouts of the dataflow panel (APM_PROF_DF_TIMEOUTS) and of the
    // TRSV (APM_PROF_TRSV_TIMEOUTS), the arrival-ticket counter (spin_words)
    if (c->mixed && c->h3) {
        c->plane_cs = 2 * np * 32 * 2 * c->outer32;  // 2 planes x rows x 2 outer32 slices x 32
        c->planes = dalloc<unsigned short>(c, 2 * B * c->plane_cs);
        {
            c->zt = dalloc<float>(c, B * 3 * 512 * 512);
            c->zplanes = dalloc<unsigned short>(c, B * 2 * 16 * 512 * 32);
        }
    }
    c->dfprog = dalloc<unsigned long long>(c, (size_t)B * (c->nb + 1) + 3);
    HIPC(hipMemset(c->dfprog, 0, sizeof(unsigned long long) * (B * (c->nb + 1) + 3)));
    // one block of 7B words, mirrored in pinned host memory and uploaded with one copy:
    // [i3: 3B int64][ca: B][cb: B][seeds: B][ctrs: B]
    c->d_i3 = dalloc<int64_t>(c, 7 * B);
    c->d_ca = reinterpret_cast<double*>(c->d_i3 + 3 * B);
    c->d_cb = c->d_ca + B;
    c->d_seeds = reinterpret_cast<uint64_t*>(c->d_i3 + 5 * B);
    c->d_ctrs = c->d_seeds + B;
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&c->hblk), (size_t)B * 56, hipHostMallocDefault));
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&c->hth),
                       sizeof(double) * (size_t)B * std::max(c->P, 1), hipHostMallocDefault));
    c->U64 = dalloc<double>(c, n * S);
    const int64_t Lsz = (np + 64) * np;
    c->Sl = SlotSet{dalloc<float>(c, n_slots * Lsz), dalloc<double>(c, n_slots * np),
                    dalloc<double>(c, n_slots * np), dalloc<double>(c, n_slots * np),
                    dalloc<double>(c, n_slots), Lsz, np,
                    nullptr, dalloc<double>(c, n_slots * np), dalloc<int>(c, n_slots),
                    dalloc<int>(c, B), APM_WIDE_Q, APM_POST32_Q};
    c->l64_d = dalloc<double*>(c, n_slots);
    c->Sl.L64 = c->l64_d;
    c->l64_h.assign((size_t)n_slots, nullptr);
    HIPC(hipMemset(c->l64_d, 0, sizeof(double*) * n_slots));
    if (const char* e = getenv("APM_WIDE_Q")) c->Sl.wide_q = atof(e);  // development knob
    if (const char* e = getenv("APM_POST32_Q")) c->Sl.post_q = atof(e);
    c->Sl.post_q = std::min(c->Sl.post_q, c->Sl.wide_q);  // (a wide slot needs the fp64 factor)
    c->Sl.icm_thr = c->icm_thr;
    HIPC(hipMemset(c->Sl.cst, 0, sizeof(double) * n_slots));
    HIPC(hipMemset(c->Sl.wide, 0, sizeof(int) * n_slots));
    c->slot_wide.assign((size_t)n_slots, 0);
    c->Up = UPool{dalloc<double>(c, n_ubufs * np * c->sp), np * c->sp, c->sp,
                  dalloc<float>(c, n_ubufs * np * c->sp)};
    HIPC(hipMemset(c->Up.base, 0, sizeof(double) * n_ubufs * np * c->sp));
    HIPC(hipMemset(c->Up.base32, 0, sizeof(float) * n_ubufs * np * c->sp));
}

void free_ctx(apm_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    // every stream drained before its buffers go (stream2 / stream3 work is joined into the main
    // stream by every call, but a call that threw may have left some behind)
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->stream2) (void)hipStreamSynchronize(c->stream2);
    if (c->stream3) (void)hipStreamSynchronize(c->stream3);
    for (void* p : c->allocs) (void)hipFree(p);
    if (c->hpin) (void)hipHostFree(c->hpin);
    if (c->hblk) (void)hipHostFree(c->hblk);
    if (c->hth) (void)hipHostFree(c->hth);
    if (c->hx) (void)hipHostFree(c->hx);
    if (c->hmask) (void)hipHostFree(c->hmask);
    for (hipEvent_t e : c->evpool) (void)hipEventDestroy(e);
    if (c->stream3) (void)hipStreamDestroy(c->stream3);
    for (hipEvent_t* e : c->ev.all())
        if (*e) (void)hipEventDestroy(*e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    delete c;
}

// stand-alone calls reuse one context per (device, n, kind) shape
std::mutex g_mu;
std::map<std::tuple<int, int64_t, int64_t, int>, apm_ctx*> g_cache;

}  // namespace

// =============================================================================== C-ABI
extern "C" {

int apm_version(void) { return APM_VERSION; }

int apm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* apm_global_error(void) { return g_err.c_str(); }

apm_ctx* apm_create(int device, int kernel_kind, const double* X, int64_t n, int64_t d,
                    int64_t ldx, const double* y, double epsilon, int64_t n_imp,
                    int64_t max_batch, int64_t n_slots, int64_t n_ubufs) {
    if (n <= 0 || d < 0 || n_imp <= 0 || max_batch <= 0 || n_slots <= 0 || n_ubufs <= 0 ||
        kernel_kind < 0 || kernel_kind > 2 || (kernel_kind != APM_KERNEL_PRECOMPUTED && !X) ||
        n_imp > 1 << 20) {
        g_err = "apm_create: invalid arguments";
        return nullptr;
    }
    apm_ctx* c = new apm_ctx();
    try {
        init_ctx(c, device, kernel_kind, X, n, d, ldx, y, epsilon, n_imp, max_batch, n_slots,
                 n_ubufs);
    } catch (const HipError& e) {
        g_err = "apm_create: " + e.msg;
        free_ctx(c);
        return nullptr;
    }
    return c;
}

void apm_destroy(apm_ctx* ctx) { free_ctx(ctx); }

const char* apm_last_error(const apm_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int64_t apm_padded_n(const apm_ctx* ctx) { return ctx ? ctx->np : -1; }

int64_t apm_theta_len(const apm_ctx* ctx) { return ctx ? ctx->P : -1; }

int apm_set_newton(apm_ctx* ctx, double diff_f_tol, int64_t max_iters) {
    if (!ctx || max_iters < 0) return fail(ctx, APM_E_INVALID, "apm_set_newton: bad arguments");
    ctx->tol = diff_f_tol;
    ctx->max_iters = max_iters;
    return APM_SUCCESS;
}

void* apm_stream(apm_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int apm_u_upload(apm_ctx* c, int64_t ubuf, const double* U, int64_t ldu) {
    if (!c || !U || ubuf < 0 || ubuf >= c->n_ubufs || ldu < c->S)
        return fail(c, APM_E_INVALID, "apm_u_upload: bad arguments");
    const SkewScope skew(c);
    try {
        HIPC(hipSetDevice(c->device));
        HIPC(hipMemcpy2DAsync(c->U64, sizeof(double) * c->S, U, sizeof(double) * ldu,
                              sizeof(double) * c->S, c->n, hipMemcpyHostToDevice, c->stream));
        launch_u_convert(c->U64, c->S, c->n, c->S, c->Up, ubuf, c->stream);
        check_launch();
        sync(c);
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_u_download(apm_ctx* c, int64_t ubuf, double* U, int64_t ldu) {
    if (!c || !U || ubuf < 0 || ubuf >= c->n_ubufs || ldu < c->S)
        return fail(c, APM_E_INVALID, "apm_u_download: bad arguments");
    try {
        HIPC(hipSetDevice(c->device));
        std::vector<double> h((size_t)c->np * c->sp);
        HIPC(hipMemcpyAsync(h.data(), c->Up.base + ubuf * c->Up.stride, sizeof(double) * h.size(),
                            hipMemcpyDeviceToHost, c->stream));
        sync(c);
        for (int i = 0; i < c->n; ++i)
            for (int s = 0; s < c->S; ++s) U[(int64_t)i * ldu + s] = h[(size_t)i * c->sp + s];
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_u_normal(apm_ctx* c, int64_t count, const int64_t* ubufs, const uint64_t* seeds,
                 const uint64_t* counters) {
    if (!c || count <= 0 || count > c->max_batch || !ubufs || !seeds || !counters)
        return fail(c, APM_E_INVALID, "apm_u_normal: bad arguments");
    if (!check_idx(c, count, ubufs, c->n_ubufs, "ubuf")) return APM_E_INVALID;
    const SkewScope skew(c);
    try {
        HIPC(hipSetDevice(c->device));
        const int64_t B = c->max_batch;
        std::memcpy(c->hblk, ubufs, sizeof(int64_t) * count);
        std::memcpy(c->hblk + 5 * B, seeds, sizeof(uint64_t) * count);
        std::memcpy(c->hblk + 6 * B, counters, sizeof(uint64_t) * count);
        HIPC(hipMemcpyAsync(c->d_i3, c->hblk, sizeof(int64_t) * 7 * B, hipMemcpyHostToDevice,
                            c->stream));
        launch_u_normal(c->Up, c->d_i3, c->d_seeds, c->d_ctrs, c->n, c->S, (int)count,
                        c->stream);
        check_launch();
        sync(c);
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_u_combine(apm_ctx* c, int64_t count, const int64_t* dst, const int64_t* a,
                  const int64_t* b, const double* ca, const double* cb) {
    if (!c || count <= 0 || count > c->max_batch || !dst || !a || !b || !ca || !cb)
        return fail(c, APM_E_INVALID, "apm_u_combine: bad arguments");
    if (!check_idx(c, count, dst, c->n_ubufs, "dst") || !check_idx(c, count, a, c->n_ubufs, "a") ||
        !check_idx(c, count, b, c->n_ubufs, "b"))
        return APM_E_INVALID;
    const SkewScope skew(c);
    try {
        HIPC(hipSetDevice(c->device));
        const int64_t B = c->max_batch;
        std::memcpy(c->hblk, dst, sizeof(int64_t) * count);
        std::memcpy(c->hblk + B, a, sizeof(int64_t) * count);
        std::memcpy(c->hblk + 2 * B, b, sizeof(int64_t) * count);
        std::memcpy(c->hblk + 3 * B, ca, sizeof(double) * count);
        std::memcpy(c->hblk + 4 * B, cb, sizeof(double) * count);
        HIPC(hipMemcpyAsync(c->d_i3, c->hblk, sizeof(int64_t) * 5 * B, hipMemcpyHostToDevice,
                            c->stream));
        launch_u_combine(c->Up, c->d_i3, c->d_i3 + c->max_batch, c->d_i3 + 2 * c->max_batch,
                         c->d_ca, c->d_cb, c->n, c->S, (int)count, c->stream);
        check_launch();
        sync(c);
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_theta_eval(apm_ctx* c, int est, int64_t count, const double* thetas, int64_t ldt,
                   const int64_t* ubufs, const int64_t* slots, double* out_logf, int* status,
                   int64_t* nops) {
    if (!c || count <= 0 || count > c->max_batch || !thetas || !out_logf || !status ||
        est < 0 || est > 2 || c->kind == APM_KERNEL_PRECOMPUTED || ldt < c->P)
        return fail(c, APM_E_INVALID, "apm_theta_eval: bad arguments");
    if (est != APM_EST_LAPLACE) {
        if (!ubufs || !slots) return fail(c, APM_E_INVALID, "apm_theta_eval: ubufs/slots required");
        if (!check_idx(c, count, slots, c->n_slots, "slot") ||
            !check_idx(c, count, ubufs, c->n_ubufs, "ubuf"))
            return APM_E_INVALID;
    }
    const SkewScope skew(c);
    try {
        HIPC(hipSetDevice(c->device));
        double* th = c->hth;  // pinned: the upload is asynchronous
        for (int64_t b = 0; b < count; ++b)
            for (int p = 0; p < c->P; ++p) th[b * c->P + p] = thetas[b * ldt + p];
        HIPC(hipMemcpyAsync(c->theta, th, sizeof(double) * count * c->P, hipMemcpyHostToDevice,
                            c->stream));
        // fp16x3 Newton updates need |L_ij| <= sqrt(1 + K_ii) < 65504 (chol32.hip): per chain;
        // the posterior bottom block's operands |L'_ij| <= sqrt(1 + n K_ii) (postcov.hip)
        for (int64_t b = 0; b < count; ++b) {
            pin_h3(c)[b] = c->h3 && th[b * c->P] < 19.0;
            pin_inv(c)[b] = 1.0 + std::exp(th[b * c->P]) + c->eps < 32768.0;
            pin_h3post(c)[b] = c->h3 && 1.0 + c->n * (std::exp(th[b * c->P]) + c->eps) < 4e8;
            pin_icm(c)[b] = c->n * (std::exp(th[b * c->P]) + c->eps) / std::max(c->icm_q, 1.0);
        }
        upload_h3(c, (int)count);
        if (est != APM_EST_LAPLACE) upload_idx(c, (int)count, slots, ubufs);
        theta_eval_impl(c, est, (int)count, true, out_logf, status, nops);
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_theta_eval_K(apm_ctx* c, int est, const double* K, int64_t ldk, int64_t ubuf,
                     int64_t slot, double* out_logf, int* status, int64_t* nops) {
    if (!c || !K || ldk < c->n || !out_logf || !status || est < 0 || est > 2)
        return fail(c, APM_E_INVALID, "apm_theta_eval_K: bad arguments");
    if (est != APM_EST_LAPLACE &&
        (slot < 0 || slot >= c->n_slots || ubuf < 0 || ubuf >= c->n_ubufs))
        return fail(c, APM_E_INVALID, "apm_theta_eval_K: slot/ubuf out of range");
    const SkewScope skew(c);
    try {
        HIPC(hipSetDevice(c->device));
        // identity-padded copy of K into chain 0's K
        std::vector<double> Kp((size_t)c->np * c->np, 0.0);
        for (int i = 0; i < c->np; ++i)
            for (int j = 0; j < c->np; ++j)
                Kp[(size_t)i * c->np + j] =
                    (i < c->n && j < c->n) ? K[(int64_t)i * ldk + j] : (i == j ? 1.0 : 0.0);
        HIPC(hipMemcpyAsync(c->K.base, Kp.data(), sizeof(double) * Kp.size(),
                            hipMemcpyHostToDevice, c->stream));
        c->k_full = true;
        double kmax = 0.0;
        for (int i = 0; i < c->n; ++i) kmax = std::max(kmax, std::fabs(Kp[(size_t)i * c->np + i]));
        pin_h3(c)[0] = c->h3 && kmax < 1.8e8;  // sqrt(1 + K_ii) < 1.4e4 (chol32.hip)
        pin_inv(c)[0] = 1.0 + kmax < 32768.0;
        pin_h3post(c)[0] = c->h3 && 1.0 + c->n * kmax < 4e8;
        pin_icm(c)[0] = c->n * kmax / std::max(c->icm_q, 1.0);
        upload_h3(c, 1);
        upload_idx(c, 1, &slot, &ubuf);  // (the pinned copy is the slot the read-back marks)
        theta_eval_impl(c, est, 1, false, out_logf, status, nops);
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_u_eval(apm_ctx* c, int64_t count, const int64_t* slots, const int64_t* ubufs,
               double* out_logf, int* status) {
    if (!c || count <= 0 || count > c->max_batch || !slots || !ubufs || !out_logf || !status)
        return fail(c, APM_E_INVALID, "apm_u_eval: bad arguments");
    if (!check_idx(c, count, slots, c->n_slots, "slot") ||
        !check_idx(c, count, ubufs, c->n_ubufs, "ubuf"))
        return APM_E_INVALID;
    const SkewScope skew(c);
    try {
        HIPC(hipSetDevice(c->device));
        upload_idx(c, (int)count, slots, ubufs);
        HIPC(hipMemsetAsync(c->status, 0, sizeof(int) * count, c->stream));
        bool wide = false;
        for (int64_t b = 0; b < count; ++b) wide |= c->slot_wide[slots[b]] != 0;
        u_eval_device(c, (int)count, wide);
        read_back(c, {RB{c->out, (int)sizeof(double) * (int)count, out_logf},
                      RB{c->status, (int)sizeof(int) * (int)count, status}});
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

// ---- cache-slot lifetimes (samplers.py:563-584: an MH sampler holds the current state's cache
// and the proposal's at once; on accept the proposal's becomes current and the old one is dropped).
// Host bookkeeping only: a slot's contents are immutable between theta-calls into it, so a copy
// of the handle is another owner of the same state, as a second reference to the reference's
// (K_chol, C_chol, f_post) tuple is.
int apm_cache_acquire(apm_ctx* c, int64_t* slot) {
    if (!c || !slot) return fail(c, APM_E_INVALID, "apm_cache_acquire: bad arguments");
    for (int i = 0; i < c->n_slots; ++i)
        if (c->slot_refs[i] == 0) {
            c->slot_refs[i] = 1;
            *slot = i;
            return APM_SUCCESS;
        }
    return fail(c, APM_E_NOMEM, "apm_cache_acquire: every cache slot is owned (raise n_slots)");
}

int apm_cache_copy(apm_ctx* c, int64_t slot) {
    if (!c || slot < 0 || slot >= c->n_slots || c->slot_refs[slot] <= 0)
        return fail(c, APM_E_INVALID, "apm_cache_copy: slot not acquired");
    ++c->slot_refs[slot];
    return APM_SUCCESS;
}

int apm_cache_release(apm_ctx* c, int64_t slot) {
    if (!c || slot < 0 || slot >= c->n_slots || c->slot_refs[slot] <= 0)
        return fail(c, APM_E_INVALID, "apm_cache_release: slot not acquired");
    --c->slot_refs[slot];
    return APM_SUCCESS;
}

int64_t apm_cache_refcount(const apm_ctx* c, int64_t slot) {
    if (!c || slot < 0 || slot >= c->n_slots) return APM_E_INVALID;
    return c->slot_refs[slot];
}

int apm_slot_read(apm_ctx* c, int64_t slot, double* L, int64_t ldl, double* f_post, double* g,
                  double* cst) {
    if (!c || slot < 0 || slot >= c->n_slots) return fail(c, APM_E_INVALID, "apm_slot_read: bad slot");
    try {
        HIPC(hipSetDevice(c->device));
        const int64_t np = c->np;
        if (L || g) {
            std::vector<float> h((size_t)((np + 64) * np));
            HIPC(hipMemcpyAsync(h.data(), c->Sl.L + slot * c->Sl.lstride, sizeof(float) * h.size(),
                                hipMemcpyDeviceToHost, c->stream));
            sync(c);
            if (L)  // (the slot keeps row i only up to its diagonal tile)
                for (int i = 0; i < c->n; ++i)
                    for (int j = 0; j < c->n; ++j)
                        L[(int64_t)i * ldl + j] = j <= i ? h[(size_t)i * np + j] : 0.0;
            if (g)
                for (int j = 0; j < c->n; ++j) g[j] = h[(size_t)np * np + j];
        }
        if (f_post) {
            HIPC(hipMemcpyAsync(f_post, c->Sl.fpost64 + slot * c->Sl.vstride, sizeof(double) * c->n,
                                hipMemcpyDeviceToHost, c->stream));
        }
        if (cst)
            HIPC(hipMemcpyAsync(cst, c->Sl.cst + slot, sizeof(double), hipMemcpyDeviceToHost,
                                c->stream));
        sync(c);
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_gram(int device, int kind, const double* X, int64_t n, int64_t d, int64_t ldx,
             const double* theta, int64_t n_theta, double eps, double* K, int64_t ldk) {
    if (n <= 0 || d <= 0 || !X || !theta || !K || ldk < n || ldx < d ||
        (kind != APM_KERNEL_ISO && kind != APM_KERNEL_ARD))
        return fail(nullptr, APM_E_INVALID, "apm_gram: bad arguments");
    const int64_t P = kind == APM_KERNEL_ISO ? 2 : d + 1;
    if (n_theta < P) return fail(nullptr, APM_E_INVALID, "apm_gram: theta too short");
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_tuple(device, n, d, kind + 16);
    apm_ctx*& c = g_cache[key];
    try {
        if (!c) {
            c = new apm_ctx();
            init_ctx(c, device, kind, X, n, d, ldx, nullptr, eps, 1, 1, 1, 1);
        } else {
            HIPC(hipSetDevice(device));
            std::vector<double> Xc((size_t)(n * d));
            for (int64_t i = 0; i < n; ++i)
                for (int64_t k = 0; k < d; ++k) Xc[i * d + k] = X[i * ldx + k];
            HIPC(hipMemcpyAsync(c->X, Xc.data(), sizeof(double) * n * d, hipMemcpyHostToDevice,
                                c->stream));
        }
        HIPC(hipMemcpyAsync(c->theta, theta, sizeof(double) * P, hipMemcpyHostToDevice, c->stream));
        HIPC(hipMemsetD32Async(c->active, 1, 1, c->stream));
        HIPC(hipMemsetAsync(c->status, 0, sizeof(int), c->stream));
        launch_gram(c->K, c->X, d, (int)n, (int)d, c->theta, P, kind, eps, c->np, live_of(c), 1,
                    c->stream, true);
        check_launch();
        HIPC(hipMemcpy2DAsync(K, sizeof(double) * ldk, c->K.base, sizeof(double) * c->np,
                              sizeof(double) * n, n, hipMemcpyDeviceToHost, c->stream));
        sync(c);
    } catch (const HipError& e) {
        if (c) {
            free_ctx(c);
            c = nullptr;
        }
        return fail(nullptr, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_laplace(int device, const double* K, int64_t n, int64_t ldk, const double* y,
                int calc_cov, int calc_lml, double diff_f_tol, int64_t max_iters, double* f_out,
                double* C_out, int64_t ldc, double* lml_out, int64_t* n_iter_out, int* status) {
    if (!K || !y || n <= 0 || ldk < n || !f_out || !status || max_iters < 0 ||
        (calc_cov && (!C_out || ldc < n)) || (calc_lml && !lml_out))
        return fail(nullptr, APM_E_INVALID, "apm_laplace: bad arguments");
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_tuple(device, n, (int64_t)0, (int)APM_KERNEL_PRECOMPUTED);
    apm_ctx*& c = g_cache[key];
    try {
        if (!c) {
            c = new apm_ctx();
            init_ctx(c, device, APM_KERNEL_PRECOMPUTED, nullptr, n, 0, 0, y, 1e-8, 1, 1, 1, 1);
        } else {
            HIPC(hipSetDevice(device));
            std::vector<double> yp((size_t)c->np, 0.0);
            for (int64_t i = 0; i < n; ++i) yp[i] = y[i];
            HIPC(hipMemcpyAsync(c->y, yp.data(), sizeof(double) * c->np, hipMemcpyHostToDevice,
                                c->stream));
        }
        c->tol = diff_f_tol;
        c->max_iters = max_iters;
        const int np = c->np;
        std::vector<double> Kp((size_t)np * np, 0.0);
        for (int i = 0; i < np; ++i)
            for (int j = 0; j < np; ++j)
                Kp[(size_t)i * np + j] =
                    (i < n && j < n) ? K[(int64_t)i * ldk + j] : (i == j ? 1.0 : 0.0);
        HIPC(hipMemcpyAsync(c->K.base, Kp.data(), sizeof(double) * Kp.size(), hipMemcpyHostToDevice,
                            c->stream));
        c->k_full = true;
        HIPC(hipMemsetD32Async(c->active, 1, 1, c->stream));
        HIPC(hipMemsetAsync(c->status, 0, sizeof(int), c->stream));
        HIPC(hipMemsetAsync(c->n_iter, 0, sizeof(int), c->stream));
        std::vector<int> st(1, 0);
        c->live_n = 1;
        newton(c, 1, st, false, 1);
        int it = 0;
        HIPC(hipMemcpyAsync(&it, c->n_iter, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        sync(c);
        *status = st[0];
        if (n_iter_out) *n_iter_out = it;
        if (st[0] != APM_STATUS_OK) return APM_SUCCESS;
        HIPC(hipMemcpyAsync(f_out, c->v.f, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
        if (calc_lml) {
            launch_laplace_lml(c->v, c->y, (int)n, c->ldet, c->lstride, c->nb, c->out, live_of(c),
                               1, c->stream);
            check_launch();
            HIPC(hipMemcpyAsync(lml_out, c->out, sizeof(double), hipMemcpyDeviceToHost, c->stream));
        }
        if (calc_cov) {
            augmented(c, 1);  // bottom-right of A now holds C = K - V^T V (lower)
            std::vector<double> Cb((size_t)np * np);
            HIPC(hipMemcpy2DAsync(Cb.data(), sizeof(double) * np,
                                  c->A.base + (int64_t)np * c->A.ld + np, sizeof(double) * c->A.ld,
                                  sizeof(double) * np, np, hipMemcpyDeviceToHost, c->stream));
            sync(c);
            for (int64_t i = 0; i < n; ++i)
                for (int64_t j = 0; j <= i; ++j) {
                    C_out[i * ldc + j] = Cb[(size_t)i * np + j];
                    C_out[j * ldc + i] = Cb[(size_t)i * np + j];
                }
        }
        sync(c);
    } catch (const HipError& e) {
        if (c) {
            free_ctx(c);
            c = nullptr;
        }
        return fail(nullptr, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_selftest_tile(int device, const double* A, const double* B, double* C) {
    if (!A || !B || !C) return fail(nullptr, APM_E_INVALID, "apm_selftest_tile: null pointer");
    double* d = nullptr;
    try {
        HIPC(hipSetDevice(device));
        HIPC(hipMalloc(&d, sizeof(double) * 3 * 4096));
        HIPC(hipMemcpy(d, A, sizeof(double) * 4096, hipMemcpyHostToDevice));
        HIPC(hipMemcpy(d + 4096, B, sizeof(double) * 4096, hipMemcpyHostToDevice));
        HIPC(hipMemcpy(d + 8192, C, sizeof(double) * 4096, hipMemcpyHostToDevice));
        launch_tile_nt_test(d, d + 4096, d + 8192, nullptr);
        check_launch();
        HIPC(hipMemcpy(C, d + 8192, sizeof(double) * 4096, hipMemcpyDeviceToHost));
        HIPC(hipFree(d));
    } catch (const HipError& e) {
        if (d) (void)hipFree(d);
        return fail(nullptr, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_selftest_philox(int device, int64_t n, const uint32_t* in, uint32_t* out) {
    if (!in || !out || n <= 0 || n > (1 << 24))
        return fail(nullptr, APM_E_INVALID, "apm_selftest_philox: bad arguments");
    uint32_t* d = nullptr;
    try {
        HIPC(hipSetDevice(device));
        HIPC(hipMalloc(&d, sizeof(uint32_t) * 10 * n));
        HIPC(hipMemcpy(d, in, sizeof(uint32_t) * 6 * n, hipMemcpyHostToDevice));
        launch_philox_test(d, d + 6 * n, n, nullptr);
        check_launch();
        HIPC(hipMemcpy(out, d + 6 * n, sizeof(uint32_t) * 4 * n, hipMemcpyDeviceToHost));
        HIPC(hipFree(d));
    } catch (const HipError& e) {
        if (d) (void)hipFree(d);
        return fail(nullptr, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_guard_read(apm_ctx* c, int64_t count, double* r) {
    if (!c || !r || count <= 0 || count > c->max_batch)
        return fail(c, APM_E_INVALID, "apm_guard_read: bad arguments");
    try {
        HIPC(hipSetDevice(c->device));
        std::vector<double> h((size_t)4 * c->max_batch);
        HIPC(hipMemcpyAsync(h.data(), c->guard + 2 * c->max_batch, sizeof(double) * h.size(),
                            hipMemcpyDeviceToHost, c->stream));
        sync(c);
        for (int64_t b = 0; b < count; ++b)
            for (int k = 0; k < 4; ++k) r[4 * b + k] = h[(size_t)k * c->max_batch + b];
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_prof_enable(apm_ctx* c, int on) {
    if (!c) return fail(c, APM_E_INVALID, "apm_prof_enable: null ctx");
    c->prof = on < 0 ? 0 : (on > 2 ? 2 : on);
    return APM_SUCCESS;
}

int apm_prof_marker(apm_ctx* c, int id) {
    if (!c || id < 0 || id > 3) return fail(c, APM_E_INVALID, "apm_prof_marker: bad arguments");
    try {
        HIPC(hipSetDevice(c->device));
        launch_marker(id, c->stream);
        check_launch();
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

int apm_prof_read(apm_ctx* c, int kind, double* total_ms, int64_t* launches, double* work,
                  int reset) {
    if (!c || kind < 0 || kind >= APM_PROF_NKINDS)
        return fail(c, APM_E_INVALID, "apm_prof_read: bad arguments");
    try {
        HIPC(hipSetDevice(c->device));
        sync(c);
        if (kind == APM_PROF_DF_TIMEOUTS || kind == APM_PROF_TRSV_TIMEOUTS) {
            unsigned long long* d = spin_words(c) + (kind == APM_PROF_TRSV_TIMEOUTS ? 1 : 0);
            unsigned long long h = 0;
            HIPC(hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost));
            if (total_ms) *total_ms = 0.0;
            if (launches) *launches = (int64_t)h;
            if (work) *work = 0.0;
            if (reset) HIPC(hipMemset(d, 0, sizeof(h)));
            return APM_SUCCESS;
        }
        if (kind == APM_PROF_POST64_RERUNS) {
            if (total_ms) *total_ms = 0.0;
            if (launches) *launches = c->n_post64;
            if (work) *work = 0.0;
            if (reset) c->n_post64 = 0;
            return APM_SUCCESS;
        }
        if (kind == APM_PROF_ICM_CHECKS || kind == APM_PROF_GUARD) {
            int64_t& n = kind == APM_PROF_GUARD ? c->n_guard : c->n_icm_check;
            if (total_ms) *total_ms = 0.0;
            if (launches) *launches = n;
            if (work) *work = 0.0;
            if (reset) n = 0;
            return APM_SUCCESS;
        }
        if (kind == APM_PROF_STATS) {
            if (total_ms) *total_ms = 0.0;
            if (launches) *launches = c->n_fp64_rerun;
            if (work) *work = (double)c->n_refine_steps;
            if (reset) c->n_fp64_rerun = c->n_refine_steps = 0;
            return APM_SUCCESS;
        }
        double ms = 0.0, wk = 0.0;
        int64_t cnt = 0;
        for (const ProfRec& r : c->recs) {
            if (r.kind != kind) continue;
            float e = 0.f;
            HIPC(hipEventElapsedTime(&e, r.a, r.b));
            ms += e;
            wk += r.work;
            ++cnt;
        }
        if (total_ms) *total_ms = ms;
        if (launches) *launches = cnt;
        if (work) *work = wk;
        if (reset) {
            c->recs.clear();
            c->evnext = 0;
        }
    } catch (const HipError& e) {
        return fail(c, APM_E_HIP, e.msg);
    }
    return APM_SUCCESS;
}

}  // extern "C"
