// Blocked right-looking Cholesky (fp64, f64 MFMA) and the Newton back-substitution.
//
// Replaces the LAPACK potrf / potrs calls of the reference hot path:
//   la.cholesky(K)  gpdemo/estimators.py:206,321    la.cholesky(B)  latent_posterior_approximations.py:92
//   la.cholesky(C)  gpdemo/estimators.py:209        la.cho_solve(L, .)  latent_posterior_approximations.py:94
// The work matrix is tiled TB x TB (TB = 64). One workgroup (4 waves) owns one output tile; each
// wave owns a 32x32 quadrant = 2x2 v_mfma_f64_16x16x4_f64 accumulators.
#include <algorithm>
#include <vector>

#include "apm_internal.h"
#include "diag.h"

// v_mfma_f64_16x16x4_f64 operand/result maps (cdna_hip_programming.md §3):
//   A: lane l holds A[row = l&15][k = l>>4]; B: lane l holds B[k = l>>4][col = l&15]
//   C/D: lane l, reg r  ->  row = (l>>4) + 4r, col = l&15
#define F64_CROW(l, r) (((l) >> 4) + 4 * (r))

__device__ __forceinline__ void tile_acc_load(d4_t (&acc)[2][2], const double* T, int64_t ld,
                                              int wr, int wc, int lane) {
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[bi][bj][r] = T[(int64_t)(32 * wr + 16 * bi + F64_CROW(lane, r)) * ld +
                                   32 * wc + 16 * bj + (lane & 15)];
}

__device__ __forceinline__ void tile_acc_store(const d4_t (&acc)[2][2], double* T, int64_t ld,
                                               int wr, int wc, int lane) {
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                T[(int64_t)(32 * wr + 16 * bi + F64_CROW(lane, r)) * ld + 32 * wc + 16 * bj +
                  (lane & 15)] = acc[bi][bj][r];
}

#ifndef UPD_ABL
#define UPD_ABL 0
#endif
#ifndef UPD_WPE
#define UPD_WPE 3  // min waves per SIMD for k_chol_update (caps VGPRs at 168)
#endif
#ifndef UPD_PF
#define UPD_PF 2   // slices of global loads in flight (1 or 2)
#endif
#ifndef UPD_LATEC
#define UPD_LATEC 1  // load the old tile behind the first slices and add it at the end
#endif
#ifndef UPD_KS
#define UPD_KS 16
#endif
#define KSUB UPD_KS
#define LPITCH (UPD_KS + 1)
struct GemmSmem {
    double a[2][64][LPITCH];
    double b[2][64][LPITCH];
};

// acc += (NEG ? -1 : 1) * A[64 x depth] * B[64 x depth]^T (+ the tile C, if given) for the
// workgroup's 64x64 tile. Operands are staged through LDS in KS-deep slices shared by the four
// waves, double-buffered, with TWO slices of global loads in flight (register sets alternate with
// the slice parity; loads are unconditional - clamped to the last slice - so the compiler's
// vmcnt waits count exactly and never drain the newer set). The old C tile, when given, is loaded
// behind the first two slices and added at the end, off the critical path of the first MFMA.
// One barrier per slice; LDS pitch KS+1 keeps the fragment reads bank-conflict free.
template <bool NEG>
__device__ __forceinline__ void tile_gemm_nt(d4_t (&acc)[2][2], const double* __restrict__ A,
                                             int64_t lda, const double* __restrict__ B,
                                             int64_t ldb, int depth, GemmSmem& sm,
                                             const double* __restrict__ C = nullptr,
                                             int64_t ldc = 0) {
    constexpr int PPR = KSUB / 2;          // 16-byte pieces per row of a slice
    constexpr int PPT = 64 * PPR / 256;    // pieces per thread per operand
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1;
    const int r16 = lane & 15, kq = lane >> 4;
    int prow[PPT], pcol[PPT];
#pragma unroll
    for (int h = 0; h < PPT; ++h) {
        const int p = tid + 256 * h;
        prow[h] = p / PPR;
        pcol[h] = (p % PPR) * 2;
    }
    auto gload = [&](int sidx, d2_t (&ra)[PPT], d2_t (&rb)[PPT]) {
#if UPD_ABL == 1  // ablation (tools/upd_bench.cpp): operands always slice 0 (L1/L2 resident)
        sidx = 0;
#endif
#pragma unroll
        for (int h = 0; h < PPT; ++h) {
            const int kc = sidx * KSUB + pcol[h];
            ra[h] = *reinterpret_cast<const d2_t*>(A + (int64_t)prow[h] * lda + kc);
            rb[h] = *reinterpret_cast<const d2_t*>(B + (int64_t)prow[h] * ldb + kc);
        }
    };
    auto sstore = [&](int buf, const d2_t (&ra)[PPT], const d2_t (&rb)[PPT]) {
#pragma unroll
        for (int h = 0; h < PPT; ++h) {
            sm.a[buf][prow[h]][pcol[h]] = NEG ? -ra[h].x : ra[h].x;
            sm.a[buf][prow[h]][pcol[h] + 1] = NEG ? -ra[h].y : ra[h].y;
            sm.b[buf][prow[h]][pcol[h]] = rb[h].x;
            sm.b[buf][prow[h]][pcol[h] + 1] = rb[h].y;
        }
    };
    auto compute = [&](int cur) {
#pragma unroll
        for (int t = 0; t < KSUB / 4; ++t) {
            double a[2], b[2];
#pragma unroll
            for (int bi = 0; bi < 2; ++bi) a[bi] = sm.a[cur][32 * wr + 16 * bi + r16][4 * t + kq];
#pragma unroll
            for (int bj = 0; bj < 2; ++bj) b[bj] = sm.b[cur][32 * wc + 16 * bj + r16][4 * t + kq];
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
                for (int bj = 0; bj < 2; ++bj)
#if UPD_ABL == 2  // ablation: no MFMA (memory + LDS + barrier pipeline only)
                    acc[bi][bj][0] += a[bi] * b[bj];
#else
                    acc[bi][bj] =
                        __builtin_amdgcn_mfma_f64_16x16x4f64(a[bi], b[bj], acc[bi][bj], 0, 0, 0);
#endif
        }
    };
    const int nsub = depth / KSUB;  // even: depth is a multiple of 64 and KS <= 32
    d4_t old[2][2];
#if UPD_PF == 2
    d2_t ra0[PPT], rb0[PPT], ra1[PPT], rb1[PPT];
    gload(0, ra0, rb0);
    gload(1, ra1, rb1);
    if (C) tile_acc_load(old, C, ldc, wr, wc, lane);
    sstore(0, ra0, rb0);
    __syncthreads();
    for (int s = 0; s < nsub; s += 2) {
        gload(min(s + 2, nsub - 1), ra0, rb0);
        compute(0);
        sstore(1, ra1, rb1);
        __syncthreads();
        gload(min(s + 3, nsub - 1), ra1, rb1);
        compute(1);
        sstore(0, ra0, rb0);  // past the end: a clamped reload into a buffer no longer read
        __syncthreads();
    }
#else
    d2_t ra0[PPT], rb0[PPT];
    gload(0, ra0, rb0);
    if (C) tile_acc_load(old, C, ldc, wr, wc, lane);
    sstore(0, ra0, rb0);
    __syncthreads();
    for (int s = 0; s < nsub; ++s) {
        gload(min(s + 1, nsub - 1), ra0, rb0);
        compute(s & 1);
        sstore((s + 1) & 1, ra0, rb0);
        __syncthreads();
    }
#endif
    if (C) {
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj) acc[bi][bj] += old[bi][bj];
    }
}

__device__ __forceinline__ bool chain_live(const Live& lv, int b) {
    return lv.active[b] != 0 && lv.status[b] == 0;
}

// ------------------------------------------------------------------------------- diagonal tile
// Stand-alone diag step (one wave per chain): tile (k, k) -> LDS, diag_compute + diag_store (diag.h). Used for
// the first column of every factorisation; every later diagonal tile is factored inside the
// update launch that produces it (k_chol_update below, fuse_diag).
template <class Mat, class TS>
__global__ __launch_bounds__(64) void k_chol_diag(Mat A, int k, TS* Dinv, int64_t dstride,
                                                  double* ldet, int64_t lstride, Live live,
                                                  int fail_code) {
    const int b = blockIdx.x;
    if (!chain_live(live, b)) return;
    __shared__ DiagSmemT<TS> S;  // fp32 tiles (Newton matrix): fp32 arithmetic
    const int lane = threadIdx.x;
    TS* At = A.base + b * A.cstride + (int64_t)(k * 64) * A.ld + k * 64;
    // 64x64 tile -> LDS: 4 rounds of 8 independent 2-element loads per lane (lane: 2 columns)
#pragma unroll
    for (int q0 = 0; q0 < 64; q0 += 16) {
        d2_t v[8];
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            const int q = q0 + 2 * h + (lane >> 5);
            v[h] = ld2(At + (int64_t)q * A.ld + 2 * (lane & 31));
        }
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            const int q = q0 + 2 * h + (lane >> 5);
            S.T[q * DP + 2 * (lane & 31)] = v[h].x;
            S.T[q * DP + 2 * (lane & 31) + 1] = v[h].y;
        }
    }
    if (!diag_compute<true>(S, lane)) {
        if (lane == 0) live.status[b] = fail_code;
        return;
    }
    diag_store<TS>(S, At, A.ld, Dinv + b * dstride + (int64_t)k * 4096, ldet + b * lstride + k,
                   lane, 64);
}

void launch_chol_diag(MatB A, int k, double* Dinv, int64_t dstride, double* ldet, int64_t lstride,
                      Live live, int fail_code, int nchains, hipStream_t s) {
    APM_LAUNCH((k_chol_diag<MatB, double>), dim3(nchains), dim3(64), 0, s, A, k, Dinv,
                       dstride, ldet, lstride, live, fail_code);
}

void launch_chol_diag32(MatF A, int k, float* Dinv, int64_t dstride, double* ldet,
                        int64_t lstride, Live live, int fail_code, int nchains, hipStream_t s) {
    APM_LAUNCH((k_chol_diag<MatF, float>), dim3(nchains), dim3(64), 0, s, A, k, Dinv,
                       dstride, ldet, lstride, live, fail_code);
}

// ------------------------------------------------------------------------------- panel TRSM
__global__ __launch_bounds__(256) void k_chol_panel(MatB A, int k, int i0, int glo, int ghi,
                                                    const double* Dinv, int64_t dstride,
                                                    Live live) {
    const int b = blockIdx.y;
    if (!chain_live(live, b)) return;
    int i = i0 + blockIdx.x;
    if (i >= glo) i += ghi - glo;  // skip the row tiles [glo, ghi) (known-zero rows)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
    double* At = A.base + b * A.cstride + (int64_t)(i * 64) * A.ld + k * 64;
    const double* D = Dinv + b * dstride + (int64_t)k * 4096;
    __shared__ GemmSmem sm;
    d4_t acc[2][2];
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = d4_t{0.0, 0.0, 0.0, 0.0};
    tile_gemm_nt<false>(acc, At, A.ld, D, 64, 64, sm);  // X = A_ik * inv(L_kk)^T
    tile_acc_store(acc, At, A.ld, wr, wc, lane);  // A_ik fully staged before the last barrier
}

void launch_chol_panel(MatB A, int k, int i0, int R, int glo, int ghi, const double* Dinv,
                       int64_t dstride, Live live, int nchains, hipStream_t s) {
    glo = std::max(glo, i0);
    ghi = std::min(ghi, R);
    if (ghi <= glo) glo = ghi = R;
    const int rows = (R - i0) - (ghi - glo);
    if (rows <= 0) return;
    APM_LAUNCH(k_chol_panel, dim3(rows, nchains), dim3(256), 0, s, A, k, i0, glo, ghi, Dinv,
                       dstride, live);
}

// ------------------------------------------------------------------------------- trailing update
// A_ij -= sum_{q<kc} A_{i,k0+q} A_{j,k0+q}^T for tiles i in [i0, R), j in [j0, min(i, jend-1)]
// (i0 >= j0): a triangular part (rows i < jend: i-j0+1 tiles) and a rectangular part (rows
// i >= jend: jend-j0 tiles).
long update_tile_count(int i0, int R, int j0, int jend) {
    if (jend <= j0 || R <= i0) return 0;
    const long a0 = i0 - j0 + 1;
    const int ntri_rows = std::max(0, std::min(R, jend) - i0);
    long n = ntri_rows * a0 + (long)ntri_rows * (ntri_rows - 1) / 2;
    const int rect_rows = R - std::max(i0, jend);
    if (rect_rows > 0) n += (long)rect_rows * (jend - j0);
    return n;
}

// Work item w -> (chain, tile) with an XCD-aware remap: workgroups are dealt round-robin over the
// 8 XCDs (MI355X_MICROARCH.md, dispatch), so XCD x = L % 8 is given the contiguous work range
// [x*q+min(x,r), ...) (bijective for any count). Consecutive work items are consecutive tiles of
// one chain in the host-built super-tile order (8x8 tiles: 8 row panels + 8 column panels = 2 MiB
// of operands per super-tile), so the operand panels a workgroup needs are in its XCD's L2.
__device__ __forceinline__ long xcd_remap(long L, long total) {
    const long xcd = L & 7, q = total >> 3, r = total & 7;
    const long base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (L >> 3);
}

// Fused diag (fd.enabled): tiles[0] must be the diagonal tile (d, d) the next column step
// factors. Workgroups 0 .. nchains-1 (dispatched first) update chain b's tile (d, d), keep it in
// LDS and factor it with wave 0 (diag_compute; all four waves store it, diag_store), so its
// latency hides under the rest of the launch;
// the other workgroups take the remaining (ntiles - 1) tiles of every chain.
__global__ __launch_bounds__(256, UPD_WPE) void k_chol_update(MatB A, int k0, int kc,
                                                              const unsigned* __restrict__ tiles,
                                                              int ntiles, int nchains, int plus,
                                                              Live live, FusedDiag<double> fd) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wr = wv >> 1, wc = wv & 1;
    __shared__ union {
        GemmSmem g;
        DiagSmem d;
    } sm;
    int b, t;
    const bool fused = fd.enabled && (int)blockIdx.x < nchains;
    if (fused) {
        b = blockIdx.x;
        t = 0;
    } else {
        const int nt = fd.enabled ? ntiles - 1 : ntiles;
        const long L = (long)blockIdx.x - (fd.enabled ? nchains : 0);
        const long w = xcd_remap(L, (long)nt * nchains);
        b = (int)(w / nt);
        t = (int)(w % nt) + (fd.enabled ? 1 : 0);
    }
    if (!chain_live(live, b)) return;
    const unsigned ij = tiles[t];
    const int i = (int)(ij >> 16), j = (int)(ij & 0xffff);
    double* Ab = A.base + b * A.cstride;
    double* Aij = Ab + (int64_t)(i * 64) * A.ld + j * 64;
    d4_t acc[2][2];
#if UPD_LATEC
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = d4_t{0.0, 0.0, 0.0, 0.0};
    const double* Cold = Aij;
#else
    tile_acc_load(acc, Aij, A.ld, wr, wc, lane);
    const double* Cold = nullptr;
#endif
    const double* Ai = Ab + (int64_t)(i * 64) * A.ld + k0 * 64;
    const double* Aj = Ab + (int64_t)(j * 64) * A.ld + k0 * 64;
    if (plus)  // A_ij += ... (the SYRK of the UL factorisation, postcov.hip)
        tile_gemm_nt<false>(acc, Ai, A.ld, Aj, A.ld, 64 * kc, sm.g, Cold, A.ld);
    else
        tile_gemm_nt<true>(acc, Ai, A.ld, Aj, A.ld, 64 * kc, sm.g, Cold, A.ld);
    if (!fused) {
        tile_acc_store(acc, Aij, A.ld, wr, wc, lane);
        return;
    }
    // tile_gemm_nt ended on a barrier: the GEMM staging area is free for the diag working set
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                sm.d.T[(32 * wr + 16 * bi + F64_CROW(lane, r)) * DP + 32 * wc + 16 * bj +
                       (lane & 15)] = acc[bi][bj][r];
    __syncthreads();
    if (wv == 0) {  // rolled pivot loops: the unrolled (DPP) form would cost this kernel a wave
        const bool ok = diag_compute<false>(sm.d, lane);
        if (lane == 0) sm.d.ok = ok;
    }
    __syncthreads();
    if (!sm.d.ok) {
        if (threadIdx.x == 0) live.status[b] = fd.fail_code;
        return;
    }
    diag_store<double>(sm.d, Aij, A.ld, fd.Dinv + b * fd.dstride + (int64_t)i * 4096,
                       fd.ldet + b * fd.lstride + i, threadIdx.x, 256);
}

void launch_chol_update(MatB A, int k0, int kc, const unsigned* tiles, int ntiles, bool plus,
                        Live live, int nchains, hipStream_t s, FusedDiag<double> fd) {
    if (ntiles <= 0) return;
    const long total = (long)ntiles * nchains;
    APM_LAUNCH(k_chol_update, dim3((unsigned)total), dim3(256), 0, s, A, k0, kc, tiles,
                       ntiles, nchains, (int)plus, live, fd);
}

// ------------------------------------------------------------------------- 128x128 trailing update
// The fp64 twin of chol32.hip's k_chol_update32_t128 (super-tile entries and validity rules of
// build_update_supertiles): one 128x128 super-tile per workgroup, each wave a 64x64 tile as 4x4
// v_mfma_f64_16x16x4_f64 accumulators (128 VGPRs). Per byte staged it feeds twice the MFMAs of the
// 64x64 kernel, whose operand-load rate co-limits it. Operands move global -> LDS with 16-byte
// LDS-DMA loads (global_load_lds_dwordx4: no staging registers, no ds_write pass), two buffers of
// KS = 16-deep slices; the LDS image is lane-linear per wave (8 rows of 128 B per instruction)
// with the 16-byte pieces XOR-swizzled by row (piece p of row r at slot p ^ (r & 7)), so the
// 16-byte fragment reads of 8 consecutive rows hit distinct banks.
#define KS64T 16
#ifndef T64_ABL
#define T64_ABL 0
#endif
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
struct __attribute__((aligned(16))) GemmSmem64T {
    double a[2][128][KS64T];
    double b[2][128][KS64T];
};

template <bool NEG, bool INIT = false>
__device__ __forceinline__ void update_t128_body(MatB A, int k0, int kc, unsigned e, int b,
                                                 bool fused, Live live, FusedDiag<double> fd,
                                                 GemmSmem64T& smg, DiagSmem& smd, MatB S) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wr = wv >> 1, wc = wv & 1;
    const int r16 = lane & 15, kq = lane >> 4;
    const int ti = (int)(e >> 18), tj = (int)((e >> 4) & 0x3fff);
    const bool rv0 = e & 1u, rv1 = e & 2u, cv0 = e & 4u, cv1 = e & 8u;
    const int ra0 = rv0 ? ti : ti + 1, ra1 = rv1 ? ti + 1 : ti;
    const int cb0 = cv0 ? tj : tj + 1, cb1 = cv1 ? tj + 1 : tj;
    double* Ab = A.base + b * A.cstride;
    const int oi = ti + wr, oj = tj + wc;
    const bool mine = (wr ? rv1 : rv0) && (wc ? cv1 : cv0) && oj <= oi;

    // LDS-DMA staging: wave wv moves operand rows 32wv .. 32wv+31 (4 instructions of 8 rows);
    // lane l takes row +l/8 and stores slot l%8, i.e. global piece (l%8) ^ (l/8)
    const int srow = 32 * wv + (lane >> 3);  // < 64 for waves 0,1 (first half), else second
    const int spiece = (lane & 7) ^ (lane >> 3);
    const int64_t ld8 = 8 * A.ld;
    const double* ga = Ab + (int64_t)((wv < 2 ? ra0 : ra1) * 64 + (srow & 63)) * A.ld + k0 * 64 +
                       2 * spiece;
    const double* gb = Ab + (int64_t)((wv < 2 ? cb0 : cb1) * 64 + (srow & 63)) * A.ld + k0 * 64 +
                       2 * spiece;
    auto glds = [&](int sidx, int buf) {
#if T64_ABL == 2  // ablation (tools/upd64_bench.cpp): no operand loads
        return;
#endif
        const int o = sidx * KS64T;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            __builtin_amdgcn_global_load_lds((glb_void_t*)(ga + q * ld8 + o),
                                             (lds_void_t*)&smg.a[buf][32 * wv + 8 * q][0], 16, 0, 0);
            __builtin_amdgcn_global_load_lds((glb_void_t*)(gb + q * ld8 + o),
                                             (lds_void_t*)&smg.b[buf][32 * wv + 8 * q][0], 16, 0, 0);
        }
    };
    d4_t acc[4][4];
    // lane group kq takes the slice's k values 4kq .. 4kq+3 (the same k for A and B): a lane's
    // fragments of two MFMA steps are one 16-byte LDS read (piece 2kq+h, swizzled by row)
    auto compute = [&](int cur) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int slot = ((2 * kq + h) ^ (r16 & 7)) * 2;
            d2_t a2[4], b2[4];
#pragma unroll
            for (int bi = 0; bi < 4; ++bi)
                a2[bi] = *reinterpret_cast<const d2_t*>(&smg.a[cur][64 * wr + 16 * bi + r16][slot]);
#pragma unroll
            for (int bj = 0; bj < 4; ++bj)
                b2[bj] = *reinterpret_cast<const d2_t*>(&smg.b[cur][64 * wc + 16 * bj + r16][slot]);
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
                for (int bi = 0; bi < 4; ++bi)
#pragma unroll
                    for (int bj = 0; bj < 4; ++bj)
#if T64_ABL == 1  // ablation: no MFMA (loads + LDS + barriers only)
                        acc[bi][bj][0] += a2[bi][q] * b2[bj][q];
#else
                        acc[bi][bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                            a2[bi][q], b2[bj][q], acc[bi][bj], 0, 0, 0);
#endif
        }
    };
    // INIT (the SYRK I + Y Y^T, Y lower triangular from column block k0): block k of Y is zero in
    // rows above it, so tiles of column j need k <= j only - one launch over the whole depth
    const int nsub = (64 * (INIT ? min(kc, max(cb0, cb1) + 1) : kc)) / KS64T;
    // old tile into acc (negated for A_ij -= ...: acc = -C + sum, result = -acc), consumed before
    // the loop so that no wait for it lands inside (see k_chol_update32_t128)
    const int li = mine ? oi : (wr ? ra1 : ra0), lj = mine ? oj : (wc ? cb1 : cb0);
    // (S.base: out of place - the old tile comes from S, e.g. K for the first trailing update of
    // chol(K), whose working copy holds the first outer panel only: capi.cpp chol_k_begin)
    const int64_t cld = S.base ? S.ld : A.ld;
    const double* Cw = (S.base ? S.base + b * S.cstride : Ab) + (int64_t)(li * 64) * cld + lj * 64;
#pragma unroll
    for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int bj = 0; bj < 4; ++bj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (INIT) {  // old tile = I (plus == 2): nothing to read
                    acc[bi][bj][r] =
                        (li * 64 + 16 * bi + F64_CROW(lane, r) == lj * 64 + 16 * bj + r16) ? 1.0
                                                                                          : 0.0;
                    continue;
                }
                const double v = Cw[(int64_t)(16 * bi + F64_CROW(lane, r)) * cld + 16 * bj + r16];
                acc[bi][bj][r] = NEG ? -v : v;
            }
#pragma unroll
    for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int bj = 0; bj < 4; ++bj) asm volatile("" : "+v"(acc[bi][bj]));
    glds(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < nsub; ++s) {
        if (s + 1 < nsub) glds(s + 1, (s + 1) & 1);  // lands while slice s is multiplied
        // a wave whose tile is dropped (diagonal super-tile's upper half, invalid half) only
        // stages; in the SYRK a wave's tile column oj needs Y's column blocks k <= oj only (the
        // rest of the workgroup's depth multiplies zeros)
        if (mine && (!INIT || (s * KS64T) / 64 <= oj)) compute(s & 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (NEG) {
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int bj = 0; bj < 4; ++bj) acc[bi][bj] = -acc[bi][bj];
    }
    double* Cout = Ab + (int64_t)(oi * 64) * A.ld + oj * 64;
    const bool diag_here = fused && wv == 0;
    if (mine && !diag_here) {
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int bj = 0; bj < 4; ++bj)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    Cout[(int64_t)(16 * bi + F64_CROW(lane, r)) * A.ld + 16 * bj + r16] =
                        acc[bi][bj][r];
    }
    if (!fused) return;
    if (wv == 0) {
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int bj = 0; bj < 4; ++bj)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    smd.T[(16 * bi + F64_CROW(lane, r)) * DP + 16 * bj + r16] = acc[bi][bj][r];
    }
    __syncthreads();
    if (wv == 0) {  // rolled pivot loops (register budget), as in k_chol_update
        const bool ok = diag_compute<false>(smd, lane);
        if (lane == 0) smd.ok = ok;
    }
    __syncthreads();
    if (!smd.ok) {
        if (tid == 0) live.status[b] = fd.fail_code;
        return;
    }
    diag_store<double>(smd, Ab + (int64_t)(ti * 64) * A.ld + tj * 64, A.ld,
                       fd.Dinv + b * fd.dstride + (int64_t)ti * 4096, fd.ldet + b * fd.lstride + ti,
                       tid, 256);
}

__global__ __launch_bounds__(256, 2) void k_chol_update_t128(MatB A, int k0, int kc,
                                                             const unsigned* __restrict__ tiles,
                                                             int ntiles, int nchains, int plus,
                                                             Live live, FusedDiag<double> fd,
                                                             MatB S) {
    __shared__ union {
        GemmSmem64T g;
        DiagSmem d;
    } sm;
    int b, t;
    const bool fused = fd.enabled && (int)blockIdx.x < nchains;
    if (fused) {
        b = blockIdx.x;
        t = 0;
    } else {
        const int nt = fd.enabled ? ntiles - 1 : ntiles;
        const long L = (long)blockIdx.x - (fd.enabled ? nchains : 0);
        const long w = xcd_remap(L, (long)nt * nchains);
        b = (int)(w / nt);
        t = (int)(w % nt) + (fd.enabled ? 1 : 0);
    }
    if (!chain_live(live, b)) return;
    if (plus == 2)  // A_ij = I_ij + Y_i Y_j^T (the SYRK of the UL factorisation, postcov.hip)
        update_t128_body<false, true>(A, k0, kc, tiles[t], b, fused, live, fd, sm.g, sm.d, S);
    else if (plus)  // A_ij += ...
        update_t128_body<false>(A, k0, kc, tiles[t], b, fused, live, fd, sm.g, sm.d, S);
    else
        update_t128_body<true>(A, k0, kc, tiles[t], b, fused, live, fd, sm.g, sm.d, S);
}

void launch_chol_update_t128(MatB A, int k0, int kc, const unsigned* tiles, int ntiles, int plus,
                             Live live, int nchains, hipStream_t s, FusedDiag<double> fd,
                             MatB S) {
    if (ntiles <= 0) return;
    const long total = (long)ntiles * nchains;
    APM_LAUNCH(k_chol_update_t128, dim3((unsigned)total), dim3(256), 0, s, A, k0, kc,
                       tiles, ntiles, nchains, plus, live, fd, S);
}

// Host: tiles (i, j), i in [i0, R), j0 <= j <= min(i, jend-1), in super-tile order (SxS tiles,
// super-rows top-down, super-columns left-right, row-major inside), packed (i << 16) | j.
std::vector<unsigned> build_update_tiles(int i0, int R, int j0, int jend, int glo, int ghi) {
    std::vector<unsigned> v;
    const int S = 8;
    for (int I = i0; I < R; I += S)
        for (int J = j0; J < jend; J += S)
            for (int i = I; i < std::min(I + S, R); ++i) {
                if (i >= glo && i < ghi) continue;
                for (int j = J; j < std::min(J + S, jend); ++j)
                    if (j <= i) v.push_back(((unsigned)i << 16) | (unsigned)j);
            }
    return v;
}

// ------------------------------------------------------------------------------- L^T z = r
// Step J of the blocked backward solve (J = nb-1 .. 0). r lives in row `rrow` of A and is
// updated in place; every workgroup first forms z_J = inv(L_JJ)^T r_J (64x64 GEMV), then
// workgroup I < J subtracts L_JI^T z_J from r_I and workgroup I == J stores z_J.
__global__ __launch_bounds__(256) void k_trsv_lt_step(MatB A, int J, int64_t rrow,
                                                      const double* Dinv, int64_t dstride,
                                                      double* z, int64_t zstride, Live live) {
    const int b = blockIdx.y;
    if (!chain_live(live, b)) return;
    const int I = blockIdx.x;
    const int tid = threadIdx.x, c = tid & 63, q = tid >> 6;
    __shared__ double rj[64];
    __shared__ double part[4][64];
    __shared__ double zj[64];
    double* Ab = A.base + b * A.cstride;
    double* r = Ab + rrow * A.ld;
    if (tid < 64) rj[tid] = r[J * 64 + tid];
    __syncthreads();
    // z_J[c] = sum_m inv(L_JJ)[m][c] * r_J[m]
    const double* D = Dinv + b * dstride + (int64_t)J * 4096;
    double s = 0.0;
    for (int m = q * 16; m < q * 16 + 16; ++m) s += D[m * 64 + c] * rj[m];
    part[q][c] = s;
    __syncthreads();
    if (tid < 64) zj[tid] = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
    __syncthreads();
    if (I == J) {
        if (tid < 64) z[b * zstride + J * 64 + tid] = zj[tid];
        return;
    }
    // r_I[c] -= sum_m L[J*64+m][I*64+c] * z_J[m]
    const double* L = Ab + (int64_t)(J * 64) * A.ld + I * 64;
    s = 0.0;
    for (int m = q * 16; m < q * 16 + 16; ++m) s += L[(int64_t)m * A.ld + c] * zj[m];
    part[q][c] = s;
    __syncthreads();
    if (tid < 64) r[I * 64 + tid] -= part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
}

void launch_trsv_lt_step(MatB A, int J, int64_t rrow, const double* Dinv, int64_t dstride,
                         double* z, int64_t zstride, Live live, int nchains, hipStream_t s) {
    APM_LAUNCH(k_trsv_lt_step, dim3(J + 1, nchains), dim3(256), 0, s, A, J, rrow, Dinv,
                       dstride, z, zstride, live);
}

// ------------------------------------------------------------------------------- test hook
__global__ __launch_bounds__(256) void k_tile_nt_test(const double* A, const double* B,
                                                      double* C) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
    __shared__ GemmSmem sm;
    d4_t acc[2][2];
    tile_acc_load(acc, C, 64, wr, wc, lane);
    tile_gemm_nt<false>(acc, A, 64, B, 64, 64, sm);
    tile_acc_store(acc, C, 64, wr, wc, lane);
}

void launch_tile_nt_test(const double* A, const double* B, double* C, hipStream_t s) {
    APM_LAUNCH(k_tile_nt_test, dim3(1), dim3(256), 0, s, A, B, C);
}

// ------------------------------------------------------------------------------- trace markers
template <int ID>
__global__ void k_apm_marker() {}

void launch_marker(int id, hipStream_t s) {
    switch (id) {
        case 0: APM_LAUNCH(k_apm_marker<0>, dim3(1), dim3(64), 0, s); break;
        case 1: APM_LAUNCH(k_apm_marker<1>, dim3(1), dim3(64), 0, s); break;
        case 2: APM_LAUNCH(k_apm_marker<2>, dim3(1), dim3(64), 0, s); break;
        default: APM_LAUNCH(k_apm_marker<3>, dim3(1), dim3(64), 0, s); break;
    }
}

// ------------------------------------------------------------------------------- chol(K) retry
// DESIGN.md §3.4 (capi.cpp retry_chol_k): a chain whose blocked factorisation of K failed
// (fail[b] == code) has K's lower triangle factored again, unblocked, in LAPACK's dpotf2 order -
// left-looking column by column, L_jj = sqrt(K_jj - L_j,:j . L_j,:j), then
// L_ij = (K_ij - L_i,:j . L_j,:j) / L_jj - each dot product with four interleaved fma
// accumulators summed pairwise, as OpenBLAS's unrolled ddot does inside the dpotf2 that decides
// the reference's LinAlgError (estimators.py:206). At the reference's two
// InvalidCovarianceMatrixError thetas (tests/golden/icm_k.npz) this order passes on the
// reference's own K where the blocked factorisation, whose panels multiply by inverted diagonal
// tiles, rounds K to indefinite; the chain then reaches the reference-route check of chol(C) as
// in the reference. One workgroup per chain (row j of L staged in LDS); success clears fail[b]
// and writes L (zeros above the diagonal inside diagonal tiles) and the per-tile log-diagonal
// sums. No inverses of diagonal tiles are written: the IS theta-call's consumers of L_K (the
// tile-parallel L_K^T a and the posterior factor's Y2 / L_K J pass) do not read them.
#define UNBLOCKED_MAXNP 512
__device__ __forceinline__ double dot4(const double* x, const double* y, int m) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int k = 0;
    for (; k + 4 <= m; k += 4) {
        a0 = fma(x[k], y[k], a0);
        a1 = fma(x[k + 1], y[k + 1], a1);
        a2 = fma(x[k + 2], y[k + 2], a2);
        a3 = fma(x[k + 3], y[k + 3], a3);
    }
    if (k < m) a0 = fma(x[k], y[k], a0);
    if (k + 1 < m) a1 = fma(x[k + 1], y[k + 1], a1);
    if (k + 2 < m) a2 = fma(x[k + 2], y[k + 2], a2);
    return (a0 + a1) + (a2 + a3);
}

__global__ __launch_bounds__(256) void k_chol_unblocked(MatB K, MatB A, int np, int* fail,
                                                        int code, double* ldet, int64_t lstride) {
    const int b = blockIdx.x, tid = threadIdx.x;
    if (fail[b] != code) return;
    __shared__ double lj[UNBLOCKED_MAXNP];
    __shared__ double ljj;
    const double* Kb = K.base + b * K.cstride;
    double* Ab = A.base + b * A.cstride;
    for (int i = tid; i < np; i += 256) {  // K's lower triangle, zeros above it in diagonal tiles
        const int cend = (i / 64 + 1) * 64;
        for (int c = 0; c < cend; ++c)
            Ab[(int64_t)i * A.ld + c] = c <= i ? Kb[(int64_t)i * K.ld + c] : 0.0;
    }
    __syncthreads();
    for (int j = 0; j < np; ++j) {
        for (int k = tid; k < j; k += 256) lj[k] = Ab[(int64_t)j * A.ld + k];
        __syncthreads();
        if (tid == 0) {
            const double d = Ab[(int64_t)j * A.ld + j] - dot4(lj, lj, j);
            ljj = d > 0.0 ? sqrt(d) : 0.0;  // (NaN fails too)
            Ab[(int64_t)j * A.ld + j] = ljj;
        }
        __syncthreads();
        if (!(ljj > 0.0)) return;  // still failed: fail[b] stays
        const double l = ljj;
        for (int i = j + 1 + tid; i < np; i += 256) {
            double* Ai = Ab + (int64_t)i * A.ld;
            Ai[j] = (Ai[j] - dot4(Ai, lj, j)) / l;
        }
        __syncthreads();
    }
    const int w = tid >> 6, lane = tid & 63;
    for (int t = w; t < np / 64; t += 4) {
        const int r = t * 64 + lane;
        const double s = wave_sum_d(log(Ab[(int64_t)r * A.ld + r]));
        if (lane == 0) ldet[b * lstride + t] = s;
    }
    if (tid == 0) fail[b] = 0;
}

bool launch_chol_unblocked(MatB K, MatB A, int np, int* fail, int code, double* ldet,
                           int64_t lstride, int nchains, hipStream_t s) {
    if (np > UNBLOCKED_MAXNP) return false;
    APM_LAUNCH(k_chol_unblocked, dim3(nchains), dim3(256), 0, s, K, A, np, fail, code, ldet,
               lstride);
    return true;
}
