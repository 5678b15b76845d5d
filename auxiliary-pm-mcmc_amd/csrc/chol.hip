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

// v_mfma_f64_16x16x4_f64 operand/result maps (cdna_hip_programming.md §3):
//   A: lane l holds A[row = l&15][k = l>>4]; B: lane l holds B[k = l>>4][col = l&15]
//   C/D: lane l, reg r  ->  row = (l>>4) + 4r, col = l&15
#define F64_CROW(l, r) (((l) >> 4) + 4 * (r))

// acc += (NEG ? -1 : 1) * A[64x64] * B[64x64]^T restricted to this wave's quadrant (wr, wc).
// Both operands are row-major [output index][inner index]. The inner index is permuted per lane
// (lane group kq handles inner k = 16*kq + t at MFMA step t) so that each lane streams 16
// contiguous doubles (128 B) per operand row with 16-byte loads; the permutation is the same for
// A and B, so the sum over the inner index is unchanged.
template <bool NEG>
__device__ __forceinline__ void tile_nt_f64(d4_t (&acc)[2][2], const double* __restrict__ A,
                                            int64_t lda, const double* __restrict__ B,
                                            int64_t ldb, int wr, int wc, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
    double a[2][16], b[2][16];
#pragma unroll
    for (int bi = 0; bi < 2; ++bi) {
        const double* p = A + (int64_t)(32 * wr + 16 * bi + r16) * lda + kq * 16;
#pragma unroll
        for (int t = 0; t < 16; t += 2) {
            const d2_t v = *reinterpret_cast<const d2_t*>(p + t);
            a[bi][t] = NEG ? -v.x : v.x;
            a[bi][t + 1] = NEG ? -v.y : v.y;
        }
    }
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
        const double* p = B + (int64_t)(32 * wc + 16 * bj + r16) * ldb + kq * 16;
#pragma unroll
        for (int t = 0; t < 16; t += 2) {
            const d2_t v = *reinterpret_cast<const d2_t*>(p + t);
            b[bj][t] = v.x;
            b[bj][t + 1] = v.y;
        }
    }
#pragma unroll
    for (int t = 0; t < 16; ++t)
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj)
                acc[bi][bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[bi][t], b[bj][t],
                                                                    acc[bi][bj], 0, 0, 0);
}

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
#ifdef APM_DIAG_STAMPS
__device__ unsigned long long g_diag_stamps[16];  // diagnostic build only (tools/diag_stamps.cpp)
#endif
#define DP 65  // LDS pitch (doubles) of the diag kernel's tile

// Broadcast lane l's value of a wave-uniform-indexed register (v_readlane x2).
__device__ __forceinline__ double rdlane(double v, int l) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// 16x16x16 products on LDS operands with one v_mfma_f64_16x16x4_f64 chain (4 steps):
//   NT: acc[r][c] += sum_k A[r][k] * B[c][k]      NN: acc[r][c] += sum_k A[r][k] * B[k][c]
template <bool NEG>
__device__ __forceinline__ void mm16_nt(d4_t& acc, const double* a, int lda, const double* b,
                                        int ldb, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const double av = a[r16 * lda + 4 * t + kq];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(NEG ? -av : av, b[r16 * ldb + 4 * t + kq], acc,
                                                   0, 0, 0);
    }
}
__device__ __forceinline__ void mm16_nn(d4_t& acc, const double* a, int lda, const double* b,
                                        int ldb, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[r16 * lda + 4 * t + kq],
                                                   b[(4 * t + kq) * ldb + r16], acc, 0, 0, 0);
}
__device__ __forceinline__ void st16(const d4_t& acc, double* dst, int ld, int lane, double sgn) {
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[((lane >> 4) + 4 * q) * ld + (lane & 15)] = sgn * acc[q];
}
__device__ __forceinline__ void st16t(const d4_t& acc, double* dst, int ld, int lane, double sgn) {
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[(lane & 15) * ld + (lane >> 4) + 4 * q] = sgn * acc[q];
}
// Products with a diagonal block X of the inverse held as (strict lower part transposed at Td,
// diagonal in xd): X[r][c] = c < r ? Td[c][r] : (c == r ? xd[r] : 0).
__device__ __forceinline__ double xblk(const double* Td, const double* xd, int r, int c) {
    return (c < r) ? Td[c * DP + r] : ((c == r) ? xd[r] : 0.0);
}
//   acc += A * X^T
__device__ __forceinline__ void mm16_nt_xb(d4_t& acc, const double* a, int lda, const double* Td,
                                           const double* xd, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[r16 * lda + 4 * t + kq],
                                                   xblk(Td, xd, r16, 4 * t + kq), acc, 0, 0, 0);
}
//   acc += A * X
__device__ __forceinline__ void mm16_nn_xb(d4_t& acc, const double* a, int lda, const double* Td,
                                           const double* xd, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[r16 * lda + 4 * t + kq],
                                                   xblk(Td, xd, 4 * t + kq, r16), acc, 0, 0, 0);
}
//   acc += X * B
__device__ __forceinline__ void mm16_nn_xa(d4_t& acc, const double* Td, const double* xd,
                                           const double* b, int ldb, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xblk(Td, xd, r16, 4 * t + kq),
                                                   b[(4 * t + kq) * ldb + r16], acc, 0, 0, 0);
}
__device__ __forceinline__ void ld16(d4_t& acc, const double* src, int ld, int lane) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = src[((lane >> 4) + 4 * q) * ld + (lane & 15)];
}

// 64x64 Cholesky + inverse of the lower factor by ONE wave (no barriers), blocked by 16:
// per 16-column block the 16x16 diagonal block is factored with lane r holding row r in
// registers (pivot by v_readlane, column broadcast through LDS, 1/sqrt by v_rsq_f64 + two Newton
// steps) and inverted (lane c substitutes column c); the 16-wide panel solve, the rank-16
// trailing update and the assembly of the full inverse X_ab = -X_aa sum_{k=b}^{a-1} L_ak X_kb are
// 16x16x16 f64-MFMA products on LDS operands. The inverse is kept transposed in the unused upper
// triangle of T (X_ab, a > b, in block (b, a); the strictly lower part of X_aa in the upper part of
// diagonal block (a, a); its diagonal in xdg): 36 KB of LDS, so that the kernel fits next to three
// padded update workgroups on a CU (lookahead, capi.cpp).
// Storage of the tile and of Dinv is fp64 (MatB) or fp32 (MatF, the mixed-precision Newton
// factorisation, chol32.hip); the factorisation itself always runs in fp64.
__device__ __forceinline__ d2_t ld2(const double* p) { return *reinterpret_cast<const d2_t*>(p); }
__device__ __forceinline__ d2_t ld2(const float* p) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    return d2_t{(double)v.x, (double)v.y};
}
template <class Mat, class TS>
__global__ __launch_bounds__(64) void k_chol_diag(Mat A, int k, TS* Dinv, int64_t dstride,
                                                  double* ldet, int64_t lstride, Live live,
                                                  int fail_code) {
    const int b = blockIdx.x;
    if (!chain_live(live, b)) return;
    __shared__ double T[64 * DP];
    __shared__ double xdg[64];
    __shared__ double Tmp[16 * 17];
    __shared__ double colb[16];
    __shared__ double dg[64];
    const int lane = threadIdx.x;
#ifdef APM_DIAG_STAMPS
    unsigned long long stamps[16];
    int ns = 0;
#define STAMP() if (lane == 0 && ns < 16) stamps[ns++] = __builtin_amdgcn_s_memtime()
#else
#define STAMP()
#endif
    STAMP();
    TS* At = A.base + b * A.cstride + (int64_t)(k * 64) * A.ld + k * 64;
    // 32 KB tile -> LDS: 4 rounds of 8 independent 16-byte loads per lane (lane covers 2 columns)
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
            T[q * DP + 2 * (lane & 31)] = v[h].x;
            T[q * DP + 2 * (lane & 31) + 1] = v[h].y;
        }
    }
    STAMP();
    const int r = lane & 15;
    for (int kb = 0; kb < 4; ++kb) {
        const int o = kb * 16;
        // (a) factor the 16x16 diagonal block
        double row[16], yv[16], dv[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) row[c] = T[(o + r) * DP + o + c];
        bool bad = false;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const double p = rdlane(row[j], j);
            bad |= !(p > 0.0);
            double y = __builtin_amdgcn_rsq(p);
            y = y * (1.5 - 0.5 * p * y * y);
            y = y * (1.5 - 0.5 * p * y * y);
            yv[j] = y;
            dv[j] = p * y;
            row[j] = (r > j) ? row[j] * y : ((r == j) ? dv[j] : row[j]);
            if (lane < 16) colb[r] = row[j];
#pragma unroll
            for (int c = j + 1; c < 16; ++c) row[c] -= row[j] * colb[c];
        }
        if (bad) {  // wave-uniform
            if (lane == 0) live.status[b] = fail_code;
            return;
        }
        if (lane < 16) {
#pragma unroll
            for (int c = 0; c < 16; ++c) T[(o + r) * DP + o + c] = (c <= r) ? row[c] : 0.0;
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < 16; ++j) dg[o + j] = dv[j];
        }
        // inverse of the 16x16 factor: lane c (< 16) solves for column c
        {
            const int c = r;
            double x[16];
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) {
                double sacc = (rr == c) ? 1.0 : 0.0;
#pragma unroll
                for (int m = 0; m < rr; ++m) sacc -= T[(o + rr) * DP + o + m] * x[m];
                x[rr] = (rr >= c) ? sacc * yv[rr] : 0.0;
            }
            if (lane < 16) {
#pragma unroll
                for (int rr = 0; rr < 16; ++rr)
                    if (rr > c) T[(o + c) * DP + o + rr] = x[rr];
                xdg[o + c] = x[c];
            }
        }
        if (kb == 3) break;
        // (b) panel: T[ib][kb] = T[ib][kb] * inv(L_kb,kb)^T for the blocks below
        for (int ib = kb + 1; ib < 4; ++ib) {
            d4_t acc = {0.0, 0.0, 0.0, 0.0};
            mm16_nt_xb(acc, &T[(16 * ib) * DP + o], DP, &T[o * DP + o], &xdg[o], lane);
            st16(acc, &T[(16 * ib) * DP + o], DP, lane, 1.0);
        }
        // (c) rank-16 trailing update of the lower blocks
        for (int ib = kb + 1; ib < 4; ++ib)
            for (int jb = kb + 1; jb <= ib; ++jb) {
                d4_t acc;
                ld16(acc, &T[(16 * ib) * DP + 16 * jb], DP, lane);
                mm16_nt<true>(acc, &T[(16 * ib) * DP + o], DP, &T[(16 * jb) * DP + o], DP, lane);
                st16(acc, &T[(16 * ib) * DP + 16 * jb], DP, lane, 1.0);
            }
        STAMP();
    }
    // off-diagonal blocks of the inverse, block row by block row
    for (int a = 1; a < 4; ++a)
        for (int bb = 0; bb < a; ++bb) {
            d4_t acc = {0.0, 0.0, 0.0, 0.0};
            mm16_nn_xb(acc, &T[(16 * a) * DP + 16 * bb], DP, &T[(16 * bb) * DP + 16 * bb],
                       &xdg[16 * bb], lane);
            for (int kk = bb + 1; kk < a; ++kk)  // X_kk,bb is stored transposed at T block (bb, kk)
                mm16_nt<false>(acc, &T[(16 * a) * DP + 16 * kk], DP, &T[(16 * bb) * DP + 16 * kk],
                               DP, lane);
            st16(acc, Tmp, 17, lane, 1.0);
            d4_t acc2 = {0.0, 0.0, 0.0, 0.0};
            mm16_nn_xa(acc2, &T[(16 * a) * DP + 16 * a], &xdg[16 * a], Tmp, 17, lane);
            st16t(acc2, &T[(16 * bb) * DP + 16 * a], DP, lane, -1.0);
        }
    STAMP();
    TS* D = Dinv + b * dstride + (int64_t)k * 4096;
    for (int q = 0; q < 64; ++q) {
        At[(int64_t)q * A.ld + lane] = (TS)((lane <= q) ? T[q * DP + lane] : 0.0);
        D[q * 64 + lane] = (TS)((lane < q) ? T[lane * DP + q] : ((lane == q) ? xdg[q] : 0.0));
    }
    const double l = wave_sum_d(log(dg[lane]));
    if (lane == 0) ldet[b * lstride + k] = l;
#ifdef APM_DIAG_STAMPS
    STAMP();
    if (lane == 0 && k == 0 && b == 0)
        for (int q = 0; q < ns; ++q) g_diag_stamps[q] = stamps[q] - stamps[0];
#endif
}

void launch_chol_diag(MatB A, int k, double* Dinv, int64_t dstride, double* ldet, int64_t lstride,
                      Live live, int fail_code, int nchains, hipStream_t s) {
    hipLaunchKernelGGL((k_chol_diag<MatB, double>), dim3(nchains), dim3(64), 0, s, A, k, Dinv,
                       dstride, ldet, lstride, live, fail_code);
}

void launch_chol_diag32(MatF A, int k, float* Dinv, int64_t dstride, double* ldet,
                        int64_t lstride, Live live, int fail_code, int nchains, hipStream_t s) {
    hipLaunchKernelGGL((k_chol_diag<MatF, float>), dim3(nchains), dim3(64), 0, s, A, k, Dinv,
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
    hipLaunchKernelGGL(k_chol_panel, dim3(rows, nchains), dim3(256), 0, s, A, k, i0, glo, ghi, Dinv,
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

__global__ __launch_bounds__(256, UPD_WPE) void k_chol_update(MatB A, int k0, int kc,
                                                     const unsigned* __restrict__ tiles, int ntiles,
                                                     int nchains, int plus, Live live) {
    const long total = (long)ntiles * nchains;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wr = wv >> 1, wc = wv & 1;
    __shared__ GemmSmem sm;
    {
        const long L = blockIdx.x;
        const long w = xcd_remap(L, total);
        const int b = (int)(w / ntiles);
        if (!chain_live(live, b)) return;
        const unsigned ij = tiles[w % ntiles];
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
            tile_gemm_nt<false>(acc, Ai, A.ld, Aj, A.ld, 64 * kc, sm, Cold, A.ld);
        else
            tile_gemm_nt<true>(acc, Ai, A.ld, Aj, A.ld, 64 * kc, sm, Cold, A.ld);
        tile_acc_store(acc, Aij, A.ld, wr, wc, lane);
    }
}

void launch_chol_update(MatB A, int k0, int kc, const unsigned* tiles, int ntiles, bool plus,
                        Live live, int nchains, hipStream_t s, int lds_pad) {
    if (ntiles <= 0) return;
    const long total = (long)ntiles * nchains;
    hipLaunchKernelGGL(k_chol_update, dim3((unsigned)total), dim3(256), lds_pad, s, A, k0, kc,
                       tiles, ntiles, nchains, (int)plus, live);
}

// ------------------------------------------------------------------------------- 128x128 update
// Outer (rank-256) updates: one workgroup per 2x2 group of 64-tiles; wave (wr, wc) owns sub-tile
// (i+wr, j+wc) as 4x4 v_mfma_f64_16x16x4 accumulators (128 VGPRs), so each 16-deep LDS slice
// feeds 64 MFMAs per wave from 8 fragment reads (twice the operand reuse of the 64x64 kernel).
// Sub-tiles outside the update region (above the diagonal, past R or jend) skip their MFMAs and
// stores; out-of-range operand rows are clamped to a valid row and their results discarded.
struct BigSmem {
    double a[2][128][17];
    double b[2][128][17];
};

__global__ __launch_bounds__(256, 2) void k_chol_update_big(MatB A, int k0, int kc,
                                                         const unsigned* __restrict__ tiles,
                                                         int ntiles, int nchains, int R, int jend,
                                                         Live live) {
    const long total = (long)ntiles * nchains;
    const long w = xcd_remap(blockIdx.x, total);
    const int b = (int)(w / ntiles);
    if (!chain_live(live, b)) return;
    const unsigned ij = tiles[w % ntiles];
    const int i0 = (int)(ij >> 16), j0 = (int)(ij & 0xffff);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wr = wv >> 1, wc = wv & 1;
    const int r16 = lane & 15, kq = lane >> 4;
    const int ti = i0 + wr, tj = j0 + wc;
    const bool valid = ti < R && tj < jend && tj <= ti;
    double* Ab = A.base + b * A.cstride;
    __shared__ BigSmem sm;
    d4_t acc[4][4];
    double* Aij = Ab + (int64_t)(ti * 64) * A.ld + tj * 64;
    if (valid) {
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int bj = 0; bj < 4; ++bj)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[bi][bj][q] = Aij[(int64_t)(16 * bi + F64_CROW(lane, q)) * A.ld + 16 * bj + r16];
    }
    // staging: 1024 pieces of 16 B per operand slice (128 rows x 128 B); thread -> 4 pieces
    const int pc = (tid & 7) * 2;
    const double* pa[4];
    const double* pb[4];
    int prow[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int row = (tid >> 3) + 32 * h;  // 0..127
        prow[h] = row;
        const int ra = min(i0 * 64 + row, R * 64 - 1);
        const int rb = min(j0 * 64 + row, R * 64 - 1);
        pa[h] = Ab + (int64_t)ra * A.ld + k0 * 64 + pc;
        pb[h] = Ab + (int64_t)rb * A.ld + k0 * 64 + pc;
    }
    d2_t ra_[4], rb_[4];
    const int nsub = 4 * kc;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        ra_[h] = *reinterpret_cast<const d2_t*>(pa[h]);
        rb_[h] = *reinterpret_cast<const d2_t*>(pb[h]);
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        sm.a[0][prow[h]][pc] = -ra_[h].x;
        sm.a[0][prow[h]][pc + 1] = -ra_[h].y;
        sm.b[0][prow[h]][pc] = rb_[h].x;
        sm.b[0][prow[h]][pc + 1] = rb_[h].y;
    }
    __syncthreads();
    for (int sl = 0; sl < nsub; ++sl) {
        const int cur = sl & 1;
        if (sl + 1 < nsub) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                ra_[h] = *reinterpret_cast<const d2_t*>(pa[h] + (sl + 1) * 16);
                rb_[h] = *reinterpret_cast<const d2_t*>(pb[h] + (sl + 1) * 16);
            }
        }
        if (valid) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                double av[4], bv[4];
#pragma unroll
                for (int bi = 0; bi < 4; ++bi) av[bi] = sm.a[cur][64 * wr + 16 * bi + r16][4 * t + kq];
#pragma unroll
                for (int bj = 0; bj < 4; ++bj) bv[bj] = sm.b[cur][64 * wc + 16 * bj + r16][4 * t + kq];
#pragma unroll
                for (int bi = 0; bi < 4; ++bi)
#pragma unroll
                    for (int bj = 0; bj < 4; ++bj)
                        acc[bi][bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[bi], bv[bj],
                                                                            acc[bi][bj], 0, 0, 0);
            }
        }
        if (sl + 1 < nsub) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                sm.a[cur ^ 1][prow[h]][pc] = -ra_[h].x;
                sm.a[cur ^ 1][prow[h]][pc + 1] = -ra_[h].y;
                sm.b[cur ^ 1][prow[h]][pc] = rb_[h].x;
                sm.b[cur ^ 1][prow[h]][pc + 1] = rb_[h].y;
            }
        }
        __syncthreads();
    }
    if (valid) {
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int bj = 0; bj < 4; ++bj)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    Aij[(int64_t)(16 * bi + F64_CROW(lane, q)) * A.ld + 16 * bj + r16] = acc[bi][bj][q];
    }
}

void launch_chol_update_big(MatB A, int k0, int kc, const unsigned* tiles, int ntiles, int R,
                            int jend, Live live, int nchains, hipStream_t s) {
    if (ntiles <= 0) return;
    const long total = (long)ntiles * nchains;
    hipLaunchKernelGGL(k_chol_update_big, dim3((unsigned)total), dim3(256), 0, s, A, k0, kc, tiles,
                       ntiles, nchains, R, jend, live);
}

// Host: 2x2 groups (top-left tile (i, j)) covering the update region, in super-tile order
std::vector<unsigned> build_update_tiles_big(int i0, int R, int j0, int jend) {
    std::vector<unsigned> v;
    const int S = 8;
    for (int I = i0; I < R; I += S)
        for (int J = j0; J < jend; J += S)
            for (int i = I; i < std::min(I + S, R); i += 2)
                for (int j = J; j < std::min(J + S, jend); j += 2)
                    if (j <= i + 1) v.push_back(((unsigned)i << 16) | (unsigned)j);
    return v;
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
    hipLaunchKernelGGL(k_trsv_lt_step, dim3(J + 1, nchains), dim3(256), 0, s, A, J, rrow, Dinv,
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
    hipLaunchKernelGGL(k_tile_nt_test, dim3(1), dim3(256), 0, s, A, B, C);
}
