// Factorisation of one 64x64 diagonal tile (Cholesky + inverse of the factor), shared by the
// stand-alone diag kernel (chol.hip) and the trailing-update kernels that fuse it into the
// workgroup that produces the tile (chol.hip, chol32.hip).
//
// One wave, no barriers, blocked by 16: per 16-column block the 16x16 diagonal block is factored
// with lane r holding row r in registers (pivot by v_readlane, column broadcast through LDS,
// 1/sqrt by v_rsq_f64 + two Newton steps) and inverted (lane c substitutes column c); the
// 16-wide panel solve, the rank-16 trailing update and the assembly of the full inverse
// X_ab = -X_aa sum_{k=b}^{a-1} L_ak X_kb are 16x16x16 f64-MFMA products on LDS operands. The
// inverse is kept transposed in the unused upper triangle of T (X_ab, a > b, in block (b, a); the
// strictly lower part of X_aa in the upper part of diagonal block (a, a); its diagonal in xdg), so
// the whole working set is 36 KB. Arithmetic is fp64 whatever the storage type of the tile.
#pragma once
#include <type_traits>
#include "apm_internal.h"

#ifndef DIAG_SKIP  // development bisection of the phase costs (tools/diag_test.cpp): bit mask
#define DIAG_SKIP 0
#endif

#define DP 65  // LDS pitch (doubles) of the diag kernel's tile

// Arithmetic type R of the factorisation: double (fp64 tiles; fp32 tiles whose factor must be
// fp64-accurate) or float (the mixed-precision Newton matrix, whose factor only has to be
// fp32-accurate: iterative refinement in fp64 follows). The float form runs the same algorithm
// on v_mfma_f32_16x16x4_f32 (32 instead of 64 cycles), single-dword broadcasts and v_rsq_f32.
template <class R>
struct V4;
template <>
struct V4<double> {
    typedef d4_t t;
};
template <>
struct V4<float> {
    typedef f4_t t;
};
template <class R>
__device__ __forceinline__ typename V4<R>::t mfma16(R a, R b, typename V4<R>::t c) {
    if constexpr (sizeof(R) == 8)
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// row of accumulator register q of lane l (16x16x4 f64: (l >> 4) + 4q; f32: 4 (l >> 4) + q)
template <class R>
__device__ __forceinline__ int crow16(int lane, int q) {
    return sizeof(R) == 8 ? (lane >> 4) + 4 * q : 4 * (lane >> 4) + q;
}

// Broadcast lane l's value of a wave-uniform-indexed register (v_readlane).
__device__ __forceinline__ double rdlane(double v, int l) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ float rdlane(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// Broadcast lane j of every 16-lane row to the whole row (DPP row_newbcast, gfx90a+).
template <int J>
__device__ __forceinline__ double row_bcast(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u & 0xffffffffull), 0x150 + J,
                                               0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), 0x150 + J, 0xf, 0xf,
                                               false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int J>
__device__ __forceinline__ float row_bcast(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                 0x150 + J, 0xf, 0xf, false));
}
// 1/sqrt(p) to the arithmetic type's precision
__device__ __forceinline__ double rsqrt_r(double p) {
    double y = __builtin_amdgcn_rsq(p);
    y = y * (1.5 - 0.5 * p * y * y);
    return y * (1.5 - 0.5 * p * y * y);
}
__device__ __forceinline__ float rsqrt_r(float p) {
    const float y = __builtin_amdgcn_rsqf(p);
    return y * (1.5f - 0.5f * p * y * y);
}
template <int J, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (J < N) {
        f(std::integral_constant<int, J>{});
        static_for<J + 1, N>(f);
    }
}

// 16x16x16 products on LDS operands with one 16x16x4 MFMA chain (4 steps):
//   NT: acc[r][c] += sum_k A[r][k] * B[c][k]      NN: acc[r][c] += sum_k A[r][k] * B[k][c]
template <bool NEG, class R>
__device__ __forceinline__ void mm16_nt(typename V4<R>::t& acc, const R* a, int lda, const R* b,
                                        int ldb, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const R av = a[r16 * lda + 4 * t + kq];
        acc = mfma16<R>(NEG ? -av : av, b[r16 * ldb + 4 * t + kq], acc);
    }
}
template <class R>
__device__ __forceinline__ void mm16_nn(typename V4<R>::t& acc, const R* a, int lda, const R* b,
                                        int ldb, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        acc = mfma16<R>(a[r16 * lda + 4 * t + kq], b[(4 * t + kq) * ldb + r16], acc);
}
template <class R>
__device__ __forceinline__ void st16(const typename V4<R>::t& acc, R* dst, int ld, int lane,
                                     R sgn) {
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[crow16<R>(lane, q) * ld + (lane & 15)] = sgn * acc[q];
}
template <class R>
__device__ __forceinline__ void st16t(const typename V4<R>::t& acc, R* dst, int ld, int lane,
                                      R sgn) {
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[(lane & 15) * ld + crow16<R>(lane, q)] = sgn * acc[q];
}
// Products with a diagonal block X of the inverse held as (strict lower part transposed at Td,
// diagonal in xd): X[r][c] = c < r ? Td[c][r] : (c == r ? xd[r] : 0).
template <class R>
__device__ __forceinline__ R xblk(const R* Td, const R* xd, int r, int c) {
    return (c < r) ? Td[c * DP + r] : ((c == r) ? xd[r] : R(0));
}
//   acc += A * X^T
template <class R>
__device__ __forceinline__ void mm16_nt_xb(typename V4<R>::t& acc, const R* a, int lda,
                                           const R* Td, const R* xd, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        acc = mfma16<R>(a[r16 * lda + 4 * t + kq], xblk(Td, xd, r16, 4 * t + kq), acc);
}
//   acc += A * X
template <class R>
__device__ __forceinline__ void mm16_nn_xb(typename V4<R>::t& acc, const R* a, int lda,
                                           const R* Td, const R* xd, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        acc = mfma16<R>(a[r16 * lda + 4 * t + kq], xblk(Td, xd, 4 * t + kq, r16), acc);
}
//   acc += X * B
template <class R>
__device__ __forceinline__ void mm16_nn_xa(typename V4<R>::t& acc, const R* Td, const R* xd,
                                           const R* b, int ldb, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        acc = mfma16<R>(xblk(Td, xd, r16, 4 * t + kq), b[(4 * t + kq) * ldb + r16], acc);
}
template <class R>
__device__ __forceinline__ void ld16(typename V4<R>::t& acc, const R* src, int ld, int lane) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = src[crow16<R>(lane, q) * ld + (lane & 15)];
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
// Tile storage is fp64 (MatB) or fp32 (MatF, the mixed-precision Newton factorisation).
__device__ __forceinline__ d2_t ld2(const double* p) { return *reinterpret_cast<const d2_t*>(p); }
__device__ __forceinline__ d2_t ld2(const float* p) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    return d2_t{(double)v.x, (double)v.y};
}

template <class R>
struct DiagSmemT {
    R T[64 * DP];
    int ok;  // fused path: the factorisation succeeded (broadcast to the storing waves)
    R xdg[64];
    R Tmp[16 * 17];
    R colb[16];
    R dg[64];
    R yv[16];
};
typedef DiagSmemT<double> DiagSmem;
typedef DiagSmemT<float> DiagSmem32;  // 18 KB

// Wave-level (lane = 0..63): factors S.T in place (L lower, inv(L) in the upper part + xdg,
// diagonal of L in dg); returns false on a non-positive pivot (wave-uniform). UNROLLED: pivot and
// inverse steps fully unrolled with DPP row broadcasts (fastest); the rolled form (select +
// __shfl) needs ~10 fewer VGPRs where a kernel is at its occupancy edge.
template <bool UNROLLED = true, class R = double>
__device__ bool diag_compute(DiagSmemT<R>& S, int lane) {
    typedef typename V4<R>::t acc_t;
    R* T = S.T;
    R* xdg = S.xdg;
    R* Tmp = S.Tmp;
    R* colb = S.colb;
    R* dg = S.dg;
    R* yv = S.yv;
#pragma unroll 1
    for (int kb = 0; kb < 4; ++kb) {
        const int o = kb * 16;
        // (a) factor the 16x16 diagonal block in registers: lane (g, c) = (lane >> 4, lane & 15)
        // holds rows 4g..4g+3 of column c. Per pivot j: v_readlane of the pivot, 1/sqrt by
        // v_rsq_f64 + two Newton steps, column j scaled by its owners (c == j) and published in
        // LDS (colb), row values L[i][j] broadcast inside each 16-lane row group by __shfl.
        const int c = lane & 15, g = lane >> 4;
        R a[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = T[(o + 4 * g + u) * DP + o + c];
        bool bad = false;
        if constexpr (!UNROLLED) {
#pragma unroll 1
            for (int j = 0; j < ((DIAG_SKIP & 1) ? 0 : 16); ++j) {
                const int ju = j & 3;
                const R aj = ju == 0 ? a[0] : (ju == 1 ? a[1] : (ju == 2 ? a[2] : a[3]));
                const R p = rdlane(aj, ((j >> 2) << 4) | j);
                bad |= !(p > R(0));
                const R y = rsqrt_r(p);
                if (lane == 0) {
                    yv[j] = y;
                    dg[o + j] = p * y;
                }
                if (c == j) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = 4 * g + u;
                        a[u] = (i > j) ? a[u] * y : ((i == j) ? p * y : a[u]);
                        colb[i] = a[u];
                    }
                }
                R lij[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) lij[u] = __shfl(a[u], (lane & 48) | j);
                const R lcj = colb[c];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = 4 * g + u;
                    if (c > j && c <= i) a[u] -= lij[u] * lcj;
                }
            }
        } else
        static_for<0, ((DIAG_SKIP & 1) ? 0 : 16)>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            int js = j;  // opaque copy: the lane masks of a step are formed in that step
            asm volatile("" : "+s"(js));
            const R p = rdlane(a[j & 3], ((j >> 2) << 4) | j);
            bad |= !(p > R(0));
            const R y = rsqrt_r(p);
            if (lane == 0) {
                yv[j] = y;
                dg[o + j] = p * y;
            }
            if (c == js) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = 4 * g + u;
                    a[u] = (i > js) ? a[u] * y : ((i == js) ? p * y : a[u]);
                    colb[i] = a[u];
                }
            }
            const R lcj = colb[c];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = 4 * g + u;
                const R lij = row_bcast<j>(a[u]);  // L[i][j]: lane j of this row group
                if (c > js && c <= i) a[u] -= lij * lcj;
            }
        });
        if (bad) return false;  // wave-uniform
        // inverse X of the 16x16 factor (L X = I) for all 16 columns at once, right-looking
        // substitution: lane (g, c) holds rows 4g..4g+3 of column c of X
        R sx[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) sx[u] = (4 * g + u == c) ? R(1) : R(0);
        if constexpr (!UNROLLED) {
#pragma unroll 1
            for (int r = 0; r < ((DIAG_SKIP & 2) ? 0 : 16); ++r) {
                const int ru = r & 3;
                const R cur =
                    (ru == 0 ? sx[0] : (ru == 1 ? sx[1] : (ru == 2 ? sx[2] : sx[3]))) * yv[r];
                const R xr = __shfl(cur, ((r >> 2) << 4) | c);
                if (g == (r >> 2)) {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (u == ru) sx[u] = cur;
                }
                R lir[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) lir[u] = __shfl(a[u], (lane & 48) | r);
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (4 * g + u > r) sx[u] -= lir[u] * xr;
            }
        } else
        static_for<0, ((DIAG_SKIP & 2) ? 0 : 16)>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            int rs = r;  // opaque copy (see the pivot loop)
            asm volatile("" : "+s"(rs));
            const R cur = sx[r & 3] * yv[r];
            const R xr = __shfl(cur, ((r >> 2) << 4) | c);  // X[r][c] (zero for c > r)
            if (g == (rs >> 2)) sx[r & 3] = cur;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const R lir = row_bcast<r>(a[u]);  // L[4g+u][r]
                if (4 * g + u > rs) sx[u] -= lir * xr;
            }
        });
        // L (lower incl. diagonal) back to T; X transposed into the upper part, diagonal to xdg
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = 4 * g + u;
            if (c <= i) T[(o + i) * DP + o + c] = a[u];
            if (i > c) T[(o + c) * DP + o + i] = sx[u];
            if (i == c) xdg[o + c] = sx[u];
        }
        if (kb == 3 || (DIAG_SKIP & 4)) continue;
        // (b) panel: T[ib][kb] = T[ib][kb] * inv(L_kb,kb)^T for the blocks below
        for (int ib = kb + 1; ib < 4; ++ib) {
            acc_t acc = {R(0), R(0), R(0), R(0)};
            mm16_nt_xb<R>(acc, &T[(16 * ib) * DP + o], DP, &T[o * DP + o], &xdg[o], lane);
            st16<R>(acc, &T[(16 * ib) * DP + o], DP, lane, R(1));
        }
        // (c) rank-16 trailing update of the lower blocks
        for (int ib = kb + 1; ib < 4; ++ib)
            for (int jb = kb + 1; jb <= ib; ++jb) {
                acc_t acc;
                ld16<R>(acc, &T[(16 * ib) * DP + 16 * jb], DP, lane);
                mm16_nt<true, R>(acc, &T[(16 * ib) * DP + o], DP, &T[(16 * jb) * DP + o], DP, lane);
                st16<R>(acc, &T[(16 * ib) * DP + 16 * jb], DP, lane, R(1));
            }
    }
    // off-diagonal blocks of the inverse, block row by block row
#pragma unroll 1
    for (int a = 1; a < ((DIAG_SKIP & 8) ? 0 : 4); ++a)
#pragma unroll 1
        for (int bb = 0; bb < a; ++bb) {
            acc_t acc = {R(0), R(0), R(0), R(0)};
            mm16_nn_xb<R>(acc, &T[(16 * a) * DP + 16 * bb], DP, &T[(16 * bb) * DP + 16 * bb],
                       &xdg[16 * bb], lane);
            for (int kk = bb + 1; kk < a; ++kk)  // X_kk,bb is stored transposed at T block (bb, kk)
                mm16_nt<false, R>(acc, &T[(16 * a) * DP + 16 * kk], DP, &T[(16 * bb) * DP + 16 * kk],
                               DP, lane);
            st16<R>(acc, Tmp, 17, lane, R(1));
            acc_t acc2 = {R(0), R(0), R(0), R(0)};
            mm16_nn_xa<R>(acc2, &T[(16 * a) * DP + 16 * a], &xdg[16 * a], Tmp, 17, lane);
            st16t<R>(acc2, &T[(16 * bb) * DP + 16 * a], DP, lane, R(-1));
        }
    return true;
}

// Stores of a factored tile by `nthr` threads (64: one wave; 256: the fused update's workgroup):
// L (zeros above the diagonal) to At, inv(L) row-major to D (16-byte stores), sum(log diag L)
// to *ldet_out (wave 0). SC1 (fp32 tiles only): L and inv(L) stored write-through (8-byte
// agent-scope stores) for a hand-off to other workgroups inside the launch (k_chol_panel_df32).
template <class TS, class R = double, bool SC1 = false>
__device__ void diag_store(DiagSmemT<R>& S, TS* At, int64_t ld, TS* D, double* ldet_out, int tid,
                           int nthr) {
    const R* T = S.T;
    const int p2 = 2 * (tid & 31);  // column pair
    for (int q = tid >> 5; q < ((DIAG_SKIP & 16) ? 0 : 64); q += nthr >> 5) {
        asm volatile("" ::: "memory");  // bounded batches of LDS reads (register pressure)
        const R l0 = (p2 <= q) ? T[q * DP + p2] : R(0);
        const R l1 = (p2 + 1 <= q) ? T[q * DP + p2 + 1] : R(0);
        const R x0 = (p2 < q) ? T[p2 * DP + q] : ((p2 == q) ? S.xdg[q] : R(0));
        const R x1 = (p2 + 1 < q) ? T[(p2 + 1) * DP + q] : ((p2 + 1 == q) ? S.xdg[q] : R(0));
        if constexpr (sizeof(TS) == 8) {
            *reinterpret_cast<d2_t*>(At + (int64_t)q * ld + p2) = d2_t{l0, l1};
            *reinterpret_cast<d2_t*>(D + q * 64 + p2) = d2_t{x0, x1};
        } else if constexpr (SC1) {
            const float2 lv{(float)l0, (float)l1}, xv{(float)x0, (float)x1};
            unsigned long long lu, xu;
            __builtin_memcpy(&lu, &lv, 8);
            __builtin_memcpy(&xu, &xv, 8);
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(At + (int64_t)q * ld + p2), lu,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(D + q * 64 + p2), xu,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            *reinterpret_cast<float2*>(At + (int64_t)q * ld + p2) = float2{(float)l0, (float)l1};
            *reinterpret_cast<float2*>(D + q * 64 + p2) = float2{(float)x0, (float)x1};
        }
    }
    if (tid < 64) {
        const double l = wave_sum_d(log((double)S.dg[tid]));
        if (tid == 0) *ldet_out = l;
    }
}

