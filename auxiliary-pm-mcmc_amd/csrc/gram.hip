// ARD / isotropic squared-exponential Gram builder (fp64), replacing gpdemo/kernels.pyx.
//
//   isotropic_squared_exponential_kernel  kernels.pyx:12-49   K_ij = s exp(-|x_i-x_j|^2 / (2 tau^2))
//   diagonal_squared_exponential_kernel   kernels.pyx:52-90   K_ij = s exp(-1/2 sum_k ((x_ik-x_jk)/tau_k)^2)
//   K_ii = s + eps. both != 0: both triangles written (the reference fills K[i,j] and K[j,i];
//   the stand-alone apm_gram); both == 0: lower tiles only (the theta-call: every consumer on the
//   device path reads K's lower tiles, so the upper half is never written - half the bytes).
// X row blocks are staged through LDS in chunks of 32 features, multiplied by 1/tau_k on the way
// in (2 fp64 VALU ops per pair and feature); the tile and its transpose are written with 32-byte
// contiguous runs per lane (two coalesced 256-byte runs per row and 8 lanes).
// Roofline: 8 B written per K element (HBM) vs ~(2D + ~40 for exp) fp64 VALU ops per lower pair.
#include "apm_internal.h"

#ifndef GRAM_ABL  // ablations (tools/gram_bench.cpp): 1 no exp, 2 no stores, 3 no distance loop
#define GRAM_ABL 0
#endif
#define GK 32       // features per LDS chunk
#define GP (128 + 2)  // LDS row pitch in doubles (16-byte aligned; the transposing staging stores
                      // of consecutive features land 4 banks apart instead of on one bank)
// lane (g = lane >> 3 or lane & 7) -> its 8 rows (columns) of the wave's 64x64 tile:
// {4g .. 4g+3, 32+4g .. 32+4g+3}, so that 8 lanes cover two contiguous 256-byte runs of a row
#define R8(g, p) (((p) >> 2) * 32 + 4 * (g) + ((p) & 3))

// One workgroup of 4 waves per lower 128x128 super-tile (si >= sj); wave w computes 64x64 tile
// (2si + w/2, 2sj + w%2) - the upper tile of a diagonal super-tile and tiles beyond the padded
// size are skipped - with an 8x8 block of pairs per lane: per feature 16 fp64 LDS values feed
// 64 (subtract, fma) pairs, so the LDS reads stay at half the VALU issue (a 4x4 block per lane
// tied them). Features are pre-scaled by 1/tau_k while staged; the sum runs over k in order
// (the same arithmetic as the reference's loop, kernels.pyx:80-88, up to the pre-scaling).
// K2 (the concurrent chol(K)'s working copy, capi.cpp chol_k_begin) receives the tiles of tile
// columns < k2cols only: the first outer panel's trailing update reads the rest from K itself.
__global__ __launch_bounds__(256, 2) void k_gram(MatB K, const double* __restrict__ X, int64_t ldx,
                                                 int n, int d, const double* __restrict__ theta,
                                                 int64_t tstride, int kind, double eps, Live live,
                                                 int both, MatB K2, int k2cols, int nb) {
    const int b = blockIdx.y;
    if (live.active[b] == 0 || live.status[b] != 0) return;
    // lower-triangular super-tile index -> (si, sj), si >= sj
    const int t = blockIdx.x;
    int si = (int)floor((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (si * (si + 1) / 2 > t) --si;
    while ((si + 1) * (si + 2) / 2 <= t) ++si;
    const int sj = t - si * (si + 1) / 2;

    __shared__ __attribute__((aligned(16))) double xi[GK][GP];
    __shared__ __attribute__((aligned(16))) double xj[GK][GP];
    __shared__ double itau[GK];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int tr = lane >> 3, tc = lane & 7;
    const int ti = 2 * si + (wv >> 1), tj = 2 * sj + (wv & 1);
    const bool mine = ti < nb && tj <= ti;
    const int ro = 64 * (wv >> 1), co = 64 * (wv & 1);
    const double* th = theta + b * tstride;
    const double sigma = exp(th[0]);

    double acc[8][8];
#pragma unroll
    for (int p = 0; p < 8; ++p)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[p][q] = 0.0;

    for (int k0 = 0; k0 < d; k0 += GK) {
        const int kc = min(GK, d - k0);
        __syncthreads();
        if (tid < kc) itau[tid] = exp(-th[kind == 0 ? 1 : 1 + k0 + tid]);
        __syncthreads();
        for (int e = tid; e < 128 * GK; e += 256) {
            const int r = e / GK, k = e % GK;  // consecutive lanes: consecutive features of a row
            const int gi = si * 128 + r, gj = sj * 128 + r;
            const double sc = (k < kc) ? itau[k] : 0.0;
            xi[k][r] = (k < kc && gi < n) ? X[(int64_t)gi * ldx + k0 + k] * sc : 0.0;
            xj[k][r] = (k < kc && gj < n) ? X[(int64_t)gj * ldx + k0 + k] * sc : 0.0;
        }
        __syncthreads();
        if (mine && GRAM_ABL != 3) {
            for (int k = 0; k < kc; ++k) {
                double a[8], c[8];
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const d2_t va = *reinterpret_cast<const d2_t*>(&xi[k][ro + R8(tr, 2 * h)]);
                    const d2_t vc = *reinterpret_cast<const d2_t*>(&xj[k][co + R8(tc, 2 * h)]);
                    a[2 * h] = va.x;
                    a[2 * h + 1] = va.y;
                    c[2 * h] = vc.x;
                    c[2 * h + 1] = vc.y;
                }
                // a row's 8 differences first, then their 8 fmas: no fma waits on the subtract
                // issued right before it (one shared temporary serialised every pair on the fp64
                // dependency latency)
#pragma unroll
                for (int p = 0; p < 8; ++p) {
                    double df[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) df[q] = a[p] - c[q];  // pre-scaled by 1/tau_k
#pragma unroll
                    for (int q = 0; q < 8; ++q) acc[p][q] = fma(df[q], df[q], acc[p][q]);
                }
            }
        }
    }
    if (!mine) return;  // (after the last barrier)

#pragma unroll
    for (int p = 0; p < 8; ++p)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int gi = ti * 64 + R8(tr, p), gj = tj * 64 + R8(tc, q);
            double val;
            if (gi < n && gj < n)
                val = (gi == gj) ? sigma + eps
                                 : (GRAM_ABL == 1 ? sigma * acc[p][q] : sigma * exp(-0.5 * acc[p][q]));
            else
                val = (gi == gj) ? 1.0 : 0.0;
            acc[p][q] = val;
        }
    auto store = [&](double* base, int64_t ld) {
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            double* dst = base + (int64_t)(ti * 64 + R8(tr, p)) * ld + tj * 64 + 4 * tc;
            *reinterpret_cast<d2_t*>(dst) = d2_t{acc[p][0], acc[p][1]};
            *reinterpret_cast<d2_t*>(dst + 2) = d2_t{acc[p][2], acc[p][3]};
            *reinterpret_cast<d2_t*>(dst + 32) = d2_t{acc[p][4], acc[p][5]};
            *reinterpret_cast<d2_t*>(dst + 34) = d2_t{acc[p][6], acc[p][7]};
        }
    };
    double* Kb = K.base + b * K.cstride;
    if (GRAM_ABL == 2 && acc[0][0] != -1.0) return;
    store(Kb, K.ld);
    if (K2.base && tj < k2cols) store(K2.base + b * K2.cstride, K2.ld);
    if (both && ti != tj) {  // transposed tile (tj, ti)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            double* dst = Kb + (int64_t)(tj * 64 + R8(tc, q)) * K.ld + ti * 64 + 4 * tr;
            *reinterpret_cast<d2_t*>(dst) = d2_t{acc[0][q], acc[1][q]};
            *reinterpret_cast<d2_t*>(dst + 2) = d2_t{acc[2][q], acc[3][q]};
            *reinterpret_cast<d2_t*>(dst + 32) = d2_t{acc[4][q], acc[5][q]};
            *reinterpret_cast<d2_t*>(dst + 34) = d2_t{acc[6][q], acc[7][q]};
        }
    }
}

void launch_gram(MatB K, const double* X, int64_t ldx, int n, int d, const double* theta,
                 int64_t tstride, int kind, double eps, int np, Live live, int nchains,
                 hipStream_t s, bool both, MatB K2, int k2cols) {
    const int nb = np / 64, ns = (nb + 1) / 2;
    APM_LAUNCH(k_gram, dim3(ns * (ns + 1) / 2, nchains), dim3(256), 0, s, K, X, ldx, n, d,
                       theta, tstride, kind, eps, live, (int)both, K2, k2cols, nb);
}
