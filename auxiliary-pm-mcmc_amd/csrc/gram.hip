// ARD / isotropic squared-exponential Gram builder (fp64), replacing gpdemo/kernels.pyx.
//
//   isotropic_squared_exponential_kernel  kernels.pyx:12-49   K_ij = s exp(-|x_i-x_j|^2 / (2 tau^2))
//   diagonal_squared_exponential_kernel   kernels.pyx:52-90   K_ij = s exp(-1/2 sum_k ((x_ik-x_jk)/tau_k)^2)
//   K_ii = s + eps. both != 0: both triangles written (the reference fills K[i,j] and K[j,i];
//   the stand-alone apm_gram); both == 0: lower tiles only (the theta-call: every consumer on the
//   device path reads K's lower tiles, so the upper half is never written - half the bytes).
// One workgroup per lower tile (i >= j) of 64x64; X row blocks are staged through LDS in chunks of
// 32 features, multiplied by 1/tau_k on the way in (2 fp64 VALU ops per pair and feature); the tile
// and its transpose are written with 32-byte contiguous runs per thread (coalesced 512-byte rows).
// Roofline: 8 B written per K element (HBM) vs ~(2D + ~40 for exp) fp64 VALU ops per lower pair.
#include "apm_internal.h"

#define GK 32  // features per LDS chunk
// thread-local index p (0..3) of thread group g -> row/column inside the 64-tile:
// {2g, 2g+1, 32+2g, 33+2g}, so that each 16-lane group reads/writes contiguous 256-byte runs
#define RO(g, p) (((p) >> 1) * 32 + 2 * (g) + ((p) & 1))

__global__ __launch_bounds__(256) void k_gram(MatB K, const double* __restrict__ X, int64_t ldx,
                                              int n, int d, const double* __restrict__ theta,
                                              int64_t tstride, int kind, double eps, Live live,
                                              int both, MatB K2) {
    const int b = blockIdx.y;
    if (live.active[b] == 0 || live.status[b] != 0) return;
    // lower-triangular tile index -> (ti, tj), ti >= tj
    const int t = blockIdx.x;
    int ti = (int)floor((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > t) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
    const int tj = t - ti * (ti + 1) / 2;

    // feature-major staging ([k][row]) so that each thread reads its 4 rows / 4 columns with two
    // 16-byte LDS reads (contiguous across the 16 lanes of a row group: conflict-free)
    __shared__ __attribute__((aligned(16))) double xi[GK][64];
    __shared__ __attribute__((aligned(16))) double xj[GK][64];
    __shared__ double itau[GK];
    const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
    const double* th = theta + b * tstride;
    const double sigma = exp(th[0]);

    double acc[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;

    for (int k0 = 0; k0 < d; k0 += GK) {
        const int kc = min(GK, d - k0);
        __syncthreads();
        if (tid < kc) itau[tid] = exp(-th[kind == 0 ? 1 : 1 + k0 + tid]);
        __syncthreads();
        for (int e = tid; e < 64 * GK; e += 256) {
            const int r = e / GK, k = e % GK;  // consecutive lanes: consecutive features of a row
            const int gi = ti * 64 + r, gj = tj * 64 + r;
            const double sc = (k < kc) ? itau[k] : 0.0;
            xi[k][r] = (k < kc && gi < n) ? X[(int64_t)gi * ldx + k0 + k] * sc : 0.0;
            xj[k][r] = (k < kc && gj < n) ? X[(int64_t)gj * ldx + k0 + k] * sc : 0.0;
        }
        __syncthreads();
        for (int k = 0; k < kc; ++k) {
            const d2_t a01 = *reinterpret_cast<const d2_t*>(&xi[k][2 * tr]);
            const d2_t a23 = *reinterpret_cast<const d2_t*>(&xi[k][32 + 2 * tr]);
            const d2_t c01 = *reinterpret_cast<const d2_t*>(&xj[k][2 * tc]);
            const d2_t c23 = *reinterpret_cast<const d2_t*>(&xj[k][32 + 2 * tc]);
            const double a[4] = {a01.x, a01.y, a23.x, a23.y};
            const double c[4] = {c01.x, c01.y, c23.x, c23.y};
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const double df = a[p] - c[q];  // features pre-scaled by 1/tau_k
                    acc[p][q] = fma(df, df, acc[p][q]);
                }
        }
    }

    double v[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int gi = ti * 64 + RO(tr, p), gj = tj * 64 + RO(tc, q);
            double val;
            if (gi < n && gj < n)
                val = (gi == gj) ? sigma + eps : sigma * exp(-0.5 * acc[p][q]);
            else
                val = (gi == gj) ? 1.0 : 0.0;
            v[p][q] = val;
        }
    double* Kb = K.base + b * K.cstride;
    // tile (ti, tj): thread row p -> RO(tr, p); columns {2tc, 2tc+1} and {32+2tc, 33+2tc}
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        double* dst = Kb + (int64_t)(ti * 64 + RO(tr, p)) * K.ld + tj * 64;
        *reinterpret_cast<d2_t*>(dst + 2 * tc) = d2_t{v[p][0], v[p][1]};
        *reinterpret_cast<d2_t*>(dst + 32 + 2 * tc) = d2_t{v[p][2], v[p][3]};
    }
    if (K2.base) {  // second copy of the lower tiles (the concurrent chol(K)'s working copy)
        double* K2b = K2.base + b * K2.cstride;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            double* dst = K2b + (int64_t)(ti * 64 + RO(tr, p)) * K2.ld + tj * 64;
            *reinterpret_cast<d2_t*>(dst + 2 * tc) = d2_t{v[p][0], v[p][1]};
            *reinterpret_cast<d2_t*>(dst + 32 + 2 * tc) = d2_t{v[p][2], v[p][3]};
        }
    }
    if (both && ti != tj) {  // transposed tile (tj, ti)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double* dst = Kb + (int64_t)(tj * 64 + RO(tc, q)) * K.ld + ti * 64;
            *reinterpret_cast<d2_t*>(dst + 2 * tr) = d2_t{v[0][q], v[1][q]};
            *reinterpret_cast<d2_t*>(dst + 32 + 2 * tr) = d2_t{v[2][q], v[3][q]};
        }
    }
}

void launch_gram(MatB K, const double* X, int64_t ldx, int n, int d, const double* theta,
                 int64_t tstride, int kind, double eps, int np, Live live, int nchains,
                 hipStream_t s, bool both, MatB K2) {
    const int nb = np / 64;
    hipLaunchKernelGGL(k_gram, dim3(nb * (nb + 1) / 2, nchains), dim3(256), 0, s, K, X, ldx, n,
                       d, theta, tstride, kind, eps, live, (int)both, K2);
}
