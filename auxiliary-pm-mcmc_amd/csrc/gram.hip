// ARD / isotropic squared-exponential Gram builder (fp64), replacing gpdemo/kernels.pyx.
//
//   isotropic_squared_exponential_kernel  kernels.pyx:12-49   K_ij = s exp(-|x_i-x_j|^2 / (2 tau^2))
//   diagonal_squared_exponential_kernel   kernels.pyx:52-90   K_ij = s exp(-1/2 sum_k ((x_ik-x_jk)/tau_k)^2)
//   K_ii = s + eps; both triangles written (the reference fills K[i,j] and K[j,i]).
// One workgroup per lower tile (i >= j) of 64x64; X row blocks are staged through LDS in chunks of
// 32 features, multiplied by 1/tau_k on the way in; the tile and its transpose are written with
// 32-byte contiguous runs per thread (coalesced 512-byte rows). HBM-bound: 8 B per K element.
#include "apm_internal.h"

#define GK 32  // features per LDS chunk

__global__ __launch_bounds__(256) void k_gram(MatB K, const double* __restrict__ X, int64_t ldx,
                                              int n, int d, const double* __restrict__ theta,
                                              int64_t tstride, int kind, double eps, Live live) {
    const int b = blockIdx.y;
    if (live.active[b] == 0 || live.status[b] != 0) return;
    // lower-triangular tile index -> (ti, tj), ti >= tj
    const int t = blockIdx.x;
    int ti = (int)floor((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > t) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
    const int tj = t - ti * (ti + 1) / 2;

    __shared__ double xi[64][GK + 1];
    __shared__ double xj[64][GK + 1];
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
            const int r = e / GK, k = e % GK;
            const int gi = ti * 64 + r, gj = tj * 64 + r;
            xi[r][k] = (k < kc && gi < n) ? X[(int64_t)gi * ldx + k0 + k] : 0.0;
            xj[r][k] = (k < kc && gj < n) ? X[(int64_t)gj * ldx + k0 + k] : 0.0;
        }
        __syncthreads();
        for (int k = 0; k < kc; ++k) {
            const double it = itau[k];
            double a[4], c[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) a[p] = xi[tr * 4 + p][k];
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] = xj[tc * 4 + q][k];
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const double df = (a[p] - c[q]) * it;
                    acc[p][q] = fma(df, df, acc[p][q]);
                }
        }
    }

    double v[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int gi = ti * 64 + tr * 4 + p, gj = tj * 64 + tc * 4 + q;
            double val;
            if (gi < n && gj < n)
                val = (gi == gj) ? sigma + eps : sigma * exp(-0.5 * acc[p][q]);
            else
                val = (gi == gj) ? 1.0 : 0.0;
            v[p][q] = val;
        }
    double* Kb = K.base + b * K.cstride;
    // tile (ti, tj): rows ti*64 + tr*4 + p, cols tj*64 + tc*4 .. +3 (32 contiguous bytes)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        double* dst = Kb + (int64_t)(ti * 64 + tr * 4 + p) * K.ld + tj * 64 + tc * 4;
        reinterpret_cast<d2_t*>(dst)[0] = d2_t{v[p][0], v[p][1]};
        reinterpret_cast<d2_t*>(dst)[1] = d2_t{v[p][2], v[p][3]};
    }
    if (ti != tj) {
        // transpose (tj, ti): rows tj*64 + tc*4 + q, cols ti*64 + tr*4 .. +3
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double* dst = Kb + (int64_t)(tj * 64 + tc * 4 + q) * K.ld + ti * 64 + tr * 4;
            reinterpret_cast<d2_t*>(dst)[0] = d2_t{v[0][q], v[1][q]};
            reinterpret_cast<d2_t*>(dst)[1] = d2_t{v[2][q], v[3][q]};
        }
    }
}

void launch_gram(MatB K, const double* X, int64_t ldx, int n, int d, const double* theta,
                 int64_t tstride, int kind, double eps, int np, Live live, int nchains,
                 hipStream_t s) {
    const int nb = np / 64;
    hipLaunchKernelGGL(k_gram, dim3(nb * (nb + 1) / 2, nchains), dim3(256), 0, s, K, X, ldx, n,
                       d, theta, tstride, kind, eps, live);
}
