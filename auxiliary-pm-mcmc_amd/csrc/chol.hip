// Blocked right-looking Cholesky (fp64, f64 MFMA) and the Newton back-substitution.
//
// Replaces the LAPACK potrf / potrs calls of the reference hot path:
//   la.cholesky(K)  gpdemo/estimators.py:206,321    la.cholesky(B)  latent_posterior_approximations.py:92
//   la.cholesky(C)  gpdemo/estimators.py:209        la.cho_solve(L, .)  latent_posterior_approximations.py:94
// The work matrix is tiled TB x TB (TB = 64). One workgroup (4 waves) owns one output tile; each
// wave owns a 32x32 quadrant = 2x2 v_mfma_f64_16x16x4_f64 accumulators.
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

__device__ __forceinline__ bool chain_live(const Live& lv, int b) {
    return lv.active[b] != 0 && lv.status[b] == 0;
}

// ------------------------------------------------------------------------------- diagonal tile
// Unblocked right-looking Cholesky of the 64x64 tile in LDS (256 threads), then the inverse of
// the lower factor by one wave with the column held in registers (fully unrolled substitution).
__global__ __launch_bounds__(256) void k_chol_diag(MatB A, int k, double* Dinv, int64_t dstride,
                                                   double* ldet, int64_t lstride, Live live,
                                                   int fail_code) {
    const int b = blockIdx.x;
    if (!chain_live(live, b)) return;
    __shared__ double T[64][65];
    const int tid = threadIdx.x;
    double* At = A.base + b * A.cstride + (int64_t)(k * 64) * A.ld + k * 64;
    for (int e = tid; e < 4096; e += 256) T[e >> 6][e & 63] = At[(int64_t)(e >> 6) * A.ld + (e & 63)];
    __syncthreads();
    double lsum = 0.0;
    for (int j = 0; j < 64; ++j) {
        const double p = T[j][j];
        if (!(p > 0.0)) {  // non-positive or NaN pivot: uniform across the block
            if (tid == 0) live.status[b] = fail_code;
            return;
        }
        const double d = sqrt(p);
        const double invd = 1.0 / d;
        lsum += log(d);
        if (tid > j && tid < 64) T[tid][j] *= invd;
        __syncthreads();
        const int m = 63 - j;
        for (int e = tid; e < m * m; e += 256) {
            const int r = j + 1 + e / m, c = j + 1 + e % m;
            if (c <= r) T[r][c] -= T[r][j] * T[c][j];
        }
        if (tid == 0) T[j][j] = d;
        __syncthreads();
    }
    // write L_kk (lower; the strict upper part of the diagonal tile is zeroed)
    for (int e = tid; e < 4096; e += 256) {
        const int r = e >> 6, c = e & 63;
        At[(int64_t)r * A.ld + c] = (c <= r) ? T[r][c] : 0.0;
    }
    if (tid == 0) ldet[b * lstride + k] = lsum;
    // inverse: lane c computes column c of inv(L) by forward substitution
    if (tid < 64) {
        const int c = tid;
        double x[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) {
            double s = (r == c) ? 1.0 : 0.0;
#pragma unroll
            for (int m = 0; m < r; ++m) s -= T[r][m] * x[m];
            x[r] = (r >= c) ? s / T[r][r] : 0.0;
        }
        double* D = Dinv + b * dstride + (int64_t)k * 4096;
#pragma unroll
        for (int r = 0; r < 64; ++r) D[r * 64 + c] = x[r];
    }
}

void launch_chol_diag(MatB A, int k, double* Dinv, int64_t dstride, double* ldet, int64_t lstride,
                      Live live, int fail_code, int nchains, hipStream_t s) {
    hipLaunchKernelGGL(k_chol_diag, dim3(nchains), dim3(256), 0, s, A, k, Dinv, dstride, ldet,
                       lstride, live, fail_code);
}

// ------------------------------------------------------------------------------- panel TRSM
__global__ __launch_bounds__(256) void k_chol_panel(MatB A, int k, int i0, const double* Dinv,
                                                    int64_t dstride, Live live) {
    const int b = blockIdx.y;
    if (!chain_live(live, b)) return;
    const int i = i0 + blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
    double* At = A.base + b * A.cstride + (int64_t)(i * 64) * A.ld + k * 64;
    const double* D = Dinv + b * dstride + (int64_t)k * 4096;
    d4_t acc[2][2];
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = d4_t{0.0, 0.0, 0.0, 0.0};
    tile_nt_f64<false>(acc, At, A.ld, D, 64, wr, wc, lane);  // X = A_ik * inv(L_kk)^T
    __syncthreads();  // every wave has read A_ik before it is overwritten
    tile_acc_store(acc, At, A.ld, wr, wc, lane);
}

void launch_chol_panel(MatB A, int k, int i0, int R, const double* Dinv, int64_t dstride,
                       Live live, int nchains, hipStream_t s) {
    if (R <= i0) return;
    hipLaunchKernelGGL(k_chol_panel, dim3(R - i0, nchains), dim3(256), 0, s, A, k, i0, Dinv,
                       dstride, live);
}

// ------------------------------------------------------------------------------- trailing update
// Tiles (i, j) with i in [i0, R), k < j <= min(i, Cb-1), enumerated as a triangular part (rows
// i < Cb, i-k tiles each) followed by a rectangular part (rows i >= Cb, Cb-1-k tiles each).
__device__ __forceinline__ void decode_update_tile(long t, int k, int i0, int R, int Cb, int& i,
                                                   int& j) {
    const int it_end = min(R, Cb);
    const int a0 = i0 - k;  // tiles in the first triangular row
    const int ntri_rows = max(0, it_end - i0);
    const long ntri = (long)ntri_rows * a0 + (long)ntri_rows * (ntri_rows - 1) / 2;
    if (t < ntri) {
        // largest p with p*a0 + p(p-1)/2 <= t
        const double aa = a0 - 0.5;
        long p = (long)floor(-aa + sqrt(aa * aa + 2.0 * (double)t));
        while (p > 0 && p * a0 + p * (p - 1) / 2 > t) --p;
        while ((p + 1) * a0 + (p + 1) * p / 2 <= t) ++p;
        i = i0 + (int)p;
        j = k + 1 + (int)(t - (p * a0 + p * (p - 1) / 2));
    } else {
        const long r = t - ntri;
        const int w = Cb - 1 - k;
        i = max(i0, Cb) + (int)(r / w);
        j = k + 1 + (int)(r % w);
    }
}

static long update_tile_count(int k, int i0, int R, int Cb) {
    const int it_end = R < Cb ? R : Cb;
    const int ntri_rows = it_end - i0 > 0 ? it_end - i0 : 0;
    const long a0 = i0 - k;
    long n = ntri_rows * a0 + (long)ntri_rows * (ntri_rows - 1) / 2;
    const int rect_rows = R - (i0 > Cb ? i0 : Cb);
    if (rect_rows > 0) n += (long)rect_rows * (Cb - 1 - k);
    return n;
}

__global__ __launch_bounds__(256) void k_chol_update(MatB A, int k, int i0, int R, int Cb,
                                                     Live live) {
    const int b = blockIdx.y;
    if (!chain_live(live, b)) return;
    int i, j;
    decode_update_tile(blockIdx.x, k, i0, R, Cb, i, j);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
    double* Ab = A.base + b * A.cstride;
    double* Aij = Ab + (int64_t)(i * 64) * A.ld + j * 64;
    const double* Aik = Ab + (int64_t)(i * 64) * A.ld + k * 64;
    const double* Ajk = Ab + (int64_t)(j * 64) * A.ld + k * 64;
    d4_t acc[2][2];
    tile_acc_load(acc, Aij, A.ld, wr, wc, lane);
    tile_nt_f64<true>(acc, Aik, A.ld, Ajk, A.ld, wr, wc, lane);
    tile_acc_store(acc, Aij, A.ld, wr, wc, lane);
}

void launch_chol_update(MatB A, int k, int i0, int R, int Cb, Live live, int nchains,
                        hipStream_t s) {
    if (i0 < k + 1) i0 = k + 1;
    const long n = update_tile_count(k, i0, R, Cb);
    if (n <= 0) return;
    hipLaunchKernelGGL(k_chol_update, dim3((unsigned)n, nchains), dim3(256), 0, s, A, k, i0, R,
                       Cb, live);
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
    d4_t acc[2][2];
    tile_acc_load(acc, C, 64, wr, wc, lane);
    tile_nt_f64<false>(acc, A, 64, B, 64, wr, wc, lane);
    tile_acc_store(acc, C, 64, wr, wc, lane);
}

void launch_tile_nt_test(const double* A, const double* B, double* C, hipStream_t s) {
    hipLaunchKernelGGL(k_tile_nt_test, dim3(1), dim3(256), 0, s, A, B, C);
}
