// Posterior-covariance factor of the IS estimator through chol(K).
//
// The reference forms C = K - (W^1/2 K)^T B^-1 (W^1/2 K) (latent_posterior_approximations.py:111-112)
// and factors it (estimators.py:209): TRSM + SYRK + potrf = 7N^3/3 flops. With K = L_K L_K^T,
//   C = L_K M^-1 L_K^T,   M = I + L_K^T W L_K   (push-through identity, W of the last iteration),
// and if M = U U^T with U UPPER triangular (the "UL" Cholesky), then C = (L_K U^-T)(L_K U^-T)^T
// where L_K U^-T is lower triangular with a positive diagonal: it IS chol(C). With J the index
// reversal, J M J = Y2 Y2^T + I for the lower-triangular Y2 = J Z^T J (Z = W^1/2 L_K), its ordinary
// Cholesky L' gives U = J L' J, and factoring [[J M J],[L_K J]] yields (L_K J) L'^-T = chol(C) J.
// Cost: chol(K) + SYRK of a triangle + chol(M) + triangular TRSM = 4N^3/3. Also
//   g = C_chol^-1 f_post = U^T L_K^-1 f_post = J L'^T J h,  h = L_K^-1 f_post,  log|B| = log|M|.
#include "apm_internal.h"

__device__ __forceinline__ bool live_pc(const Live& lv, int b) {
    return lv.active[b] != 0 && lv.status[b] == 0;
}

// rows [row0, row0+64) of A over columns [0, ncols): row row0 = vec, the others 0
__global__ __launch_bounds__(256) void k_set_rhs(MatB A, int64_t row0, int ncols,
                                                 const double* __restrict__ vec, int64_t vstride,
                                                 Live live) {
    const int b = blockIdx.y;
    if (!live_pc(live, b)) return;
    double* Ab = A.base + b * A.cstride;
    const int c0 = blockIdx.x * 64;
    for (int e = threadIdx.x; e < 4096; e += 256) {
        const int rr = e >> 6, c = c0 + (e & 63);
        if (c < ncols) Ab[(row0 + rr) * A.ld + c] = (rr == 0) ? vec[b * vstride + c] : 0.0;
    }
}

void launch_set_rhs(MatB A, int64_t row0, int ncols, const double* vec, int64_t vstride,
                    Live live, int nchains, hipStream_t s) {
    APM_LAUNCH(k_set_rhs, dim3((ncols + 63) / 64, nchains), dim3(256), 0, s, A, row0, ncols,
                       vec, vstride, live);
}

// copy one row of A (row `row`, columns [0, n)) of every chain into a vector
__global__ __launch_bounds__(256) void k_get_row(MatB A, int64_t row, int n, double* out,
                                                 int64_t ostride, Live live) {
    const int b = blockIdx.y;
    if (!live_pc(live, b)) return;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c < n) out[b * ostride + c] = A.base[b * A.cstride + row * A.ld + c];
}

void launch_get_row(MatB A, int64_t row, int n, double* out, int64_t ostride, Live live,
                    int nchains, hipStream_t s) {
    APM_LAUNCH(k_get_row, dim3((n + 255) / 256, nchains), dim3(256), 0, s, A, row, n, out,
                       ostride, live);
}

// Y2[a][k'] = W^1/2[np-1-k'] * L[np-1-k'][np-1-a] for k' <= a, 0 above (all np x np of dst from
// column dcol0): lower tile (ta, tk') of dst is the reversed transpose of the source tile
// (nb-1-tk', nb-1-ta), staged through LDS. In the same pass L is overwritten in place by
// Y = L J (L's lower triangle only, the rest read as zero). Workgroup (sr, c1), c1 <= c2 = nb-1-c1,
// holds P = L(sr, c1) and Q = L(sr, c2), writes their Y2 tiles into dst and the column-reversed
// tiles Y(sr, c2) = rev(P), Y(sr, c1) = rev(Q) back into L; every load is consumed into LDS ahead
// of a barrier before any thread writes L. One read of L's lower triangle in all.
__device__ __forceinline__ void load_lower_tile(const double* Lr, int64_t ld, int sr, int sc,
                                                d2_t v[8]) {
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const int e = threadIdx.x + 256 * h, r = e >> 5, c = 2 * (e & 31);
        d2_t x = d2_t{0.0, 0.0};
        if (sc <= sr) x = *reinterpret_cast<const d2_t*>(Lr + (int64_t)r * ld + sc * 64 + c);
        v[h] = d2_t{(sr > sc || c <= r) ? x.x : 0.0, (sr > sc || c + 1 <= r) ? x.y : 0.0};
    }
}

// Y2 tile of source tile (sr, sc) (as k_form_y2); T must be free on entry
__device__ __forceinline__ void y2_tile(double (*T)[65], const d2_t v[8], int sr, int sc,
                                        double* dbase, int64_t ld, int64_t dcol0,
                                        const double* w, int nb, int zero_all) {
    const int ta = nb - 1 - sc, tk = nb - 1 - sr, np = nb * 64;
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const int e = threadIdx.x + 256 * h, r = e >> 5, c = 2 * (e & 31);
        T[r][c] = v[h].x;
        T[r][c + 1] = v[h].y;
    }
    __syncthreads();
    double* D = dbase + (int64_t)(ta * 64) * ld + dcol0 + tk * 64;
    if (tk > ta) {  // upper tile of Y2: zero where the SYRK reads it
        if (!zero_all && tk != ta + 1) return;
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            const int e = threadIdx.x + 256 * h;
            *reinterpret_cast<d2_t*>(D + (int64_t)(e >> 5) * ld + 2 * (e & 31)) = d2_t{0.0, 0.0};
        }
        return;
    }
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const int e = threadIdx.x + 256 * h;
        const int al = e >> 5, kl = 2 * (e & 31);
        const int kg = tk * 64 + kl;
        *reinterpret_cast<d2_t*>(D + (int64_t)al * ld + kl) =
            d2_t{w[np - 1 - kg] * T[63 - kl][63 - al], w[np - 2 - kg] * T[62 - kl][63 - al]};
    }
}

__global__ __launch_bounds__(256) void k_form_y2_rev(MatB L, MatB dst, int64_t dcol0,
                                                     const double* __restrict__ Ws,
                                                     int64_t vstride, int nb, Live live,
                                                     int zero_all) {
    const int b = blockIdx.y;
    if (!live_pc(live, b)) return;
    const int half = (nb + 1) / 2;
    const int sr = blockIdx.x / half, c1 = blockIdx.x % half, c2 = nb - 1 - c1;
    double* Lr = L.base + b * L.cstride + (int64_t)(sr * 64) * L.ld;
    double* dbase = dst.base + b * dst.cstride;
    const double* w = Ws + b * vstride;
    __shared__ double T[64][65];
    d2_t p[8], q[8];
    load_lower_tile(Lr, L.ld, sr, c1, p);
    if (c2 != c1) load_lower_tile(Lr, L.ld, sr, c2, q);
    y2_tile(T, p, sr, c1, dbase, dst.ld, dcol0, w, nb, zero_all);
    __syncthreads();
    if (c2 != c1) {
        y2_tile(T, q, sr, c2, dbase, dst.ld, dcol0, w, nb, zero_all);
    } else {
#pragma unroll
        for (int h = 0; h < 8; ++h) q[h] = p[h];
    }
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const int e = threadIdx.x + 256 * h, r = e >> 5, k = e & 31;
        double* row = Lr + (int64_t)r * L.ld + 2 * (31 - k);
        *reinterpret_cast<d2_t*>(row + c1 * 64) = d2_t{q[h].y, q[h].x};
        *reinterpret_cast<d2_t*>(row + c2 * 64) = d2_t{p[h].y, p[h].x};
    }
}

void launch_form_y2_rev(MatB L, MatB dst, int64_t dcol0, const double* Ws, int64_t vstride,
                        int np, Live live, int nchains, hipStream_t s, bool zero_all) {
    const int nb = np / 64;
    APM_LAUNCH(k_form_y2_rev, dim3(nb * ((nb + 1) / 2), nchains), dim3(256), 0, s, L, dst,
                       dcol0, Ws, vstride, nb, live, (int)zero_all);
}

// lower tiles of M <- I
__global__ __launch_bounds__(256) void k_identity_lower(MatB M, Live live) {
    const int b = blockIdx.y;
    if (!live_pc(live, b)) return;
    int ti = (int)floor((sqrt(8.0 * blockIdx.x + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > (int)blockIdx.x) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= (int)blockIdx.x) ++ti;
    const int tj = blockIdx.x - ti * (ti + 1) / 2;
    double* D = M.base + b * M.cstride + (int64_t)(ti * 64) * M.ld + tj * 64;
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const int e = threadIdx.x + 256 * h, r = e >> 5, c = 2 * (e & 31);
        *reinterpret_cast<d2_t*>(D + (int64_t)r * M.ld + c) =
            d2_t{(ti == tj && r == c) ? 1.0 : 0.0, (ti == tj && r == c + 1) ? 1.0 : 0.0};
    }
}

void launch_identity_lower(MatB M, int np, Live live, int nchains, hipStream_t s) {
    const int nb = np / 64;
    APM_LAUNCH(k_identity_lower, dim3(nb * (nb + 1) / 2, nchains), dim3(256), 0, s, M, live);
}

// g = J L'^T J h: g[np-1-c] = sum_{r >= c} L'[r][c] h[np-1-r] (REV), or out[c] = sum_{r >= c}
// L[r][c] x[r] (h = L_K^T a), from L's lower tiles in parallel (a workgroup per column strip
// walks 64-KB-strided rows and leaves most CUs idle): workgroup (ti, tj), ti >= tj, loads its tile into registers
// (thread: rows 4rg..+3, columns 4cg..+3, 16-byte loads) and writes the column partials
// sum_r L[r][c] x(r) of the tile (lower part only on the diagonal) to part[tj][ti]; k_trmv_reduce
// adds them over ti in a fixed order (deterministic). x(r) = REV ? h[np-1-r] : x[r].
template <bool REV>
__global__ __launch_bounds__(256) void k_trmv_part(MatB L, const double* __restrict__ x,
                                                   int64_t vstride, double* __restrict__ part,
                                                   int64_t pstride, int nb, Live live) {
    const int b = blockIdx.y;
    if (!live_pc(live, b)) return;
    const int t = blockIdx.x;
    int ti = (int)floor((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > t) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
    const int tj = t - ti * (ti + 1) / 2;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rg = tid >> 4, cg = tid & 15;
    const int np = nb * 64;
    const double* Lt = L.base + b * L.cstride + (int64_t)(ti * 64 + 4 * rg) * L.ld + tj * 64 + 4 * cg;
    d2_t v[4][2];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        v[r][0] = *reinterpret_cast<const d2_t*>(Lt + (int64_t)r * L.ld);
        v[r][1] = *reinterpret_cast<const d2_t*>(Lt + (int64_t)r * L.ld + 2);
    }
    const double* xb = x + b * vstride;
    double xv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int gr = ti * 64 + 4 * rg + r;
        xv[r] = xb[REV ? np - 1 - gr : gr];
    }
    const bool diag = ti == tj;
    double cs[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double lv = c < 2 ? (c == 0 ? v[r][0].x : v[r][0].y) : (c == 2 ? v[r][1].x : v[r][1].y);
            if (!diag || 4 * rg + r >= 4 * cg + c) s = fma(lv, xv[r], s);
        }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        cs[c] = s;
    }
    __shared__ double red[4][64];
    if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 4; ++c) red[w][4 * lane + c] = cs[c];
    }
    __syncthreads();
    if (tid < 64)
        part[b * pstride + ((int64_t)tj * nb + ti) * 64 + tid] =
            red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
}

template <bool REV>
__global__ __launch_bounds__(256) void k_trmv_reduce(const double* __restrict__ part,
                                                     int64_t pstride, int nb,
                                                     double* __restrict__ out, int64_t vstride,
                                                     Live live) {
    const int b = blockIdx.y;
    if (!live_pc(live, b)) return;
    const int c = blockIdx.x * 256 + threadIdx.x;
    const int np = nb * 64;
    if (c >= np) return;
    const int tj = c >> 6;
    const double* pb = part + b * pstride + (int64_t)tj * nb * 64 + (c & 63);
    double s = 0.0;
    for (int ti = tj; ti < nb; ++ti) s += pb[(int64_t)ti * 64];
    out[b * vstride + (REV ? np - 1 - c : c)] = s;
}

void launch_trmv_tiles(bool rev, MatB L, const double* x, double* out, int64_t vstride, int np,
                       double* part, int64_t pstride, Live live, int nchains, hipStream_t s) {
    const int nb = np / 64;
    const dim3 gp(nb * (nb + 1) / 2, nchains), gr((np + 255) / 256, nchains);
    if (rev) {
        APM_LAUNCH(k_trmv_part<true>, gp, dim3(256), 0, s, L, x, vstride, part, pstride,
                           nb, live);
        APM_LAUNCH(k_trmv_reduce<true>, gr, dim3(256), 0, s, part, pstride, nb, out,
                           vstride, live);
    } else {
        APM_LAUNCH(k_trmv_part<false>, gp, dim3(256), 0, s, L, x, vstride, part, pstride,
                           nb, live);
        APM_LAUNCH(k_trmv_reduce<false>, gr, dim3(256), 0, s, part, pstride, nb, out,
                           vstride, live);
    }
}

// fp32 working copy for the posterior factor's bottom block (apm_internal.h). Grid x per chain:
// [0, T) the top's tiles (i, j), j in [k0, k1), i >= j (rectangular index, upper ones skipped),
// [T, T + k1 - k0) the diagonal-tile inverses of those columns, then (bottom) the bottom's tiles
// (I, k), those before the outer panel of the row's first nonzero tile column nb - 1 - I skipped
// (never read by the bottom's walks and updates). pl.base: the top's tiles below the panel's
// diagonal block (rows >= k1: the trailing update's column operands) also go to the fp16x3
// operand planes (Planes16, slice 2 (j - k0) + c / 32), split as the update would split the fp32
// value (hi = fp16(x), lo = fp16(x - hi)).
__global__ __launch_bounds__(256) void k_post32_convert(MatB A, MatF S, const double* __restrict__ D64,
                                                        int64_t d64stride, float* __restrict__ D32,
                                                        int64_t d32stride, int nb, int outer,
                                                        int k0, int k1, Live live, Planes16 pl) {
    const int b = blockIdx.y;
    if (!live_pc(live, b)) return;
    const int nc = k1 - k0, T = (nb - k0) * nc;
    const int t = blockIdx.x;
    const double* src;
    int64_t sld;
    float* dst;
    int64_t dld;
    unsigned short* hp = nullptr;  // the tile's planes (top tiles below the diagonal block)
    if (t < T) {
        const int ti = k0 + t / nc, tj = k0 + t % nc;
        if (tj > ti) return;
        if (pl.base && ti >= k1)
            hp = pl.base + b * pl.cstride + ((int64_t)(2 * (tj - k0)) * pl.rows + ti * 64) * 32;
        src = A.base + b * A.cstride + (int64_t)(ti * 64) * A.ld + tj * 64;
        sld = A.ld;
        dst = S.base + b * S.cstride + (int64_t)(ti * 64) * S.ld + tj * 64;
        dld = S.ld;
    } else if (t < T + nc) {
        const int k = k0 + t - T;
        src = D64 + b * d64stride + (int64_t)k * 4096;
        sld = 64;
        dst = D32 + b * d32stride + (int64_t)k * 4096;
        dld = 64;
    } else {
        const int u = t - T - nc, I = u / nb, k = u % nb;
        const int kz = nb - 1 - I;  // first nonzero tile column of bottom row tile I
        if (k < (kz / outer) * outer) return;
        src = A.base + b * A.cstride + (int64_t)((nb + I) * 64) * A.ld + k * 64;
        sld = A.ld;
        dst = S.base + b * S.cstride + (int64_t)((nb + I) * 64) * S.ld + k * 64;
        dld = S.ld;
    }
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const int e = threadIdx.x + 256 * h, r = e >> 5, c = 2 * (e & 31);
        const d2_t v = *reinterpret_cast<const d2_t*>(src + (int64_t)r * sld + c);
        const f2_t f{(float)v.x, (float)v.y};
        *reinterpret_cast<f2_t*>(dst + (int64_t)r * dld + c) = f;
        if (hp) {  // slice 2 (tj - k0) + c / 32, row r, halves c % 32 .. +1
            const _Float16 h0 = (_Float16)f.x, h1 = (_Float16)f.y;
            const _Float16 l0 = (_Float16)(f.x - (float)h0), l1 = (_Float16)(f.y - (float)h1);
            unsigned short* q = hp + ((int64_t)(c >> 5) * pl.rows + r) * 32 + (c & 31);
            *reinterpret_cast<unsigned*>(q) =
                __builtin_bit_cast(unsigned short, h0) |
                ((unsigned)__builtin_bit_cast(unsigned short, h1) << 16);
            *reinterpret_cast<unsigned*>(q + pl.lo) =
                __builtin_bit_cast(unsigned short, l0) |
                ((unsigned)__builtin_bit_cast(unsigned short, l1) << 16);
        }
    }
}

void launch_post32_convert(MatB A, MatF S32, const double* D64, int64_t d64stride, float* D32,
                           int64_t d32stride, int nb, int outer, int k0, int k1, bool bottom,
                           Live live, int nchains, hipStream_t s, Planes16 pl) {
    const int nc = k1 - k0, T = (nb - k0) * nc;
    const int grid = T + nc + (bottom ? nb * nb : 0);
    if (grid <= 0) return;
    APM_LAUNCH(k_post32_convert, dim3(grid, nchains), dim3(256), 0, s, A, S32, D64,
                       d64stride, D32, d32stride, nb, outer, k0, k1, live, pl);
}

__global__ void k_merge_status(int* status, const int* other, int code, int nchains) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nchains && other[b] != 0) status[b] = code;
}

void launch_merge_status(int* status, const int* other, int code, int nchains, hipStream_t s) {
    APM_LAUNCH(k_merge_status, dim3((nchains + 255) / 256), dim3(256), 0, s, status, other,
                       code, nchains);
}
