// Laplace-approximation Newton iteration (fp64) and the theta-call plumbing around the Cholesky.
//
// Follows gpdemo/latent_posterior_approximations.py:81-124 (Rasmussen & Williams Alg. 3.1 form):
//   v = phi(f)/Phi(yf) (:86), grad = v y, W = v^2 + grad f (:87-88), B = I + W^1/2 K W^1/2 (:89-91),
//   L = chol(B) (:92), b = W f + grad (:93), a = b - W^1/2 L^-T L^-1 W^1/2 K b (:94), f <- K a (:95),
//   stop when mean((f_new - f)^2) < tol (:96-97).
// The forward solve L^-1 (W^1/2 K b) is produced by the Cholesky itself: W^1/2 K b is appended as an
// extra row below B, so the factorisation of the (np+64) x np trapezoid returns it in that row.
#include "apm_internal.h"

__device__ __forceinline__ bool live_b(const Live& lv, int b) {
    return lv.active[b] != 0 && lv.status[b] == 0;
}

// ------------------------------------------------------------------------------- vectors
__global__ __launch_bounds__(256) void k_newton_prep(NewtonVecs v, const double* __restrict__ y,
                                                     int n, int np, Live live) {
    const int b = blockIdx.y;
    if (!live_b(live, b)) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= np) return;
    const int64_t o = b * v.vstride + i;
    double W = 0.0, Ws = 0.0, bb = 0.0;
    if (i < n) {
        const double f = v.f[o], yi = y[i];
        const double vv = exp(-0.5 * f * f - log_ndtr_d(yi * f) - 0.91893853320467274178);
        const double grad = vv * yi;
        W = vv * vv + grad * f;
        Ws = sqrt(W);
        bb = W * f + grad;
    }
    v.W[o] = W;
    v.Ws[o] = Ws;
    v.b[o] = bb;
}

void launch_newton_prep(NewtonVecs v, const double* y, int n, int np, Live live, int nchains,
                        hipStream_t s) {
    APM_LAUNCH(k_newton_prep, dim3((np + 255) / 256, nchains), dim3(256), 0, s, v, y, n,
                       np, live);
}

// out = M x for a full np x np row-major M; one wave per row, 16-byte loads
__global__ __launch_bounds__(256) void k_gemv(MatB M, const double* __restrict__ x,
                                              int64_t xstride, double* __restrict__ out,
                                              int64_t ostride, int np, Live live) {
    const int b = blockIdx.y;
    if (!live_b(live, b)) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double* xb = x + b * xstride;
    for (int row = blockIdx.x * 16 + w * 4; row < blockIdx.x * 16 + w * 4 + 4; ++row) {
        const double* Mr = M.base + b * M.cstride + (int64_t)row * M.ld;
        double s = 0.0;
        for (int c = lane * 2; c < np; c += 128) {
            const d2_t m = *reinterpret_cast<const d2_t*>(Mr + c);
            const d2_t xx = *reinterpret_cast<const d2_t*>(xb + c);
            s = fma(m.x, xx.x, s);
            s = fma(m.y, xx.y, s);
        }
        s = wave_sum_d(s);
        if (lane == 0) out[b * ostride + row] = s;
    }
}

void launch_gemv(MatB M, const double* x, int64_t xstride, double* out, int64_t ostride, int np,
                 Live live, int nchains, hipStream_t s) {
    APM_LAUNCH(k_gemv, dim3(np / 16, nchains), dim3(256), 0, s, M, x, xstride, out,
                       ostride, np, live);
}

__device__ __forceinline__ void tri_decode(int t, int& ti, int& tj) {
    int i = (int)floor((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (i * (i + 1) / 2 > t) --i;
    while ((i + 1) * (i + 2) / 2 <= t) ++i;
    ti = i;
    tj = t - i * (i + 1) / 2;
}

// B = I + W^1/2 K W^1/2 into the lower tiles of A's top-left np x np, and the extra row block
// rows [np, np+64): row np = W^1/2 (K b) (the Newton right-hand side), the others zero.
__global__ __launch_bounds__(256) void k_form_B(MatB K, MatB A, NewtonVecs v, int nb,
                                                Live live) {
    const int b = blockIdx.y;
    if (!live_b(live, b)) return;
    const int t = blockIdx.x, ntri = nb * (nb + 1) / 2;
    const double* Kb = K.base + b * K.cstride;
    double* Ab = A.base + b * A.cstride;
    const double* Ws = v.Ws + b * v.vstride;
    const int tid = threadIdx.x;
    if (t < ntri) {
        int ti, tj;
        tri_decode(t, ti, tj);
        for (int e = tid; e < 4096; e += 256) {
            const int r = ti * 64 + (e >> 6), c = tj * 64 + (e & 63);
            const double kv = Kb[(int64_t)r * K.ld + c];
            Ab[(int64_t)r * A.ld + c] = (r == c ? 1.0 : 0.0) + (Ws[r] * kv) * Ws[c];
        }
    } else {
        const int tj = t - ntri;
        const int64_t r0 = (int64_t)nb * 64;
        const double* Kbv = v.Kb + b * v.vstride;
        for (int e = tid; e < 4096; e += 256) {
            const int rr = e >> 6, c = tj * 64 + (e & 63);
            Ab[(r0 + rr) * A.ld + c] = (rr == 0) ? Ws[c] * Kbv[c] : 0.0;
        }
    }
}

void launch_form_B(MatB K, MatB A, NewtonVecs v, int np, Live live, int nchains, hipStream_t s) {
    const int nb = np / 64;
    APM_LAUNCH(k_form_B, dim3(nb * (nb + 1) / 2 + nb, nchains), dim3(256), 0, s, K, A, v,
                       nb, live);
}

__global__ __launch_bounds__(256) void k_newton_update(NewtonVecs v, int np, Live live) {
    const int b = blockIdx.y;
    if (!live_b(live, b)) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= np) return;
    const int64_t o = b * v.vstride + i;
    v.a[o] = v.b[o] - v.Ws[o] * v.z[o];
}

void launch_newton_update(NewtonVecs v, int np, Live live, int nchains, hipStream_t s) {
    APM_LAUNCH(k_newton_update, dim3((np + 255) / 256, nchains), dim3(256), 0, s, v, np,
                       live);
}

// diff = mean((f_new - f)^2) over the n real entries; f <- f_new; converged chains drop out.
__global__ __launch_bounds__(256) void k_newton_check(NewtonVecs v, int n, int np, double tol,
                                                      int* active, const int* status,
                                                      int* n_iter) {
    const int b = blockIdx.x;
    if (active[b] == 0 || status[b] != 0) return;
    __shared__ double red[4];
    const double* fn = v.fnew + b * v.vstride;
    double* f = v.f + b * v.vstride;
    double s = 0.0;
#pragma unroll 4  // (loads of 4 steps in flight; the sum keeps its order)
    for (int i = threadIdx.x; i < n; i += 256) {
        const double d = fn[i] - f[i];
        s += d * d;
    }
    s = block_sum_d(s, red);
    __syncthreads();
    for (int i = threadIdx.x; i < np; i += 256) f[i] = fn[i];
    if (threadIdx.x == 0) {
        n_iter[b] += 1;
        if (s / n < tol) active[b] = 0;
    }
}

void launch_newton_check(NewtonVecs v, int n, int np, double tol, int* active, const int* status,
                         int* n_iter, int nchains, hipStream_t s) {
    APM_LAUNCH(k_newton_check, dim3(nchains), dim3(256), 0, s, v, n, np, tol, active,
                       status, n_iter);
}

// lower tiles of src's np x np -> dst (PriorMC: factor K itself)
__global__ __launch_bounds__(256) void k_copy_lower(MatB src, MatB dst, Live live) {
    const int b = blockIdx.y;
    if (!live_b(live, b)) return;
    int ti, tj;
    tri_decode(blockIdx.x, ti, tj);
    const double* S = src.base + b * src.cstride;
    double* D = dst.base + b * dst.cstride;
    d2_t v[8];  // 16-byte pieces, all loads in flight before the stores
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const int e = threadIdx.x + 256 * h;  // piece: row e / 32, columns 2 (e % 32) .. +1
        const int r = ti * 64 + (e >> 5), c = tj * 64 + 2 * (e & 31);
        v[h] = *reinterpret_cast<const d2_t*>(S + (int64_t)r * src.ld + c);
    }
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const int e = threadIdx.x + 256 * h;
        const int r = ti * 64 + (e >> 5), c = tj * 64 + 2 * (e & 31);
        *reinterpret_cast<d2_t*>(D + (int64_t)r * dst.ld + c) = v[h];
    }
}

void launch_copy_lower(MatB src, MatB dst, int np, Live live, int nchains, hipStream_t s) {
    const int nb = np / 64;
    APM_LAUNCH(k_copy_lower, dim3(nb * (nb + 1) / 2, nchains), dim3(256), 0, s, src, dst,
                       live);
}

// Augmented matrix for the posterior covariance factor:
//   [[ B          .  ]        chol       [[ L      0      ]
//    [ K W^1/2    K  ]   ---------->      [ V^T    C_chol ]      V = L^-1 W^1/2 K,
//    [ 0      f_post^T]]                  [ 0      g^T    ]]     C = K - V^T V, g = C_chol^-1 f_post
// The top-left (L of the last Newton iteration) is already factored; this fills rows [np, 2np+64).
// lower_only: K holds its lower tiles only (the theta-call's Gram); the upper block of K W^1/2
// then reads K's symmetric entry
__global__ __launch_bounds__(256) void k_form_aug(MatB K, MatB A, NewtonVecs v, int nb,
                                                  Live live, int lower_only) {
    const int b = blockIdx.y;
    if (!live_b(live, b)) return;
    const int t = blockIdx.x;
    const int nbl = nb * nb, ntri = nb * (nb + 1) / 2;
    const double* Kb = K.base + b * K.cstride;
    double* Ab = A.base + b * A.cstride;
    const double* Ws = v.Ws + b * v.vstride;
    const int64_t np = (int64_t)nb * 64;
    const int tid = threadIdx.x;
    if (t < nbl) {  // bottom-left: (K W^1/2)[r][c] = K[r][c] * W^1/2[c]
        const int ti = t / nb, tj = t % nb;
        for (int e = tid; e < 4096; e += 256) {
            const int r = ti * 64 + (e >> 6), c = tj * 64 + (e & 63);
            const double kv = (lower_only && c > r) ? Kb[(int64_t)c * K.ld + r]
                                                    : Kb[(int64_t)r * K.ld + c];
            Ab[(np + r) * A.ld + c] = kv * Ws[c];
        }
    } else if (t < nbl + ntri) {  // bottom-right lower tiles: K
        int ti, tj;
        tri_decode(t - nbl, ti, tj);
        for (int e = tid; e < 4096; e += 256) {
            const int r = ti * 64 + (e >> 6), c = tj * 64 + (e & 63);
            Ab[(np + r) * A.ld + np + c] = Kb[(int64_t)r * K.ld + c];
        }
    } else {  // extra row block at 2np: row 0 = [0 | f_post^T]
        const int tj = t - nbl - ntri;  // 0 .. 2nb-1
        const double* f = v.f + b * v.vstride;
        for (int e = tid; e < 4096; e += 256) {
            const int rr = e >> 6, c = tj * 64 + (e & 63);
            Ab[(2 * np + rr) * A.ld + c] = (rr == 0 && c >= np) ? f[c - np] : 0.0;
        }
    }
}

void launch_form_aug(MatB K, MatB A, NewtonVecs v, int np, Live live, int nchains,
                     hipStream_t s, bool lower_only) {
    const int nb = np / 64;
    APM_LAUNCH(k_form_aug, dim3(nb * nb + nb * (nb + 1) / 2 + 2 * nb, nchains), dim3(256),
                       0, s, K, A, v, nb, live, (int)lower_only);
}

// Laplace LML (latent_posterior_approximations.py:103-106), with -sum log L_ii = -sum_k ldet[k]
__global__ __launch_bounds__(256) void k_laplace_lml(NewtonVecs v, const double* __restrict__ y,
                                                     int n, const double* ldet, int64_t lstride,
                                                     int nb, double* out, Live live) {
    const int b = blockIdx.x;
    if (live.status[b] != 0) return;
    __shared__ double red[4];
    const double* f = v.f + b * v.vstride;
    const double* a = v.a + b * v.vstride;
    double s1 = 0.0, s2 = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) {
        s1 += a[i] * f[i];
        s2 += log_ndtr_d(y[i] * f[i]);
    }
    s1 = block_sum_d(s1, red);
    __syncthreads();
    s2 = block_sum_d(s2, red);
    if (threadIdx.x == 0) {
        double ld = 0.0;
        for (int k = 0; k < nb; ++k) ld += ldet[b * lstride + k];
        out[b] = -0.5 * s1 + s2 - ld;
    }
}

void launch_laplace_lml(NewtonVecs v, const double* y, int n, const double* ldet,
                        int64_t lstride, int nb, double* out, Live live, int nchains,
                        hipStream_t s) {
    APM_LAUNCH(k_laplace_lml, dim3(nchains), dim3(256), 0, s, v, y, n, ldet, lstride, nb,
                       out, live);
}

// ------------------------------------------------------------------------------- cache slots
// mode 1 (PriorMC):       L = K_chol (A top-left), row np of L = 0
// mode 2 (IS, chol(K)):   L = (block at rows np.., cols 0..) J, row np = g^T (vector v.Kb)
// Rows are written whole (upper part zero) because the u-path GEMM streams full row segments.
// mode 3 (IS, fp32 bottom): L = (rows np.. of S32) J, row np = g^T
// mode 2 / 3 also write the guard's row residuals e_r = (C_chol g)_r - f_post_r (fp32 factor
// row, fp64 g = C_chol^-1 f_post from the fp64 posterior factors and f_post from the Newton
// vectors; k_guard_check): every row of the factor is checked against two fp64 quantities it
// was not computed from, so a tile of C_chol that was read before it was final shows
__global__ __launch_bounds__(256) void k_slot_write_L(MatB A, SlotSet S,
                                                      const int64_t* __restrict__ slots, int mode,
                                                      int np, const double* __restrict__ gvec,
                                                      int64_t gstride, Live live, MatF S32,
                                                      const double* __restrict__ fvec,
                                                      double* rowe) {
    const int b = blockIdx.y;
    if (live.status[b] != 0 || live.active[b] == 0) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * 4 + w;  // 0 .. np+63
    const double* Ab = A.base + b * A.cstride;
    float* L = S.L + slots[b] * S.lstride + (int64_t)r * np;
    double q = 0.0;  // squared norm of factor row r (the wide-slot test, k_slot_write_vec)
    double pg = 0.0;  // (C_chol g)_r of the fp32 row (the guard)
    // rows stop at the end of their diagonal tile: k_ugemm reads row r up to column
    // 64 (r / 64 + 1) only (apm_slot_read zeroes the rest on the host)
    const int cend = (r / 64 + 1) * 64;
    const double* g = gvec + b * gstride;
    if (r < np && mode == 3) {  // as mode 2, from the fp32 bottom block
        const float* src = S32.base + b * S32.cstride + ((int64_t)np + r) * S32.ld;
        for (int c = lane; c < cend; c += 64) {
            const float x = (c <= r) ? src[np - 1 - c] : 0.0f;
            L[c] = x;
            q += (double)x * (double)x;
            pg += (double)x * g[c];
        }
    } else if (r < np && mode == 2) {  // chol(C) = (chol(C) J) J: row r of the block at (np, 0), reversed
        const double* src = Ab + ((int64_t)np + r) * A.ld;
        for (int c = lane; c < cend; c += 64) {
            const double x = (c <= r) ? src[np - 1 - c] : 0.0;
            L[c] = (float)x;
            q += x * x;
            pg += (double)(float)x * g[c];
        }
    } else if (r < np) {
        const double* src = Ab + (int64_t)r * A.ld;
        for (int c = lane; c < cend; c += 64) {
            const double x = (c <= r) ? src[c] : 0.0;
            L[c] = (float)x;
            q += x * x;
        }
    } else if (r == np && mode >= 2) {
        const double* g = gvec + b * gstride;
        for (int c = lane; c < np; c += 64) L[c] = (float)g[c];
    } else {
        for (int c = lane; c < np; c += 64) L[c] = 0.0f;
    }
    if (r < np) {
        q = wave_sum_d(q);
        if (lane == 0) S.rowq[slots[b] * S.vstride + r] = q;
        if (mode >= 2 && rowe) {
            pg = wave_sum_d(pg);
            if (lane == 0) rowe[b * (int64_t)np + r] = pg - fvec[b * gstride + r];
        }
    }
}

// the fp64 factor of the call's wide slots (k_slot_write_vec decided), for k_ugemm64
__global__ __launch_bounds__(256) void k_slot_write_L64(MatB A, SlotSet S,
                                                        const int64_t* __restrict__ slots,
                                                        int mode, int np, Live live) {
    const int b = blockIdx.y;
    if (live.status[b] != 0 || live.active[b] == 0 || !S.wide[slots[b]] || mode == 3) return;
    double* const L0 = S.L64[slots[b]];
    if (!L0) return;  // no buffer yet: the host attaches one and writes the slot again
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * 4 + w;  // 0 .. np-1
    const double* Ab = A.base + b * A.cstride;
    double* L = L0 + (int64_t)r * np;
    const int cend = (r / 64 + 1) * 64;  // as k_slot_write_L: k_ugemm64 reads no further
    if (mode == 2) {
        const double* src = Ab + ((int64_t)np + r) * A.ld;
        for (int c = lane; c < cend; c += 64) L[c] = (c <= r) ? src[np - 1 - c] : 0.0;
    } else {
        const double* src = Ab + (int64_t)r * A.ld;
        for (int c = lane; c < cend; c += 64) L[c] = (c <= r) ? src[c] : 0.0;
    }
}

// fp64 slot vectors of the self-consistent IS epilogue (ugemm.hip): f_post, W (last Newton
// iteration, the one C is built with: latent_posterior_approximations.py:107-112) and
// z = C^-1 f_post = K^-1 f_post + W f_post = a + W f_post (f_post = K a exactly, lpa.py:95), and
// cst = 1/2 f_post^T z - 1/2 log|B| (= 1/2 |C_chol^-1 f_post|^2 - 1/2 log|B|); PriorMC: zeros.
__global__ __launch_bounds__(256) void k_slot_write_vec(MatB A, NewtonVecs v, const double* ldet,
                                                        int64_t lstride, int nb, SlotSet S,
                                                        const int64_t* __restrict__ slots,
                                                        int mode, int n, Live live) {
    (void)A;
    const int b = blockIdx.x;
    if (live.status[b] != 0 || live.active[b] == 0) return;
    __shared__ double red[4];
    const int64_t np = (int64_t)nb * 64;
    const int64_t so = slots[b] * S.vstride;
    double fz = 0.0, tq = 0.0;
    for (int i = threadIdx.x; i < np; i += 256) {
        tq += S.rowq[so + i];
        const bool is = (mode != 1) && i < n;
        const double f = is ? v.f[b * v.vstride + i] : 0.0;
        const double W = is ? v.W[b * v.vstride + i] : 0.0;
        const double z = is ? v.a[b * v.vstride + i] + W * f : 0.0;
        S.fpost64[so + i] = f;
        S.W64[so + i] = W;
        S.z64[so + i] = z;
        fz += f * z;
    }
    fz = block_sum_d(fz, red);
    __syncthreads();
    tq = block_sum_d(tq, red);
    if (threadIdx.x == 0) {
        // (an fp32 bottom block above post_q is recomputed in fp64 and rewritten in mode 2)
        // bit 0: wide now; bit 1: fp32 bottom to recompute; bit 2: wide once it is (the host
        // attaches an fp64 buffer to the slot of every chain with bit 2)
        const int wd = tq > S.wide_q && mode != 3 ? 1 : 0;
        S.wide[slots[b]] = wd;
        // bit 3: C's mean diagonal below 1e-3 of K's (cancellation in the reference's K - V^T V)
        S.chain_wide[b] = wd | (mode == 3 && tq > S.post_q ? 2 : 0) | (tq > S.wide_q ? 4 : 0) |
                          (S.icm_thr && mode != 1 && tq < S.icm_thr[b] ? 8 : 0);
        double c = 0.0;
        if (mode != 1) {
            double ld = 0.0;
            for (int k = 0; k < nb; ++k) ld += ldet[b * lstride + k];
            c = 0.5 * fz - ld;
        }
        S.cst[slots[b]] = c;
    }
}

void launch_slot_write(MatB A, NewtonVecs v, const double* ldet, int64_t lstride, int nb,
                       SlotSet S, const int64_t* slots, int mode, int n, int np, Live live,
                       int nchains, hipStream_t s, MatF S32, double* rowe) {
    APM_LAUNCH(k_slot_write_L, dim3((np + 64) / 4, nchains), dim3(256), 0, s, A, S, slots,
                       mode, np, v.Kb, v.vstride, live, S32, (const double*)v.f, rowe);
    APM_LAUNCH(k_slot_write_vec, dim3(nchains), dim3(256), 0, s, A, v, ldet, lstride, nb,
                       S, slots, mode, n, live);
    launch_slot_write_L64(A, S, slots, mode, np, live, nchains, s);
}

void launch_slot_write_L64(MatB A, SlotSet S, const int64_t* slots, int mode, int np, Live live,
                           int nchains, hipStream_t s) {
    APM_LAUNCH(k_slot_write_L64, dim3(np / 4, nchains), dim3(256), 0, s, A, S, slots, mode,
                       np, live);
}

// Per-call read-back of small per-chain arrays (Newton flags, refinement mask, estimates,
// status, iteration counts): one launch writes up to three device arrays straight into mapped,
// coherent pinned host memory, replacing one hipMemcpyAsync each (every small D2H copy left the
// GPU idle ~77 us before its blit, profiles/r02_idle_gaps.txt). The host reads after the
// stream synchronisation that follows.
__global__ __launch_bounds__(256) void k_export(Export e) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    int off = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (t >= off && t < off + e.words[k]) e.dst[t] = e.src[k][t - off];
        off += e.words[k];
    }
    __threadfence_system();
}

void launch_export(const Export& e, hipStream_t s) {
    const int tot = e.words[0] + e.words[1] + e.words[2] + e.words[3];
    if (tot <= 0) return;
    APM_LAUNCH(k_export, dim3((tot + 255) / 256), dim3(256), 0, s, e);
}

// ------------------------------------------------------------------------------------ the guard
// DESIGN.md §11. Identities between independently computed parts of an IS theta-call; a chain
// that breaks one beyond the rounding of its precisions fails with APM_STATUS_GUARD instead of
// returning its value. G[k * B + b]: k = 0: 1/2 log|B| of the last Newton factor, summed after
// the Newton loop (the factor the posterior's M = I + L_K^T W L_K shares its eigenvalues with,
// W being the last iteration's); k = 1: 1/2 log|K| after chol(K); k = 2..4: the residuals.
__global__ __launch_bounds__(64) void k_guard_save(const double* __restrict__ ldet,
                                                   int64_t lstride, int off, int nb, double* G,
                                                   int B, int k, Live live, int nchains) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= nchains || live.status[b] != 0) return;  // (converged chains are inactive here)
    double s = 0.0;  // (the order of k_slot_write_vec's sum)
    for (int q = 0; q < nb; ++q) s += ldet[b * lstride + off + q];
    G[(int64_t)k * B + b] = s;
}

void launch_guard_save(const double* ldet, int64_t lstride, int off, int nb, double* G, int B,
                       int k, Live live, int nchains, hipStream_t s) {
    APM_LAUNCH(k_guard_save, dim3((nchains + 63) / 64), dim3(64), 0, s, ldet, lstride, off, nb, G,
               B, k, live, nchains);
}

// r1 = |G0 - 1/2 log|M||, r2 = | |g|^2 - f_post^T z | / max(1, |f_post^T z|) (g = chol(C)^-1
// f_post from L' and L_K, v.Kb; z = a + W f_post from the Newton vectors, in the slot), r3 =
// |sum log diag(C_chol) - (G1 - 1/2 log|M|)| (C_chol = L_K U^-T: its diagonal is L_K,ii / U_ii;
// from the fp32 slot; skipped for a chain whose bottom block is recomputed in fp64, bit 1 of
// chain_wide). 1/2 log|M| is the ldet sum the slot's cst was formed with.
__global__ __launch_bounds__(256) void k_guard_check(const double* __restrict__ ldet,
                                                     int64_t lstride, int nb, const double* gvec,
                                                     int64_t gstride, SlotSet S,
                                                     const int64_t* __restrict__ slots, double* G,
                                                     int B, double t1, double t2, double t3,
                                                     double t4, const double* rowe,
                                                     const double* fvec, int fail_code,
                                                     Live live) {
    const int b = blockIdx.x;
    if (live.status[b] != 0 || live.active[b] == 0) return;
    __shared__ double red[4];
    const int64_t np = (int64_t)nb * 64;
    const int64_t sl = slots[b];
    const int64_t so = sl * S.vstride;
    const float* L = S.L + sl * S.lstride;
    double gg = 0.0, fz = 0.0, lc = 0.0, em = 0.0, fm = 0.0;
    for (int64_t i = threadIdx.x; i < np; i += 256) {
        const double g = gvec[b * gstride + i];
        gg += g * g;
        fz += S.fpost64[so + i] * S.z64[so + i];
        lc += log((double)L[i * np + i]);
        em = fmax(em, fabs(rowe[b * np + i]));  // (a NaN row makes em NaN: fmax drops it, so
        if (rowe[b * np + i] != rowe[b * np + i]) em = INFINITY;  // it is caught here)
        fm = fmax(fm, fabs(fvec[b * gstride + i]));
    }
    gg = block_sum_d(gg, red);
    __syncthreads();
    fz = block_sum_d(fz, red);
    __syncthreads();
    lc = block_sum_d(lc, red);
    __syncthreads();
    em = block_max_d(em, red);
    __syncthreads();
    fm = block_max_d(fm, red);
    if (threadIdx.x == 0) {
        double ldm = 0.0;
        for (int q = 0; q < nb; ++q) ldm += ldet[b * lstride + q];
        const double r1 = fabs(G[b] - ldm);
        const double r2 = fabs(gg - fz) / fmax(1.0, fabs(fz));
        const bool fp64_bottom = S.chain_wide[b] & 2;  // (recomputed in fp64 after this)
        const double r3 = fp64_bottom ? 0.0 : fabs(lc - (G[B + b] - ldm));
        const double r4 = fp64_bottom ? 0.0 : em / fmax(1.0, fm);
        G[2 * (int64_t)B + b] = r1;
        G[3 * (int64_t)B + b] = r2;
        G[4 * (int64_t)B + b] = r3;
        G[5 * (int64_t)B + b] = r4;
        // (!(r <= t): a NaN residual fails as well)
        if (!(r1 <= t1) || !(r2 <= t2) || !(r3 <= t3) || !(r4 <= t4))
            live.status[b] = fail_code;
    }
}

void launch_guard_check(const double* ldet, int64_t lstride, int nb, const double* gvec,
                        int64_t gstride, SlotSet S, const int64_t* slots, double* G, int B,
                        double t1, double t2, double t3, double t4, const double* rowe,
                        const double* fvec, int fail_code, Live live, int nchains,
                        hipStream_t s) {
    APM_LAUNCH(k_guard_check, dim3(nchains), dim3(256), 0, s, ldet, lstride, nb, gvec, gstride, S,
               slots, G, B, t1, t2, t3, t4, rowe, fvec, fail_code, live);
}

// APM_SKEW (tests only): a kernel that only waits, `us` microseconds of the 100 MHz constant
// clock (s_memrealtime), one wave
__global__ __launch_bounds__(64) void k_delay(long long ticks) {
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void launch_delay(int us, hipStream_t s) {
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, (long long)us * 100);
}
