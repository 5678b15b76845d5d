// Importance-sampling u-path: f_s = f_post + L U (fp32 MFMA), probit epilogue, log-mean-exp.
//
// Replaces gpdemo/estimators.py:221-241 (ApproxPosteriorIS, theta- and cached u-calls) and
// :323-325 (PriorMC) in the algebraically identical, self-consistent form of DESIGN.md §3.2:
//   log w_s = sum_n [log Phi(y_n f_sn) + 1/2 W_n f_sn^2 - z_n f_sn] + cst,
//   z = C^-1 f_post = a + W f_post,  cst = 1/2 f_post^T z - 1/2 log|B|   (IS)
//   W = 0, z = 0, cst = 0                                               (PriorMC)
// i.e. the reference's log p(y|f) + log p(f) - log q(f) evaluated AT the computed f_s (with
// K^-1 = C^-1 - W and |C|/|K| = 1/|B|): no term uses u_s itself, so the fp32 rounding of L, U and
// the MFMA accumulation moves f_s but not the consistency of the three terms, whose sum has a
// vanishing gradient in f_s at the Laplace mode - as in the reference's own evaluation. The large
// terms (1/2 W f^2, z f, the -x^2/2 of log Phi) are formed and summed in fp64.
#include "apm_internal.h"

// ------------------------------------------------------------------------------- U buffers
__global__ __launch_bounds__(256) void k_u_convert(const double* __restrict__ U, int64_t ldu,
                                                   int n, int S, double* __restrict__ dst,
                                                   float* __restrict__ dst32, int sp, int np) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)np * sp) return;
    const int r = (int)(e / sp), c = (int)(e % sp);
    const double v = (r < n && c < S) ? U[(int64_t)r * ldu + c] : 0.0;
    dst[e] = v;
    dst32[e] = (float)v;
}

void launch_u_convert(const double* U64, int64_t ldu, int n, int S, UPool P, int64_t ubuf,
                      hipStream_t s) {
    const int np = (int)(P.stride / P.sp);
    const int64_t tot = (int64_t)np * P.sp;
    APM_LAUNCH(k_u_convert, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, U64, ldu,
                       n, S, P.base + ubuf * P.stride, P.base32 + ubuf * P.stride, P.sp, np);
}

// Philox4x32-10 (Salmon et al., SC'11) + Box-Muller: counter = (e/4, ctr_lo, ctr_hi, 0)
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// raw Philox4x32-10 blocks (apm_selftest_philox): in = {ctr0..3, key0, key1} per block
__global__ __launch_bounds__(256) void k_philox_test(const uint32_t* __restrict__ in,
                                                     uint32_t* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t c[4] = {in[6 * i], in[6 * i + 1], in[6 * i + 2], in[6 * i + 3]};
    philox4x32_10(c, in[6 * i + 4], in[6 * i + 5]);
#pragma unroll
    for (int h = 0; h < 4; ++h) out[4 * i + h] = c[h];
}

void launch_philox_test(const uint32_t* in, uint32_t* out, int64_t n, hipStream_t s) {
    APM_LAUNCH(k_philox_test, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out,
                       n);
}

__global__ __launch_bounds__(256) void k_u_normal(UPool P, const int64_t* __restrict__ ubufs,
                                                  const uint64_t* __restrict__ seeds,
                                                  const uint64_t* __restrict__ counters, int n,
                                                  int S) {
    const int b = blockIdx.y;
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // group of 4 normals
    const int64_t tot = (int64_t)n * S;
    if (q * 4 >= tot) return;
    const uint64_t sd = seeds[b], ct = counters[b];
    uint32_t c[4] = {(uint32_t)q, (uint32_t)ct, (uint32_t)(ct >> 32), (uint32_t)(q >> 32)};
    philox4x32_10(c, (uint32_t)sd, (uint32_t)(sd >> 32));
    float z[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const float u1 = ((float)c[2 * h] + 0.5f) * 2.3283064365386963e-10f;
        const float u2 = ((float)c[2 * h + 1] + 0.5f) * 2.3283064365386963e-10f;
        const float rr = sqrtf(-2.0f * logf(u1));
        float sn, cs;
        sincosf(6.283185307179586f * u2, &sn, &cs);
        z[2 * h] = rr * cs;
        z[2 * h + 1] = rr * sn;
    }
    double* dst = P.base + ubufs[b] * P.stride;
    float* dst32 = P.base32 + ubufs[b] * P.stride;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int64_t e = q * 4 + h;
        if (e < tot) {
            dst[(e / S) * P.sp + (e % S)] = (double)z[h];
            dst32[(e / S) * P.sp + (e % S)] = z[h];
        }
    }
}

void launch_u_normal(UPool P, const int64_t* ubufs, const uint64_t* seeds,
                     const uint64_t* counters, int n, int S, int nchains, hipStream_t s) {
    const int64_t groups = ((int64_t)n * S + 3) / 4;
    APM_LAUNCH(k_u_normal, dim3((unsigned)((groups + 255) / 256), nchains), dim3(256), 0, s,
                       P, ubufs, seeds, counters, n, S);
}

__global__ __launch_bounds__(256) void k_u_combine(UPool P, const int64_t* __restrict__ dst,
                                                   const int64_t* __restrict__ a,
                                                   const int64_t* __restrict__ bb,
                                                   const double* __restrict__ ca,
                                                   const double* __restrict__ cb, int64_t tot) {
    const int b = blockIdx.y;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= tot) return;
    const double x = P.base[a[b] * P.stride + e], v = P.base[bb[b] * P.stride + e];
    const double u = ca[b] * x + cb[b] * v;
    P.base[dst[b] * P.stride + e] = u;
    P.base32[dst[b] * P.stride + e] = (float)u;
}

void launch_u_combine(UPool P, const int64_t* dst, const int64_t* a, const int64_t* b,
                      const double* ca, const double* cb, int n, int S, int nchains,
                      hipStream_t s) {
    (void)n;
    (void)S;
    const int64_t tot = P.stride;  // padded entries are 0 in both inputs, stay 0
    APM_LAUNCH(k_u_combine, dim3((unsigned)((tot + 255) / 256), nchains), dim3(256), 0, s,
                       P, dst, a, b, ca, cb, tot);
}

// ------------------------------------------------------------------------------- L . U + epilogue
// v_mfma_f32_16x16x4_f32: A lane l -> A[l&15][k=l>>4], B lane l -> B[k=l>>4][l&15],
// C/D lane l, reg r -> (row = (l>>4)*4 + r, col = l&15)
#define UP 65  // LDS row pitch (floats) of the staged U tile: conflict-free B-fragment reads

// one entry of the per-sample sum: log Phi(y f) + 1/2 W f^2 - z f, the large terms in fp64
__device__ __forceinline__ double is_term(double f, double y, double W, double z) {
    return log_ndtr_mixed(y * f) + (0.5 * W * f - z) * f;
}

// One 64 x 64 output tile (row block i, sample block sb) per workgroup, waves 32 x 32 (a 64 x 128
// tile that read L once per two sample blocks was measured slower from 8 chains up: half the
// workgroups, 2 instead of 4 per CU - DESIGN.md §5).
__global__ __launch_bounds__(256) void k_ugemm(SlotSet S, const int64_t* __restrict__ slots,
                                               UPool P, const int64_t* __restrict__ ubufs,
                                               const double* __restrict__ y, int n, int np,
                                               double* __restrict__ partial, int64_t pstride,
                                               const int* __restrict__ status, int nsb,
                                               int nchains) {
    // XCD-aware order (as k_chol_update's xcd_remap): dispatch slot s runs on XCD s % 8, and
    // consecutive work items land on the same XCD. Items run chain-major, then row block
    // (heaviest, i.e. longest K range, first; consecutive row blocks read nearly the same rows
    // of U), then sample block fastest - so the nsb
    // workgroups that share row block i's slice of L run together on one XCD and read it once
    // from its L2, and a chain's U stays within one XCD's L2 / the Infinity Cache.
    constexpr int NSW = 1;
    const int nb = np / 64;
    const int nsg = nsb / NSW;  // sample groups
    const long total = (long)nb * nsg * nchains;
    const long slot_id = blockIdx.x, xcd = slot_id & 7, q = total >> 3, rem = total & 7;
    const long item = nchains < 8 ? slot_id  // too few chains to fill 8 XCDs evenly: plain order
                      : (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (slot_id >> 3);
    const int b = (int)(item / ((long)nb * nsg));
    const int rest = (int)(item % ((long)nb * nsg));
    if (status[b] != 0) return;
    const int i = nb - 1 - rest / nsg;
    const int sb = (rest % nsg) * NSW;  // first sample block
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1;
    const int r16 = lane & 15, kq = lane >> 4;
    constexpr int SW = 64 * NSW;  // samples per workgroup
    __shared__ float Ut[2][64][SW + 1];
    __shared__ double csum[2][SW];

    const int64_t slot = slots[b];
    if (S.wide[slot]) return;  // k_ugemm64
    const float* L = S.L + slot * S.lstride;
    const float* U = P.base32 + ubufs[b] * P.stride;
    const int sp = P.sp;
    const int kend = (i + 1) * 64;

    f4_t acc[2][2 * NSW];
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2 * NSW; ++bj) acc[bi][bj] = f4_t{0.f, 0.f, 0.f, 0.f};

    // U[kk:kk+64][sb*64 : sb*64+SW] (16 KB per sample block, 16-byte loads) and the A fragments
    // (straight from global: 16 contiguous floats per lane and row) of the next slice are loaded
    // into registers while the current one is multiplied; U goes through two LDS buffers, one
    // barrier per slice
    constexpr int PR = 16 * NSW;  // 16-byte pieces per U row
    f4_t un[4 * NSW];
    f4_t an[2][4];
    auto gload = [&](int kk) {
#pragma unroll
        for (int h = 0; h < 4 * NSW; ++h) {
            const int e = tid + h * 256;  // 4-element piece
            un[h] = *reinterpret_cast<const f4_t*>(U + (int64_t)(kk + e / PR) * sp + sb * 64 +
                                                   (e % PR) * 4);
        }
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
            const float* p = L + (int64_t)(i * 64 + 32 * wr + 16 * bi + r16) * np + kk + kq * 16;
#pragma unroll
            for (int t = 0; t < 4; ++t) an[bi][t] = *reinterpret_cast<const f4_t*>(p + 4 * t);
        }
    };
    gload(0);
    for (int kk = 0, cur = 0; kk < kend; kk += 64, cur ^= 1) {
#pragma unroll
        for (int h = 0; h < 4 * NSW; ++h) {
            const int e = tid + h * 256;
            const int r = e / PR, c4 = (e % PR) * 4;
            Ut[cur][r][c4] = un[h][0];
            Ut[cur][r][c4 + 1] = un[h][1];
            Ut[cur][r][c4 + 2] = un[h][2];
            Ut[cur][r][c4 + 3] = un[h][3];
        }
        float a[2][16];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int t = 0; t < 16; ++t) a[bi][t] = an[bi][t >> 2][t & 3];
        __syncthreads();
        if (kk + 64 < kend) gload(kk + 64);
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            float bv[2 * NSW];
#pragma unroll
            for (int bj = 0; bj < 2 * NSW; ++bj)
                bv[bj] = Ut[cur][kq * 16 + t][32 * NSW * wc + 16 * bj + r16];
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
                for (int bj = 0; bj < 2 * NSW; ++bj)
                    acc[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[bi][t], bv[bj],
                                                                       acc[bi][bj], 0, 0, 0);
        }
    }

    double* pb = partial + b * pstride;
    const double* fp = S.fpost64 + slot * S.vstride;
    const double* Wv = S.W64 + slot * S.vstride;
    const double* zv = S.z64 + slot * S.vstride;
    double colsum[2 * NSW];
#pragma unroll
    for (int bj = 0; bj < 2 * NSW; ++bj) {
        double d = 0.0;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = i * 64 + 32 * wr + 16 * bi + kq * 4 + r;
                if (row < n) d += is_term(fp[row] + (double)acc[bi][bj][r], y[row], Wv[row], zv[row]);
            }
        d += __shfl_xor(d, 16, 64);
        d += __shfl_xor(d, 32, 64);
        colsum[bj] = d;
    }
    if (kq == 0) {
#pragma unroll
        for (int bj = 0; bj < 2 * NSW; ++bj) csum[wr][32 * NSW * wc + 16 * bj + r16] = colsum[bj];
    }
    __syncthreads();
    if (tid < SW) pb[(int64_t)i * sp + sb * 64 + tid] = csum[0][tid] + csum[1][tid];
}

// The same product and epilogue on f64 MFMA (v_mfma_f64_16x16x4_f64) for the call's WIDE slots
// (S.wide: trace(L L^T) > APM_WIDE_Q, set by k_slot_write_vec), from the slot's fp64 factor and
// the fp64 U buffer: where the entries of f_s are large (sigma = e^18.5: |f_s| ~ 1e4), the fp32
// rounding of L and U alone moves log f by ~10 nats. Rare (extreme theta),
// so plainly staged: 64x64 output tile per workgroup, L and U slices of 16 through LDS.
__global__ __launch_bounds__(256) void k_ugemm64(SlotSet S, const int64_t* __restrict__ slots,
                                                 UPool P, const int64_t* __restrict__ ubufs,
                                                 const double* __restrict__ y, int n, int np,
                                                 double* __restrict__ partial, int64_t pstride,
                                                 const int* __restrict__ status, int nsb) {
    const int nb = np / 64;
    const int b = blockIdx.y;
    if (status[b] != 0) return;
    const int64_t slot = slots[b];
    if (!S.wide[slot]) return;
    const int i = (int)blockIdx.x / nsb, sb = (int)blockIdx.x % nsb;
    (void)nb;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1;
    const int r16 = lane & 15, kq = lane >> 4;
    __shared__ double La[64][17];
    __shared__ double Ub[16][65];
    __shared__ double csum[2][64];
    const double* L = S.L64[slot];
    if (!L) return;  // wide by this call, buffer not attached yet: recomputed after it is
    const double* U = P.base + ubufs[b] * P.stride;
    const int sp = P.sp;
    d4_t acc[2][2];
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = d4_t{0.0, 0.0, 0.0, 0.0};
    const int kend = (i + 1) * 64;
    for (int kk = 0; kk < kend; kk += 16) {
        for (int e = tid; e < 64 * 16; e += 256) {
            const int r = e >> 4, c = e & 15;
            La[r][c] = L[(int64_t)(i * 64 + r) * np + kk + c];
            Ub[e >> 6][e & 63] = U[(int64_t)(kk + (e >> 6)) * sp + sb * 64 + (e & 63)];
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
                for (int bj = 0; bj < 2; ++bj)
                    acc[bi][bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                        La[32 * wr + 16 * bi + r16][4 * t + kq],
                        Ub[4 * t + kq][32 * wc + 16 * bj + r16], acc[bi][bj], 0, 0, 0);
        }
        __syncthreads();
    }
    // f64 MFMA output map: lane l, reg r -> row (l >> 4) + 4r, col l & 15
    double* pb = partial + b * pstride;
    const double* fp = S.fpost64 + slot * S.vstride;
    const double* Wv = S.W64 + slot * S.vstride;
    const double* zv = S.z64 + slot * S.vstride;
    double colsum[2];
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
        double d = 0.0;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = i * 64 + 32 * wr + 16 * bi + kq + 4 * r;
                if (row < n) d += is_term(fp[row] + acc[bi][bj][r], y[row], Wv[row], zv[row]);
            }
        d += __shfl_xor(d, 16, 64);
        d += __shfl_xor(d, 32, 64);
        colsum[bj] = d;
    }
    if (kq == 0) {
        csum[wr][32 * wc + r16] = colsum[0];
        csum[wr][32 * wc + 16 + r16] = colsum[1];
    }
    __syncthreads();
    if (tid < 64) pb[(int64_t)i * sp + sb * 64 + tid] = csum[0][tid] + csum[1][tid];
}

void launch_ugemm(SlotSet S, const int64_t* slots, UPool P, const int64_t* ubufs,
                  const double* y, int n, int np, double* partial, int64_t pstride,
                  const int* status, int nchains, bool wide, hipStream_t s) {
    const int nb = np / 64, nsb = P.sp / 64;
    const long total = (long)nb * nsb * nchains;
    APM_LAUNCH(k_ugemm, dim3((unsigned)total), dim3(256), 0, s, S, slots, P, ubufs, y, n,
                       np, partial, pstride, status, nsb, nchains);
    if (wide)
        APM_LAUNCH(k_ugemm64, dim3((unsigned)(nb * nsb), nchains), dim3(256), 0, s, S,
                           slots, P, ubufs, y, n, np, partial, pstride, status, nsb);
}

// logsumexp_s(lw_s) - log S per chain
__global__ __launch_bounds__(256) void k_lme(const double* __restrict__ partial, int64_t pstride,
                                             int nb, int S, int sp, SlotSet Sl,
                                             const int64_t* __restrict__ slots,
                                             double* __restrict__ out,
                                             const int* __restrict__ status) {
    const int b = blockIdx.x;
    if (status[b] != 0) return;
    __shared__ double red[4];
    __shared__ double lw[1024];
    const double* pb = partial + b * pstride;
    const double cst = Sl.cst[slots[b]];
    double mx = -INFINITY;
    for (int s = threadIdx.x; s < S; s += 256) {
        double v = cst;
        int i = 0;
        for (; i + 16 <= nb; i += 16) {  // 16 loads in flight, added in order
            double t[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) t[q] = pb[(int64_t)(i + q) * sp + s];
#pragma unroll
            for (int q = 0; q < 16; ++q) v += t[q];
        }
        for (; i < nb; ++i) v += pb[(int64_t)i * sp + s];
        if (s < 1024) lw[s] = v;
        mx = fmax(mx, v);
    }
    mx = block_max_d(mx, red);
    __syncthreads();
    double se = 0.0;
    for (int s = threadIdx.x; s < S; s += 256) {
        double v;
        if (s < 1024) {
            v = lw[s];
        } else {
            v = cst;
            for (int i = 0; i < nb; ++i) v += pb[(int64_t)i * sp + s];
        }
        se += exp(v - mx);
    }
    se = block_sum_d(se, red);
    if (threadIdx.x == 0) out[b] = (isfinite(mx) ? mx + log(se) : mx) - log((double)S);
}

void launch_lme(const double* partial, int64_t pstride, int nb, int S, int sp, SlotSet Sl,
                const int64_t* slots, double* out, const int* status, int nchains,
                hipStream_t s) {
    APM_LAUNCH(k_lme, dim3(nchains), dim3(256), 0, s, partial, pstride, nb, S, sp, Sl,
                       slots, out, status);
}
