// Importance-sampling u-path: f_s = f_post + L U (fp32 MFMA), probit epilogue, log-mean-exp.
//
// Replaces gpdemo/estimators.py:221-241 (ApproxPosteriorIS, theta- and cached u-calls) and
// :323-325 (PriorMC) in the algebraically identical form of DESIGN.md §3:
//   log w_s = sum_n [log Phi(y_n f_sn) + 1/2 W_n f_sn^2] - g^T u_s + cst,
//   cst = -1/2 |g|^2 - 1/2 log|B|          (IS);     W = 0, g = 0, cst = 0   (PriorMC)
// g^T u_s comes out of the same GEMM: g^T is stored as row np of the slot's factor, so the extra
// 64-row block of the output holds it in its first row.
#include "apm_internal.h"

// ------------------------------------------------------------------------------- U buffers
// Device layout of an auxiliary-variable buffer: sample-major, element (row i, sample s) at
// s * np + i (zero padded to sp x np). The L.U kernel then reads both of its operands (rows of
// L, rows of U^T) as k-contiguous 16-byte pieces. The logical matrix (N x S, reference layout
// estimators.py:223) is unchanged: upload/download convert.
__global__ __launch_bounds__(256) void k_u_convert(const double* __restrict__ U, int64_t ldu,
                                                   int n, int S, float* __restrict__ dst, int sp,
                                                   int np) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)np * sp) return;
    const int sidx = (int)(e / np), i = (int)(e % np);
    dst[e] = (i < n && sidx < S) ? (float)U[(int64_t)i * ldu + sidx] : 0.0f;
}

void launch_u_convert(const double* U64, int64_t ldu, int n, int S, UPool P, int64_t ubuf,
                      hipStream_t s) {
    const int np = (int)(P.stride / P.sp);
    const int64_t tot = (int64_t)np * P.sp;
    hipLaunchKernelGGL(k_u_convert, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, U64, ldu,
                       n, S, P.base + ubuf * P.stride, P.sp, np);
}

// Philox4x32-10 (Salmon et al., SC'11) + Box-Muller: counter = (q, ctr_lo, ctr_hi, q >> 32) gives
// the 4 normals of logical elements 4q .. 4q+3 of the row-major N x S matrix.
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

__device__ __forceinline__ void philox_normals(int64_t q, uint64_t sd, uint64_t ct, float z[4]) {
    uint32_t c[4] = {(uint32_t)q, (uint32_t)ct, (uint32_t)(ct >> 32), (uint32_t)(q >> 32)};
    philox4x32_10(c, (uint32_t)sd, (uint32_t)(sd >> 32));
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
}

// S % 4 == 0: thread t -> row i = t % np, sample group m = t / np (q = i * S/4 + m), so a wave
// writes 64 consecutive rows of 4 sample-major rows (coalesced). Otherwise one thread per q.
__global__ __launch_bounds__(256) void k_u_normal(UPool P, const int64_t* __restrict__ ubufs,
                                                  const uint64_t* __restrict__ seeds,
                                                  const uint64_t* __restrict__ counters, int n,
                                                  int S, int np) {
    const int b = blockIdx.y;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t sd = seeds[b], ct = counters[b];
    float* dst = P.base + ubufs[b] * P.stride;
    float z[4];
    if ((S & 3) == 0) {
        const int G = S >> 2;
        if (t >= (int64_t)np * G) return;
        const int i = (int)(t % np), m = (int)(t / np);
        if (i >= n) return;
        philox_normals((int64_t)i * G + m, sd, ct, z);
#pragma unroll
        for (int h = 0; h < 4; ++h) dst[(int64_t)(4 * m + h) * np + i] = z[h];
        return;
    }
    const int64_t tot = (int64_t)n * S;
    if (t * 4 >= tot) return;
    philox_normals(t, sd, ct, z);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int64_t e = t * 4 + h;
        if (e < tot) dst[(e % S) * np + (e / S)] = z[h];
    }
}

void launch_u_normal(UPool P, const int64_t* ubufs, const uint64_t* seeds,
                     const uint64_t* counters, int n, int S, int nchains, hipStream_t s) {
    const int np = (int)(P.stride / P.sp);
    const int64_t threads = (S % 4 == 0) ? (int64_t)np * (S / 4) : ((int64_t)n * S + 3) / 4;
    hipLaunchKernelGGL(k_u_normal, dim3((unsigned)((threads + 255) / 256), nchains), dim3(256), 0,
                       s, P, ubufs, seeds, counters, n, S, np);
}

__global__ __launch_bounds__(256) void k_u_combine(UPool P, const int64_t* __restrict__ dst,
                                                   const int64_t* __restrict__ a,
                                                   const int64_t* __restrict__ bb,
                                                   const double* __restrict__ ca,
                                                   const double* __restrict__ cb, int64_t tot) {
    const int b = blockIdx.y;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= tot) return;
    const float x = P.base[a[b] * P.stride + e], v = P.base[bb[b] * P.stride + e];
    P.base[dst[b] * P.stride + e] = (float)ca[b] * x + (float)cb[b] * v;
}

void launch_u_combine(UPool P, const int64_t* dst, const int64_t* a, const int64_t* b,
                      const double* ca, const double* cb, int n, int S, int nchains,
                      hipStream_t s) {
    (void)n;
    (void)S;
    const int64_t tot = P.stride;  // padded entries are 0 in both inputs, stay 0
    hipLaunchKernelGGL(k_u_combine, dim3((unsigned)((tot + 255) / 256), nchains), dim3(256), 0, s,
                       P, dst, a, b, ca, cb, tot);
}

// ------------------------------------------------------------------------------- L . U + epilogue
// F = L U^T-read GEMM: F[i][s] = sum_k L[i][k] U[s][k] (U buffers are sample-major), then the
// probit epilogue. One 512-thread workgroup owns 128 rows x 256 samples (8 waves, 2 x 4, each
// 64 x 64 = 4 x 4 tiles of v_mfma_f32_16x16x4_f32; 2 x 2 and 2 x 1 waves for S <= 128 and
// S <= 64): L is read once per launch for S <= 256, and
// 48 KB of operands are staged per 128 x 256 x 32 slice (a 64 x 64 tile per workgroup stages
// 32 KB per 64 x 64 x 64: 2.7x more bytes per MAC).
// Staging: 16-byte LDS-DMA loads (global_load_lds_dwordx4: no staging registers, no ds_write
// pass) into two buffers of 32-deep slices; one instruction moves 8 rows of 128 B, lane-linear, with
// the 16-byte pieces XOR-swizzled by row (piece p of row r at slot p ^ (r & 7)) so the 16-byte
// fragment reads of 8 consecutive rows hit distinct banks. Lane group kq of a fragment owns
// k = 8kq .. 8kq+7 of the slice (pieces 2kq, 2kq+1; any k order common to both operands gives the
// same sums): two ds_read_b128 per fragment and slice.
// Rows past the end of L's slot (np + 64 rows) or of U (sp samples) are clamped to a valid row:
// only waves that own no output read them.
// Epilogue: f_post, W and y of the block's 128 rows sit in LDS (loaded before the main loop, so
// the epilogue has no global-load latency); every wave reduces its own 64 rows per sample (probit
// term in fp64 per element, branch-free log Phi) and writes its 64-row-block partial directly
// (partial[b][i][s], i < nb; k_lme is unchanged); the wave holding output row np writes g^T u_s
// (g^T is row np of the slot factor).
// Grid: 1-D, remapped so that each XCD processes a contiguous range of (chain, row block, sample
// block) - the row blocks of one chain share its U (4 MB at S = 256) in that XCD's L2 - with the
// heaviest (longest k range) row blocks of each chain first.
// Measured (tools/ugemm_bench.cpp, 64 chains, N = 4096, S = 256): MFMA + barriers alone 2.08 ms;
// the register-staged version of this kernel 3.03 ms (+0.58 ms staging, +0.37 ms epilogue).
#define UG_BM 128
#ifndef UG_KS
#define UG_KS 32  // slice depth (floats): 32 (1 workgroup per CU) or 16 (2 per CU)
#endif
#define UG_PPR (UG_KS / 4)     // 16-byte pieces per staged row
#define UG_RPI (64 / UG_PPR)   // rows per LDS-DMA instruction (1 KB)
// swizzle: piece p of row r at slot p ^ sw(r); 16-byte reads of 8 consecutive rows are distinct
#if UG_KS == 32
#define UG_SW(r) ((r) & 7)
#else
#define UG_SW(r) (((r) >> 2) & 3)
#endif
#ifndef UG_ABL
#define UG_ABL 0  // tools/ugemm_bench.cpp ablations: 1 no MFMA, 2 no global loads, 5 = no loads,
                  // no LDS fragment reads, no epilogue
#endif
typedef __attribute__((address_space(3))) void ug_lds_t;
typedef __attribute__((address_space(1))) void ug_glb_t;
template <int WC>
struct __attribute__((aligned(16))) UgSmem {
    float a[2][UG_BM][UG_KS];
    float b[2][64 * WC][UG_KS];
    float fp[UG_BM], w[UG_BM], y[UG_BM];
};

// WC = waves across samples: the tile is 128 x 64*WC (WC = 4 for S > 128; 2 and 1 keep narrow
// sample counts, e.g. N_imp = 64, from idling three quarters of the waves)
template <int WC>
__global__ __launch_bounds__(128 * WC) void k_ugemm(SlotSet S, const int64_t* __restrict__ slots,
                                               UPool P, const int64_t* __restrict__ ubufs,
                                               const double* __restrict__ y, int n, int np,
                                               double* __restrict__ partial, int64_t pstride,
                                               const int* __restrict__ status, int nI, int nJ,
                                               int total) {
    int lin = blockIdx.x;
    if ((total & 7) == 0) lin = (lin & 7) * (total >> 3) + (lin >> 3);
    const int jb = lin % nJ;
    const int rest = lin / nJ;
    const int I = nI - 1 - rest % nI;
    const int b = rest / nI;
    if (status[b] != 0) return;
    extern __shared__ __attribute__((aligned(16))) float ug_sm[];
    UgSmem<WC>& sm = *reinterpret_cast<UgSmem<WC>*>(ug_sm);
    constexpr int BN = 64 * WC;
    constexpr int NA = UG_BM / UG_RPI / (2 * WC);  // DMA instructions per wave and slice: L
    constexpr int NB = BN / UG_RPI / (2 * WC);     // and U

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w / WC, wc = w % WC;
    const int r16 = lane & 15, kq = lane >> 4;
    const int nb = np / 64, sp = P.sp;
    const int64_t slot = slots[b];
    const float* L = S.L + slot * S.lstride;
    const float* U = P.base + ubufs[b] * P.stride;
    const int row0 = I * UG_BM;
    const int rows_avail = np + 64 - row0;  // slot rows: np + 64 (row np = g^T, then zeros)
    const int kend = min(row0 + UG_BM, np);
    const int col0 = jb * BN;
    const int cols_avail = min(BN, sp - col0);
    const int h = 2 * I + wr;  // this wave's 64-row block
    const bool active = h <= nb && 64 * wc < cols_avail;

    if (tid < UG_BM) {
        const int row = row0 + tid;
        const bool in = row < n;
        sm.fp[tid] = in ? S.fpost[slot * S.vstride + row] : 0.f;
        sm.w[tid] = in ? S.W[slot * S.vstride + row] : 0.f;
        sm.y[tid] = in ? (float)y[row] : 0.f;  // y = 0 marks a padded row
    }

    // LDS-DMA: lane l of an instruction takes row RPI*c + l/PPR of chunk c and the global piece
    // stored at slot l%PPR. Chunks: L 128/RPI (NA per wave), U BN/RPI (NB per wave).
    const int lrow = lane / UG_PPR, spiece = (lane % UG_PPR) ^ UG_SW(lrow);
    const float* ga[NA];
    const float* gb[NB];
#pragma unroll
    for (int q = 0; q < NA; ++q) {
        const int r = UG_RPI * (NA * w + q) + lrow;
        ga[q] = L + (int64_t)(row0 + min(r, rows_avail - 1)) * np + 4 * spiece;
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        const int r = UG_RPI * (NB * w + q) + lrow;
        gb[q] = U + (int64_t)(col0 + min(r, cols_avail - 1)) * np + 4 * spiece;
    }
    auto glds = [&](int kk, int buf) {
        if (UG_ABL == 2 || UG_ABL == 5) return;
#pragma unroll
        for (int q = 0; q < NA; ++q)
            __builtin_amdgcn_global_load_lds((ug_glb_t*)(ga[q] + kk),
                                             (ug_lds_t*)&sm.a[buf][UG_RPI * (NA * w + q)][0],
                                             16, 0, 0);
#pragma unroll
        for (int q = 0; q < NB; ++q)
            __builtin_amdgcn_global_load_lds((ug_glb_t*)(gb[q] + kk),
                                             (ug_lds_t*)&sm.b[buf][UG_RPI * (NB * w + q)][0],
                                             16, 0, 0);
    };

    f4_t acc[4][4];
#pragma unroll
    for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int bj = 0; bj < 4; ++bj) acc[bi][bj] = f4_t{0.f, 0.f, 0.f, 0.f};

    // fragment rows of this lane: A rows 64wr + 16x + r16, U rows 64wc + 16x + r16 (the swizzle
    // depends on r16 only); lane group kq owns pieces kq*NG .. kq*NG+NG-1 of the slice
    constexpr int NG = UG_PPR / 4;
    const int sw = UG_SW(r16);
    auto compute = [&](int cur) {
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int sl = ((NG * kq + g) ^ sw) * 4;
            f4_t fa[4], fb[4];
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                if (UG_ABL == 5) {
                    fa[x] = f4_t{1.f, 1.f, 1.f, (float)g};
                    fb[x] = f4_t{1.f, 1.f, (float)cur, 1.f};
                } else {
                    fa[x] = *reinterpret_cast<const f4_t*>(&sm.a[cur][64 * wr + 16 * x + r16][sl]);
                    fb[x] = *reinterpret_cast<const f4_t*>(&sm.b[cur][64 * wc + 16 * x + r16][sl]);
                }
            }
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int bi = 0; bi < 4; ++bi)
#pragma unroll
                    for (int bj = 0; bj < 4; ++bj)
                        acc[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[bi][t], fb[bj][t],
                                                                           acc[bi][bj], 0, 0, 0);
        }
    };
    const int ns = kend / UG_KS;
    glds(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < ns; ++s) {
        if (s + 1 < ns) glds((s + 1) * UG_KS, (s + 1) & 1);  // lands while slice s is multiplied
        if (active && UG_ABL != 1) compute(s & 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (!active) return;
    if (UG_ABL == 5) {  // ablation: no epilogue (every accumulator stays live)
        float z = 0.f;
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int bj = 0; bj < 4; ++bj)
                z += acc[bi][bj][0] + acc[bi][bj][1] + acc[bi][bj][2] + acc[bi][bj][3];
        if (z == 12345.f) partial[b] = (double)z;
        return;
    }

    double* pbuf = partial + b * pstride;
    const int cbase = col0 + 64 * wc + r16;
    if (h == nb) {  // output row np (= first row of this block) is g^T u_s
        if (kq == 0) {
#pragma unroll
            for (int bj = 0; bj < 4; ++bj)
                pbuf[(int64_t)nb * sp + cbase + 16 * bj] = (double)acc[0][bj][0];
        }
        return;
    }
#pragma unroll
    for (int bj = 0; bj < 4; ++bj) {
        double d = 0.0;
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int lr = 64 * wr + 16 * bi + 4 * kq + r;
                const float yv = sm.y[lr];
                if (yv != 0.f) {
                    const float f = sm.fp[lr] + acc[bi][bj][r];
                    d += (double)(log_ndtr_fast(yv * f) + 0.5f * sm.w[lr] * f * f);
                }
            }
        d += __shfl_xor(d, 16, 64);
        d += __shfl_xor(d, 32, 64);
        if (kq == 0) pbuf[(int64_t)h * sp + cbase + 16 * bj] = d;
    }
}

template <int WC>
static void launch_ugemm_wc(SlotSet S, const int64_t* slots, UPool P, const int64_t* ubufs,
                            const double* y, int n, int np, double* partial, int64_t pstride,
                            const int* status, int nchains, hipStream_t s) {
    static bool attr = false;
    const size_t lds = sizeof(UgSmem<WC>);
    if (!attr) {  // dynamic LDS above the default 64 KiB cap
        (void)hipFuncSetAttribute((const void*)k_ugemm<WC>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    const int nb = np / 64;
    const int nI = (nb + 2) / 2, nJ = (P.sp + 64 * WC - 1) / (64 * WC);
    const int total = nI * nJ * nchains;
    hipLaunchKernelGGL(k_ugemm<WC>, dim3(total), dim3(128 * WC), lds, s, S, slots, P, ubufs, y, n,
                       np, partial, pstride, status, nI, nJ, total);
}

void launch_ugemm(SlotSet S, const int64_t* slots, UPool P, const int64_t* ubufs,
                  const double* y, int n, int np, double* partial, int64_t pstride,
                  const int* status, int nchains, hipStream_t s) {
    if (P.sp <= 64)
        launch_ugemm_wc<1>(S, slots, P, ubufs, y, n, np, partial, pstride, status, nchains, s);
    else if (P.sp <= 128)
        launch_ugemm_wc<2>(S, slots, P, ubufs, y, n, np, partial, pstride, status, nchains, s);
    else
        launch_ugemm_wc<4>(S, slots, P, ubufs, y, n, np, partial, pstride, status, nchains, s);
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
        double v = cst - pb[(int64_t)nb * sp + s];
        for (int i = 0; i < nb; ++i) v += pb[(int64_t)i * sp + s];
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
            v = cst - pb[(int64_t)nb * sp + s];
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
    hipLaunchKernelGGL(k_lme, dim3(nchains), dim3(256), 0, s, partial, pstride, nb, S, sp, Sl,
                       slots, out, status);
}
