// fp64 trailing updates of the Cholesky factorisations on int8 MFMA, exactly (Ozaki scheme II:
// Ozaki, Uchino, Imamura, "Ozaki Scheme II: A GEMM-oriented emulation of floating-point matrix
// multiplication using an integer modular technique", 2024).
//
// C -= A B^T (or C += A B^T) for the 128x128 super-tiles of k_chol_update_t128 (chol.hip), where
// A and B are rows of one fp64 panel L[:, k0*64 : (k0+kc)*64]:
//   1. split (k_oz_split, once per panel): row r is scaled by 2^E_r so that its largest entry
//      lies in [2^(beta-1), 2^beta) and rounded to integers x_rk (|x| <= 2^beta <= 2^53, exact
//      in fp64: the only rounding of the scheme, 2^-beta relative to the row's largest entry);
//      x is stored as its residues modulo NM pairwise coprime moduli m_i <= 256 (int8 planes).
//   2. update (k_oz_update_t128): for each modulus, P_i = sum_k r_i(x_a) r_i(x_b) on
//      v_mfma_i32_16x16x64_i8 - exact in int32 (|P| < depth * 128^2 = 2^23 for depth 512);
//      the integer product X = sum_k x_a x_b (|X| < depth * 2^(2 beta) < M / 2, M = prod m_i) is
//      the unique CRT solution: X / M = frac(sum_i t_i y_i / m_i), t_i = P_i mod m_i,
//      y_i = (M / m_i)^-1 mod m_i. The fraction is accumulated exactly in fp64 (weights y_i / m_i
//      split into a 40-bit head, exact products and sums, and a tail), so X comes out with
//      fp64 relative precision; C +-= X 2^-(E_a + E_b).
// The result equals the exact product of the rounded operands, i.e. differs from fp64 GEMM only
// by the operand rounding at 2^-beta of each row's maximum (fp64 GEMM: k * 2^-53 of the summed
// magnitudes). 15 moduli (log2 M = 118.57) give beta = 53 at depth 512.
// Work: NM int8 GEMMs at 2048 ops/clk/SIMD (64x the f64 MFMA rate) + ~7 VALU ops per output
// element and modulus.
#include <cmath>
#include <vector>

#include "apm_internal.h"
#include "diag.h"

typedef int i4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

struct OzConst {
    float m[OZ_NM];
    float minv[OZ_NM];
    double dm[OZ_NM];
    double whi[OZ_NM], wlo[OZ_NM];
    double M, log2M;
};
__constant__ OzConst ozc;

static const int kOzModuli[OZ_NM] = {256, 255, 253, 251, 247, 241, 239, 233,
                                     229, 227, 223, 211, 199, 197, 193};

static OzConst oz_host_consts() {
    OzConst c{};
    double M = 1.0, l2 = 0.0;
    for (int i = 0; i < OZ_NM; ++i) {
        M *= kOzModuli[i];
        l2 += std::log2((double)kOzModuli[i]);
    }
    for (int i = 0; i < OZ_NM; ++i) {
        const int m = kOzModuli[i];
        long Mi = 1;  // (M / m_i) mod m_i
        for (int j = 0; j < OZ_NM; ++j)
            if (j != i) Mi = (Mi * (kOzModuli[j] % m)) % m;
        int y = 1;  // Mi^-1 mod m (m is small: search)
        while ((Mi * y) % m != 1) ++y;
        const double w = (double)y / m;
        const double whi = std::floor(w * 1099511627776.0) / 1099511627776.0;  // 40 fraction bits
        c.m[i] = (float)m;
        c.minv[i] = 1.0f / (float)m;
        c.dm[i] = (double)m;
        c.whi[i] = whi;
        c.wlo[i] = ((double)y - (double)m * whi) / (double)m;  // (y - m whi) exact, / m rounded
    }
    c.M = M;
    c.log2M = l2;
    return c;
}

double oz_log2M() {
    static const double l2 = oz_host_consts().log2M;
    return l2;
}

// largest beta with depth * 2^(2 beta) < M / 2 (margin 1/4 bit), at most 53 (x exact in fp64)
int oz_beta(int depth) {
    const double b = std::floor((oz_log2M() - 1.25 - std::log2((double)depth)) / 2.0);
    return (int)std::min(53.0, b);
}

hipError_t oz_init_device() {
    static const OzConst c = oz_host_consts();
    return hipMemcpyToSymbol(HIP_SYMBOL(ozc), &c, sizeof(c));
}

// ------------------------------------------------------------------------------------- split
// One wave per panel row: rows [row0, row0 + nrows) of A, columns [col0, col0 + depth) (depth a
// multiple of 64); lane l takes columns 8l + 512j .. +7 (one 8-byte store per plane).
#define OZ_EXP_BAD (-100000)
__global__ __launch_bounds__(256) void k_oz_split(MatB A, int row0, int nrows, int col0, int depth,
                                                  OzPlanes P, int beta, Live live) {
    const int b = blockIdx.y;
    if (!(live.active[b] != 0 && live.status[b] == 0)) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * 4 + w;
    if (r >= nrows) return;
    const double* src = A.base + b * A.cstride + (int64_t)(row0 + r) * A.ld + col0;
    const int nj = (depth + 511) / 512;
    double mx = 0.0;
    for (int j = 0; j < nj; ++j) {
        const int c0 = 512 * j + 8 * lane;
        if (c0 < depth)
#pragma unroll
            for (int e = 0; e < 8; ++e) mx = fmax(mx, fabs(src[c0 + e]));
    }
    mx = wave_max_d(mx);
    int ex = 0;
    const bool bad = !isfinite(mx);
    if (mx > 0.0 && !bad) {
        frexp(mx, &ex);  // mx < 2^ex
        ex = beta - ex;  // |x| = |v| 2^ex < 2^beta
    }
    int8_t* pl = P.base + b * P.cstride + (int64_t)(row0 + r - P.row0) * depth;
    if (lane == 0) P.exps[b * P.estride + row0 + r - P.row0] = bad ? OZ_EXP_BAD : ex;
    for (int j = 0; j < nj; ++j) {
        const int c0 = 512 * j + 8 * lane;
        if (c0 >= depth) break;
        double x[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = bad ? 0.0 : rint(ldexp(src[c0 + e], ex));
#pragma unroll
        for (int i = 0; i < OZ_NM; ++i) {
            const double m = ozc.dm[i], mh = 0.5 * m;
            uint64_t packed = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const double q = rint(x[e] * (1.0 / m));
                double t = fma(-q, m, x[e]);  // exact: |q m| <= 2^53
                // symmetric residue: [-m/2, m/2) for even m, [-(m-1)/2, (m-1)/2] for odd m
                if (t >= mh) t -= m;
                if (t < -mh) t += m;
                packed |= (uint64_t)(uint8_t)(int8_t)(int)t << (8 * e);
            }
            *reinterpret_cast<uint64_t*>(pl + (int64_t)i * P.mstride + c0) = packed;
        }
    }
}

void launch_oz_split(MatB A, int row0, int nrows, int col0, int depth, OzPlanes P, int beta,
                     Live live, int nchains, hipStream_t s) {
    if (nrows <= 0) return;
    hipLaunchKernelGGL(k_oz_split, dim3((nrows + 3) / 4, nchains), dim3(256), 0, s, A, row0,
                       nrows, col0, depth, P, beta, live);
}

// ------------------------------------------------------------------------------------ update
// v_mfma_i32_16x16x64_i8: lane l holds A[row l&15][k 16(l>>4) .. +15] and B[k ..][col l&15]
// (16 bytes each); C/D lane l, reg r -> (row 4(l>>4) + r, col l&15).
// One pipeline step stages a 256-deep chunk of one modulus's planes (4 MFMA k-steps): LDS image
// per operand and buffer 128 rows x 256 bytes, piece p (16 bytes) of row r at slot p ^ (r & 15),
// so that the 16-byte fragment reads of each ds_read_b128 lane group hit 16 distinct bank groups.
#define OZ_KB 256
struct __attribute__((aligned(16))) OzSmem {
    int8_t a[2][128][OZ_KB];
    int8_t b[2][128][OZ_KB];
};
#define OZ_CROW(l, r) (4 * ((l) >> 4) + (r))

__device__ __forceinline__ int oz_slot(int row, int piece) { return piece ^ (row & 15); }

// t = P mod m (|t| < 1.5 m, exact in fp32 for |P| < 2^24) into the exact CRT head and the tail
__device__ __forceinline__ void oz_crt(const int p_i, float m, float minv, double whi, double wlo,
                                       double& shi, double& slo) {
    const float p = (float)p_i;
    const float t = fmaf(-rintf(p * minv), m, p);
    const double td = (double)t;
    shi = fma(td, whi, shi);
    slo = fma(td, wlo, slo);
}

// 8 waves per 128x128 super-tile: wave (wr, wc) = (wv >> 2, wv & 3) owns rows 64 wr .. +63 and
// columns 32 wc .. +31 (4 x 2 blocks of 16 x 16): its CRT sums (2 x 32 doubles per lane) and two
// sets of int32 accumulators fit 2 waves per SIMD. The CRT step of modulus i runs interleaved
// with the MFMAs of modulus i + 1 (accumulators `pend` / `acc`), so VALU and MFMA overlap.
template <bool NEG>
__device__ __forceinline__ void oz_update_body(MatB A, OzPlanes P, int depth, unsigned e, int b,
                                               bool fused, Live live, FusedDiag<double> fd,
                                               OzSmem& smg, DiagSmem& smd) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wr = wv >> 2, wc = wv & 3;
    const int r16 = lane & 15, kq = lane >> 4;
    const int ti = (int)(e >> 18), tj = (int)((e >> 4) & 0x3fff);
    const bool rv0 = e & 1u, rv1 = e & 2u, cv0 = e & 4u, cv1 = e & 8u;
    const int ra0 = rv0 ? ti : ti + 1, ra1 = rv1 ? ti + 1 : ti;
    const int cb0 = cv0 ? tj : tj + 1, cb1 = cv1 ? tj + 1 : tj;
    double* Ab = A.base + b * A.cstride;
    const int ch = wc >> 1, hc = 32 * (wc & 1);  // column tile half and offset inside it
    const int oi = ti + wr, oj = tj + ch;
    const bool mine = (wr ? rv1 : rv0) && (ch ? cv1 : cv0) && oj <= oi;

    // LDS-DMA: wave wv moves rows 16wv .. 16wv+15 of both operands (4 instructions of 4 rows x
    // 256 B each); lane l lands at row +4q + l/16, slot l%16, so it loads piece (l%16) ^ row%16
    const int8_t* pb = P.base + b * P.cstride;
    // rows 16 wv .. +15 lie in one operand half (wv < 4: the first); row 16 wv + 4q + l/16
    const int rbase = 16 * wv + (lane >> 4);
    const int8_t* ga = pb + (int64_t)((wv < 4 ? ra0 : ra1) * 64 - P.row0 + (rbase & 63)) * depth;
    const int8_t* gbp = pb + (int64_t)((wv < 4 ? cb0 : cb1) * 64 - P.row0 + (rbase & 63)) * depth;
    const int nch = depth / OZ_KB;  // steps per modulus (depth: a multiple of 256 here)
    const int nsteps = OZ_NM * nch;
    auto glds = [&](int s, int buf) {
        const int i = s / nch, c = s - i * nch;
        const int64_t o = (int64_t)i * P.mstride + OZ_KB * c;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int piece = (lane & 15) ^ ((rbase + 4 * q) & 15);
            const int64_t oq = o + (int64_t)(4 * q) * depth + 16 * piece;
            __builtin_amdgcn_global_load_lds((glb_void_t*)(ga + oq),
                                             (lds_void_t*)&smg.a[buf][16 * wv + 4 * q][0], 16, 0, 0);
            __builtin_amdgcn_global_load_lds((glb_void_t*)(gbp + oq),
                                             (lds_void_t*)&smg.b[buf][16 * wv + 4 * q][0], 16, 0, 0);
        }
    };
    i4_t acc[4][2], pend[4][2];
    double shi[4][2][4], slo[4][2][4];
#pragma unroll
    for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) {
            acc[bi][bj] = pend[bi][bj] = i4_t{0, 0, 0, 0};
#pragma unroll
            for (int r = 0; r < 4; ++r) shi[bi][bj][r] = slo[bi][bj][r] = 0.0;
        }
    int pend_i = -1;  // modulus whose sums wait in `pend`
    glds(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        const int cur = s & 1;
        if (s + 1 < nsteps) glds(s + 1, cur ^ 1);
        const int i = s / nch;
        if (mine) {
            const bool do_crt = pend_i >= 0;
            float m = 0.f, minv = 0.f;
            double whi = 0.0, wlo = 0.0;
            if (do_crt) {
                m = ozc.m[pend_i];
                minv = ozc.minv[pend_i];
                whi = ozc.whi[pend_i];
                wlo = ozc.wlo[pend_i];
            }
#pragma unroll
            for (int kk = 0; kk < OZ_KB / 64; ++kk) {
                i4_t af[4], bf[2];
#pragma unroll
                for (int bi = 0; bi < 4; ++bi) {
                    const int row = 64 * wr + 16 * bi + r16;
                    af[bi] = *reinterpret_cast<const i4_t*>(
                        &smg.a[cur][row][16 * oz_slot(row, 4 * kk + kq)]);
                }
#pragma unroll
                for (int bj = 0; bj < 2; ++bj) {
                    const int row = 64 * ch + hc + 16 * bj + r16;
                    bf[bj] = *reinterpret_cast<const i4_t*>(
                        &smg.b[cur][row][16 * oz_slot(row, 4 * kk + kq)]);
                }
#pragma unroll
                for (int bi = 0; bi < 4; ++bi)
#pragma unroll
                    for (int bj = 0; bj < 2; ++bj) {
                        acc[bi][bj] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[bi], bf[bj],
                                                                           acc[bi][bj], 0, 0, 0);
                        // a quarter of the previous modulus's CRT per k-step, between the MFMAs
                        if (do_crt && (bi >> 1) == (kk >> 1) && (bi & 1) == (kk & 1))
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                oz_crt(pend[bi][bj][r], m, minv, whi, wlo, shi[bi][bj][r],
                                       slo[bi][bj][r]);
                    }
            }
            if (do_crt && nch > 0) pend_i = -1;
            if (s - i * nch == nch - 1) {  // modulus i complete: its sums wait for the next step
#pragma unroll
                for (int bi = 0; bi < 4; ++bi)
#pragma unroll
                    for (int bj = 0; bj < 2; ++bj) {
                        pend[bi][bj] = acc[bi][bj];
                        acc[bi][bj] = i4_t{0, 0, 0, 0};
                    }
                pend_i = i;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (mine && pend_i >= 0) {  // the last modulus
        const float m = ozc.m[pend_i], minv = ozc.minv[pend_i];
        const double whi = ozc.whi[pend_i], wlo = ozc.wlo[pend_i];
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    oz_crt(pend[bi][bj][r], m, minv, whi, wlo, shi[bi][bj][r], slo[bi][bj][r]);
    }
    // X = M frac(S), C +-= X 2^-(E_row + E_col); the result overwrites the CRT sums in place
    const int* ex = P.exps + b * P.estride;
    const double* Cw = Ab + (int64_t)(oi * 64) * A.ld + oj * 64 + hc;
    if (mine) {
#pragma unroll
        for (int bi = 0; bi < 4; ++bi) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * bi + OZ_CROW(lane, r);
                const int er = ex[oi * 64 + row - P.row0];
#pragma unroll
                for (int bj = 0; bj < 2; ++bj) {
                    const int col = 16 * bj + r16;
                    const int ec = ex[oj * 64 + hc + col - P.row0];
                    const double sh = shi[bi][bj][r];
                    const double fr = (sh - rint(sh)) + slo[bi][bj][r];
                    double d = ldexp(fr * ozc.M, -(er + ec));
                    if (er == OZ_EXP_BAD || ec == OZ_EXP_BAD) d = NAN;
                    const double old = Cw[(int64_t)row * A.ld + col];
                    shi[bi][bj][r] = NEG ? old - d : old + d;
                }
            }
        }
    }
    double* Cout = Ab + (int64_t)(oi * 64) * A.ld + oj * 64 + hc;
    const bool diag_here = fused && wr == 0 && ch == 0;  // the (d, d) tile: through the diag step
    if (mine && !diag_here) {
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    Cout[(int64_t)(16 * bi + OZ_CROW(lane, r)) * A.ld + 16 * bj + r16] =
                        shi[bi][bj][r];
    }
    if (!fused) return;
    if (diag_here) {
#pragma unroll
        for (int bi = 0; bi < 4; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    smd.T[(16 * bi + OZ_CROW(lane, r)) * DP + hc + 16 * bj + r16] = shi[bi][bj][r];
    }
    __syncthreads();
    if (wv == 0) {
        const bool ok = diag_compute<false>(smd, lane);
        if (lane == 0) smd.ok = ok;
    }
    __syncthreads();
    if (!smd.ok) {
        if (tid == 0) live.status[b] = fd.fail_code;
        return;
    }
    diag_store<double>(smd, Ab + (int64_t)(ti * 64) * A.ld + tj * 64, A.ld,
                       fd.Dinv + b * fd.dstride + (int64_t)ti * 4096, fd.ldet + b * fd.lstride + ti,
                       tid, 512);
}

__device__ __forceinline__ long oz_xcd_remap(long L, long total) {
    const long xcd = L & 7, q = total >> 3, r = total & 7;
    const long base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (L >> 3);
}

__global__ __launch_bounds__(512, 1) void k_oz_update_t128(MatB A, OzPlanes P, int depth,
                                                           const unsigned* __restrict__ tiles,
                                                           int ntiles, int nchains, int plus,
                                                           Live live, FusedDiag<double> fd) {
    __shared__ union {
        OzSmem g;
        DiagSmem d;
    } sm;
    int b, t;
    const bool fused = fd.enabled && (int)blockIdx.x < nchains;
    if (fused) {
        b = blockIdx.x;
        t = 0;
    } else {
        const int nt = fd.enabled ? ntiles - 1 : ntiles;
        const long L = (long)blockIdx.x - (fd.enabled ? nchains : 0);
        const long w = oz_xcd_remap(L, (long)nt * nchains);
        b = (int)(w / nt);
        t = (int)(w % nt) + (fd.enabled ? 1 : 0);
    }
    if (!(live.active[b] != 0 && live.status[b] == 0)) return;
    if (plus)
        oz_update_body<false>(A, P, depth, tiles[t], b, fused, live, fd, sm.g, sm.d);
    else
        oz_update_body<true>(A, P, depth, tiles[t], b, fused, live, fd, sm.g, sm.d);
}

void launch_oz_update_t128(MatB A, OzPlanes P, int depth, const unsigned* tiles, int ntiles,
                           int plus, Live live, int nchains, hipStream_t s, FusedDiag<double> fd) {
    if (ntiles <= 0) return;
    const long total = (long)ntiles * nchains;
    hipLaunchKernelGGL(k_oz_update_t128, dim3((unsigned)total), dim3(512), 0, s, A, P, depth,
                       tiles, ntiles, nchains, plus, live, fd);
}
