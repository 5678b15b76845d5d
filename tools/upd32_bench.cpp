// Microbenchmark of the Newton factorisation's rank-512 trailing update (k_chol_update32_t128,
// fp16x3 operands) at the stationary theta-call shape: 64 chains, N = 4096, the outer panel K's
// update of every tile column right of it (the appended right-hand-side row block included, as
// in chol_range32). Development tool: prints ms per launch, fp32-equivalent TFLOP/s (lower
// triangle, the bench's roofline accounting) and an output checksum (variants must match it).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip tools/upd32_bench.cpp -o tools/upd32.bin
//   tools/upd32.bin [chains=64] [K=0] [reps=10]
#define APM_TOOL_NO_SKEW
#include "../auxiliary-pm-mcmc_amd/csrc/chol32.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"

// the fp16x3 planes of panel columns [k0*64, k0*64 + 64kc) of rows < np (Planes16 layout)
__global__ void k_fill_planes(const float* A, int64_t ld, int64_t cs, int np, int k0, int kc,
                              Planes16 pl) {
    const int64_t n = (int64_t)np * 64 * kc;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (e >= n) return;
    const int r = (int)(e / (64 * kc)), col = (int)(e % (64 * kc));
    const float v = A[b * cs + (int64_t)r * ld + k0 * 64 + col];
    const _Float16 h = (_Float16)v, l = (_Float16)(v - (float)h);
    const int64_t o = b * pl.cstride + ((int64_t)(col >> 5) * pl.rows + r) * 32 + (col & 31);
    pl.base[o] = __builtin_bit_cast(unsigned short, h);
    pl.base[o + pl.lo] = __builtin_bit_cast(unsigned short, l);
}

static double upd_flops(int i0, int R, int j0, int jend, int kc) {
    double f = 0.0;
    for (int i = i0; i < R; ++i)
        for (int j = j0; j <= std::min(i, jend - 1); ++j)
            f += (i == j) ? 64.0 * 65.0 * 64.0 * kc : 2.0 * 64.0 * 64.0 * 64.0 * kc;
    return f;
}

int main(int argc, char** argv) {
    const int chains = argc > 1 ? atoi(argv[1]) : 64, K = argc > 2 ? atoi(argv[2]) : 0;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    // UPD_OUTER: the outer panel width in tiles (8 in the library; 16 measures what 1024-wide
    // panels would give the trailing update: half the old-tile passes per unit of depth)
    const int np = 4096, nb = np / 64, outer = getenv("UPD_OUTER") ? atoi(getenv("UPD_OUTER")) : 8;
    const int64_t ld = np, cs = (int64_t)(np + 64) * np;
    float* A;
    hipMalloc(&A, sizeof(float) * cs * chains);
    float* A0;
    hipMalloc(&A0, sizeof(float) * cs * chains);
    std::vector<float> h((size_t)cs);
    // a private generator: libc rand() is shared with the HIP runtime's threads, which made the
    // input (and so the checksum) differ from process to process
    uint64_t lcg = 7;
    auto rnd = [&]() {
        lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
        return (double)(lcg >> 11) * (1.0 / 9007199254740992.0);
    };
    for (int b = 0; b < chains; ++b) {
        for (int64_t e = 0; e < cs; ++e) {
            const int64_t r = e / ld;
            h[e] = (r >= np && r != np) ? 0.f : (float)((rnd() - 0.5) * 2.0);
        }
        hipMemcpy(A0 + b * cs, h.data(), sizeof(float) * cs, hipMemcpyHostToDevice);
    }
    int *act, *st, *h3;
    hipMalloc(&act, 4 * chains);
    hipMalloc(&st, 4 * chains);
    hipMalloc(&h3, 4 * chains);
    std::vector<int> one(chains, 1), zero(chains, 0);
    hipMemcpy(act, one.data(), 4 * chains, hipMemcpyHostToDevice);
    hipMemcpy(st, zero.data(), 4 * chains, hipMemcpyHostToDevice);
    hipMemcpy(h3, one.data(), 4 * chains, hipMemcpyHostToDevice);
    const int k0 = K * outer, kc = outer, Kend = k0 + kc, R = nb + 1, rhs = nb;
    std::vector<unsigned> sl = build_update_supertiles(Kend, R, Kend, nb, 0, 0, rhs);
    unsigned* dsl;
    hipMalloc(&dsl, sizeof(unsigned) * sl.size());
    hipMemcpy(dsl, sl.data(), sizeof(unsigned) * sl.size(), hipMemcpyHostToDevice);
    const MatF M{A, ld, cs};
    const Live lv{act, st};
    const FusedDiag<float> fd{0, nullptr, 0, nullptr, 0, 0};
    // UPD_PLANES=1: operands from fp16x3 planes (filled from the pristine matrix before each
    // checked launch; the timed launches reuse them) - the checksum must equal the split path's
    Planes16 pl{nullptr, 0, 0, 0};
    const char* pe = getenv("UPD_PLANES");
    if (pe && atoi(pe)) {
        const int64_t pcs = (int64_t)2 * np * 64 * kc;
        hipMalloc(&pl.base, sizeof(unsigned short) * pcs * chains);
        pl = Planes16{pl.base, pcs, pcs / 2, np};
    }
    auto fill = [&]() {
        if (!pl.base) return;
        hipLaunchKernelGGL(k_fill_planes, dim3((unsigned)(((int64_t)np * 64 * kc + 255) / 256), chains),
                           dim3(256), 0, 0, A0, ld, cs, np, k0, kc, pl);
    };
    // UPD_Q256=1 (with UPD_PLANES=1): 256x256 quad tiles for the rows above the right-hand side,
    // the 128-row kernel for that row alone
    const char* qe = getenv("UPD_Q256");
    const bool q256 = qe && atoi(qe) && pl.base;
    std::vector<unsigned> ql = build_update_quads(Kend, nb, Kend, nb);
    std::vector<unsigned> rl = build_update_supertiles(nb, R, Kend, nb, 0, 0, rhs);
    unsigned *dql, *drl;
    hipMalloc(&dql, sizeof(unsigned) * ql.size());
    hipMemcpy(dql, ql.data(), sizeof(unsigned) * ql.size(), hipMemcpyHostToDevice);
    hipMalloc(&drl, sizeof(unsigned) * rl.size());
    hipMemcpy(drl, rl.data(), sizeof(unsigned) * rl.size(), hipMemcpyHostToDevice);
    auto launch = [&]() {
        if (q256) {
            launch_chol_update32_q256(M, k0, kc, dql, (int)ql.size(), lv, chains, nullptr, h3, pl);
            launch_chol_update32_t128(M, k0, kc, drl, (int)rl.size(), lv, chains, nullptr, fd, nb,
                                      h3, rhs, 0, pl);
        } else {
            launch_chol_update32_t128(M, k0, kc, dsl, (int)sl.size(), lv, chains, nullptr, fd, nb,
                                      h3, rhs, 0, pl);
        }
    };
    // checksum of one launch from the pristine matrix
    hipMemcpy(A, A0, sizeof(float) * cs * chains, hipMemcpyDeviceToDevice);
    fill();
    launch();
    hipDeviceSynchronize();
    std::vector<float> out((size_t)cs);
    double sum = 0.0;
    unsigned long long hsh = 1469598103934665603ull;
    for (int b = 0; b < chains; b += std::max(1, chains / 4)) {
        hipMemcpy(out.data(), A + b * cs, sizeof(float) * cs, hipMemcpyDeviceToHost);
        for (int64_t e = 0; e < cs; ++e) {
            sum += std::fabs((double)out[e]);
            unsigned u;
            std::memcpy(&u, &out[e], 4);
            hsh = (hsh ^ u) * 1099511628211ull;
        }
    }
    if (argc > 4) {  // determinism check: launch again from the pristine matrix, compare all
        std::vector<float> first((size_t)cs * chains), second((size_t)cs * chains);
        hipMemcpy(first.data(), A, sizeof(float) * cs * chains, hipMemcpyDeviceToHost);
        hipMemcpy(A, A0, sizeof(float) * cs * chains, hipMemcpyDeviceToDevice);
        launch();
        hipDeviceSynchronize();
        hipMemcpy(second.data(), A, sizeof(float) * cs * chains, hipMemcpyDeviceToHost);
        long nd = 0;
        for (int64_t e = 0; e < cs * chains; ++e)
            if (std::memcmp(&first[e], &second[e], 4)) {
                if (nd < 12) {
                    const int64_t b = e / cs, r = (e % cs) / ld, c = e % ld;
                    printf("  differs: chain %ld row %ld col %ld (tile %ld, %ld): %.9g vs %.9g\n",
                           (long)b, (long)r, (long)c, (long)(r / 64), (long)(c / 64), first[e],
                           second[e]);
                }
                ++nd;
            }
        printf("determinism: %ld of %ld elements differ between two launches\n", nd,
               (long)(cs * chains));
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 2; ++w) launch();
    hipEventRecord(e0, nullptr);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(e1, nullptr);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double fl = upd_flops(Kend, R - 1, Kend, nb, kc) * chains;  // (rhs row: not credited)
    printf("%sK=%d chains=%d supertiles=%zu: %.4f ms/launch  %.1f TFLOP/s fp32-eq  sum %.9e hash "
           "%016llx\n", q256 ? "q256 " : pl.base ? "planes " : "", K, chains, sl.size(), ms / reps, fl / (ms / reps * 1e-3) / 1e12, sum, hsh);
    return 0;
}
