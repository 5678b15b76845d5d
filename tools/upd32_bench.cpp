// Microbenchmark of the Newton factorisation's rank-512 trailing update (k_chol_update32_t128,
// fp16x3 operands) at the stationary theta-call shape: 64 chains, N = 4096, the outer panel K's
// update of every tile column right of it (the appended right-hand-side row block included, as
// in chol_range32). Development tool: prints ms per launch, fp32-equivalent TFLOP/s (lower
// triangle, the bench's roofline accounting) and an output checksum (variants must match it).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip tools/upd32_bench.cpp -o tools/upd32.bin
//   tools/upd32.bin [chains=64] [K=0] [reps=10]
#include "../auxiliary-pm-mcmc_amd/csrc/chol32.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"

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
    const int np = 4096, nb = np / 64, outer = 8;
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
    auto launch = [&]() {
        launch_chol_update32_t128(M, k0, kc, dsl, (int)sl.size(), lv, chains, nullptr, fd, nb, h3,
                                  rhs);
    };
    // checksum of one launch from the pristine matrix
    hipMemcpy(A, A0, sizeof(float) * cs * chains, hipMemcpyDeviceToDevice);
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
    printf("K=%d chains=%d supertiles=%zu: %.4f ms/launch  %.1f TFLOP/s fp32-eq  sum %.9e hash "
           "%016llx\n", K, chains, sl.size(), ms / reps, fl / (ms / reps * 1e-3) / 1e12, sum, hsh);
    return 0;
}
