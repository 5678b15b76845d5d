// Microbenchmark of the Gram builder (k_gram) at the theta-call shape (N=4096, D=32, 64 chains,
// lower tiles only, K2 copy of the first 8 tile columns) - development tool. Ablations:
// -DGRAM_ABL=1 no exp, =2 no stores, =3 no distance loop.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip tools/gram_bench.cpp -o tools/gram.bin
#define APM_TOOL_NO_SKEW
#include "../auxiliary-pm-mcmc_amd/csrc/gram.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"

int main(int argc, char** argv) {
    const int n = 4096, d = argc > 2 ? atoi(argv[2]) : 32, chains = argc > 1 ? atoi(argv[1]) : 64;
    const int np = n, nb = np / 64, P = d + 1;
    const int64_t cs = (int64_t)np * np;
    double *K, *K2, *X, *th;
    hipMalloc(&K, sizeof(double) * cs * chains);
    hipMalloc(&K2, sizeof(double) * cs * chains);
    hipMalloc(&X, sizeof(double) * n * d);
    hipMalloc(&th, sizeof(double) * P * chains);
    std::vector<double> hx((size_t)n * d), ht((size_t)P * chains);
    srand(1);
    for (auto& v : hx) v = (rand() / (double)RAND_MAX - 0.5) * 3.0;
    for (int b = 0; b < chains; ++b)
        for (int k = 0; k < P; ++k) ht[b * P + k] = k == 0 ? 0.0 : 1.7 + 0.01 * k;
    hipMemcpy(X, hx.data(), sizeof(double) * hx.size(), hipMemcpyHostToDevice);
    hipMemcpy(th, ht.data(), sizeof(double) * ht.size(), hipMemcpyHostToDevice);
    int *act, *st;
    hipMalloc(&act, 4 * chains); hipMalloc(&st, 4 * chains);
    std::vector<int> one(chains, 1), zero(chains, 0);
    hipMemcpy(act, one.data(), 4 * chains, hipMemcpyHostToDevice);
    hipMemcpy(st, zero.data(), 4 * chains, hipMemcpyHostToDevice);
    MatB MK{K, np, cs}, MK2{K2, np, cs};
    Live lv{act, st};
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int k2c[2] = {8, 0};
    std::vector<double> Kh[2];
    for (int mf = 0; mf < 2; ++mf)
    for (int v = 0; v < 2; ++v) {
        for (int w = 0; w < 3; ++w)
            launch_gram(MK, X, d, n, d, th, P, 1, 1e-8, np, lv, chains, 0, false,
                        k2c[v] ? MK2 : MatB{nullptr, 0, 0}, k2c[v], mf);
        hipEventRecord(e0, 0);
        const int reps = 10;
        for (int r = 0; r < reps; ++r)
            launch_gram(MK, X, d, n, d, th, P, 1, 1e-8, np, lv, chains, 0, false,
                        k2c[v] ? MK2 : MatB{nullptr, 0, 0}, k2c[v], mf);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        const double bytes = 8.0 * ((double)n * (n + 1) / 2) * chains;
        printf("%s ABL=%d k2cols=%d chains=%d d=%d: %.3f ms  %.2f TB/s (lower-tile bytes)\n",
               mf ? "k_gram_mfma" : "k_gram     ", GRAM_ABL, k2c[v], chains, d, ms,
               bytes / (ms * 1e-3) / 1e12);
        if (v == 0) {  // last chain's K: GEMM form vs direct form (lower triangle)
            Kh[mf].resize((size_t)cs);
            hipMemcpy(Kh[mf].data(), K + (chains - 1) * cs, sizeof(double) * cs,
                      hipMemcpyDeviceToHost);
        }
    }
    double worst = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            const double a = Kh[1][(size_t)i * np + j], r = Kh[0][(size_t)i * np + j];
            const double sc = fmax(1.0, fabs(log(fmax(r, 1e-300))));
            worst = fmax(worst, fabs(a - r) / (sc * fabs(r) + 1e-300));
        }
    printf("GEMM form vs direct form: max |dK| / (K max(1, |log K|)) = %.3g\n", worst);
    return 0;
}
