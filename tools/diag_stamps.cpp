// Diagnostic build: phase timestamps (s_memtime) of the 64x64 diagonal-tile kernel.
// hipcc --offload-arch=gfx950 -O3 -DAPM_DIAG_STAMPS -x hip tools/diag_stamps.cpp -o /tmp/diag
#include "../auxiliary-pm-mcmc_amd/csrc/chol.hip"
#include <cstdio>
#include <vector>
int main() {
    const int n = 64;
    std::vector<double> h(n * n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) h[i * n + j] = (i == j ? n : 0.0) + 1.0 / (1 + i + j);
    double *A, *Dinv, *ldet;
    int *act, *st;
    hipMalloc(&A, 8 * n * n); hipMalloc(&Dinv, 8 * n * n); hipMalloc(&ldet, 8);
    hipMalloc(&act, 4); hipMalloc(&st, 4);
    int one = 1, zero = 0;
    hipMemcpy(act, &one, 4, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        hipMemcpy(A, h.data(), 8 * n * n, hipMemcpyHostToDevice);
        hipMemcpy(st, &zero, 4, hipMemcpyHostToDevice);
        MatB M{A, n, n * n};
        launch_chol_diag(M, 0, Dinv, 4096, ldet, 1, Live{act, st}, 1, 1, nullptr);
        hipDeviceSynchronize();
        unsigned long long s[16];
        hipMemcpyFromSymbol(s, HIP_SYMBOL(g_diag_stamps), sizeof(s));
        printf("rep %d stamps (cycles @100MHz memtime?):", rep);
        for (int q = 0; q < 10; ++q) printf(" %llu", s[q]);
        printf("\n");
    }
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    for (int rep = 0; rep < 100; ++rep) {
        MatB M{A, n, n * n};
        hipMemcpyAsync(A, h.data(), 8 * n * n, hipMemcpyHostToDevice);
        launch_chol_diag(M, 0, Dinv, 4096, ldet, 1, Live{act, st}, 1, 1, nullptr);
    }
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("avg per (copy+diag) %.2f us\n", ms * 10);
    return 0;
}
