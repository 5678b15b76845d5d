// Development timing of the stand-alone diag kernel (64 chains); build with -DDIAG_SKIP=mask to
// drop phases (1: pivots, 2: 16x16 inverse, 4: panel+trailing, 8: off-diagonal inverse, 16: stores).
#define APM_TOOL_NO_SKEW
#include "../auxiliary-pm-mcmc_amd/csrc/chol.hip"
#include <cstdio>
#include <vector>
int main() {
    const int n = 64, B = 64;
    std::vector<double> M((size_t)B * n * n);
    for (int b = 0; b < B; ++b)
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) M[(size_t)b * n * n + i * n + j] = (i == j) ? 64.0 : 1.0 / (1 + i + j);
    double *dA, *dA0, *dD, *dl;
    int *act, *st;
    hipMalloc(&dA, 8 * M.size()); hipMalloc(&dA0, 8 * M.size()); hipMalloc(&dD, 8 * M.size()); hipMalloc(&dl, 8 * B * 4);
    hipMalloc(&act, 4 * B); hipMalloc(&st, 4 * B);
    std::vector<int> one(B, 1), zero(B, 0);
    hipMemcpy(act, one.data(), 4 * B, hipMemcpyHostToDevice);
    hipMemcpy(dA0, M.data(), 8 * M.size(), hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float best = 1e9;
    for (int rep = 0; rep < 20; ++rep) {
        hipMemcpy(dA, dA0, 8 * M.size(), hipMemcpyDeviceToDevice);
        hipMemcpy(st, zero.data(), 4 * B, hipMemcpyHostToDevice);
        hipEventRecord(e0);
        launch_chol_diag(MatB{dA, n, n * n}, 0, dD, n * n, dl, 4, Live{act, st}, 7, B, 0);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    printf("DIAG_SKIP=%d  diag kernel fp64 %.1f us (64 chains, best of 20)\n", DIAG_SKIP, best * 1e3);
    // the fp32 twin (the Newton matrix)
    std::vector<float> Mf(M.begin(), M.end());
    float *fA, *fA0, *fD;
    hipMalloc(&fA, 4 * Mf.size()); hipMalloc(&fA0, 4 * Mf.size()); hipMalloc(&fD, 4 * Mf.size());
    hipMemcpy(fA0, Mf.data(), 4 * Mf.size(), hipMemcpyHostToDevice);
    best = 1e9;
    for (int rep = 0; rep < 20; ++rep) {
        hipMemcpy(fA, fA0, 4 * Mf.size(), hipMemcpyDeviceToDevice);
        hipMemcpy(st, zero.data(), 4 * B, hipMemcpyHostToDevice);
        hipEventRecord(e0);
        launch_chol_diag32(MatF{fA, n, n * n}, 0, fD, n * n, dl, 4, Live{act, st}, 7, B, 0);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    printf("DIAG_SKIP=%d  diag kernel fp32 %.1f us (64 chains, best of 20)\n", DIAG_SKIP, best * 1e3);
    return 0;
}
