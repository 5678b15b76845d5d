// Microbenchmark of the L.U kernel k_ugemm (128x256 tile per workgroup) on random data at the
// bench shape (N=4096, S=256, 64 chains). Development tool; ablations:
// -DUG_ABL=1 no MFMA, =2 no global loads, =3 operands always slice 0 (cache resident).
// hipcc --offload-arch=gfx950 -O3 -x hip tools/ugemm_bench.cpp -o tools/ugemm.bin
#include "../auxiliary-pm-mcmc_amd/csrc/ugemm.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

__global__ void fillf(float* p, size_t n, unsigned seed, float sc) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = ((float)(x & 0xffffff) / 16777216.0f - 0.5f) * sc;
    }
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096, S = argc > 2 ? atoi(argv[2]) : 256;
    const int chains = argc > 3 ? atoi(argv[3]) : 64;
    const int np = (n + 63) / 64 * 64, sp = (S + 63) / 64 * 64;
    SlotSet Sl{};
    Sl.lstride = (int64_t)(np + 64) * np;
    Sl.vstride = np;
    hipMalloc(&Sl.L, sizeof(float) * Sl.lstride * chains);
    hipMalloc(&Sl.fpost, sizeof(float) * np * chains);
    hipMalloc(&Sl.W, sizeof(float) * np * chains);
    hipMalloc(&Sl.cst, sizeof(double) * chains);
    UPool P{};
    P.sp = sp;
    P.stride = (int64_t)np * sp;
    hipMalloc(&P.base, sizeof(float) * P.stride * chains);
    fillf<<<4096, 256>>>(Sl.L, Sl.lstride * chains, 3u, 0.05f);
    fillf<<<4096, 256>>>(P.base, P.stride * chains, 5u, 2.0f);
    fillf<<<256, 256>>>(Sl.fpost, (size_t)np * chains, 7u, 1.0f);
    fillf<<<256, 256>>>(Sl.W, (size_t)np * chains, 9u, 0.5f);
    std::vector<double> yh(np, 0.0);
    for (int i = 0; i < n; ++i) yh[i] = (i % 3) ? 1.0 : -1.0;
    double* y;
    hipMalloc(&y, sizeof(double) * np);
    hipMemcpy(y, yh.data(), sizeof(double) * np, hipMemcpyHostToDevice);
    std::vector<int64_t> ids(chains);
    for (int b = 0; b < chains; ++b) ids[b] = b;
    int64_t* dids;
    hipMalloc(&dids, sizeof(int64_t) * chains);
    hipMemcpy(dids, ids.data(), sizeof(int64_t) * chains, hipMemcpyHostToDevice);
    int* st;
    hipMalloc(&st, sizeof(int) * chains);
    hipMemset(st, 0, sizeof(int) * chains);
    const int64_t ps = (int64_t)(np / 64 + 1) * sp;
    double* part;
    hipMalloc(&part, sizeof(double) * ps * chains);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double fl = (double)n * (n + 1) * S * chains;
    {
        auto run = [&]() { launch_ugemm(Sl, dids, P, dids, y, n, np, part, ps, st, chains, 0); };
        for (int w = 0; w < 2; ++w) run();
        const int reps = 10;
        hipEventRecord(e0);
        for (int w = 0; w < reps; ++w) run();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("ABL=%d KS=%d 128x256 N=%d S=%d chains=%d: %8.3f ms/launch %7.2f TFLOP/s (algorithmic)\n",
               UG_ABL, UG_KS, n, S, chains, ms / reps,
               fl / (ms / reps * 1e-3) / 1e12);
    }
    return 0;
}
