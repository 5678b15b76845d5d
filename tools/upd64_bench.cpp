// Microbenchmark of the fp64 128x128 trailing update (k_chol_update_t128) on random data at the
// chol(K) shape of N=4096 (development tool). Ablations: -DT64_ABL=1 no MFMA, =2 no operand loads.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip tools/upd64_bench.cpp \
//     auxiliary-pm-mcmc_amd/build/chol32.hip.o -o tools/upd64.bin
#define APM_TOOL_NO_SKEW
#include "../auxiliary-pm-mcmc_amd/csrc/chol.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"

__global__ void filld(double* p, size_t n, unsigned seed) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = ((double)(x & 0xffffff) / 16777216.0 - 0.5) * 0.01;
    }
}

static double flops_of(int i0, int R, int j0, int jend, int kc) {
    double f = 0;
    for (int i = i0; i < R; ++i)
        for (int j = j0; j <= std::min(i, jend - 1); ++j)
            f += (i == j) ? 64.0 * 65 * 64 * kc : 2.0 * 64 * 64 * 64 * kc;
    return f;
}

int main(int argc, char** argv) {
    const int nb = 64, chains = argc > 1 ? atoi(argv[1]) : 64;
    const int R = nb, Cb = nb;
    const int64_t ld = 64 * nb, rows = 64 * (nb + 1);
    const int64_t cs = rows * ld;
    double* A;
    if (hipMalloc(&A, sizeof(double) * cs * chains) != hipSuccess) { printf("oom\n"); return 1; }
    filld<<<4096, 256>>>(A, (size_t)cs * chains, 7u);
    int *act, *st;
    hipMalloc(&act, 4 * chains); hipMalloc(&st, 4 * chains);
    std::vector<int> one(chains, 1), zero(chains, 0);
    hipMemcpy(act, one.data(), 4 * chains, hipMemcpyHostToDevice);
    hipMemcpy(st, zero.data(), 4 * chains, hipMemcpyHostToDevice);
    MatB M{A, ld, cs};
    Live lv{act, st};
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    struct Cfg { int k0, kc, i0; const char* name; };
    Cfg cfgs[] = {{0, 8, 8, "K=0 rank512"}, {16, 8, 24, "K=16 rank512"}, {32, 8, 40, "K=32 rank512"}};
    for (const Cfg& c : cfgs) {
        std::vector<unsigned> t = build_update_supertiles(c.i0, R, c.i0, Cb, 0, 0);
        unsigned* dt;
        hipMalloc(&dt, 4 * t.size());
        hipMemcpy(dt, t.data(), 4 * t.size(), hipMemcpyHostToDevice);
        auto run = [&]() {
            launch_chol_update_t128(M, c.k0, c.kc, dt, (int)t.size(), false, lv, chains, 0,
                                    FusedDiag<double>{0, nullptr, 0, nullptr, 0, 0});
        };
        for (int w = 0; w < 2; ++w) run();
        hipEventRecord(e0);
        const int reps = 5;
        for (int w = 0; w < reps; ++w) run();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double fl = flops_of(c.i0, R, c.i0, Cb, c.kc) * chains * reps;
        printf("ABL=%d %-14s supertiles %5zu x %d: %8.3f ms/launch %7.2f TFLOP/s\n", T64_ABL,
               c.name, t.size(), chains, ms / reps, fl / (ms * 1e-3) / 1e12);
        hipFree(dt);
    }
    return 0;
}
