// Microbenchmark of the f64-MFMA trailing-update kernels on random data (development tool).
// hipcc --offload-arch=gfx950 -O3 -DUPD_KS=16 -x hip tools/upd_bench.cpp -o tools/upd_ks16.bin
#define APM_TOOL_NO_SKEW
#include "../auxiliary-pm-mcmc_amd/csrc/chol.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void fill(double* p, size_t n, unsigned seed) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = ((double)(x & 0xffffff) / 16777216.0 - 0.5) * 0.01;
    }
}

static double flops_of(const std::vector<unsigned>& t, int kc) {
    double f = 0;
    for (unsigned ij : t) {
        int i = ij >> 16, j = ij & 0xffff;
        f += (i == j) ? 64.0 * 65 * 64 * kc : 2.0 * 64 * 64 * 64 * kc;
    }
    return f;
}

int main(int argc, char** argv) {
    const int nb = 64, chains = argc > 1 ? atoi(argv[1]) : 32;
    const int R = nb + 1, Cb = nb;           // Newton shape: B plus the rhs row block
    const int64_t ld = 64 * (nb + 1), rows = 64 * (nb + 1);
    const int64_t cs = rows * ld;
    double* A;
    if (hipMalloc(&A, sizeof(double) * cs * chains) != hipSuccess) { printf("oom\n"); return 1; }
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, A, (size_t)cs * chains, 7u);
    int *act, *st;
    hipMalloc(&act, 4 * chains); hipMalloc(&st, 4 * chains);
    std::vector<int> one(chains, 1), zero(chains, 0);
    hipMemcpy(act, one.data(), 4 * chains, hipMemcpyHostToDevice);
    hipMemcpy(st, zero.data(), 4 * chains, hipMemcpyHostToDevice);
    MatB M{A, ld, cs};
    Live lv{act, st};
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    struct Cfg { int k0, kc, i0, j0, jend; const char* name; };
    Cfg cfgs[] = {{0, 4, 4, 4, Cb, "outer K=0 rank256"}, {32, 4, 36, 36, Cb, "outer K=32 rank256"},
                  {0, 1, 1, 1, 4, "inner k=0 rank64"}};
    for (const Cfg& c : cfgs) {
        std::vector<unsigned> t = build_update_tiles(c.i0, R, c.j0, c.jend);
        unsigned* dt;
        hipMalloc(&dt, 4 * t.size());
        hipMemcpy(dt, t.data(), 4 * t.size(), hipMemcpyHostToDevice);
        for (int w = 0; w < 2; ++w) launch_chol_update(M, c.k0, c.kc, dt, (int)t.size(), false, lv, chains, 0);
        hipEventRecord(e0);
        const int reps = 5;
        for (int w = 0; w < reps; ++w) launch_chol_update(M, c.k0, c.kc, dt, (int)t.size(), false, lv, chains, 0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double fl = flops_of(t, c.kc) * chains * reps;
        printf("KS=%d %-22s tiles %6zu x %d chains: %8.3f ms/launch  %6.2f TFLOP/s\n", UPD_KS, c.name,
               t.size(), chains, ms / reps, fl / (ms * 1e-3) / 1e12);
    }
    return 0;
}
