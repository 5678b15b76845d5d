// Development tool: the int8 Ozaki-II emulation of the fp64 rank-512 trailing update
// (csrc/ozaki.hip) against the f64-MFMA kernel (k_chol_update_t128) at the chol(K) shape of
// N=4096: exactness on integer data (operand maps), accuracy on scaled random panels (vs a CPU
// long-double reference on sampled tiles), and launch times.
//   make -C auxiliary-pm-mcmc_amd/csrc && hipcc --offload-arch=gfx950 -O3 -std=c++17 \
//     -I auxiliary-pm-mcmc_amd/csrc tools/ozaki_bench.cpp -L auxiliary-pm-mcmc_amd/lib -lapm \
//     -Wl,-rpath,$PWD/auxiliary-pm-mcmc_amd/lib -o tools/ozaki_bench.bin
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "apm_internal.h"

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            printf("HIP error %s at %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

static double flops_of(const std::vector<unsigned>& st) {
    double f = 0;
    for (unsigned e : st) {
        const int ti = (int)(e >> 18), tj = (int)((e >> 4) & 0x3fff);
        const bool rv[2] = {(e & 1u) != 0, (e & 2u) != 0}, cv[2] = {(e & 4u) != 0, (e & 8u) != 0};
        for (int a = 0; a < 2; ++a)
            for (int c = 0; c < 2; ++c)
                if (rv[a] && cv[c] && tj + c <= ti + a)
                    f += (tj + c == ti + a) ? 64.0 * 65 * 64 : 2.0 * 64 * 64 * 64;
    }
    return f;
}

int main(int argc, char** argv) {
    const int nb = 64, chains = argc > 1 ? atoi(argv[1]) : 64;
    const int kc = 8;
    const int64_t ld = 64 * nb, rows = 64 * (nb + 1), cs = rows * ld;
    const size_t nel = (size_t)cs * chains;
    CK(oz_init_device());
    double *A1, *A2;
    CK(hipMalloc(&A1, sizeof(double) * nel));
    CK(hipMalloc(&A2, sizeof(double) * nel));
    int *act, *st;
    CK(hipMalloc(&act, 4 * chains));
    CK(hipMalloc(&st, 4 * chains));
    std::vector<int> one(chains, 1), zero(chains, 0);
    CK(hipMemcpy(act, one.data(), 4 * chains, hipMemcpyHostToDevice));
    CK(hipMemcpy(st, zero.data(), 4 * chains, hipMemcpyHostToDevice));
    Live lv{act, st};
    // plane storage for rows [64 k, 64 nb) of one panel
    const int depth = 64 * kc;
    OzPlanes P{};
    const int64_t prow = 64 * nb;
    P.mstride = prow * depth;
    P.cstride = (int64_t)OZ_NM * P.mstride;
    CK(hipMalloc(&P.base, (size_t)P.cstride * chains));
    P.estride = prow;
    CK(hipMalloc(&P.exps, sizeof(int) * prow * chains));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const FusedDiag<double> nofd{0, nullptr, 0, nullptr, 0, 0};

    // host data: chain-major, (rows x ld) per chain; mode 0 = small integers (exact test),
    // mode 1 = scaled random reals (rows of magnitudes 2^-20 .. 2^20, a few tiny entries)
    std::vector<double> h((size_t)cs * std::min(chains, 2));
    for (int mode = 0; mode < 2; ++mode) {
        std::mt19937_64 g(1234 + mode);
        std::uniform_real_distribution<double> U(-1.0, 1.0);
        const int chk = std::min(chains, 2);
        for (int c = 0; c < chk; ++c)
            for (int64_t r = 0; r < rows; ++r) {
                const double sc = mode ? std::ldexp(1.0, (int)(r * 7919 % 41) - 20) : 1.0;
                for (int64_t k = 0; k < ld; ++k) {
                    double v = mode ? U(g) * sc : std::floor(U(g) * 200.0);
                    if (mode && (k % 97) == 3) v *= 1e-30;
                    h[(size_t)c * cs + r * ld + k] = v;
                }
            }
        CK(hipMemcpy(A1, h.data(), sizeof(double) * cs * chk, hipMemcpyHostToDevice));
        CK(hipMemcpy(A2, h.data(), sizeof(double) * cs * chk, hipMemcpyHostToDevice));
        const int k0 = 16, i0 = k0 + kc;  // panel columns [64 k0, 64 (k0+kc)), trailing from i0
        std::vector<unsigned> t = build_update_supertiles(i0, nb, i0, nb, 0, 0, -1);
        unsigned* dt;
        CK(hipMalloc(&dt, 4 * t.size()));
        CK(hipMemcpy(dt, t.data(), 4 * t.size(), hipMemcpyHostToDevice));
        MatB M1{A1, ld, cs}, M2{A2, ld, cs};
        launch_chol_update_t128(M1, k0, kc, dt, (int)t.size(), 0, lv, chk, 0, nofd);
        P.row0 = 64 * i0;
        const int beta = oz_beta(depth);
        launch_oz_split(M2, 64 * i0, 64 * (nb - i0), 64 * k0, depth, P, beta, lv, chk, 0);
        launch_oz_update_t128(M2, P, depth, dt, (int)t.size(), 0, lv, chk, 0, nofd);
        CK(hipDeviceSynchronize());
        std::vector<double> r1((size_t)cs * chk), r2((size_t)cs * chk);
        CK(hipMemcpy(r1.data(), A1, sizeof(double) * cs * chk, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r2.data(), A2, sizeof(double) * cs * chk, hipMemcpyDeviceToHost));
        // CPU long-double reference on sampled entries of the trailing lower triangle
        double e_f64 = 0, e_oz = 0, scale = 0;
        long cnt = 0;
        std::mt19937 gs(7);
        for (int q = 0; q < 4000; ++q) {
            const int c = q % chk;
            int i = 64 * i0 + (int)(gs() % (64 * (nb - i0)));
            int j = 64 * i0 + (int)(gs() % (64 * (nb - i0)));
            if (j > i) std::swap(i, j);
            long double s = 0, sa = 0;
            for (int k = 64 * k0; k < 64 * (k0 + kc); ++k) {
                const long double p = (long double)h[(size_t)c * cs + (int64_t)i * ld + k] *
                                      h[(size_t)c * cs + (int64_t)j * ld + k];
                s += p;
                sa += fabsl(p);
            }
            const long double ref = (long double)h[(size_t)c * cs + (int64_t)i * ld + j] - s;
            const size_t o = (size_t)c * cs + (int64_t)i * ld + j;
            // error relative to the sum of |products| (the fp64 GEMM error scale)
            const double den = (double)sa + 1e-300;
            e_f64 = std::max(e_f64, (double)fabsl(r1[o] - ref) / den);
            e_oz = std::max(e_oz, (double)fabsl(r2[o] - ref) / den);
            scale = std::max(scale, (double)sa);
            ++cnt;
        }
        printf("mode %d (%s) beta %d: max |err| / sum|a b|  f64-MFMA %.3e  ozaki %.3e  (%ld entries)\n",
               mode, mode ? "scaled reals" : "integers", beta, e_f64, e_oz, cnt);
        CK(hipFree(dt));
    }

    // timing at full batch, panel positions K = 0, 16, 32, 48
    for (int k0 : {0, 16, 32, 48}) {
        const int i0 = k0 + kc;
        if (i0 >= nb) break;
        std::vector<unsigned> t = build_update_supertiles(i0, nb, i0, nb, 0, 0, -1);
        unsigned* dt;
        CK(hipMalloc(&dt, 4 * t.size()));
        CK(hipMemcpy(dt, t.data(), 4 * t.size(), hipMemcpyHostToDevice));
        MatB M1{A1, ld, cs};
        P.row0 = 64 * i0;
        const int beta = oz_beta(depth);
        auto run64 = [&]() {
            launch_chol_update_t128(M1, k0, kc, dt, (int)t.size(), 0, lv, chains, 0, nofd);
        };
        auto runsplit = [&]() {
            launch_oz_split(M1, 64 * i0, 64 * (nb - i0), 64 * k0, depth, P, beta, lv, chains, 0);
        };
        auto runoz = [&]() {
            launch_oz_update_t128(M1, P, depth, dt, (int)t.size(), 0, lv, chains, 0, nofd);
        };
        float ms[3];
        auto timeit = [&](auto&& f) {
            f();
            f();
            CK(hipEventRecord(e0));
            const int reps = 5;
            for (int w = 0; w < reps; ++w) f();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float m;
            CK(hipEventElapsedTime(&m, e0, e1));
            return m / reps;
        };
        // restore the matrix between kinds is unnecessary for timing (values stay finite: the
        // data are small and repeated updates add at most a few units of magnitude)
        CK(hipMemset(A1, 0, sizeof(double) * nel));
        ms[0] = timeit(run64);
        ms[1] = timeit(runsplit);
        ms[2] = timeit(runoz);
        const double fl = flops_of(t) * kc * chains;
        printf("K=%2d supertiles %5zu x %d: f64 %.3f ms (%.1f TF) | split %.3f ms + oz %.3f ms "
               "(%.1f TF-eq, %.1f incl. split)\n",
               k0, t.size(), chains, ms[0], fl / (ms[0] * 1e-3) / 1e12, ms[1], ms[2],
               fl / (ms[2] * 1e-3) / 1e12, fl / ((ms[1] + ms[2]) * 1e-3) / 1e12);
        CK(hipFree(dt));
    }
    CK(hipGetLastError());
    printf("ok\n");
    return 0;
}
