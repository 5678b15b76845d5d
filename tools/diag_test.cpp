// Development check of the 64x64 diagonal-tile factorisation (diag.h) against a CPU Cholesky.
// hipcc --offload-arch=gfx950 -O3 -x hip tools/diag_test.cpp -o tools/diag_test.bin
#define APM_TOOL_NO_SKEW
#include "../auxiliary-pm-mcmc_amd/csrc/chol.hip"
#include <cmath>
#include <cstdio>
#include <vector>

int main() {
    const int n = 64;
    std::vector<double> M(n * n), L(n * n, 0.0);
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 65536.0 - 0.5; };
    std::vector<double> G(n * n);
    for (auto& g : G) g = rnd();
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = (i == j) ? 4.0 : 0.0;
            for (int k = 0; k < n; ++k) acc += G[i * n + k] * G[j * n + k];
            M[i * n + j] = acc;
        }
    for (int j = 0; j < n; ++j) {  // CPU Cholesky
        double d = M[j * n + j];
        for (int k = 0; k < j; ++k) d -= L[j * n + k] * L[j * n + k];
        L[j * n + j] = std::sqrt(d);
        for (int i = j + 1; i < n; ++i) {
            double v = M[i * n + j];
            for (int k = 0; k < j; ++k) v -= L[i * n + k] * L[j * n + k];
            L[i * n + j] = v / L[j * n + j];
        }
    }
    double *dA, *dD, *dl;
    int *act, *st;
    hipMalloc(&dA, 8 * n * n); hipMalloc(&dD, 8 * n * n); hipMalloc(&dl, 8 * 4);
    hipMalloc(&act, 4); hipMalloc(&st, 4);
    int one = 1, zero = 0;
    hipMemcpy(act, &one, 4, hipMemcpyHostToDevice);
    hipMemcpy(st, &zero, 4, hipMemcpyHostToDevice);
    hipMemcpy(dA, M.data(), 8 * n * n, hipMemcpyHostToDevice);
    launch_chol_diag(MatB{dA, n, n * n}, 0, dD, n * n, dl, 4, Live{act, st}, 7, 1, 0);
    std::vector<double> Lg(n * n), Dg(n * n);
    int stat;
    hipMemcpy(Lg.data(), dA, 8 * n * n, hipMemcpyDeviceToHost);
    hipMemcpy(Dg.data(), dD, 8 * n * n, hipMemcpyDeviceToHost);
    hipMemcpy(&stat, st, 4, hipMemcpyDeviceToHost);
    double el = 0, ei = 0;
    int worst = -1;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            const double e = std::fabs(Lg[i * n + j] - L[i * n + j]);
            if (e > el) { el = e; worst = i * n + j; }
        }
    for (int i = 0; i < n; ++i)  // |Dinv * L - I|
        for (int j = 0; j < n; ++j) {
            double acc = 0;
            for (int k = 0; k < n; ++k) acc += Dg[i * n + k] * L[k * n + j];
            ei = std::fmax(ei, std::fabs(acc - (i == j)));
        }
    for (int bi = 0; bi < 4; ++bi) {
        for (int bj = 0; bj <= bi; ++bj) {
            double e = 0;
            for (int i = 16 * bi; i < 16 * bi + 16; ++i)
                for (int j = 16 * bj; j < 16 * bj + 16 && j <= i; ++j)
                    e = std::fmax(e, std::fabs(Lg[i * n + j] - L[i * n + j]));
            printf("  blk(%d,%d) %.1e", bi, bj, e);
        }
        printf("\n");
    }
    {   // inverse of the first 16x16 block vs CPU substitution
        double e = 0;
        for (int c = 0; c < 16; ++c) {
            double x[16];
            for (int r = 0; r < 16; ++r) {
                double acc = (r == c);
                for (int m = 0; m < r; ++m) acc -= L[r * n + m] * x[m];
                x[r] = acc / L[r * n + r];
                e = std::fmax(e, std::fabs(x[r] - Dg[r * n + c]));
            }
        }
        printf("Dinv blk(0,0) err %.3e  Dinv[1][0]=%.6f Dinv[0][0]=%.6f Dinv[1][1]=%.6f\n", e, Dg[n], Dg[0], Dg[n + 1]);
    }
    printf("status %d  max|L-Lcpu| %.3e (at %d,%d: %.6f vs %.6f)  max|Dinv L - I| %.3e\n", stat,
           el, worst / n, worst % n, worst >= 0 ? Lg[worst] : 0.0, worst >= 0 ? L[worst] : 0.0, ei);
    return (stat == 0 && el < 1e-10 && ei < 1e-10) ? 0 : 1;
}
