// Development probe: the Newton factorisation's rank-512 trailing update (outer panel K of the
// 64-chain N = 4096 theta-call) as hipBLASLt GEMMs on fp16 operand planes - per row the panel's
// 512 fp32 values split into hi = fp16(x), lo = fp16(x - hi), stored [hi | lo | hi | hi] (2048
// halves), so that the fp16x3 product hi.hi^T + hi.lo^T + lo.hi^T of two rows is ONE K' = 1536
// contraction of the windows [0, 1536) and [512, 2048). C (fp32, row-major, ld 4096) -= L_I L_J^T
// over the lower block triangle: one strided-batched GEMM (64 chains) per 512-wide block column.
// Prints ms per update and fp32-equivalent TFLOP/s of the lower-triangle work, as
// tools/upd32_bench.cpp does for k_chol_update32_t128.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip tools/hblt_bench.cpp -lhipblaslt -o /tmp/hblt
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        auto e_ = (x);                                                                 \
        if ((int)e_ != 0) {                                                            \
            printf("error %d at %s:%d: %s\n", (int)e_, __FILE__, __LINE__, #x);        \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void k_fill(_Float16* P, int64_t n, unsigned seed) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    unsigned s = (unsigned)(i * 2654435761u) ^ seed;
    s ^= s >> 13; s *= 0x5bd1e995; s ^= s >> 15;
    P[i] = (_Float16)((s & 0xffff) / 65536.0f - 0.5f);
}

int main(int argc, char** argv) {
    const int chains = argc > 1 ? atoi(argv[1]) : 64, K = argc > 2 ? atoi(argv[2]) : 0;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const int np = 4096, outer = 512, KP = 1536, PW = 2048;
    const int64_t ldc = np, cstride = (int64_t)(np + 64) * np;
    const int row0 = (K + 1) * outer;  // first row / column of the trailing matrix
    const int m = np - row0;           // its size
    const int64_t pstride = (int64_t)np * PW;
    _Float16* P;
    float* C;
    CK(hipMalloc(&P, sizeof(_Float16) * pstride * chains));
    CK(hipMalloc(&C, sizeof(float) * cstride * chains));
    hipLaunchKernelGGL(k_fill, dim3((pstride * chains + 255) / 256), dim3(256), 0, 0, P,
                       pstride * chains, 7u);
    CK(hipMemset(C, 0, sizeof(float) * cstride * chains));
    hipblasLtHandle_t h;
    CK(hipblasLtCreate(&h));
    size_t wsz = 64ull << 20;
    void* ws;
    CK(hipMalloc(&ws, wsz));
    const int nblk = m / outer;
    struct G {
        hipblasLtMatmulDesc_t d;
        hipblasLtMatrixLayout_t a, b, c;
        hipblasLtMatmulAlgo_t algo;
        const void *A, *B;
        float* Cp;
    };
    std::vector<G> gs(nblk);
    for (int c = 0; c < nblk; ++c) {
        G& g = gs[c];
        const int r0 = row0 + c * outer, M = np - r0;  // rows r0 .. np of block column c
        CK(hipblasLtMatmulDescCreate(&g.d, HIPBLAS_COMPUTE_32F, HIP_R_32F));
        hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
        CK(hipblasLtMatmulDescSetAttribute(g.d, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
        CK(hipblasLtMatmulDescSetAttribute(g.d, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
        // column-major view: D (512 x M) = A^T (512 x K') B (K' x M); A = the block column's
        // rows' right window, B = the M rows' left window
        CK(hipblasLtMatrixLayoutCreate(&g.a, HIP_R_16F, KP, outer, PW));
        CK(hipblasLtMatrixLayoutCreate(&g.b, HIP_R_16F, KP, M, PW));
        CK(hipblasLtMatrixLayoutCreate(&g.c, HIP_R_32F, outer, M, ldc));
        int32_t bc = chains;
        for (auto L : {g.a, g.b, g.c})
            CK(hipblasLtMatrixLayoutSetAttribute(L, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc,
                                                 sizeof(bc)));
        int64_t sp = pstride, sc = cstride;
        CK(hipblasLtMatrixLayoutSetAttribute(g.a, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET,
                                             &sp, sizeof(sp)));
        CK(hipblasLtMatrixLayoutSetAttribute(g.b, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET,
                                             &sp, sizeof(sp)));
        CK(hipblasLtMatrixLayoutSetAttribute(g.c, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET,
                                             &sc, sizeof(sc)));
        hipblasLtMatmulPreference_t pref;
        CK(hipblasLtMatmulPreferenceCreate(&pref));
        CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES,
                                                 &wsz, sizeof(wsz)));
        hipblasLtMatmulHeuristicResult_t res[8];
        int nres = 0;
        CK(hipblasLtMatmulAlgoGetHeuristic(h, g.d, g.a, g.b, g.c, g.c, pref, 8, res, &nres));
        if (nres == 0) {
            printf("no algorithm for block %d\n", c);
            return 1;
        }
        g.algo = res[0].algo;
        g.A = P + (int64_t)r0 * PW + outer;  // right window of the block column's rows
        g.B = P + (int64_t)r0 * PW;          // left window of rows r0 ..
        g.Cp = C + (int64_t)r0 * ldc + r0;
    }
    const float alpha = -1.f, beta = 1.f;
    auto run = [&]() {
        for (G& g : gs)
            CK(hipblasLtMatmul(h, g.d, &alpha, g.A, g.a, g.B, g.b, &beta, g.Cp, g.c, g.Cp, g.c,
                               &g.algo, ws, wsz, 0));
    };
    run();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) run();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // fp32-equivalent lower-triangle flops of the update (the bench's accounting: m^2 x 512 x 2 / 2)
    const double fl = (double)m * (m + 64) * outer * chains;
    double f16 = 0;
    for (int c = 0; c < nblk; ++c) f16 += 2.0 * (np - row0 - c * outer) * outer * KP * chains;
    printf("K=%d chains=%d blocks=%d: %.4f ms/update  %.1f TFLOP/s fp32-eq lower  (%.1f TFLOP/s "
           "fp16 executed)\n", K, chains, nblk, ms / reps, fl / (ms / reps * 1e-3) / 1e12,
           f16 / (ms / reps * 1e-3) / 1e12);
    return 0;
}
