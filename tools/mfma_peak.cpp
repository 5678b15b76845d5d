// Peak throughput of v_mfma_f64_16x16x4_f64 and v_mfma_f32_16x16x4_f32 (register operands,
// independent accumulators, random data) — calibrates the roofline peaks used by bench.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void kf64(double* out, int iters, double seed) {
    d4 acc[8] = {};
    double a = seed + threadIdx.x * 1e-3, b = 1.0 - seed * threadIdx.x * 1e-4;
    for (int i = 0; i < iters / 2; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    }
    double s = 0;
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void kf32(float* out, int iters, float seed) {
    f4 acc[4] = {};
    float a = seed + threadIdx.x * 1e-3f, b = 1.0f - seed * threadIdx.x * 1e-4f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
    }
    float s = 0;
    for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main(int argc, char** argv) {
    const int per_cu = argc > 1 ? atoi(argv[1]) : 8;
    const int blocks = 256 * per_cu, iters = 4096;
    double* o; hipMalloc(&o, 8 * blocks * 256);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(kf64, dim3(blocks), dim3(256), 0, 0, o, iters, 0.37);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double fl = (double)blocks * 4 /*waves*/ * iters * 4 * 16 * 16 * 4 * 2;
        printf("f64 16x16x4: %.2f TFLOP/s\n", fl / (ms * 1e-3) / 1e12);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kf32, dim3(blocks), dim3(256), 0, 0, (float*)o, iters, 0.37f);
        hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("f32 16x16x4: %.2f TFLOP/s\n", fl / (ms * 1e-3) / 1e12);
    }
    return 0;
}
