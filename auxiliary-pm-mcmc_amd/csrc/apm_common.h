// Shared definitions for the MI355X (gfx950) APM hot path.
//
// Layout conventions:
//   * every matrix is row-major, fp64 unless stated, padded to Np = ceil(N/64)*64 so kernels
//     need no bounds checks; padded rows/cols are the identity (matrices) or zero (vectors);
//   * the lower triangle is the meaningful part of every factor; TB = 64 is the tile edge;
//   * batched objects carry an explicit per-chain stride and a `chain` grid dimension.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define APM_TB 64

typedef double d4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef float f2_t __attribute__((ext_vector_type(2)));
typedef double d2_t __attribute__((ext_vector_type(2)));

// per-chain status codes (mirrored in gpdemo/_native.py)
enum {
    APM_OK = 0,
    APM_ERR_CHOL_K = 1,        // chol(K) failed           -> numpy.linalg.LinAlgError
    APM_ERR_CHOL_B = 2,        // chol(B) failed (Newton)  -> numpy.linalg.LinAlgError
    APM_ERR_CHOL_C = 3,        // chol(C) failed           -> InvalidCovarianceMatrixError
    APM_ERR_MAXITER = 4,       // Newton did not converge  -> MaximumIterationsExceededError
};

// ---------------------------------------------------------------------------------------------
// log Phi(z) = log_ndtr(z), accurate over the whole real line (scipy.special.log_ndtr semantics):
//   z <  0 : log(erfcx(-z/sqrt2)/2) - z^2/2      (no underflow for very negative z)
//   z >= 0 : log1p(-erfc(z/sqrt2)/2)
__device__ __forceinline__ double log_ndtr_d(double z) {
    const double rs2 = 0.70710678118654752440;
    if (z < 0.0) return log(0.5 * erfcx(-z * rs2)) - 0.5 * z * z;
    return log1p(-0.5 * erfc(z * rs2));
}

__device__ __forceinline__ float log_ndtr_f(float z) {
    const float rs2 = 0.70710678118654752440f;
    if (z < 0.0f) return __logf(0.5f * erfcxf(-z * rs2)) - 0.5f * z * z;
    return log1pf(-0.5f * erfcf(z * rs2));
}

// log Phi(z) with the -z^2/2 of the negative branch in fp64 and the O(log|z|) remainder in fp32
// (the u-path epilogue, ugemm.hip: the large terms of the per-sample sum cancel in fp64; the
// fp32 part is bounded by ~1 + log|z| in magnitude, so its rounding stays below 1e-6 per entry)
__device__ __forceinline__ double log_ndtr_mixed(double z) {
    const float rs2 = 0.70710678118654752440f;
    const float zf = (float)z;
    if (z < 0.0) return (double)__logf(0.5f * erfcxf(-zf * rs2)) - 0.5 * z * z;
    return (double)log1pf(-0.5f * erfcf(zf * rs2));
}

// wave64 reductions
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

// block (<=1024 threads) sum into every thread; `red` needs blockDim/64 doubles of LDS
__device__ __forceinline__ double block_sum_d(double v, double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_sum_d(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < nw; ++i) s += red[i];
    return s;
}
__device__ __forceinline__ double block_max_d(double v, double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_max_d(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double s = -INFINITY;
    for (int i = 0; i < nw; ++i) s = fmax(s, red[i]);
    return s;
}
