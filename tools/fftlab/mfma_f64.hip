// Micro-benchmark: throughput of v_mfma_f64_16x16x4f64 and fp64 VALU FMA on
// one MI355X (cycles per instruction per SIMD).  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void k_mfma(double *out, int iters) {
    const int lane = threadIdx.x & 63;
    double a = 1.0 + lane * 1e-3, b = 2.0 - lane * 1e-3;
    f64x4 d0 = {0, 0, 0, 0}, d1 = d0, d2 = d0, d3 = d0;
    for (int i = 0; i < iters; ++i) {
        d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d1, 0, 0, 0);
        d2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d2, 0, 0, 0);
        d3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d3, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = d0[0] + d1[1] + d2[2] + d3[3];
}

__global__ void k_fma(double *out, int iters) {
    const int lane = threadIdx.x & 63;
    double x[8];
    for (int j = 0; j < 8; ++j) x[j] = lane + j;
    const double m = 0.999999, c = 1e-9;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fma(x[j], m, c);
    double s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    double *out;
    hipMalloc(&out, sizeof(double) * 256 * 64 * 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    int iters = 20000;
    for (int wps : {1, 2, 4}) {       // waves per SIMD
        int blocks = 256 * 4 * wps;  // one-wave blocks
        hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(64), 0, 0, out, 100);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(64), 0, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double n = (double)blocks * iters * 4;
        printf("mfma_f64_16x16x4: waves/SIMD %d: %.2f TFLOP/s, %.1f ns per MFMA per SIMD\n", wps,
               n * 2048 / (ms * 1e-3) / 1e12, ms * 1e6 / (n / 1024.0));
        hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(64), 0, 0, out, 100);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(64), 0, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        n = (double)blocks * iters * 8;
        printf("v_fma_f64: waves/SIMD %d: %.2f TFLOP/s, %.2f ns per wave-FMA per SIMD\n", wps,
               n * 128 / (ms * 1e-3) / 1e12, ms * 1e6 / (n / 1024.0));
    }
    return 0;
}
