// Micro-benchmark: per-wave fp64 VALU issue rate vs independent chains and
// waves per SIMD (MI355X).  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHECK(x) (void)(x)

template <int C>
__global__ void k_fma(double *out, int iters) {
    const int lane = threadIdx.x & 63;
    double x[C];
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] = lane + j;
    const double m = 0.999999, c = 1e-9;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int j = 0; j < C; ++j) x[j] = fma(x[j], m, c);
    double s = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int C>
__global__ void k_fma32(float *out, int iters) {
    const int lane = threadIdx.x & 63;
    float x[C];
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] = lane + j;
    const float m = 0.999999f, c = 1e-9f;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int j = 0; j < C; ++j) x[j] = fmaf(x[j], m, c);
    float s = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename T>
static void run(const char *name, void (*kern)(T *, int), T *out, int chains, int wps) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    const int iters = 4000, blocks = 256 * 4 * wps;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, 10);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    double n = (double)blocks * iters * chains;   // wave-instructions
    printf("%-8s chains %2d waves/SIMD %d: %.2f ns per wave-instr per SIMD (%.1f TFLOP/s)\n", name, chains, wps,
           ms * 1e6 / (n / 1024.0), n * 128 / (ms * 1e-3) / 1e12);
}

int main() {
    void *out;
    CHECK(hipMalloc(&out, sizeof(double) * 256 * 64 * 16));
    for (int wps : {1, 2, 4}) {
        run("fma64", k_fma<4>, (double *)out, 4, wps);
        run("fma64", k_fma<8>, (double *)out, 8, wps);
        run("fma64", k_fma<16>, (double *)out, 16, wps);
        run("fma64", k_fma<32>, (double *)out, 32, wps);
        run("fma32", k_fma32<16>, (float *)out, 16, wps);
    }
    return 0;
}
