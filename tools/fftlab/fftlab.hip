// fftlab.hip -- A/B harness for the 1024-point wave FFT engines (GPU box).
//
// Every variant reads rows of 2048 f32 samples from HBM (next row in flight),
// transforms them (2048-point real FFT = 1024-point complex FFT + real
// post-pass) and writes per row the get_noise_PS power sum (k >= 768) and
// sum_{k>=1} |D_k|^2; the first NCHK rows also write their whole spectrum,
// which the host checks against a direct DFT in double precision.
//   cur   : wfft::fft_row (ppf_wfft.hpp, three LDS exchanges) + LDS post-pass
//   nat   : wf2::fft1024 (one exchange) + natural-order LDS post-pass
//   perm  : wf2::fft1024 + wf2::pairs (permlane32 partner swap, no LDS)
//   read  : the loads alone (HBM reference)
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast
//        -I../../pulseportraiture_amd/csrc fftlab.hip -o fftlab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ppf_wfft2.hpp"

using namespace ppf;

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                  \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr int N = 1024, NH = 1025, KC = 768, NCHK = 8, WG = 4;
typedef float vf2 __attribute__((ext_vector_type(2)));

struct Args {
    const vf2 *rows;
    long long nrows;
    double *out;          // [nrows][2]
    double2 *chk;         // [NCHK][NH]
    const double2 *T;     // e^{-2 pi i k/1024}, k < 256
};

__device__ __forceinline__ void rpair(double2 zk, double2 zn, double2 w, double2 &Dlo, double2 &Dhi) {
    const double2 e = cmk(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y));
    const double2 o = cmk(0.5 * (zk.x - zn.x), 0.5 * (zk.y + zn.y));
    const double2 wo = cmul(w, o);
    Dlo = cmk(e.x + wo.y, e.y - wo.x);
    Dhi = cmk(e.x - wo.y, -(e.y + wo.x));
}

__device__ __forceinline__ double2 wpi(int k) {   // e^{-i pi k / N}
    double s, c;
    sincospi(-(double)k / (double)N, &s, &c);
    return cmk(c, s);
}

// natural-order post-pass from buf[pad(k)] (the current engine's)
__device__ __forceinline__ void post_nat(const double2 *buf, int lane, double2 wseed, double2 wstep,
                                         double &pn, double &pd, double2 *chk) {
    double2 w = wseed;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int klo = lane + 64 * i, khi = N - klo;
        const double2 zk = buf[wfft::pad<10>(klo)];
        const double2 zn = buf[klo == 0 ? 0 : wfft::pad<10>(khi)];
        double2 Dlo, Dhi;
        rpair(zk, zn, w, Dlo, Dhi);
        w = cmul(w, wstep);
        const double p0 = cabs2(Dlo), p1 = cabs2(Dhi);
        if (klo >= KC) pn += p0;
        if (khi >= KC) pn += p1;
        if (klo >= 1) pd += p0;
        pd += p1;
        if (chk) { chk[klo] = Dlo; chk[khi] = Dhi; }
    }
    if (lane == 0) {
        const double2 zm = buf[wfft::pad<10>(N / 2)];
        const double2 Dm = cmk(zm.x, -zm.y);
        if (N / 2 >= KC) pn += cabs2(Dm);
        pd += cabs2(Dm);
        if (chk) chk[N / 2] = Dm;
    }
}

template <int VAR, int WPE>
__global__ __launch_bounds__(64 * WG) __attribute__((amdgpu_waves_per_eu(WPE))) void k_lab(Args a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int lane0 = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int SLW = VAR == 0 ? wfft::buf_slots<10>()
                                 : (wf2::kXSlots + wf2::kSpSlots > wfft::buf_slots<10>()
                                        ? wf2::kXSlots + wf2::kSpSlots
                                        : wfft::buf_slots<10>());
    double2 *buf = lds + wave * SLW;
    double2 *tw = lds + WG * SLW;
    if (VAR == 0) {
        for (int i = threadIdx.x; i < 256; i += 64 * WG) tw[i] = a.T[i];
        __syncthreads();
    }
    const wf2::Seeds sd = wf2::make_seeds(lane0);
    const double2 wstep = wpi(64);
    const double2 wseed_nat = wpi(lane0);
    const double2 wseed_pair = wpi(wf2::pair_k0(lane0));
    const long long nw = (long long)gridDim.x * WG;
    long long row = (long long)blockIdx.x * WG + wave;
    vf2 zr[16];
    auto fetch = [&](long long rr) {
        const vf2 *src = a.rows + rr * N;
#pragma unroll
        for (int q = 0; q < 16; ++q) zr[q] = src[lane0 + 64 * q];
    };
    if (row < a.nrows) fetch(row);
    for (; row < a.nrows; row += nw) {
        double2 x[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) x[q] = cmk((double)zr[q].x, (double)zr[q].y);
        if (row + nw < a.nrows) fetch(row + nw);
        double2 *chk = row < NCHK ? a.chk + row * NH : nullptr;
        double pn = 0.0, pd = 0.0;
        // opaque lane: per-lane indices re-derived every row (hoisted out of
        // the row loop they hold dozens of VGPRs)
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        if constexpr (VAR == 3) {
            // loads only: fold the row into the sums so nothing is dead
#pragma unroll
            for (int q = 0; q < 16; ++q) { pn += x[q].x; pd += x[q].y; }
        } else if constexpr (VAR == 0) {
            wfft::fft_row<10>(x, buf, tw, lane0);
            post_nat(buf, lane, wseed_nat, wstep, pn, pd, chk);
        } else if constexpr (VAR == 1) {
            wf2::fft1024(x, buf, lane, sd);
            // natural order: k = out_index(lane, m)
#pragma unroll
            for (int m = 0; m < 16; ++m) buf[wfft::pad<10>(wf2::out_index(lane, m))] = x[m];
            wfft::wave_sync();
            post_nat(buf, lane, wseed_nat, wstep, pn, pd, chk);
            wfft::wave_sync();
        } else {
            wf2::fft1024(x, buf, lane, sd);
            double2 zm = cmk(0.0, 0.0);
            wf2::pairs(x, buf + wf2::kXSlots, lane, zm);
            const int k0 = wf2::pair_k0(lane);
            double2 w = wseed_pair;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int klo = k0 + 64 * i, khi = N - klo;
                double2 Dlo, Dhi;
                rpair(x[i], x[i + 8], w, Dlo, Dhi);
                w = cmul(w, wstep);
                const double p0 = cabs2(Dlo), p1 = cabs2(Dhi);
                if (klo >= KC) pn += p0;
                if (khi >= KC) pn += p1;
                if (klo >= 1) pd += p0;
                pd += p1;
                if (chk) { chk[klo] = Dlo; chk[khi] = Dhi; }
            }
            if (lane == 0) {
                const double2 Dm = cmk(zm.x, -zm.y);
                if (N / 2 >= KC) pn += cabs2(Dm);
                pd += cabs2(Dm);
                if (chk) chk[N / 2] = Dm;
            }
        }
        pn = wave_sum(pn);
        pd = wave_sum(pd);
        if (lane == 0) {
            a.out[row * 2] = pn;
            a.out[row * 2 + 1] = pd;
        }
    }
}

__global__ void k_fill(float *x, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long h = (unsigned long long)i * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    h ^= h >> 31; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 27; h *= 0x94D049BB133111EBull; h ^= h >> 31;
    const float u = (float)((h >> 40) * (1.0 / 16777216.0)) - 0.5f;
    const long long c = i % 2048;
    // a pulse near bin 700 plus noise
    const float d = (float)(c - 700);
    x[i] = 3.0f * expf(-d * d / 200.0f) + u;
}

template <int VAR, int WPE>
static float run(const Args &a, int grid, size_t lds, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipFuncSetAttribute((const void *)k_lab<VAR, WPE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((k_lab<VAR, WPE>), dim3(grid), dim3(64 * WG), lds, 0, a);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((k_lab<VAR, WPE>), dim3(grid), dim3(64 * WG), lds, 0, a);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
    const long long nrows = argc > 1 ? atoll(argv[1]) : 1048576;
    const int gmul = argc > 2 ? atoi(argv[2]) : 16;
    const long long n = nrows * 2048;
    float *rows;
    double *out;
    double2 *chk, *T;
    CK(hipMalloc(&rows, n * 4));
    CK(hipMalloc(&out, nrows * 16));
    CK(hipMalloc(&chk, (size_t)NCHK * NH * 16));
    CK(hipMalloc(&T, 256 * 16));
    hipLaunchKernelGGL(k_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, rows, n);
    std::vector<double2> hT(256);
    for (int k = 0; k < 256; ++k) hT[k] = cmk(cos(-2 * M_PI * k / 1024.0), sin(-2 * M_PI * k / 1024.0));
    CK(hipMemcpy(T, hT.data(), 256 * 16, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    // host reference spectra of the check rows
    std::vector<float> hx((size_t)NCHK * 2048);
    CK(hipMemcpy(hx.data(), rows, hx.size() * 4, hipMemcpyDeviceToHost));
    std::vector<double> cs(2048), sn(2048);
    for (int j = 0; j < 2048; ++j) { cs[j] = cos(2 * M_PI * j / 2048.0); sn[j] = -sin(2 * M_PI * j / 2048.0); }
    std::vector<double2> ref((size_t)NCHK * NH);
    std::vector<double> refp((size_t)NCHK * 2);
    for (int r = 0; r < NCHK; ++r) {
        double pn = 0, pd = 0;
        for (int k = 0; k < NH; ++k) {
            long double re = 0, im = 0;
            for (int j = 0; j < 2048; ++j) {
                const int t = (int)(((long long)j * k) & 2047);
                re += (long double)hx[r * 2048 + j] * cs[t];
                im += (long double)hx[r * 2048 + j] * sn[t];
            }
            ref[r * NH + k] = cmk((double)re, (double)im);
            const double p = (double)(re * re + im * im);
            if (k >= KC) pn += p;
            if (k >= 1) pd += p;
        }
        refp[r * 2] = pn;
        refp[r * 2 + 1] = pd;
    }
    Args a{reinterpret_cast<const vf2 *>(rows), nrows, out, chk, T};
    const size_t lds_cur = (size_t)(WG * wfft::buf_slots<10>() + 256) * 16;
    const size_t slw_new = std::max<size_t>(wf2::kXSlots + wf2::kSpSlots, wfft::buf_slots<10>());
    const size_t lds_new = (size_t)(WG * slw_new + 256) * 16;
    const int grid = (int)std::min<long long>((nrows + WG - 1) / WG, 256LL * gmul);
    const double scale = 5120000.0 / (double)nrows;   // ms per C2 launch (10k x 512 rows)
    auto check = [&](const char *name, float ms) {
        std::vector<double2> hc((size_t)NCHK * NH);
        std::vector<double> ho((size_t)NCHK * 2);
        CK(hipMemcpy(hc.data(), chk, hc.size() * 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ho.data(), out, ho.size() * 8, hipMemcpyDeviceToHost));
        double emax = 0, dmax = 0, perr = 0;
        for (size_t i = 0; i < hc.size(); ++i) {
            emax = std::max(emax, std::hypot(hc[i].x - ref[i].x, hc[i].y - ref[i].y));
            dmax = std::max(dmax, std::hypot(ref[i].x, ref[i].y));
        }
        for (size_t i = 0; i < ho.size(); ++i) perr = std::max(perr, std::fabs(ho[i] / refp[i] - 1));
        printf("%-5s %8.3f ms  (%7.2f ms per 5.12M rows, %6.2f TB/s)  D err %.2e rel, sums %.2e rel\n", name, ms,
               ms * scale, (double)nrows * 8192 / ms / 1e9, emax / dmax, perr);
        CK(hipMemset(chk, 0, (size_t)NCHK * NH * 16));
        CK(hipMemset(out, 0, (size_t)nrows * 16));
    };
    const int reps = 5;
    printf("rows %lld, grid %d\n", nrows, grid);
    check("read", run<3, 2>(a, grid, lds_new, reps));
    check("cur", run<0, 2>(a, grid, lds_cur, reps));
    check("nat", run<1, 2>(a, grid, lds_new, reps));
    check("perm", run<2, 2>(a, grid, lds_new, reps));
    return 0;
}
