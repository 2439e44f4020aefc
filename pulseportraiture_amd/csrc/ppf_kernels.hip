// ppf_kernels.hip -- gfx950 kernels of the wideband FFTFIT engine.
//
// Pipeline of one ppf_fit_batch call:
//   k_twiddles      (once per nbin, cached by the context)
//   k_rfft_rows     model portraits -> model spectra M[model][chan][k]
//   k_xspec         data rows -> rfft (LDS Stockham) -> PS noise -> cross
//                   spectrum X = D conj(M) / sigma~^2, Sd_n, S0_n; optional
//                   dedispersed-profile accumulators for the phase guess
//   k_guess         brute grid + Nelder-Mead on the mean profile (GetTOAs)
//   k_solve         one workgroup per sub-integration: scipy trust-ncg replica
//                   whose every objective/gradient/Hessian evaluation is one
//                   streaming pass over X; then zero-covariance frequencies,
//                   output transform, O(nchan) Schur covariance, scales, S/N
// Standalone kernels: k_rotate, k_noise, k_phase_shift, k_synth.
#include <cstdlib>
#include <type_traits>

#include "ppf_device.hpp"
#include "ppf_internal.hpp"

namespace ppf {

// ===========================================================================
// common row loading: z_j = x_{2j} + i x_{2j+1} (even nbin); z_j = x_j + 0 i
// (odd nbin, rfft_len)
// ===========================================================================
__device__ __forceinline__ void load_row(double2 *buf, const void *src, int dtype, int64_t row,
                                         int nbin) {
    const int N = nbin >> 1;
    if (nbin & 1) {
        if (dtype == 0) {
            const float *s = reinterpret_cast<const float *>(src) + row * (int64_t)nbin;
            for (int j = threadIdx.x; j < nbin; j += kBlock) buf[j] = cmk((double)s[j], 0.0);
        } else {
            const double *s = reinterpret_cast<const double *>(src) + row * (int64_t)nbin;
            for (int j = threadIdx.x; j < nbin; j += kBlock) buf[j] = cmk(s[j], 0.0);
        }
        return;
    }
    if (dtype == 0) {
        const float2 *s = reinterpret_cast<const float2 *>(src) + row * (int64_t)N;
        for (int j = threadIdx.x; j < N; j += kBlock) {
            float2 v = s[j];
            buf[j] = cmk((double)v.x, (double)v.y);
        }
    } else {
        const double2 *s = reinterpret_cast<const double2 *>(src) + row * (int64_t)N;
        for (int j = threadIdx.x; j < N; j += kBlock) buf[j] = s[j];
    }
}

// X_k (k <= nbin / 2) of the row load_row + lds_fft_n(rfft_len(nbin)) left in buf
__device__ __forceinline__ double2 rbin(const double2 *buf, int nbin, const double2 *__restrict__ T2, int k) {
    return (nbin & 1) ? buf[k] : rfft_bin(buf, nbin >> 1, T2, k);
}
// odd nbin: Y_k (k <= nbin / 2) into the Hermitian full-length buffer of the
// inverse transform, whose real part is then the row (the imaginary part of
// Y_0 drops out, as numpy.fft.irfft ignores it)
__device__ __forceinline__ void herm_put(double2 *buf, int nbin, int k, double2 Y) {
    buf[k] = Y;
    if (k) buf[nbin - k] = cconj(Y);
}

// ===========================================================================
// twiddles: T[t] = exp(-2 pi i t/N), T2[k] = exp(-i pi k/N), t,k < N
// ===========================================================================
__global__ void k_twiddles(int N, double2 *T, double2 *T2) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= N) return;
    double s, c;
    sincospi(2.0 * (double)t / (double)N, &s, &c);
    T[t] = cmk(c, -s);
    sincospi((double)t / (double)N, &s, &c);
    T2[t] = cmk(c, -s);
}

// ===========================================================================
// rfft of fp64 rows -> full half spectrum [row][N+1] (model portraits)
// ===========================================================================
template <bool MX>
__global__ __launch_bounds__(kBlock) void k_rfft_rows(RfftArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int N = a.nbin >> 1;
    const int64_t row = blockIdx.x;
    load_row(lds, a.in, a.dtype, row, a.nbin);
    __syncthreads();
    lds_fft_n<MX>(lds, rfft_len(a.nbin), a.T, false);
    double2 *o = a.out + row * (int64_t)(N + 1);
    for (int k = threadIdx.x; k <= N; k += kBlock) o[k] = rbin(lds, a.nbin, a.T2, k);
}

// ===========================================================================
// k_xspec: one workgroup per (sub-integration, block of channels)
// ===========================================================================
template <int LOG2N, int DT>
__global__ __launch_bounds__(kBlock) void k_xspec(XspecArgs a) {
    constexpr int N = 1 << LOG2N, NH = N + 1;
    constexpr bool TWL = (N <= 1024);                 // twiddles in LDS
    constexpr int ZP = (N + kBlock - 1) / kBlock;      // row elements / thread
    constexpr int KM = (NH + kBlock - 1) / kBlock;     // harmonics / thread
    using RowT = typename std::conditional<DT == 0, float2, double2>::type;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double red[kWaves * 4];
    double2 *buf = lds;
    const int tid = threadIdx.x;
    if (TWL) {
        for (int j = tid; j < N; j += kBlock) { lds[N + j] = a.T[j]; lds[2 * N + j] = a.T2[j]; }
    }
    const double2 *T = TWL ? lds + N : a.T;
    const double2 *T2 = TWL ? lds + 2 * N : a.T2;
    // XCD-aware block -> (sub-int, channel block): blocks b and b+8 share an
    // XCD, so each XCD keeps only its channel blocks' model rows in its L2
    int s, cb;
    if (a.xcd_swizzle) {
        const int per = a.nblk / 8, x = blockIdx.x % 8, r = blockIdx.x / 8;
        cb = x * per + r % per;
        s = r / per;
    } else {
        s = blockIdx.x / a.nblk;
        cb = blockIdx.x % a.nblk;
    }
    const int c0 = cb * a.cb, c1 = min(a.nchan, c0 + a.cb);
    const int mi = a.model_index ? a.model_index[s] : 0;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double sqrt_half_nbin = sqrt((double)(2 * N) / 2.0);
    const RowT *rows = reinterpret_cast<const RowT *>(a.data);

    auto skip_masked = [&](int n) {
        while (n < c1 && mask && !mask[n]) {
            if (tid < 4) a.chan[((int64_t)s * a.nchan + n) * 4 + tid] = 0.0;
            ++n;
        }
        return n;
    };
    RowT zr[ZP];
    auto prefetch = [&](int n) {
        const RowT *src = rows + ((int64_t)s * a.nchan + n) * N;
#pragma unroll
        for (int q = 0; q < ZP; ++q) {
            const int j = tid + q * kBlock;
            if (j < N) zr[q] = src[j];
        }
    };
    int n = skip_masked(c0);
    if (n < c1) prefetch(n);
    while (n < c1) {
        const int64_t crow = (int64_t)s * a.nchan + n;
#pragma unroll
        for (int q = 0; q < ZP; ++q) {
            const int j = tid + q * kBlock;
            if (j < N) buf[j] = cmk((double)zr[q].x, (double)zr[q].y);
        }
        const int nn = skip_masked(n + 1);
        if (nn < c1) prefetch(nn);              // next row in flight during this FFT
        const double2 *Mrow = a.Mft + ((int64_t)mi * a.nchan + n) * NH;
        double2 Mv[KM];
#pragma unroll
        for (int i = 0; i < KM; ++i) {
            const int k = tid + i * kBlock;
            if (k <= N) Mv[i] = Mrow[k];
        }
        __syncthreads();
        lds_fft_t<LOG2N, false>(buf, T);
        // pass 1 over my harmonics: power sums
        double acc[2] = {0.0, 0.0};
#pragma unroll
        for (int i = 0; i < KM; ++i) {
            const int k = tid + i * kBlock;
            if (k <= N) {
                const double2 D = rfft_bin(buf, N, T2, k);
                const double p2 = cabs2(D);
                if (k >= a.kc) acc[0] += p2;
                if (k >= 1) acc[1] += p2;
            }
        }
        block_sum<2>(acc, red);                 // buf is not modified here
        double errs_FT;
        if (a.errs) errs_FT = a.errs[crow] * sqrt_half_nbin;
        else errs_FT = sqrt(acc[0] / (double)(NH - a.kc) / (double)(2 * N)) * sqrt_half_nbin;
        const double inv_e2 = 1.0 / (errs_FT * errs_FT);
        double2 *Xrow = a.X + (int64_t)(a.xslot ? a.xslot[s] : s) * NH * a.nchan + n;   // X[slot][k][n]
        const int64_t xs = a.nchan;
        double mpow[1] = {0.0};
        // pass 2: cross spectrum (D recomputed from the LDS spectrum)
#pragma unroll
        for (int i = 0; i < KM; ++i) {
            const int k = tid + i * kBlock;
            if (k <= N) {
                const double2 M = Mv[i];
                if (k == 0) {
                    Xrow[0] = cmk(0.0, 0.0);       // F0_fact = 0 (pplib.py:82)
                } else {
                    mpow[0] += cabs2(M);
                    Xrow[k * xs] = cscale(cmulc(rfft_bin(buf, N, T2, k), M), inv_e2);
                }
            }
        }
        block_sum<1>(mpow, red);
        if (tid == 0) {
            double *chan = a.chan + crow * 4;
            chan[0] = errs_FT;
            chan[1] = inv_e2;
            chan[2] = acc[1] * inv_e2;     // Sd_n
            chan[3] = mpow[0] * inv_e2;    // S_n at tau = 0
        }
        n = nn;
    }
}

// ===========================================================================
// k_xspec_any: k_xspec for nbin / 2 not a power of two (mixed-radix LDS FFT,
// lds_fft_n): the same per-row arithmetic, rows loaded straight into LDS
// ===========================================================================
template <int DT>
__global__ __launch_bounds__(kBlock) void k_xspec_any(XspecArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double red[kWaves * 4];
    const int N = a.nbin >> 1, NH = N + 1;
    const int tid = threadIdx.x;
    int s, cb;
    if (a.xcd_swizzle) {
        const int per = a.nblk / 8, x = blockIdx.x % 8, r = blockIdx.x / 8;
        cb = x * per + r % per;
        s = r / per;
    } else {
        s = blockIdx.x / a.nblk;
        cb = blockIdx.x % a.nblk;
    }
    if (a.needx && !a.needx[s]) return;
    const int c0 = cb * a.cb, c1 = min(a.nchan, c0 + a.cb);
    const int mi = a.model_index ? a.model_index[s] : 0;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double sqrt_half_nbin = sqrt((double)a.nbin / 2.0);
    for (int n = c0; n < c1; ++n) {
        const int64_t crow = (int64_t)s * a.nchan + n;
        if (mask && !mask[n]) {
            if (tid < 4) a.chan[crow * 4 + tid] = 0.0;
            continue;
        }
        load_row(lds, a.data, DT, crow, a.nbin);
        __syncthreads();
        lds_fft_n(lds, rfft_len(a.nbin), a.T, false);
        double acc[2] = {0.0, 0.0};
        for (int k = tid; k <= N; k += kBlock) {
            const double p2 = cabs2(rbin(lds, a.nbin, a.T2, k));
            if (k >= a.kc) acc[0] += p2;
            if (k >= 1) acc[1] += p2;
        }
        block_sum<2>(acc, red);
        double errs_FT;
        if (a.errs) errs_FT = a.errs[crow] * sqrt_half_nbin;
        else errs_FT = sqrt(acc[0] / (double)(NH - a.kc) / (double)a.nbin) * sqrt_half_nbin;
        const double inv_e2 = 1.0 / (errs_FT * errs_FT);
        double2 *Xrow = a.X + (int64_t)(a.xslot ? a.xslot[s] : s) * NH * a.nchan + n;
        const double2 *Mrow = a.Mft + ((int64_t)mi * a.nchan + n) * NH;
        double mpow[1] = {0.0};
        for (int k = tid; k <= N; k += kBlock) {
            if (k == 0) {
                Xrow[0] = cmk(0.0, 0.0);
            } else {
                const double2 M = Mrow[k];
                mpow[0] += cabs2(M);
                Xrow[(int64_t)k * a.nchan] = cscale(cmulc(rbin(lds, a.nbin, a.T2, k), M), inv_e2);
            }
        }
        block_sum<1>(mpow, red);          // (its barriers also end this row's reads)
        if (tid == 0) {
            double *chan = a.chan + crow * 4;
            chan[0] = errs_FT;
            chan[1] = inv_e2;
            chan[2] = acc[1] * inv_e2;
            chan[3] = mpow[0] * inv_e2;
        }
    }
}

// the guess profiles of long rows: prof[s][t] = sum_b gP[s][b][t] (the
// block partials of k_dsum in k_guess's order), for their long rFFT
__global__ __launch_bounds__(kBlock) void k_gsum(int nblkd, int nbin, const double *gP, double *prof) {
    const int64_t s = blockIdx.y;
    for (int t = blockIdx.x * kBlock + threadIdx.x; t < nbin; t += gridDim.x * kBlock) {
        double p = 0.0;
        for (int b = 0; b < nblkd; ++b) p += gP[((int64_t)s * nblkd + b) * nbin + t];
        prof[s * nbin + t] = p;
    }
}

hipError_t launch_gsum(int nsub, int nblkd, int nbin, const double *gP, double *prof, hipStream_t st) {
    hipLaunchKernelGGL(k_gsum, dim3((unsigned)((nbin + kBlock - 1) / kBlock), (unsigned)nsub), dim3(kBlock), 0,
                       st, nblkd, nbin, gP, prof);
    return hipGetLastError();
}

// ===========================================================================
// k_xspec_spec: k_xspec_any's per-row arithmetic on rows whose rFFT was
// taken beforehand (a.spec, the long-row transforms of ppf_longfft.hip:
// even nbin > 8192, odd > 4095; round 6) -- noise, Sd_n, S_n and X from the
// stored bins, no LDS transform
// ===========================================================================
__global__ __launch_bounds__(kBlock) void k_xspec_spec(XspecArgs a) {
    __shared__ double red[kWaves * 4];
    const int N = a.nbin >> 1, NH = N + 1;
    const int tid = threadIdx.x;
    const int s = blockIdx.x / a.nblk, cb = blockIdx.x % a.nblk;
    if (a.needx && !a.needx[s]) return;
    const int c0 = cb * a.cb, c1 = min(a.nchan, c0 + a.cb);
    const int mi = a.model_index ? a.model_index[s] : 0;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double sqrt_half_nbin = sqrt((double)a.nbin / 2.0);
    for (int n = c0; n < c1; ++n) {
        const int64_t crow = (int64_t)s * a.nchan + n;
        if (mask && !mask[n]) {
            if (tid < 4) a.chan[crow * 4 + tid] = 0.0;
            continue;
        }
        const double2 *D = a.spec + crow * NH;
        double acc[2] = {0.0, 0.0};
        for (int k = tid; k <= N; k += kBlock) {
            const double p2 = cabs2(D[k]);
            if (k >= a.kc) acc[0] += p2;
            if (k >= 1) acc[1] += p2;
        }
        block_sum<2>(acc, red);
        double errs_FT;
        if (a.errs) errs_FT = a.errs[crow] * sqrt_half_nbin;
        else errs_FT = sqrt(acc[0] / (double)(NH - a.kc) / (double)a.nbin) * sqrt_half_nbin;
        const double inv_e2 = 1.0 / (errs_FT * errs_FT);
        double2 *Xrow = a.X + (int64_t)(a.xslot ? a.xslot[s] : s) * NH * a.nchan + n;
        const double2 *Mrow = a.Mft + ((int64_t)mi * a.nchan + n) * NH;
        double mpow[1] = {0.0};
        for (int k = tid; k <= N; k += kBlock) {
            if (k == 0) {
                Xrow[0] = cmk(0.0, 0.0);
            } else {
                const double2 M = Mrow[k];
                mpow[0] += cabs2(M);
                Xrow[(int64_t)k * a.nchan] = cscale(cmulc(D[k], M), inv_e2);
            }
        }
        block_sum<1>(mpow, red);
        if (tid == 0) {
            double *chan = a.chan + crow * 4;
            chan[0] = errs_FT;
            chan[1] = inv_e2;
            chan[2] = acc[1] * inv_e2;
            chan[3] = mpow[0] * inv_e2;
        }
    }
}

hipError_t launch_xspec_spec(const XspecArgs &a, hipStream_t st) {
    hipLaunchKernelGGL(k_xspec_spec, dim3((unsigned)((int64_t)a.nsub * a.nblk)), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}

// ===========================================================================
// 1-D FFTFIT objective and scipy brute + fmin replica (pplib.py:1294-1306,
// 2136-2182; scipy.optimize.brute / _minimize_neldermead), one workgroup.
// xm[k] = D_k conj(M_k) (k = 0 zeroed), in LDS.
// ===========================================================================
// wave-level evaluation of -Re sum_k xm_k exp(2 pi i k phase) / err2
__device__ double wave_fps_eval(const double2 *xm, int nharm, double phase, double inv_err2) {
    const int lane = threadIdx.x & 63;
    double2 E = cexp2pi((double)lane * phase);
    const double2 W = cexp2pi(64.0 * phase);
    double acc = 0.0;
    for (int k = lane; k < nharm; k += 64) {
        double2 x = xm[k];
        acc = fma(x.x, E.x, fma(-x.y, E.y, acc));
        E = cmul(E, W);
    }
    return -wave_sum(acc) * inv_err2;
}

// Brute grid over Ns points of [lo, hi] (all waves), then fmin polish (wave
// 0).  Returns the phase in every thread; fval/nfev via pointers (thread 0).
// exp(i pi m^2 / L), m^2 reduced mod 2L in integers (exact phase; 32-bit:
// |m|, L < 2^13 here, so r^2 < 2^28)
__device__ __forceinline__ double2 cz_chirp(int m, int L) {
    int r = m % (2 * L);
    if (r < 0) r += 2 * L;
    const int e = (r * r) % (2 * L);
    double s, c;
    sincospi((double)e / (double)L, &s, &c);
    return cmk(c, s);
}

// the chirp z-transform's P-point FFTs: the compile-time-size Stockham
// passes, a k_guess instantiation per size (CZL = log2 P: 9, 10, 11 for
// nbin 512, 1024, 2048).  In one kernel beside each other (or as the
// runtime-size lds_fft) they took k_guess from four waves per SIMD to three
// or two; alone, the 1024-point one keeps it at four.
template <int CZL, bool INV>
__device__ __forceinline__ void cz_fft(double2 *buf, const double2 *T) {
    lds_fft_t<CZL, INV>(buf, T);
}

// The brute grid of a whole turn as a chirp z-transform (round 6).  With
// L = Ns - 1 and phi_j = lo + j / L, e^{2 pi i k phi_j} = e^{2 pi i k lo}
// nu^{k^2} nu^{j^2} nu^{-(j-k)^2}, nu = e^{i pi / L}, so
//   S_j = Re sum_k xm_k e^{2 pi i k phi_j} = Re nu^{j^2} (a * b)_j,
//   a_k = xm_k e^{2 pi i k lo} nu^{k^2}, b_m = nu^{-m^2}:
// per chunk of J outputs one P-point circular convolution against the
// chunk's precomputed FFT_P(b) (k_cz_table), 2 Q block FFTs in all
// instead of Ns x nharm phasor products.  buf: P double2 of LDS.
// (inline: out of line, as a function compiled without the kernel's occupancy
// target, it took 248 VGPRs + spills)
template <int CZL>
__device__ __forceinline__ void cz_grid(const double2 *xm, int nharm, double inv_err2, int Ns, double lo,
                                     double *sh, double2 *buf, const double2 *czB, const double2 *czT, int J,
                                     int Q, int K) {
    constexpr int P = 1 << CZL;
    const int L = Ns - 1;
    // per chunk: FFT_P(a) (rebuilt: kept in registers it would pin
    // kMaxFftN / kBlock complex values per thread), times the chunk's
    // FFT_P(b), inverse, the chunk's outputs
    for (int q = 0; q < Q; ++q) {
        for (int k = threadIdx.x; k < P; k += kBlock) {
            double2 a = cmk(0.0, 0.0);
            if (k < nharm && k < K) a = cmul(cmul(xm[k], cexp2pi((double)k * lo)), cz_chirp(k, L));
            buf[k] = a;
        }
        __syncthreads();
        cz_fft<CZL, false>(buf, czT);
        __syncthreads();
        const double2 *Bq = czB + (int64_t)q * P;
        for (int t = threadIdx.x; t < P; t += kBlock) buf[t] = cmul(buf[t], Bq[t]);
        __syncthreads();
        cz_fft<CZL, true>(buf, czT);
        __syncthreads();
        for (int t = threadIdx.x; t < J; t += kBlock) {
            const int j = q * J + t;
            if (j < Ns) {
                const double2 c = buf[t + K - 1];
                const double2 w = cz_chirp(j, L);
                sh[j] = -(c.x * w.x - c.y * w.y) * inv_err2;
            }
        }
        __syncthreads();
    }
}

// FFT_P of each chunk's chirp kernel b'_t = nu^{-(t + qJ - (K-1))^2}
// (t < K + J - 1; 0 past), scaled by 1/P: one block per chunk
__global__ __launch_bounds__(kBlock) void k_cz_table(CzPlan c, double2 *B, const double2 *T) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int q = blockIdx.x;
    const int L = c.Ns - 1;
    for (int t = threadIdx.x; t < c.P; t += kBlock) {
        double2 b = cmk(0.0, 0.0);
        if (t < c.K + c.J - 1) b = cconj(cz_chirp(t + q * c.J - (c.K - 1), L));
        lds[t] = b;
    }
    __syncthreads();
    int log2P = 0;
    while ((1 << log2P) < c.P) ++log2P;
    lds_fft(lds, log2P, T, false);
    __syncthreads();
    for (int t = threadIdx.x; t < c.P; t += kBlock) B[(int64_t)q * c.P + t] = cscale(lds[t], 1.0 / (double)c.P);
}

hipError_t launch_cz_table(const CzPlan &c, double2 *B, const double2 *T, hipStream_t st) {
    hipLaunchKernelGGL(k_cz_table, dim3((unsigned)c.Q), dim3(kBlock), sizeof(double2) * (size_t)c.P, st, c, B, T);
    return hipGetLastError();
}

// grid_done: sh[0..Ns) already holds the grid (cz_grid)
__device__ double brute_fmin(const double2 *xm, int nharm, double inv_err2, int Ns, double lo,
                             double hi, double *sh /*LDS >= 2*Ns+8*/, double *fval, int *nfev,
                             bool grid_done = false) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double step = (Ns != 1) ? (hi - lo) / (double)(Ns - 1) : 1.0;
#ifndef PPF_GUESS_DIAG
#define PPF_GUESS_DIAG 0    // timing-only builds: 1 no brute grid, 2 no polish
#endif
    if (PPF_GUESS_DIAG & 1) {
        for (int j = threadIdx.x; j < Ns; j += kBlock) sh[j] = (double)j;
    } else if (grid_done) {
    } else if (Ns >= 2 * kBlock) {
        // large grids (ppalign: Ns = nbin): one point per lane, two points
        // in flight; harmonics broadcast from LDS, phasor e^{2 pi i k ph} by
        // recurrence, re-seeded exactly every 64 harmonics
        for (int j0 = threadIdx.x; j0 < Ns; j0 += 2 * kBlock) {
            const int j1 = j0 + kBlock;
            const double ph0 = (double)j0 * step + lo;
            const double ph1 = (double)(j1 < Ns ? j1 : j0) * step + lo;
            const double2 W0 = cexp2pi(ph0), W1 = cexp2pi(ph1);
            double acc0 = 0.0, acc1 = 0.0;
            for (int kb = 0; kb < nharm; kb += 64) {
                double2 E0 = cexp2pi((double)kb * ph0), E1 = cexp2pi((double)kb * ph1);
                const int ke = min(nharm, kb + 64);
                for (int k = kb; k < ke; ++k) {
                    const double2 x = xm[k];
                    acc0 = fma(x.x, E0.x, fma(-x.y, E0.y, acc0));
                    acc1 = fma(x.x, E1.x, fma(-x.y, E1.y, acc1));
                    E0 = cmul(E0, W0);
                    E1 = cmul(E1, W1);
                }
            }
            sh[j0] = -acc0 * inv_err2;
            if (j1 < Ns) sh[j1] = -acc1 * inv_err2;
        }
    } else {
        for (int j = wave; j < Ns; j += kWaves) {
            double ph = (double)j * step + lo;
            double f = wave_fps_eval(xm, nharm, ph, inv_err2);
            if (lane == 0) sh[j] = f;
        }
    }
    __syncthreads();
    if (wave == 0) {
        // argmin (first occurrence), computed redundantly by the wave
        int jmin = 0;
        double fmin_ = sh[0];
        for (int j = 1; j < Ns; ++j)
            if (sh[j] < fmin_) { fmin_ = sh[j]; jmin = j; }
        double x0 = (double)jmin * step + lo;
        // Nelder-Mead, N = 1, rho=1 chi=2 psi=0.5 sigma=0.5, xatol=fatol=1e-4,
        // maxiter = maxfun = 200 (scipy fmin defaults)
        double sim0 = x0, sim1 = (x0 != 0.0) ? 1.05 * x0 : 0.00025;
        int nf = 0;
        double f0 = wave_fps_eval(xm, nharm, sim0, inv_err2); ++nf;
        double f1 = wave_fps_eval(xm, nharm, sim1, inv_err2); ++nf;
        if (f1 < f0) { double t = sim0; sim0 = sim1; sim1 = t; t = f0; f0 = f1; f1 = t; }
        int iters = 1;
        while (!(PPF_GUESS_DIAG & 2) && nf < 200 && iters < 200) {
            if (fabs(sim1 - sim0) <= 1e-4 && fabs(f0 - f1) <= 1e-4) break;
            double xbar = sim0;
            double xr = 2.0 * xbar - sim1;
            double fxr = wave_fps_eval(xm, nharm, xr, inv_err2); ++nf;
            bool shrink = false;
            if (fxr < f0) {
                double xe = 3.0 * xbar - 2.0 * sim1;
                double fxe = wave_fps_eval(xm, nharm, xe, inv_err2); ++nf;
                if (fxe < fxr) { sim1 = xe; f1 = fxe; } else { sim1 = xr; f1 = fxr; }
            } else {
                // N = 1: fsim[-2] is fsim[0], so "fxr < fsim[-2]" is never true
                if (fxr < f1) {
                    double xc = 1.5 * xbar - 0.5 * sim1;
                    double fxc = wave_fps_eval(xm, nharm, xc, inv_err2); ++nf;
                    if (fxc <= fxr) { sim1 = xc; f1 = fxc; } else shrink = true;
                } else {
                    double xcc = 0.5 * xbar + 0.5 * sim1;
                    double fxcc = wave_fps_eval(xm, nharm, xcc, inv_err2); ++nf;
                    if (fxcc < f1) { sim1 = xcc; f1 = fxcc; } else shrink = true;
                }
                if (shrink) {
                    sim1 = sim0 + 0.5 * (sim1 - sim0);
                    f1 = wave_fps_eval(xm, nharm, sim1, inv_err2); ++nf;
                }
            }
            ++iters;
            if (f1 < f0) { double t = sim0; sim0 = sim1; sim1 = t; t = f0; f0 = f1; f1 = t; }
        }
        if (lane == 0) { sh[Ns] = sim0; sh[Ns + 1] = fmin(f0, f1); sh[Ns + 2] = (double)nf; }
    }
    __syncthreads();
    double ph = sh[Ns];
    if (fval) *fval = sh[Ns + 1];
    if (nfev) *nfev = (int)sh[Ns + 2];
    __syncthreads();
    return ph;
}

// ===========================================================================
// k_dsum: the GetTOAs guess profile (pptoas.py:461-464): the portrait
// rotated by the guess DM relative to the mean usable frequency and
// averaged with the channel weights, rot_prof(t) = sum_n w_n x_n(t + tau_n) /
// sum_n w_n, tau_n = nbin Dconst DM/P (nu_n^-2 - nu_mean^-2).  The shift is
// applied in the time domain by linear interpolation between bins (the
// reference rotates each channel in the Fourier domain): this profile only
// seeds the phase of the trust-region fit, whose converged result does not
// depend on it, and the pass then streams the data once at HBM rate with no
// per-channel FFT.  Grid: (sub-int, block of cbd channels); thread t owns
// bins t + 256 j; output: the block's partial sum (fixed channel order).
// ===========================================================================
template <int DT, int JB>
__global__ __launch_bounds__(kBlock) void k_dsum(DsumArgs a) {
    using ElT = typename std::conditional<DT == 0, float, double>::type;
    __shared__ double red[kWaves * 4];
    const int tid = threadIdx.x;
    const int s = blockIdx.x / a.nblkd, blk = blockIdx.x % a.nblkd;
    if (a.gflag && a.gflag[s]) return;        // guess fused into k_xspec_w
    const int nbin = a.nbin;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double *fr = a.freqs + (int64_t)s * a.nchan;
    double v[2] = {0.0, 0.0};
    for (int n = tid; n < a.nchan; n += kBlock)
        if (!mask || mask[n]) { v[0] += fr[n]; v[1] += 1.0; }
    block_sum<2>(v, red);
    const double Dg = kDconst * a.guess_DM[s] / a.P[s];
    double nu_mean_m2 = pow(v[0] / v[1], -2.0);
    if (a.guess_ref) {                       // ppalign: dedisperse at nu_fit
        const double nf = a.nu_fits[(int64_t)s * 3];
        if (nf == nf) nu_mean_m2 = pow(nf, -2.0);
    }
    const int c0 = blk * a.cbd, c1 = min(a.nchan, c0 + a.cbd);
    const ElT *rows = reinterpret_cast<const ElT *>(a.data) + (int64_t)s * a.nchan * nbin;
    double wsum = 0.0, wcnt = 0.0;
    for (int t0 = 0; t0 < nbin; t0 += JB * kBlock) {
        double p[JB];
#pragma unroll
        for (int j = 0; j < JB; ++j) p[j] = 0.0;
        for (int n = c0; n < c1; ++n) {
            if (mask && !mask[n]) continue;
            const double w = a.guess_weights[(int64_t)s * a.nchan + n];
            const double tau = (double)nbin * Dg * (pow(fr[n], -2.0) - nu_mean_m2);
            const double fl = floor(tau);
            const double f = tau - fl;
            const int i0 = (int)(fl - (double)nbin * floor(fl / (double)nbin));   // mod nbin
            const double wa = w * (1.0 - f), wb = w * f;
            const ElT *x = rows + (int64_t)n * nbin;
#pragma unroll
            for (int j = 0; j < JB; ++j) {
                const int t = t0 + tid + j * kBlock;
                if (t < nbin) {
                    // (t + i0) mod nbin and its successor (any nbin)
                    const int ia = t + i0 >= nbin ? t + i0 - nbin : t + i0;
                    const int ib = ia + 1 == nbin ? 0 : ia + 1;
                    p[j] = fma(wa, (double)x[ia], fma(wb, (double)x[ib], p[j]));
                }
            }
            if (t0 == 0) { wsum += w; wcnt += 1.0; }
        }
        double *out = a.gP + ((int64_t)s * a.nblkd + blk) * nbin;
#pragma unroll
        for (int j = 0; j < JB; ++j) {
            const int t = t0 + tid + j * kBlock;
            if (t < nbin) out[t] = p[j];
        }
    }
    if (tid == 0) {
        a.gw[((int64_t)s * a.nblkd + blk) * 2 + 0] = wsum;
        a.gw[((int64_t)s * a.nblkd + blk) * 2 + 1] = wcnt;
    }
}

// nu_ref^-2 of sub-int s for the wave-per-row guess passes: the mean usable
// frequency (GetTOAs, pptoas.py:461-464) or nu_fit (ppalign), one wave's
// fixed-order sum.  At many channels (C5: 16,384) every workgroup of
// k_dsum_w repeating this over the whole band cost more than its rows'
// loads, so k_nu_ref forms it once per sub-int (same arithmetic, same bits).
__device__ __forceinline__ double nu_ref_m2(const DsumArgs &a, int s, int lane) {
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double *fr = a.freqs + (int64_t)s * a.nchan;
    double v0 = 0.0, v1 = 0.0;
    // (loads unconditional, so that eight channels' loads are in flight;
    // adding 0.0 for a masked channel leaves the sums' bits unchanged)
#pragma unroll 8
    for (int n = lane; n < a.nchan; n += 64) {
        const double f = fr[n];
        const bool ok = !mask || mask[n];
        v0 += ok ? f : 0.0;
        v1 += ok ? 1.0 : 0.0;
    }
    v0 = wave_sum(v0);
    v1 = wave_sum(v1);
    const double mu = v0 / v1;
    double nu_mean_m2 = 1.0 / (mu * mu);
    if (a.guess_ref) {                       // ppalign: dedisperse at nu_fit
        const double nf = a.nu_fits[(int64_t)s * 3];
        if (nf == nf) nu_mean_m2 = 1.0 / (nf * nf);
    }
    return nu_mean_m2;
}

__global__ __launch_bounds__(64) void k_nu_ref(DsumArgs a) {
    const int s = blockIdx.x;
    if (a.gflag && a.gflag[s]) return;
    const double v = nu_ref_m2(a, s, threadIdx.x);
    if (threadIdx.x == 0) a.nuref[s] = v;
}

// ===========================================================================
// k_dsum_w: k_dsum with one wave per channel row (256 <= nbin <= 2048).
// Each wave streams its rows (channels c0 + wave + 4 i) with 16-B loads, one
// row in flight ahead of the one being summed, stages the row in its own LDS
// slice and accumulates the shifted, interpolated row into nbin/64 register
// accumulators per lane (output bin t = lane + 64 j); no workgroup barrier in
// the row loop.  The four waves' sums are added in wave order through LDS
// (deterministic) and the block's partial profile is written once.
// ===========================================================================
// rows in flight per wave (1: the one being summed has a successor loading;
// 2 measured slower: C5 k_dsum_w 9.25 vs 8.39 ms per 500 sub-ints, the
// extra VGPRs cost occupancy)
#ifndef PPF_DSUM_DEPTH
#define PPF_DSUM_DEPTH 1
#endif
template <int DT, int LOG2NB>
// (capped at four waves per SIMD -- 128 VGPRs, nine spills -- it measured
// 8.2 vs 7.1 ms per 10,000 C2 sub-ints)
__global__ __launch_bounds__(kBlock) void k_dsum_w(DsumArgs a) {
    using ElT = typename std::conditional<DT == 0, float, double>::type;
    // native vector types: arrays of HIP_vector_type structs carried across
    // the row loop are not promoted to VGPRs (they land in scratch)
    typedef float vf4 __attribute__((ext_vector_type(4)));
    typedef double vd2 __attribute__((ext_vector_type(2)));
    using VecT = typename std::conditional<DT == 0, vf4, vd2>::type;
    constexpr int NB = 1 << LOG2NB, J = NB / 64, VW = 16 / (int)sizeof(ElT);
    constexpr int NL = NB / (64 * VW);                 // 16-B loads per lane per row
    extern __shared__ __attribute__((aligned(16))) double dlds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    ElT *xs = reinterpret_cast<ElT *>(dlds) + wave * NB;
    const int s = blockIdx.x / a.nblkd, blk = blockIdx.x % a.nblkd;
    if (a.gflag && a.gflag[s]) return;        // guess fused into k_xspec_w
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double *fr = a.freqs + (int64_t)s * a.nchan;
    const double *gwt = a.guess_weights + (int64_t)s * a.nchan;
    const double Dg = (double)NB * kDconst * a.guess_DM[s] / a.P[s];
    const double nu_mean_m2 = a.nuref ? a.nuref[s] : nu_ref_m2(a, s, lane);
    const int c0 = blk * a.cbd, c1 = min(a.nchan, c0 + a.cbd);
    const VecT *rows = reinterpret_cast<const VecT *>(a.data) + (int64_t)s * a.nchan * (NB / VW);
    // the block's channel scalars in lane registers (channel c0 + lane + 64 k,
    // cbd <= 128), broadcast by readlane: a global load of the weight or the
    // frequency after the next row's prefetch would wait for that prefetch
    // (vmcnt counts in order), i.e. only one row would be in flight
    double t_w[2], t_f[2];
    int t_m[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int ch = c0 + lane + 64 * k;
        const bool in = ch < c1;
        t_w[k] = in ? gwt[ch] : 0.0;
        t_f[k] = in ? fr[ch] : 1.0;
        t_m[k] = (in && (!mask || mask[ch])) ? 1 : 0;
    }
    auto usable = [&](int n) {
        const int r = n - c0;
        return n < c1 && __builtin_amdgcn_readlane(r < 64 ? t_m[0] : t_m[1], r & 63) != 0;
    };
    double acc[J];
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = 0.0;
    double wsum = 0.0, wcnt = 0.0;
#if PPF_DSUM_DEPTH >= 2
    // two rows in flight per wave: the row being summed comes from one
    // register buffer while the next two are loading (the second buffer and
    // the refill of the first)
    auto next_usable = [&](int m) {
        m += kWaves;
        while (m < c1 && !usable(m)) m += kWaves;
        return m;
    };
    auto load = [&](VecT (&p)[NL], int m) {
        // unconditional (a valid row when past the block): keeps p in VGPRs
        const VecT *src = rows + (int64_t)(m < c1 ? m : c1 - 1) * (NB / VW);
#pragma unroll
        for (int i = 0; i < NL; ++i) p[i] = ld_stream(src + lane + 64 * i);
    };
    auto row = [&](VecT (&p)[NL], int m, int m2) {
        wave_lds_sync();                      // the previous row's reads are issued
#pragma unroll
        for (int i = 0; i < NL; ++i) reinterpret_cast<VecT *>(xs)[lane + 64 * i] = p[i];
        load(p, m2);
        const int r = m - c0;
        const double w = readlane_d(r < 64 ? t_w[0] : t_w[1], r & 63),
                     f0 = readlane_d(r < 64 ? t_f[0] : t_f[1], r & 63);
        const double tau = Dg * (1.0 / (f0 * f0) - nu_mean_m2);
        const double fl = floor(tau), f = tau - fl;
        const int i0 = (int)(fl - (double)NB * floor(fl / (double)NB));   // mod nbin
        const double wa = w * (1.0 - f), wb = w * f;
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int ia = (lane + 64 * j + i0) & (NB - 1);
            acc[j] = fma(wa, (double)xs[ia], fma(wb, (double)xs[(ia + 1) & (NB - 1)], acc[j]));
        }
        wsum += w;
        wcnt += 1.0;
    };
    int n = c0 + wave;
    while (n < c1 && !usable(n)) n += kWaves;
    int n1 = next_usable(n);
    VecT pa[NL], pb[NL];
    load(pa, n);
    load(pb, n1);
    while (n < c1) {
        int n2 = next_usable(n1);
        row(pa, n, n2);                       // pa: n -> n2
        n = n1;
        n1 = n2;
        if (n >= c1) break;
        n2 = next_usable(n1);
        row(pb, n, n2);                       // pb: n -> the row after n1
        n = n1;
        n1 = n2;
    }
#else
    int n = c0 + wave;
    while (n < c1 && !usable(n)) n += kWaves;
    VecT pre[NL];
    {
        const VecT *src = rows + (int64_t)min(n, c1 - 1) * (NB / VW);
#pragma unroll
        for (int i = 0; i < NL; ++i) pre[i] = src[lane + 64 * i];
    }
    while (n < c1) {
        wave_lds_sync();                      // the previous row's reads are issued
#pragma unroll
        for (int i = 0; i < NL; ++i) reinterpret_cast<VecT *>(xs)[lane + 64 * i] = pre[i];
        int nn = n + kWaves;
        while (nn < c1 && !usable(nn)) nn += kWaves;
        {
            // next row in flight during this one (unconditional load: keeps
            // pre[] in VGPRs)
            const VecT *src = rows + (int64_t)(nn < c1 ? nn : n) * (NB / VW);
#pragma unroll
            for (int i = 0; i < NL; ++i) pre[i] = src[lane + 64 * i];
        }
        const int r = n - c0;
        const double w = readlane_d(r < 64 ? t_w[0] : t_w[1], r & 63),
                     f0 = readlane_d(r < 64 ? t_f[0] : t_f[1], r & 63);
        const double tau = Dg * (1.0 / (f0 * f0) - nu_mean_m2);
        const double fl = floor(tau), f = tau - fl;
        const int i0 = (int)(fl - (double)NB * floor(fl / (double)NB));   // mod nbin
        const double wa = w * (1.0 - f), wb = w * f;
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int ia = (lane + 64 * j + i0) & (NB - 1);
            acc[j] = fma(wa, (double)xs[ia], fma(wb, (double)xs[(ia + 1) & (NB - 1)], acc[j]));
        }
        wsum += w;
        wcnt += 1.0;
        n = nn;
    }
#endif
    // fixed-order sum of the four waves' profiles (LDS reused as NB doubles)
    __syncthreads();
    double *part = dlds;
    for (int w2 = 0; w2 < kWaves; ++w2) {
        if (wave == w2) {
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int t = lane + 64 * j;
                part[t] = w2 == 0 ? acc[j] : part[t] + acc[j];
            }
        }
        __syncthreads();
    }
    double *out = a.gP + ((int64_t)s * a.nblkd + blk) * NB;
    for (int t = threadIdx.x; t < NB; t += kBlock) out[t] = part[t];
    __shared__ double wred[kWaves * 2];
    if (lane == 0) { wred[wave * 2] = wsum; wred[wave * 2 + 1] = wcnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s0 = 0.0, s1 = 0.0;
        for (int w2 = 0; w2 < kWaves; ++w2) { s0 += wred[w2 * 2]; s1 += wred[w2 * 2 + 1]; }
        a.gw[((int64_t)s * a.nblkd + blk) * 2 + 0] = s0;
        a.gw[((int64_t)s * a.nblkd + blk) * 2 + 1] = s1;
    }
}

// ===========================================================================
// k_dsum_wn: k_dsum_w for any nbin <= NBMAX (nbin not a power of two: 1000,
// 1536, 1022 ...; round 5).  The same wave-per-row streaming (next row in
// flight, channel scalars in lane registers, fixed-order wave sums), with
// per-lane element loads and the (t + i0) mod nbin index by compare-subtract.
// ===========================================================================
template <int DT, int NBMAX>
__global__ __launch_bounds__(kBlock) void k_dsum_wn(DsumArgs a) {
    using ElT = typename std::conditional<DT == 0, float, double>::type;
    constexpr int J = NBMAX / 64;
    extern __shared__ __attribute__((aligned(16))) double dlds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb = a.nbin;
    ElT *xs = reinterpret_cast<ElT *>(dlds) + wave * NBMAX;
    const int s = blockIdx.x / a.nblkd, blk = blockIdx.x % a.nblkd;
    if (a.gflag && a.gflag[s]) return;        // guess fused into the spectrum pass
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double *fr = a.freqs + (int64_t)s * a.nchan;
    const double *gwt = a.guess_weights + (int64_t)s * a.nchan;
    const double Dg = (double)nb * kDconst * a.guess_DM[s] / a.P[s];
    const double nu_mean_m2 = a.nuref ? a.nuref[s] : nu_ref_m2(a, s, lane);
    const int c0 = blk * a.cbd, c1 = min(a.nchan, c0 + a.cbd);
    const ElT *rows = reinterpret_cast<const ElT *>(a.data) + (int64_t)s * a.nchan * nb;
    double t_w[2], t_f[2];
    int t_m[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int ch = c0 + lane + 64 * k;
        const bool in = ch < c1;
        t_w[k] = in ? gwt[ch] : 0.0;
        t_f[k] = in ? fr[ch] : 1.0;
        t_m[k] = (in && (!mask || mask[ch])) ? 1 : 0;
    }
    auto usable = [&](int n) {
        const int r = n - c0;
        return n < c1 && __builtin_amdgcn_readlane(r < 64 ? t_m[0] : t_m[1], r & 63) != 0;
    };
    double acc[J];
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = 0.0;
    double wsum = 0.0, wcnt = 0.0;
    // element t = lane + 64 i of a row; past nbin: element nbin - 1 again
    // (unconditional loads keep the prefetch in VGPRs)
    auto load = [&](ElT (&p)[J], int m) {
        const ElT *src = rows + (int64_t)m * nb;
#pragma unroll
        for (int i = 0; i < J; ++i) {
            const int t = lane + 64 * i;
            p[i] = src[t < nb ? t : nb - 1];
        }
    };
    int n = c0 + wave;
    while (n < c1 && !usable(n)) n += kWaves;
    ElT pre[J];
    load(pre, min(n, c1 - 1));
    while (n < c1) {
        wave_lds_sync();                      // the previous row's reads are issued
#pragma unroll
        for (int i = 0; i < J; ++i) xs[lane + 64 * i] = pre[i];
        int nn = n + kWaves;
        while (nn < c1 && !usable(nn)) nn += kWaves;
        load(pre, nn < c1 ? nn : n);          // next row in flight during this one
        const int r = n - c0;
        const double w = readlane_d(r < 64 ? t_w[0] : t_w[1], r & 63),
                     f0 = readlane_d(r < 64 ? t_f[0] : t_f[1], r & 63);
        const double tau = Dg * (1.0 / (f0 * f0) - nu_mean_m2);
        const double fl = floor(tau), f = tau - fl;
        const int i0 = (int)(fl - (double)nb * floor(fl / (double)nb));   // mod nbin
        const double wa = w * (1.0 - f), wb = w * f;
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int t = lane + 64 * j;
            int ia = t + i0;
            ia -= ia >= nb ? nb : 0;
            const int ib = ia + 1 == nb ? 0 : ia + 1;
            if (t < nb) acc[j] = fma(wa, (double)xs[ia], fma(wb, (double)xs[ib], acc[j]));
        }
        wsum += w;
        wcnt += 1.0;
        n = nn;
    }
    // fixed-order sum of the four waves' profiles (LDS reused as NBMAX doubles)
    __syncthreads();
    double *part = dlds;
    for (int w2 = 0; w2 < kWaves; ++w2) {
        if (wave == w2) {
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int t = lane + 64 * j;
                part[t] = w2 == 0 ? acc[j] : part[t] + acc[j];
            }
        }
        __syncthreads();
    }
    double *out = a.gP + ((int64_t)s * a.nblkd + blk) * nb;
    for (int t = threadIdx.x; t < nb; t += kBlock) out[t] = part[t];
    __shared__ double wred[kWaves * 2];
    if (lane == 0) { wred[wave * 2] = wsum; wred[wave * 2 + 1] = wcnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s0 = 0.0, s1 = 0.0;
        for (int w2 = 0; w2 < kWaves; ++w2) { s0 += wred[w2 * 2]; s1 += wred[w2 * 2 + 1]; }
        a.gw[((int64_t)s * a.nblkd + blk) * 2 + 0] = s0;
        a.gw[((int64_t)s * a.nblkd + blk) * 2 + 1] = s1;
    }
}

// ===========================================================================
// k_guess: GetTOAs initial phase (pptoas.py:461-499): FFTFIT of the weighted,
// dedispersed mean profile against the mean model profile, then
// phase_transform to nu_fit_DM (pplib.py:2688-2712).
// ===========================================================================
// the block-partial sums of k_guess (fixed order, so bit-identical either
// way) unrolled 8 deep: their loads independent, in flight together instead
// of one latency each (PPF_GUESS_UNROLL 0: as through round 6's first builds)
#ifndef PPF_GUESS_UNROLL
#define PPF_GUESS_UNROLL 1
#endif
#if PPF_GUESS_UNROLL
#define PPF_GU _Pragma("unroll 8")
#else
#define PPF_GU _Pragma("unroll 1")
#endif
template <bool MX, int CZL = 0, bool GS = false>
__global__ __launch_bounds__(kBlock) void k_guess(GuessArgs a) {
    // lds: z[max(rfft_len, czP)] (packed profile, FFT in place; then the
    // chirp z-transform's buffer; none with gspec) | xm[N+1] | sh[Ns+8]
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double red[kWaves * 4];
    const int N = a.nbin >> 1, nharm = N + 1, s = blockIdx.x, tid = threadIdx.x;
    const bool odd = a.nbin & 1;
    const bool pre = a.gspec != nullptr;      // (uniform) the profile's rFFT given
    double2 *z = lds,
            *xm = lds + (pre ? 0 : (a.czB && a.czP > rfft_len(a.nbin) ? a.czP : rfft_len(a.nbin)));
    // GS (long rows, a grid past the LDS): sh in global memory
    double *sh = GS ? a.gsh + (int64_t)s * (a.Ns + 8) : reinterpret_cast<double *>(xm + nharm + 1);
    // fused (k_xspec_w accumulated the guess spectrum of its rows in the
    // Fourier domain): the block partials of the covered harmonics
    const bool fused = a.gflag && a.gflag[s];
    const int NL = guess_slots(a.log2N);
    if (tid == 0) {
        double w0 = 0.0, w1 = 0.0, w2 = 0.0;
        if (fused) {
            PPF_GU
            for (int b = 0; b < a.nblk; ++b) {
                w0 += a.gwx[((int64_t)s * a.nblk + b) * 3 + 0];
                w1 += a.gwx[((int64_t)s * a.nblk + b) * 3 + 1];
                w2 += a.gwx[((int64_t)s * a.nblk + b) * 3 + 2];
            }
        } else {
            PPF_GU
            for (int b = 0; b < a.nblkd; ++b) {
                w0 += a.gw[((int64_t)s * a.nblkd + b) * 2 + 0];
                w1 += a.gw[((int64_t)s * a.nblkd + b) * 2 + 1];
            }
        }
        sh[0] = w0; sh[1] = w1; sh[2] = w2;
    }
    if (!fused && !pre) {
        // weighted dedispersed profile: sum of the k_dsum block partials
        // (fixed order), packed z_j = p_2j + i p_2j+1 for the real FFT
        // (odd nbin: z_j = p_j)
        for (int j = tid; odd && j < a.nbin; j += kBlock) {
            double pj = 0.0;
            PPF_GU
            for (int b = 0; b < a.nblkd; ++b) pj += a.gP[((int64_t)s * a.nblkd + b) * a.nbin + j];
            z[j] = cmk(pj, 0.0);
        }
        for (int j = tid; !odd && j < N; j += kBlock) {
            double pe = 0.0, po = 0.0;
            PPF_GU
            for (int b = 0; b < a.nblkd; ++b) {
                const double *pp = a.gP + ((int64_t)s * a.nblkd + b) * a.nbin;
                pe += pp[2 * j];
                po += pp[2 * j + 1];
            }
            z[j] = cmk(pe, po);
        }
    }
    __syncthreads();
    const double wsum = sh[0], cnt = sh[1];
    if (!fused && !pre) lds_fft_n<MX>(z, rfft_len(a.nbin), a.T, false);
    // R_k of the fused partials (k < NL; 0 above: past every channel's cutoff)
    auto fused_bin = [&](int k) {
        double2 r = cmk(0.0, 0.0);
        if (k >= 1 && k < NL) {
            PPF_GU
            for (int b = 0; b < a.nblk; ++b) r = cadd(r, a.gpart[((int64_t)s * a.nblk + b) * NL + k]);
        }
        return r;
    };
    double pw[1] = {0.0};
    const int mi = a.model_index ? a.model_index[s] : 0;
    const double2 *Mm = a.Mft + (int64_t)mi * a.nchan * nharm;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const int lane = tid & 63;
    // the mean model has no harmonic above the largest channel cutoff
    // (k_model_cut): the FFTFIT sums stop there
    double kmx[1] = {1.0};
    if (a.KC)
        for (int n = tid; n < a.nchan; n += kBlock)
            kmx[0] = fmax(kmx[0], (double)a.KC[(int64_t)mi * a.nchan + n]);
    else
        kmx[0] = (double)nharm;
    block_max<1>(kmx, red);
    // fused: the noise comes from the channels (below), so only the
    // harmonics the FFTFIT sums read (k < kmx) are formed; otherwise every
    // harmonic, for the power above kc
    const int kloop = fused ? (int)kmx[0] : nharm;
    // uniform trip count: the mask ballots below need every lane active
    for (int k0 = 0; k0 < kloop; k0 += kBlock) {
        const int k = k0 + tid;
        const bool kv = k <= N;
        // mean model profile of the usable channels: the batch sum minus the
        // masked channels' rows in increasing channel order (the masked
        // channels of each 64-channel group found with one ballot)
        double2 M = kv ? a.Msum[(int64_t)mi * nharm + k] : cmk(0.0, 0.0);
        if (mask) {
            for (int n0 = 0; n0 < a.nchan; n0 += 64) {
                const int nl = n0 + lane;
                unsigned long long bits = __ballot(nl < a.nchan && !mask[nl]);
                while (bits) {
                    const int b = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    if (kv) M = csub(M, Mm[(int64_t)(n0 + b) * nharm + k]);
                }
            }
        }
        if (!kv || k >= kloop) continue;
        double2 R = cscale(fused ? fused_bin(k) : (pre ? a.gspec[(int64_t)s * nharm + k] : rbin(z, a.nbin, a.T2, k)),
                           1.0 / wsum);
        M = cscale(M, 1.0 / cnt);
        if (a.guess_tau && a.guess_tau[s] != 0.0) {   // scattered model profile
            double u = kTwoPi * (double)k * a.guess_tau[s];
            double dd = 1.0 / fma(u, u, 1.0);
            M = cmul(M, cmk(dd, -u * dd));
        }
        if (k == N && !odd) R.y = 0.0;   // irfft drops the imaginary Nyquist part
        if (k >= a.kc) pw[0] += cabs2(R);
        xm[k] = (k == 0) ? cmk(0.0, 0.0) : cmulc(R, M);
    }
    block_sum<1>(pw, red);
    const double sig = sqrt(pw[0] / (double)(nharm - a.kc) / (double)a.nbin);
    // fused: the profile's expected noise, sqrt(sum w^2 errs_FT^2) / W
    const double err = fused ? sqrt(sh[2]) / wsum : sig * sqrt((double)a.nbin / 2.0);
    if constexpr (CZL > 0) {
        if (!(PPF_GUESS_DIAG & 1))
            cz_grid<CZL>(xm, (int)kmx[0], 1.0 / (err * err), a.Ns, -0.5, sh, z, a.czB, a.czT, a.czJ, a.czQ,
                         a.czK);
    }
    const double phase = brute_fmin(xm, (int)kmx[0], 1.0 / (err * err), a.Ns, -0.5, 0.5, sh, nullptr,
                                    nullptr, CZL > 0);
    // nu_mean of the usable channels (block reduction: 16384-channel
    // portraits made a serial loop here cost ~0.2 ms per sub-int)
    double nv[2] = {0.0, 0.0};
    {
        const double *fr = a.freqs + (int64_t)s * a.nchan;
        const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
        for (int n = tid; n < a.nchan; n += kBlock)
            if (!mask || mask[n]) { nv[0] += fr[n]; nv[1] += 1.0; }
    }
    block_sum<2>(nv, red);
    if (tid == 0) {
        double nu_mean = nv[0] / nv[1];
        double nu_fit = a.nu_fits[(int64_t)s * 3 + 0];
        if (nu_fit != nu_fit) nu_fit = nu_mean;
        double DM = a.guess_DM[s], P = a.P[s];
        double out = phase;
        if (!a.guess_ref) {     // GetTOAs: phase_transform(..., mod=True)
            out = phase + kDconst * DM * pow(P, -1.0) * (pow(nu_fit, -2.0) - pow(nu_mean, -2.0));
            if (fabs(out) >= 0.5) out = out - floor(out);   // python % 1
            if (out >= 0.5) out -= 1.0;
        }
        a.x0[(int64_t)s * 8 + 0] = out;
    }
}

// ===========================================================================
// k_rotate: out = irfft(rfft(in) * exp(2 pi i k phase_row))
// ===========================================================================
template <int KMAX, bool MX>
__global__ __launch_bounds__(kBlock) void k_rotate(RotateArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int N = a.nbin >> 1;
    const bool odd = a.nbin & 1;
    const int KH = odd ? N + 1 : N;        // harmonic slots: k < KH
    const int64_t row = blockIdx.x;
    load_row(lds, a.in, a.dtype, row, a.nbin);
    __syncthreads();
    lds_fft_n<MX>(lds, rfft_len(a.nbin), a.T, false);
    double2 Xk[KMAX], Xn[KMAX];
    const double ph = a.phases[row];
    // harmonics handled by this thread: k = tid + 256 i, k < N (pre-pass
    // pairs k, N-k); odd nbin: k <= N, no pairs
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        int k = threadIdx.x + i * kBlock;
        if (k < KH) {
            double2 X1 = cmul(rbin(lds, a.nbin, a.T2, k), cexp2pi((double)k * ph));
            double2 X2 = cmk(0.0, 0.0);
            if (!odd) X2 = cmul(rfft_bin(lds, N, a.T2, N - k), cexp2pi((double)(N - k) * ph));
            if (k == 0) { X1.y = 0.0; X2.y = 0.0; }   // DC and Nyquist: real parts only
            Xk[i] = X1;
            Xn[i] = X2;
        }
    }
    __syncthreads();
    if (odd && a.ref_len) {
        // the reference's irfft without a length: 2 N = nbin - 1 samples
        // from X_0..X_N, X_N as the Nyquist term (imaginary part dropped):
        // the even-length packed inverse with the nbin - 1 twiddles (as
        // k_gauss_port's scattered rows)
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
            const int k = threadIdx.x + i * kBlock;
            if (k < KH) lds[k] = Xk[i];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
            const int k = threadIdx.x + i * kBlock;
            if (k < N) {
                Xk[i] = lds[k];
                Xn[i] = lds[N - k];
                if (k == 0) Xn[i].y = 0.0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
            const int k = threadIdx.x + i * kBlock;
            if (k < N) lds[k] = irfft_prebin(Xk[i], Xn[i], a.T2e[k]);
        }
        __syncthreads();
        lds_fft_n<MX>(lds, N, a.Te, true);
        const double sc = 1.0 / (double)N;
        double2 *o = reinterpret_cast<double2 *>(a.out) + row * (int64_t)N;
        for (int j = threadIdx.x; j < N; j += kBlock) o[j] = cscale(lds[j], sc);
        return;
    }
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        int k = threadIdx.x + i * kBlock;
        if (k < KH) {
            if (odd) herm_put(lds, a.nbin, k, Xk[i]);
            else lds[k] = irfft_prebin(Xk[i], Xn[i], a.T2[k]);
        }
    }
    __syncthreads();
    lds_fft_n<MX>(lds, rfft_len(a.nbin), a.T, true);
    if (odd) {
        const double sc = 1.0 / (double)a.nbin;
        double *o = reinterpret_cast<double *>(a.out) + row * (int64_t)a.nbin;
        for (int j = threadIdx.x; j < a.nbin; j += kBlock) o[j] = lds[j].x * sc;
        return;
    }
    const double sc = 1.0 / (double)N;
    double2 *o = reinterpret_cast<double2 *>(a.out) + row * (int64_t)N;
    for (int j = threadIdx.x; j < N; j += kBlock) o[j] = cscale(lds[j], sc);
}

// ===========================================================================
// k_noise: get_noise_PS per row
// ===========================================================================
template <bool MX>
__global__ __launch_bounds__(kBlock) void k_noise(NoiseArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double red[kWaves * 2];
    const int N = a.nbin >> 1;
    const int64_t row = blockIdx.x;
    load_row(lds, a.in, a.dtype, row, a.nbin);
    __syncthreads();
    lds_fft_n<MX>(lds, rfft_len(a.nbin), a.T, false);
    double acc[1] = {0.0};
    for (int k = threadIdx.x + a.kc; k <= N; k += kBlock) acc[0] += cabs2(rbin(lds, a.nbin, a.T2, k));
    block_sum<1>(acc, red);
    if (threadIdx.x == 0) a.out[row] = sqrt(acc[0] / (double)a.nbin / (double)(N + 1 - a.kc));
}

// ===========================================================================
// k_phase_shift: pplib.fit_phase_shift per profile
// ===========================================================================
template <bool MX, bool GS = false>
__global__ __launch_bounds__(kBlock) void k_phase_shift(PhaseShiftArgs a) {
    // [rfft_len] fft | [N+1] xm | sh
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double red[kWaves * 4];
    const bool pre = a.Dspec != nullptr;   // (uniform) rFFTs given: long rows
    const int N = a.nbin >> 1, nharm = N + 1, NF = pre ? 0 : rfft_len(a.nbin);
    const int64_t prof = blockIdx.x;
    double *sh = GS ? a.gsh + prof * (a.Ns + 8) : reinterpret_cast<double *>(lds + NF + N + 2);
    double2 *fbuf = lds, *xm = lds + NF;
    // model spectrum first (into xm as M_k)
    const int mi = a.model_index ? a.model_index[prof] : 0;
    if (!pre) {
        load_row(fbuf, a.model, 1, mi, a.nbin);
        __syncthreads();
        lds_fft_n<MX>(fbuf, NF, a.T, false);
    }
    double pp[1] = {0.0};
    for (int k = threadIdx.x; k <= N; k += kBlock) {
        double2 M = pre ? a.Mspec[(int64_t)mi * nharm + k] : rbin(fbuf, a.nbin, a.T2, k);
        xm[k] = M;
        if (k >= 1) pp[0] += cabs2(M);
    }
    __syncthreads();
    if (!pre) {
        load_row(fbuf, a.data, a.dtype, prof, a.nbin);
        __syncthreads();
        lds_fft_n<MX>(fbuf, NF, a.T, false);
    }
    double acc[3] = {0.0, 0.0, pp[0]};
    for (int k = threadIdx.x; k <= N; k += kBlock) {
        double2 D = pre ? a.Dspec[prof * nharm + k] : rbin(fbuf, a.nbin, a.T2, k);
        double p2 = cabs2(D);
        if (k >= a.kc) acc[0] += p2;
        if (k >= 1) acc[1] += p2;
        xm[k] = (k == 0) ? cmk(0.0, 0.0) : cmulc(D, xm[k]);
    }
    block_sum<3>(acc, red);
    double err;
    if (a.noise) err = a.noise[prof] * sqrt((double)a.nbin / 2.0);
    else err = sqrt(acc[0] / (double)a.nbin / (double)(nharm - a.kc)) * sqrt((double)a.nbin / 2.0);
    const double inv_err2 = 1.0 / (err * err);
    const double d = acc[1] * inv_err2, p = acc[2] * inv_err2;
    double fval = 0.0;
    int nfev = 0;
    const double phase = brute_fmin(xm, nharm, inv_err2, a.Ns, a.lo, a.hi, sh, &fval, &nfev);
    // second derivative at phase: -Re sum (-(2 pi k)^2) xm e^{..} / err^2
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double d2 = 0.0;
    if (wave == 0) {
        double2 E = cexp2pi((double)lane * phase);
        const double2 W = cexp2pi(64.0 * phase);
        double s2 = 0.0;
        for (int k = lane; k < nharm; k += 64) {
            double2 x = xm[k];
            double re = fma(x.x, E.x, -x.y * E.y);
            s2 = fma((double)k * (double)k, re, s2);
            E = cmul(E, W);
        }
        d2 = 4.0 * kPi * kPi * wave_sum(s2) * inv_err2;
    }
    if (threadIdx.x == 0) {
        double scale = -fval / p;
        double* o = a.out + prof * 8;
        o[0] = phase;
        o[1] = pow(scale * d2, -0.5);
        o[2] = scale;
        o[3] = pow(p, -0.5);
        o[4] = pow(scale * scale * p, 0.5);
        o[5] = (d - fval * fval / p) / (double)(a.nbin - 2);
        o[6] = (double)nfev;
        o[7] = 0.0;
    }
}

// ===========================================================================
// k_synth: synthetic sub-integrations (bench / tests)
// ===========================================================================
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ double u01(uint64_t h) {   // (0, 1]
    return ((double)(h >> 11) + 1.0) * (1.0 / 9007199254740992.0);
}

template <bool MX>
__global__ __launch_bounds__(kBlock) void k_synth(SynthArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int N = a.nbin >> 1;
    const int s = blockIdx.x / a.nchan, n = blockIdx.x % a.nchan;
    const double2 *Mrow = a.Mft + (int64_t)n * (N + 1);
    // phase of this row: rotate_data(model, -phi, -DM, P, freq, nu_ref)
    const double D = kDconst * (-a.DM[s]) / a.P[s];
    const double ph = -a.phi[s] + D * (pow(a.freqs[n], -2.0) - pow(a.nu_ref, -2.0));
    const int64_t row = (int64_t)s * a.nchan + n;
    if (a.nbin & 1) {      // odd nbin: Hermitian full-length inverse, one normal deviate per bin
        for (int k = threadIdx.x; k <= N; k += kBlock) {
            double2 X = cmul(Mrow[k], cexp2pi((double)k * ph));
            if (k == 0) X.y = 0.0;
            herm_put(lds, a.nbin, k, X);
        }
        __syncthreads();
        lds_fft_n<MX>(lds, a.nbin, a.T, true);
        const double sc = 1.0 / (double)a.nbin;
        for (int j = threadIdx.x; j < a.nbin; j += kBlock) {
            const uint64_t grow = (uint64_t)(a.first + s) * (uint64_t)a.nchan + (uint64_t)n;
            uint64_t h = splitmix64(a.seed ^ splitmix64(grow * 0x100000001B3ull + (uint64_t)j));
            double u1 = u01(h), u2 = u01(splitmix64(h));
            double sn, cs;
            sincospi(2.0 * u2, &sn, &cs);
            const double z = lds[j].x * sc + a.noise * sqrt(-2.0 * log(u1)) * cs;
            if (a.dtype == 0) reinterpret_cast<float *>(a.out)[row * a.nbin + j] = (float)z;
            else reinterpret_cast<double *>(a.out)[row * a.nbin + j] = z;
        }
        return;
    }
    for (int k = threadIdx.x; k < N; k += kBlock) {
        double2 X1 = cmul(Mrow[k], cexp2pi((double)k * ph));
        double2 X2 = cmul(Mrow[N - k], cexp2pi((double)(N - k) * ph));
        if (k == 0) { X1.y = 0.0; X2.y = 0.0; }
        lds[k] = irfft_prebin(X1, X2, a.T2[k]);
    }
    __syncthreads();
    lds_fft_n<MX>(lds, a.nbin >> 1, a.T, true);
    const double sc = 1.0 / (double)N;
    for (int j = threadIdx.x; j < N; j += kBlock) {
        const uint64_t grow = (uint64_t)(a.first + s) * (uint64_t)a.nchan + (uint64_t)n;
        uint64_t h = splitmix64(a.seed ^ splitmix64(grow * 0x100000001B3ull + (uint64_t)j));
        double u1 = u01(h), u2 = u01(splitmix64(h));
        double r = sqrt(-2.0 * log(u1));
        double sn, cs;
        sincospi(2.0 * u2, &sn, &cs);
        double2 z = cscale(lds[j], sc);
        z.x += a.noise * r * cs;
        z.y += a.noise * r * sn;
        if (a.dtype == 0) reinterpret_cast<float2 *>(a.out)[row * N + j] = make_float2((float)z.x, (float)z.y);
        else reinterpret_cast<double2 *>(a.out)[row * N + j] = z;
    }
}

// ===========================================================================
// k_gauss_port: pplib.gen_gaussian_portrait (pplib.py:886-963, join_ichans
// = []), one workgroup per (portrait, channel) row.  Per component: the
// evolved loc/wid/amp (evolve_parameter pplib.py:1032-1084), the wrapped,
// truncated Gaussian of gaussian_profile (pplib.py:801-856) with its unit-peak
// factor taken at the first argmax (a block reduction), accumulated into the
// LDS row in component order as gen_gaussian_profile does (pplib.py:859-883).
// A non-zero tau then convolves the row with the one-sided exponential
// (rfft * 1/(1 + 2 pi i k tau_n) -> irfft, pplib.py:951-957, 4212-4260).
// FP contraction is off so each product/sum rounds as NumPy's does.
// ===========================================================================
__device__ __forceinline__ double gp_evolve(double f, double nu_ref, double v, double e, int code) {
#pragma clang fp contract(off)
    if (code == 0) return exp((log(f) - log(nu_ref)) * e + 1.0 * log(v));   // power_law_evolution
    return (f - nu_ref) * e + 1.0 * v;                                    // linear_evolution
}

__device__ __forceinline__ double gp_bin_center(int j, int nbin) {
#pragma clang fp contract(off)
    // np.linspace(1/(2 nbin), 1 - 1/(2 nbin), nbin) (get_bin_centers, pplib.py:694-707)
    const double lo = 1.0 / (double)(nbin * 2), hi = 1.0 - 1.0 / (double)(nbin * 2);
    if (j == nbin - 1) return hi;
    const double step = (hi - lo) / (double)(nbin - 1);
    return (double)j * step + lo;
}

// unnormalised retval of gaussian_profile at bin j (0 outside |z| < 20);
// *xw receives the wrapped bin centre
__device__ __forceinline__ double gp_raw(int j, int nbin, double mean, double sigma, double *xw) {
#pragma clang fp contract(off)
    double x = gp_bin_center(j, nbin);
    if (mean < 0.5) { if (x > mean + 0.5) x = x - 1.0; }
    else if (x < mean - 0.5) x = x + 1.0;
    *xw = x;
    const double z = (x - mean) / sigma;
    if (!(fabs(z) < 20.0)) return 0.0;
    return exp(-0.5 * (z * z)) / (sigma * 2.5066282746310002);   // sqrt(2 pi)
}


template <int KMAX, bool MX>
__global__ __launch_bounds__(kBlock) void k_gauss_port(GaussArgs a) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double red[kWaves * 2];
    double *row = reinterpret_cast<double *>(lds);
    const int nbin = a.nbin, N = nbin >> 1;
    const int p = blockIdx.x / a.nchan, n = blockIdx.x % a.nchan;
    const double *prm = a.params + (int64_t)p * a.npar;
    const double f = a.freqs[(int64_t)p * a.nchan + n], nu_ref = a.nu_ref[p];
    const double dc = prm[0];
    for (int j = threadIdx.x; j < nbin; j += kBlock) row[j] = dc;   // zeros + DC
    const double fwhm = 2.0 * sqrt(2.0 * log(2.0));
    for (int g = 0; g < a.ngauss; ++g) {
        const double *c = prm + 2 + 6 * g;
        const double L = gp_evolve(f, nu_ref, c[0], c[1], a.code[0]);
        const double W = gp_evolve(f, nu_ref, c[2], c[3], a.code[1]);
        const double A = gp_evolve(f, nu_ref, c[4], c[5], a.code[2]);
        if (!(W > 0.0)) {   // wid <= 0 (zeroout) or NaN: amp * zeros
            for (int j = threadIdx.x; j < nbin; j += kBlock) row[j] = row[j] + A * 0.0;
            continue;
        }
        const double sigma = W / fwhm;
        double mean = fmod(L, 1.0);                  // Python/NumPy L % 1.0
        if (mean != 0.0 && mean < 0.0) mean += 1.0;
        // first argmax of the unnormalised profile
        double lmax = -1.0, xw;
        int lidx = nbin;
        for (int j = threadIdx.x; j < nbin; j += kBlock) {
            const double r = gp_raw(j, nbin, mean, sigma, &xw);
            if (r > lmax) { lmax = r; lidx = j; }
        }
        double v[1] = {lmax};
        block_max<1>(v, red);
        const double gmax = v[0];
        double vi[1] = {lmax == gmax ? -(double)lidx : -(double)nbin};
        block_max<1>(vi, red);
        const int imax = (int)(-vi[0]);
        double fact = 1.0;                            // all-zero profile: returned as is
        if (gmax != 0.0) {
            double xi;
            (void)gp_raw(imax, nbin, mean, sigma, &xi);
            const double zz = (xi - L) / sigma;
            fact = exp(-0.5 * (zz * zz)) / gmax;
        }
        for (int j = threadIdx.x; j < nbin; j += kBlock) {
            const double r = gp_raw(j, nbin, mean, sigma, &xw);
            row[j] = row[j] + A * (fact * r);
        }
    }
    const double tau = prm[1];
    if (a.taus_out) {
        // long rows: tau_n for the convolution on the long transforms
        if (threadIdx.x == 0)
            a.taus_out[blockIdx.x] = tau != 0.0 ? tau / (double)nbin * pow(f / nu_ref, a.scat_index[p]) : 0.0;
    } else if (tau != 0.0) {
        // taus = (tau / nbin) * (freqs / nu_ref)**alpha; B_k = 1 / (1 + 2 pi i k tau_n)
        const double tn = tau / (double)nbin * pow(f / nu_ref, a.scat_index[p]);
        const bool odd = nbin & 1;
        const int KH = odd ? N + 1 : N;
        __syncthreads();
        if (odd) {
            // the real row (doubles) -> complex points in place: all reads first
            double v[2 * KMAX];
#pragma unroll
            for (int i = 0; i < 2 * KMAX; ++i) {
                const int j = threadIdx.x + i * kBlock;
                if (j < nbin) v[i] = row[j];
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 2 * KMAX; ++i) {
                const int j = threadIdx.x + i * kBlock;
                if (j < nbin) lds[j] = cmk(v[i], 0.0);
            }
            __syncthreads();
        }
        lds_fft_n<MX>(lds, rfft_len(nbin), a.T, false);
        double2 Xk[KMAX], Xn[KMAX];
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
            const int k = threadIdx.x + i * kBlock;
            if (k < KH) {
                double2 X1 = rbin(lds, nbin, a.T2, k);
                double2 X2 = odd ? cmk(0.0, 0.0) : rfft_bin(lds, N, a.T2, N - k);
                if (tn != 0.0) {
                    X1 = cmul(X1, scat_recip((2.0 * kPi * (double)k) * tn));
                    if (!odd) X2 = cmul(X2, scat_recip((2.0 * kPi * (double)(N - k)) * tn));
                }
                if (k == 0) { X1.y = 0.0; X2.y = 0.0; }   // irfft keeps DC, Nyquist real parts
                Xk[i] = X1;
                Xn[i] = X2;
            }
        }
        __syncthreads();
        if (odd) {
            // the reference's irfft takes no length (pplib.py:957): 2 N =
            // nbin - 1 bins from X_0..X_N, X_N as the Nyquist term (its
            // imaginary part dropped); the even-length packed inverse with
            // the nbin - 1 twiddles, the row's last column zero
#pragma unroll
            for (int i = 0; i < KMAX; ++i) {
                const int k = threadIdx.x + i * kBlock;
                if (k < KH) lds[k] = Xk[i];
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < KMAX; ++i) {
                const int k = threadIdx.x + i * kBlock;
                if (k < N) {
                    Xk[i] = lds[k];
                    Xn[i] = lds[N - k];
                    if (k == 0) Xn[i].y = 0.0;
                }
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < KMAX; ++i) {
                const int k = threadIdx.x + i * kBlock;
                if (k < N) lds[k] = irfft_prebin(Xk[i], Xn[i], a.T2e[k]);
            }
            __syncthreads();
            lds_fft_n<MX>(lds, N, a.Te, true);
            const double sc = 1.0 / (double)N;
            double *o = a.out + (int64_t)blockIdx.x * nbin;
            for (int j = threadIdx.x; j < N; j += kBlock) {
                const double2 z = cscale(lds[j], sc);
                o[2 * j] = z.x;
                o[2 * j + 1] = z.y;
            }
            if (threadIdx.x == 0) o[nbin - 1] = 0.0;
            return;
        }
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
            const int k = threadIdx.x + i * kBlock;
            if (k < KH) lds[k] = irfft_prebin(Xk[i], Xn[i], a.T2[k]);
        }
        __syncthreads();
        lds_fft_n<MX>(lds, rfft_len(nbin), a.T, true);
        const double sc = 1.0 / (double)N;
        double2 *o = reinterpret_cast<double2 *>(a.out) + (int64_t)blockIdx.x * N;
        for (int j = threadIdx.x; j < N; j += kBlock) o[j] = cscale(lds[j], sc);
        return;
    }
    __syncthreads();
    if (nbin & 1) {
        double *o = a.out + (int64_t)blockIdx.x * nbin;
        for (int j = threadIdx.x; j < nbin; j += kBlock) o[j] = row[j];
        return;
    }
    double2 *o = reinterpret_cast<double2 *>(a.out) + (int64_t)blockIdx.x * N;
    for (int j = threadIdx.x; j < N; j += kBlock) o[j] = lds[j];
}

// ===========================================================================
// host-side launchers
// ===========================================================================
// per-thread harmonic slots of the block kernels' KMAX instantiations (1, 2,
// 4, 8, 16): the smallest that holds ceil(N / kBlock)
static inline int kmax_pow2(int N) {
    int q = (N + kBlock - 1) / kBlock, k = 1;
    while (k < q) k <<= 1;
    return k;
}
static inline int log2i(int n) {
    int l = 0;
    while ((1 << l) < n) ++l;
    return l;
}

// launch KER<A, MX> with MX = mx (the mixed-radix FFT compiled in only when
// nbin / 2 is not a power of two; lds_fft_n)
#define MXL(mx, KER, A, ...)                                          \
    do {                                                              \
        if (mx) hipLaunchKernelGGL((KER<A, true>), __VA_ARGS__);      \
        else hipLaunchKernelGGL((KER<A, false>), __VA_ARGS__);        \
    } while (0)

hipError_t launch_twiddles(int N, double2 *T, double2 *T2, hipStream_t st) {
    hipLaunchKernelGGL(k_twiddles, dim3((N + 255) / 256), dim3(256), 0, st, N, T, T2);
    return hipGetLastError();
}
hipError_t launch_rfft_rows(const RfftArgs &a, int64_t nrows, hipStream_t st) {
    size_t lds = (size_t)rfft_len(a.nbin) * sizeof(double2);
    if (is_pow2(rfft_len(a.nbin))) hipLaunchKernelGGL(k_rfft_rows<false>, dim3((unsigned)nrows), dim3(kBlock), lds, st, a);
    else hipLaunchKernelGGL(k_rfft_rows<true>, dim3((unsigned)nrows), dim3(kBlock), lds, st, a);
    return hipGetLastError();
}
template <int L2>
static void launch_xspec_t(const XspecArgs &a, hipStream_t st) {
    constexpr int N = 1 << L2;
    size_t lds = (size_t)N * sizeof(double2) * (N <= 1024 ? 3 : 1);
    dim3 g((unsigned)((int64_t)a.nsub * a.nblk)), b(kBlock);
    if (a.dtype == 0) hipLaunchKernelGGL((k_xspec<L2, 0>), g, b, lds, st, a);
    else hipLaunchKernelGGL((k_xspec<L2, 1>), g, b, lds, st, a);
}

hipError_t launch_xspec(const XspecArgs &a, hipStream_t st) {
    switch (a.log2N) {
        case 4: launch_xspec_t<4>(a, st); break;
        case 5: launch_xspec_t<5>(a, st); break;
        case 6: launch_xspec_t<6>(a, st); break;
        case 7: launch_xspec_t<7>(a, st); break;
        case 8: launch_xspec_t<8>(a, st); break;
        case 9: launch_xspec_t<9>(a, st); break;
        case 10: launch_xspec_t<10>(a, st); break;
        case 11: launch_xspec_t<11>(a, st); break;
        case 12: launch_xspec_t<12>(a, st); break;
        case 0: {      // nbin / 2 not a power of two
#ifndef PPF_XSPEC_WM
#define PPF_XSPEC_WM 1
#endif
            // wave per row (k_xspec_wm) up to N = 1024; the block kernel above
            if (PPF_XSPEC_WM && xspec_wm_supported(a.nbin) && a.cb <= 64) return launch_xspec_wm(a, st);
            dim3 g((unsigned)((int64_t)a.nsub * a.nblk)), b(kBlock);
            const size_t lds = (size_t)rfft_len(a.nbin) * sizeof(double2);
            if (a.dtype == 0) hipLaunchKernelGGL((k_xspec_any<0>), g, b, lds, st, a);
            else hipLaunchKernelGGL((k_xspec_any<1>), g, b, lds, st, a);
            break;
        }
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
bool dsum_wave_supported(int nbin) { return nbin >= 256 && nbin <= 2048 && is_pow2(nbin); }
// k_dsum_wn for the other nbin <= 2048 (0: the block kernel k_dsum)
#ifndef PPF_DSUM_WN
#define PPF_DSUM_WN 1
#endif

template <int DT, int L2>
static void launch_dsum_w(const DsumArgs &a, hipStream_t st) {
    constexpr int NB = 1 << L2;
    const size_t row = (size_t)kWaves * NB * (DT == 0 ? 4 : 8);
    const size_t lds = row > (size_t)NB * 8 ? row : (size_t)NB * 8;
    hipLaunchKernelGGL((k_dsum_w<DT, L2>), dim3((unsigned)((int64_t)a.nsub * a.nblkd)), dim3(kBlock),
                       lds, st, a);
}

#ifndef PPF_NUREF
#define PPF_NUREF 1
#endif
hipError_t launch_dsum(const DsumArgs &a_in, hipStream_t st) {
    DsumArgs a = a_in;
    // many channels: nu_ref once per sub-int (the wave-per-row kernels read it)
    if (PPF_NUREF && a.nuref && a.nchan >= 2048 && a.nbin <= 2048 &&
        (dsum_wave_supported(a.nbin) || PPF_DSUM_WN)) {
        hipLaunchKernelGGL(k_nu_ref, dim3((unsigned)a.nsub), dim3(64), 0, st, a);
    } else {
        a.nuref = nullptr;
    }
    if (dsum_wave_supported(a.nbin)) {
        switch (__builtin_ctz((unsigned)a.nbin) * 2 + a.dtype) {
            case 16: launch_dsum_w<0, 8>(a, st); break;
            case 17: launch_dsum_w<1, 8>(a, st); break;
            case 18: launch_dsum_w<0, 9>(a, st); break;
            case 19: launch_dsum_w<1, 9>(a, st); break;
            case 20: launch_dsum_w<0, 10>(a, st); break;
            case 21: launch_dsum_w<1, 10>(a, st); break;
            case 22: launch_dsum_w<0, 11>(a, st); break;
            case 23: launch_dsum_w<1, 11>(a, st); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    dim3 g((unsigned)((int64_t)a.nsub * a.nblkd)), b(kBlock);
    if (PPF_DSUM_WN && a.nbin <= 2048 && a.cbd <= 128) {
        // wave-per-row pass at any nbin (k_dsum_wn), NBMAX 1024 or 2048
        const int nbm = a.nbin <= 1024 ? 1024 : 2048;
        const size_t row = (size_t)kWaves * nbm * (a.dtype == 0 ? 4 : 8);
        const size_t lds = row > (size_t)nbm * 8 ? row : (size_t)nbm * 8;
        if (nbm == 1024) {
            if (a.dtype == 0) hipLaunchKernelGGL((k_dsum_wn<0, 1024>), g, b, lds, st, a);
            else hipLaunchKernelGGL((k_dsum_wn<1, 1024>), g, b, lds, st, a);
        } else {
            if (a.dtype == 0) hipLaunchKernelGGL((k_dsum_wn<0, 2048>), g, b, lds, st, a);
            else hipLaunchKernelGGL((k_dsum_wn<1, 2048>), g, b, lds, st, a);
        }
        return hipGetLastError();
    }
    const int jb = a.nbin >= 2048 ? 8 : (a.nbin + kBlock - 1) / kBlock;
    if (a.dtype == 0) {
        if (jb >= 8) hipLaunchKernelGGL((k_dsum<0, 8>), g, b, 0, st, a);
        else if (jb >= 4) hipLaunchKernelGGL((k_dsum<0, 4>), g, b, 0, st, a);
        else if (jb >= 2) hipLaunchKernelGGL((k_dsum<0, 2>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_dsum<0, 1>), g, b, 0, st, a);
    } else {
        if (jb >= 8) hipLaunchKernelGGL((k_dsum<1, 8>), g, b, 0, st, a);
        else if (jb >= 4) hipLaunchKernelGGL((k_dsum<1, 4>), g, b, 0, st, a);
        else if (jb >= 2) hipLaunchKernelGGL((k_dsum<1, 2>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_dsum<1, 1>), g, b, 0, st, a);
    }
    return hipGetLastError();
}

// ppalign's rotation phases and weights (ppf_align_phases, ppalign.py:
// 222-247): a thread per (sub-int, channel)
__global__ __launch_bounds__(kBlock) void k_align_phases(int nsub, int nchan, const double *results,
                                                         const double *freqs, const double *P,
                                                         const uint8_t *mask, const double *scales,
                                                         const double *errs, double *phases, double *weights) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= (int64_t)nsub * nchan) return;
    const int64_t s = i / nchan;
    const double *r = results + s * (int64_t)(sizeof(ppf_result) / sizeof(double));
    const double phi = r[offsetof(ppf_result, params) / sizeof(double)];
    const double DM = r[offsetof(ppf_result, params) / sizeof(double) + 1];
    const double nu_ref = r[offsetof(ppf_result, nu_out) / sizeof(double)];
    const bool ok = !mask || mask[i];
    phases[i] = ok ? phi + kDconst * DM / P[s] * (pow(freqs[i], -2.0) - pow(nu_ref, -2.0)) : 0.0;
    weights[i] = ok ? scales[i] / (errs[i] * errs[i]) : 0.0;
}

hipError_t launch_align_phases(int nsub, int nchan, const double *results, const double *freqs, const double *P,
                               const uint8_t *mask, const double *scales, const double *errs, double *phases,
                               double *weights, hipStream_t st) {
    const int64_t n = (int64_t)nsub * nchan;
    hipLaunchKernelGGL(k_align_phases, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, nsub,
                       nchan, results, freqs, P, mask, scales, errs, phases, weights);
    return hipGetLastError();
}

hipError_t launch_guess(const GuessArgs &a, hipStream_t st) {
    const int zs = a.gspec ? 0 : ((a.czB && a.czP > rfft_len(a.nbin)) ? a.czP : rfft_len(a.nbin));
    size_t lds = (size_t)(zs + a.nbin / 2 + 2) * sizeof(double2) +
                 (a.gsh ? 0 : (size_t)(a.Ns + 8) * sizeof(double));
    const dim3 g((unsigned)a.nsub), b(kBlock);
    if (a.gsh) {
        // the brute grid in global memory (long rows: gspec given, no
        // transform runs in the kernel)
        if (a.gspec || is_pow2(rfft_len(a.nbin))) hipLaunchKernelGGL((k_guess<false, 0, true>), g, b, lds, st, a);
        else hipLaunchKernelGGL((k_guess<true, 0, true>), g, b, lds, st, a);
    } else if (a.czB && is_pow2(rfft_len(a.nbin))) {
        switch (a.czP) {
            case 512: hipLaunchKernelGGL((k_guess<false, 9>), g, b, lds, st, a); break;
            case 1024: hipLaunchKernelGGL((k_guess<false, 10>), g, b, lds, st, a); break;
            case 2048: hipLaunchKernelGGL((k_guess<false, 11>), g, b, lds, st, a); break;
            default: return hipErrorInvalidValue;
        }
    } else if (is_pow2(rfft_len(a.nbin))) {
        hipLaunchKernelGGL((k_guess<false, 0>), g, b, lds, st, a);
    } else {
        hipLaunchKernelGGL((k_guess<true, 0>), g, b, lds, st, a);
    }
    return hipGetLastError();
}
hipError_t launch_gauss_port(const GaussArgs &a, hipStream_t st) {
    size_t lds = (size_t)rfft_len(a.nbin) * sizeof(double2);
    dim3 g((unsigned)((int64_t)a.nport * a.nchan)), b(kBlock);
    if (!fft_len_supported(rfft_len(a.nbin))) {
        // long rows, unscattered models (checked by the caller): the row in
        // LDS only; the smallest instantiation (its transform never runs)
        hipLaunchKernelGGL((k_gauss_port<1, false>), g, b, (size_t)a.nbin * sizeof(double), st, a);
        return hipGetLastError();
    }
    const bool mx = !is_pow2(rfft_len(a.nbin));
    switch (kmax_pow2(a.nbin / 2 + (a.nbin & 1))) {
        case 1: MXL(mx, k_gauss_port, 1, g, b, lds, st, a); break;
        case 2: MXL(mx, k_gauss_port, 2, g, b, lds, st, a); break;
        case 4: MXL(mx, k_gauss_port, 4, g, b, lds, st, a); break;
        case 8: MXL(mx, k_gauss_port, 8, g, b, lds, st, a); break;
        case 16: MXL(mx, k_gauss_port, 16, g, b, lds, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_rotate(const RotateArgs &a, int64_t nrows, hipStream_t st) {
    size_t lds = (size_t)rfft_len(a.nbin) * sizeof(double2);
    dim3 g((unsigned)nrows), b(kBlock);
    const bool mx = !is_pow2(rfft_len(a.nbin));
    switch (kmax_pow2(a.nbin / 2 + (a.nbin & 1))) {
        case 1: MXL(mx, k_rotate, 1, g, b, lds, st, a); break;
        case 2: MXL(mx, k_rotate, 2, g, b, lds, st, a); break;
        case 4: MXL(mx, k_rotate, 4, g, b, lds, st, a); break;
        case 8: MXL(mx, k_rotate, 8, g, b, lds, st, a); break;
        case 16: MXL(mx, k_rotate, 16, g, b, lds, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
// ===========================================================================
// ppalign accumulation.  k_align_part: workgroup = (channel n, group g of
// sub-ints); for each of its sub-ints in order, rfft of the row, times
// w exp(2 pi i k phase), summed in registers (the rotate-then-sum of the
// reference is linear, so the sum is taken before the single inverse FFT).
// k_align_fin: per channel, the group partials in group order, DC and
// Nyquist imaginary parts dropped (as numpy irfft does), irfft, added to out.
// ===========================================================================
int align_groups(int nsub, int nchan) {
    int g = (2048 + nchan - 1) / nchan;       // >= 2048 workgroups in flight
    if (g > nsub) g = nsub;
    return g < 1 ? 1 : g;
}

template <int KMAX, bool MX>
__global__ __launch_bounds__(kBlock) void k_align_part(AlignArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int N = a.nbin >> 1;
    const bool odd = a.nbin & 1;
    const int KH = odd ? N + 1 : N;
    const int n = blockIdx.x % a.nchan, g = blockIdx.x / a.nchan;
    const int per = (a.nsub + a.ngroup - 1) / a.ngroup;
    const int s0 = g * per, s1 = min(a.nsub, s0 + per);
    double2 Ak[KMAX], An[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) Ak[i] = An[i] = cmk(0.0, 0.0);
    double wtot = 0.0;
    for (int s = s0; s < s1; ++s) {
        const int64_t row = (int64_t)s * a.nchan + n;
        const double w = a.weights[row];
        if (w == 0.0) continue;                     // uniform per workgroup
        const double ph = a.phases[row];
        wtot += w;
        load_row(lds, a.in, a.dtype, row, a.nbin);
        __syncthreads();
        lds_fft_n<MX>(lds, rfft_len(a.nbin), a.T, false);
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
            const int k = threadIdx.x + i * kBlock;
            if (k < KH) {
                const double2 X1 = cmul(rbin(lds, a.nbin, a.T2, k), cexp2pi((double)k * ph));
                Ak[i] = cadd(Ak[i], cscale(X1, w));
                if (!odd) {
                    const double2 X2 =
                        cmul(rfft_bin(lds, N, a.T2, N - k), cexp2pi((double)(N - k) * ph));
                    An[i] = cadd(An[i], cscale(X2, w));
                }
            }
        }
        __syncthreads();
    }
    double2 *P = a.part + ((int64_t)g * a.nchan + n) * (N + 1);
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        const int k = threadIdx.x + i * kBlock;
        if (k < KH) {
            P[k] = Ak[i];
            if (odd) continue;
            if (k == 0) P[N] = An[i];               // (k, N - k) = (0, N)
            else P[N - k] = An[i];
        }
    }
    if (threadIdx.x == 0) a.wpart[(int64_t)g * a.nchan + n] = wtot;
}

template <int KMAX, bool MX>
__global__ __launch_bounds__(kBlock) void k_align_fin(AlignArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int N = a.nbin >> 1, n = blockIdx.x;
    const bool odd = a.nbin & 1;
    const int KH = odd ? N + 1 : N;
    double2 Xk[KMAX], Xn[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        const int k = threadIdx.x + i * kBlock;
        if (k < KH) {
            double2 s1 = cmk(0.0, 0.0), s2 = s1;
            for (int g = 0; g < a.ngroup; ++g) {
                const double2 *P = a.part + ((int64_t)g * a.nchan + n) * (N + 1);
                s1 = cadd(s1, P[k]);
                if (!odd) s2 = cadd(s2, P[N - k]);
            }
            if (k == 0) { s1.y = 0.0; s2.y = 0.0; }  // DC and Nyquist: real parts only
            Xk[i] = s1;
            Xn[i] = s2;
        }
    }
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        const int k = threadIdx.x + i * kBlock;
        if (k < KH) {
            if (odd) herm_put(lds, a.nbin, k, Xk[i]);
            else lds[k] = irfft_prebin(Xk[i], Xn[i], a.T2[k]);
        }
    }
    __syncthreads();
    lds_fft_n<MX>(lds, rfft_len(a.nbin), a.T, true);
    if (odd) {
        const double sc = 1.0 / (double)a.nbin;
        double *o = a.out + (int64_t)n * a.nbin;
        for (int j = threadIdx.x; j < a.nbin; j += kBlock) o[j] += lds[j].x * sc;
    } else {
        const double sc = 1.0 / (double)N;
        double2 *o = reinterpret_cast<double2 *>(a.out) + (int64_t)n * N;
        for (int j = threadIdx.x; j < N; j += kBlock) o[j] = cadd(o[j], cscale(lds[j], sc));
    }
    if (threadIdx.x == 0) {
        double w = 0.0;
        for (int g = 0; g < a.ngroup; ++g) w += a.wpart[(int64_t)g * a.nchan + n];
        a.wsum[n] += w;
    }
}

hipError_t launch_align(const AlignArgs &a, hipStream_t st) {
    const size_t lds = (size_t)rfft_len(a.nbin) * sizeof(double2);
    dim3 gp((unsigned)((int64_t)a.ngroup * a.nchan)), gf((unsigned)a.nchan), b(kBlock);
    // wave-per-row partials where the register FFT covers nbin; the
    // block-FFT k_align_part otherwise
    const bool wave = align_wave_supported(a.log2N);
    if (wave) {
        hipError_t e = launch_align_part_w(a, st);
        if (e != hipSuccess) return e;
    }
    const bool mx = !is_pow2(rfft_len(a.nbin));
    switch (kmax_pow2(a.nbin / 2 + (a.nbin & 1))) {
        case 1: if (!wave) MXL(mx, k_align_part, 1, gp, b, lds, st, a);
                MXL(mx, k_align_fin, 1, gf, b, lds, st, a); break;
        case 2: if (!wave) MXL(mx, k_align_part, 2, gp, b, lds, st, a);
                MXL(mx, k_align_fin, 2, gf, b, lds, st, a); break;
        case 4: if (!wave) MXL(mx, k_align_part, 4, gp, b, lds, st, a);
                MXL(mx, k_align_fin, 4, gf, b, lds, st, a); break;
        case 8: if (!wave) MXL(mx, k_align_part, 8, gp, b, lds, st, a);
                MXL(mx, k_align_fin, 8, gf, b, lds, st, a); break;
        case 16: if (!wave) MXL(mx, k_align_part, 16, gp, b, lds, st, a);
                 MXL(mx, k_align_fin, 16, gf, b, lds, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ===========================================================================
// k_resid_chi2: get_red_chi2(rotate_portrait_full(x)[n], scale_n model_n,
// err_n, dof) per row (pplib.py:754-779): rotation as k_rotate (rfft,
// phasor, irfft dropping the DC / Nyquist imaginary parts), then the
// residual sum of squares over the bins with a fixed-order block reduction.
// ===========================================================================
template <int KMAX, bool MX>
__global__ __launch_bounds__(kBlock) void k_resid_chi2(ResidArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double red[kWaves * 4];
    const int N = a.nbin >> 1;
    const bool odd = a.nbin & 1;
    const int KH = odd ? N + 1 : N;
    const int64_t row = blockIdx.x;
    load_row(lds, a.in, a.dtype, row, a.nbin);
    __syncthreads();
    lds_fft_n<MX>(lds, rfft_len(a.nbin), a.T, false);
    double2 Xk[KMAX], Xn[KMAX];
    const double ph = a.phases[row];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        int k = threadIdx.x + i * kBlock;
        if (k < KH) {
            double2 X1 = cmul(rbin(lds, a.nbin, a.T2, k), cexp2pi((double)k * ph));
            double2 X2 = cmk(0.0, 0.0);
            if (!odd) X2 = cmul(rfft_bin(lds, N, a.T2, N - k), cexp2pi((double)(N - k) * ph));
            if (k == 0) { X1.y = 0.0; X2.y = 0.0; }
            Xk[i] = X1;
            Xn[i] = X2;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        int k = threadIdx.x + i * kBlock;
        if (k < KH) {
            if (odd) herm_put(lds, a.nbin, k, Xk[i]);
            else lds[k] = irfft_prebin(Xk[i], Xn[i], a.T2[k]);
        }
    }
    __syncthreads();
    lds_fft_n<MX>(lds, rfft_len(a.nbin), a.T, true);
    const double sc = 1.0 / (double)N, s = a.scales[row];
    const double *m = a.model + (int64_t)a.model_row[row] * a.nbin;
    double acc[1] = {0.0};
    for (int j = threadIdx.x; odd && j < a.nbin; j += kBlock) {
        const double r0 = lds[j].x * (1.0 / (double)a.nbin) - s * m[j];
        acc[0] = fma(r0, r0, acc[0]);
    }
    for (int j = threadIdx.x; !odd && j < N; j += kBlock) {
        const double2 x = cscale(lds[j], sc);
        const double r0 = x.x - s * m[2 * j], r1 = x.y - s * m[2 * j + 1];
        acc[0] = fma(r0, r0, fma(r1, r1, acc[0]));
    }
    block_sum<1>(acc, red);
    if (threadIdx.x == 0) {
        const double e = a.errs[row];
        a.out[row] = acc[0] / (e * e) / a.dof;
    }
}

hipError_t launch_resid_chi2(const ResidArgs &a, int64_t nrows, hipStream_t st) {
    size_t lds = (size_t)rfft_len(a.nbin) * sizeof(double2);
    dim3 g((unsigned)nrows), b(kBlock);
    const bool mx = !is_pow2(rfft_len(a.nbin));
    switch (kmax_pow2(a.nbin / 2 + (a.nbin & 1))) {
        case 1: MXL(mx, k_resid_chi2, 1, g, b, lds, st, a); break;
        case 2: MXL(mx, k_resid_chi2, 2, g, b, lds, st, a); break;
        case 4: MXL(mx, k_resid_chi2, 4, g, b, lds, st, a); break;
        case 8: MXL(mx, k_resid_chi2, 8, g, b, lds, st, a); break;
        case 16: MXL(mx, k_resid_chi2, 16, g, b, lds, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_noise(const NoiseArgs &a, int64_t nrows, hipStream_t st) {
    size_t lds = (size_t)rfft_len(a.nbin) * sizeof(double2);
    if (is_pow2(rfft_len(a.nbin))) hipLaunchKernelGGL(k_noise<false>, dim3((unsigned)nrows), dim3(kBlock), lds, st, a);
    else hipLaunchKernelGGL(k_noise<true>, dim3((unsigned)nrows), dim3(kBlock), lds, st, a);
    return hipGetLastError();
}
hipError_t launch_phase_shift(const PhaseShiftArgs &a, int nprof, hipStream_t st) {
    size_t lds = (size_t)((a.Dspec ? 0 : rfft_len(a.nbin)) + a.nbin / 2 + 2) * sizeof(double2) +
                 (a.gsh ? 0 : (size_t)(a.Ns + 8) * sizeof(double));
    if (a.gsh) {   // the brute grid in global memory
        if (a.Dspec || is_pow2(rfft_len(a.nbin)))
            hipLaunchKernelGGL((k_phase_shift<false, true>), dim3((unsigned)nprof), dim3(kBlock), lds, st, a);
        else hipLaunchKernelGGL((k_phase_shift<true, true>), dim3((unsigned)nprof), dim3(kBlock), lds, st, a);
    } else if (is_pow2(rfft_len(a.nbin))) hipLaunchKernelGGL(k_phase_shift<false>, dim3((unsigned)nprof), dim3(kBlock), lds, st, a);
    else hipLaunchKernelGGL(k_phase_shift<true>, dim3((unsigned)nprof), dim3(kBlock), lds, st, a);
    return hipGetLastError();
}
hipError_t launch_synth(const SynthArgs &a, hipStream_t st) {
    size_t lds = (size_t)rfft_len(a.nbin) * sizeof(double2);
    if (is_pow2(rfft_len(a.nbin))) hipLaunchKernelGGL(k_synth<false>, dim3((unsigned)(a.nsub * a.nchan)), dim3(kBlock), lds, st, a);
    else hipLaunchKernelGGL(k_synth<true>, dim3((unsigned)(a.nsub * a.nchan)), dim3(kBlock), lds, st, a);
    return hipGetLastError();
}


// ===========================================================================
// k_spline_port: pplib.gen_spline_portrait (pplib.py:966-990) per row
// (portrait p, channel n).  Thread 0 evaluates the B-spline curve at
// x = freqs[p][n] exactly as FITPACK's splev (ext = 0: the end intervals
// extrapolate) with fpbspl's Cox-de Boor recursion; every thread then forms
// port[j] = mean_prof[j] + sum_c proj[c] eigvec[j][c] (np.dot(proj,
// eigvec.T) + mean_prof).  With nbin != nbin_model the row is resampled as
// scipy.signal.resample(port, nbin) (rfft; keep min(num, Nx)//2 + 1
// harmonics, the old Nyquist halved when upsampling / doubled when
// downsampling; irfft; x num/Nx) and then rotated by rotate_portrait(port,
// 0.5 (1/nbin - 1/nbin_model)): both are folded into one spectrum
// (the resampled spectrum with the DC and Nyquist imaginary parts dropped,
// as the irfft -> rfft round trip does, times the phasor), one irfft.
// ===========================================================================
template <bool MX>
__global__ __launch_bounds__(kBlock) void k_spline_port(SplineArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double proj[kSplineMaxComp];
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;                   // p * nchan + n
    const int N0 = a.nbin_model >> 1, N1 = a.nbin >> 1;
    if (tid == 0) {
        const double x = a.freqs[row];
        const int k = a.degree, n = a.nknots;
        const double *t = a.knots;
        // knot interval t[l] <= x < t[l+1], l in [k, n - k - 2] (0-based)
        int l = k;
        while (l < n - k - 2 && x >= t[l + 1]) ++l;
        double h[kSplineMaxDeg + 2], hh[kSplineMaxDeg + 2];
        h[0] = 1.0;
        for (int j = 1; j <= k; ++j) {
            for (int i = 0; i < j; ++i) hh[i] = h[i];
            h[0] = 0.0;
            for (int i = 1; i <= j; ++i) {
                const int li = l + i, lj = li - j;
                if (t[li] != t[lj]) {
                    const double f = hh[i - 1] / (t[li] - t[lj]);
                    h[i - 1] += f * (t[li] - x);
                    h[i] = f * (x - t[lj]);
                } else {
                    h[i] = 0.0;
                }
            }
        }
        for (int c = 0; c < a.ncomp; ++c) {
            const double *cc = a.coefs + (int64_t)c * n;
            double sp = 0.0;
            for (int j = 0; j <= k; ++j) sp += cc[l - k + j] * h[j];
            proj[c] = sp;
        }
    }
    __syncthreads();
    auto value = [&](int j) {
        double v = 0.0;
        const double *e = a.eigvec + (int64_t)j * a.ncomp;
        for (int c = 0; c < a.ncomp; ++c) v = fma(proj[c], e[c], v);
        return v + a.mean_prof[j];
    };
    double *o = a.out + row * (int64_t)a.nbin;
    if (a.nbin == a.nbin_model) {
        for (int j = tid; j < a.nbin; j += kBlock) o[j] = value(j);
        return;
    }
    // resample + rotate
    const int NM = N0 > N1 ? N0 : N1;
    double2 *buf = lds;                    // complex FFT buffer (max N0, N1)
    double2 *spec = lds + NM;              // output spectrum Y_k, k <= N1
    for (int j = tid; j < N0; j += kBlock) buf[j] = cmk(value(2 * j), value(2 * j + 1));
    __syncthreads();
    lds_fft_n<MX>(buf, a.nbin_model >> 1, a.T0, false);
    const int num = a.nbin, Nx = a.nbin_model;
    const int Nm = num < Nx ? num : Nx, nyq = Nm / 2 + 1;
    const double scale = (double)num / (double)Nx;
    const double shift = 0.5 * (1.0 / (double)num - 1.0 / (double)Nx);
    for (int k = tid; k <= N1; k += kBlock) {
        double2 Y = cmk(0.0, 0.0);
        if (k < nyq) {
            Y = rfft_bin(buf, N0, a.T20, k);
            if (k == Nm / 2) Y = cscale(Y, num < Nx ? 2.0 : 0.5);   // Nm even (powers of 2)
        }
        Y = cscale(Y, scale);
        if (k == 0 || k == N1) Y.y = 0.0;          // irfft -> rfft round trip
        spec[k] = cmul(Y, cexp2pi((double)k * shift));
    }
    __syncthreads();
    for (int k = tid; k < N1; k += kBlock) {
        double2 Xk = spec[k], Xn = spec[N1 - k];
        if (k == 0) { Xk.y = 0.0; Xn.y = 0.0; }    // irfft: DC and Nyquist real parts
        buf[k] = irfft_prebin(Xk, Xn, a.T21[k]);
    }
    __syncthreads();
    lds_fft_n<MX>(buf, a.nbin >> 1, a.T1, true);
    const double sc = 1.0 / (double)N1;
    double2 *o2 = reinterpret_cast<double2 *>(o);
    for (int j = tid; j < N1; j += kBlock) o2[j] = cscale(buf[j], sc);
}

hipError_t launch_spline_port(const SplineArgs &a, hipStream_t st) {
    const int N0 = a.nbin_model >> 1, N1 = a.nbin >> 1;
    const int NM = N0 > N1 ? N0 : N1;
    const size_t lds = a.nbin == a.nbin_model ? 16 : (size_t)(NM + N1 + 1) * sizeof(double2);
    if (is_pow2(N0) && is_pow2(N1))
        hipLaunchKernelGGL(k_spline_port<false>, dim3((unsigned)((int64_t)a.nport * a.nchan)), dim3(kBlock),
                           lds, st, a);
    else
        hipLaunchKernelGGL(k_spline_port<true>, dim3((unsigned)((int64_t)a.nport * a.nchan)), dim3(kBlock),
                           lds, st, a);
    return hipGetLastError();
}

// ===========================================================================
// k_scales: pptoaslib.get_scales_full (pptoaslib.py:953-971) -- a_n = C_n/S_n
// at given parameters from given spectra, one wave per (sub-int, channel):
//   phi_n = phase_shifts(phi, DM, GM, nu_n, nu_DM, nu_GM, P)  (pptoaslib.py:195-228)
//   tau_n = tau (nu_n / nu_tau)^alpha                         (pplib.py:4212-4216)
//   B_k = 1 / (1 + 2 pi i k tau_n), 1 where tau_n == 0        (pplib.py:4219-4260)
//   S_n = sum_k |B_k|^2 |M_k|^2 / e_n^2                        (Sbp, pptoaslib.py:421-428)
//   C_n = Re sum_k D_k conj(M_k) conj(B_k) e^{2 pi i k phi_n} / e_n^2  (Cdbp, 458-469)
// The phasor is taken with exact argument reduction (cexp2pi); the lanes'
// partial sums are reduced in fixed order.
// ===========================================================================
__global__ __launch_bounds__(kBlock) void k_scales(ScalesArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (row >= (int64_t)a.nsub * a.nchan) return;
    const int s = (int)(row / a.nchan), n = (int)(row % a.nchan);
    const double *pr = a.params + (int64_t)s * 5;
    const double P = a.P[s], nu = a.freqs[row];
    const double nuDM = a.nus[s * 3 + 0], nuGM = a.nus[s * 3 + 1], nutau = a.nus[s * 3 + 2];
    const double phi_n = pr[0] + kDconst * pr[1] * (pow(nu, -2.0) - pow(nuDM, -2.0)) / P +
                         kDconst * kDconst * pr[2] * (pow(nu, -4.0) - pow(nuGM, -4.0)) / P;
    const double tau = a.log10_tau ? pow(10.0, pr[3]) : pr[3];
    const double tau_n = tau * pow(nu / nutau, pr[4]);
    const int mi = a.model_index ? a.model_index[s] : 0;
    const double2 *D = a.D + row * a.nharm;
    const double2 *M = a.M + ((int64_t)mi * a.nchan + n) * a.nharm;
    double C = 0.0, S = 0.0;
    for (int k = lane; k < a.nharm; k += 64) {
        const double2 m = M[k];
        const double2 y = cmulc(D[k], m);
        const double2 e = cexp2pi((double)k * phi_n);
        double2 t = cmul(y, e);
        double b2 = 1.0;
        if (tau_n != 0.0) {
            // conj(B) = 1 / (1 - i u), u = 2 pi k tau_n: (1 + i u) / (1 + u^2)
            const double u = kTwoPi * (double)k * tau_n, den = 1.0 / (1.0 + u * u);
            t = cmul(t, cmk(den, u * den));
            b2 = den;
        }
        C += t.x;
        S += b2 * cabs2(m);
    }
    C = wave_sum(C);
    S = wave_sum(S);
    if (lane == 0) {
        if (a.errs_FT) {
            const double e2 = a.errs_FT[row] * a.errs_FT[row];
            C /= e2;
            S /= e2;
        }
        a.out[row] = C / S;
    }
}

hipError_t launch_scales(const ScalesArgs &a, hipStream_t st) {
    const int64_t rows = (int64_t)a.nsub * a.nchan;
    hipLaunchKernelGGL(k_scales, dim3((unsigned)((rows + kWaves - 1) / kWaves)), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}

}  // namespace ppf
