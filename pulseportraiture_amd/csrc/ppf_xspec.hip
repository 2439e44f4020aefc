// ppf_xspec.hip -- wave-per-row cross-spectrum kernel (128 <= nbin/2 <= 1024).
//
// k_xspec_w<LOG2N, DT, GUESS>: workgroup = 8 waves = one (sub-integration,
// block of CB channels); each wave takes CB/8 consecutive channel rows and,
// per row, with no workgroup barrier:
//   global f32/f64 row (prefetched one row ahead)  -> registers
//   wave FFT of the N = nbin/2 complex points (ppf_wfft.hpp)
//   real-FFT post-pass on (k, N-k) pairs -> D_k, D_{N-k}
//   get_noise_PS noise (pplib.py:2312-2332), Sd_n, S_n(tau=0)
//   X_k = D_k conj(M_k) / sigma~_n^2 (pptoaslib.py:1014-1031), k = 0 zeroed
//   [GUESS] accumulate w_n D_k exp(2 pi i k phi_n) for the dedispersed mean
//           profile of GetTOAs' initial phase (pptoas.py:461-499)
// The mean model spectrum of the guess is model-only: k_model_sum forms
// sum_n M_nk once per call and k_guess subtracts the masked channels.
//
// The 8 waves of a workgroup take the block's channels in rounds (round r:
// channel base + 8 r + wave); in GUESS mode each round's 8 contributions are
// summed into a block accumulator in LDS in wave order (deterministic).
// LDS: 8 padded wave buffers (17/16 N x 16 B) [+ the N+1 accumulator] =
// 136 [152] KiB at N = 1024: one workgroup (8 waves, 2 per SIMD) per CU.
#include <type_traits>

#include "ppf_internal.hpp"
#include "ppf_wfft.hpp"

namespace ppf {

constexpr int kXW = 8;                 // waves per workgroup
#ifndef PPF_SCHED_CUT
#define PPF_SCHED_CUT 1
#endif
#if PPF_SCHED_CUT
#define SCHED_CUT() __builtin_amdgcn_sched_barrier(0)
#else
#define SCHED_CUT()
#endif

template <int LOG2N, int DT, bool GUESS>
__global__ __launch_bounds__(64 * kXW) void k_xspec_w(XspecArgs a) {
    using P = wfft::Plan<LOG2N>;
    constexpr int N = P::N, R = P::R, NH = N + 1;
    constexpr int NP = N / 128;                       // (k, N-k) pairs per lane
    constexpr int SL = wfft::buf_slots<LOG2N>();      // padded wave buffer
    using RowT = typename std::conditional<DT == 0, float2, double2>::type;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double2 *buf = lds + wave * SL;
    double2 *racc = lds + kXW * SL;                   // [N+1] block guess accumulator
    double *tail = reinterpret_cast<double *>(racc + NH);   // [kXW][2]

    int s, cb;
    if (a.xcd_swizzle) {
        const int per = a.nblk / 8, x = blockIdx.x % 8, r = blockIdx.x / 8;
        cb = x * per + r % per;
        s = r / per;
    } else {
        s = blockIdx.x / a.nblk;
        cb = blockIdx.x % a.nblk;
    }
    // rounds: in round r wave w takes channel cb*CB + r*kXW + w
    const int cbase = cb * a.cb, cend = min(a.nchan, cbase + a.cb);
    const int nround = (a.cb + kXW - 1) / kXW;
    const int mi = a.model_index ? a.model_index[s] : 0;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double *fr = a.freqs + (int64_t)s * a.nchan;
    const double sqrtN = sqrt((double)N);
    const RowT *rows = reinterpret_cast<const RowT *>(a.data);
    // rfft post-pass twiddles w_k = exp(-i pi k / N), k = lane + 64 i, by
    // recurrence from w_lane (T2) with step exp(-i pi 64 / N) = T2[64]
    const double2 w_seed = a.T2[lane], w_step = a.T2[64];

    double Dg = 0.0, nu_mean_m2 = 0.0, wsum = 0.0, wcnt = 0.0;
    if constexpr (GUESS) {
        double v0 = 0.0, v1 = 0.0;
        for (int n = lane; n < a.nchan; n += 64)
            if (!mask || mask[n]) { v0 += fr[n]; v1 += 1.0; }
        v0 = wave_sum(v0);
        v1 = wave_sum(v1);
        Dg = kDconst * a.guess_DM[s] / a.P[s];
        const double nm = v0 / v1;
        nu_mean_m2 = 1.0 / (nm * nm);
        for (int k = tid; k < NH; k += 64 * kXW) racc[k] = cmk(0.0, 0.0);
    }

    auto usable = [&](int n) { return n < cend && (!mask || mask[n]); };
    RowT zr[R];
    auto fetch = [&](int n) {
        const RowT *src = rows + ((int64_t)s * a.nchan + n) * N;
#pragma unroll
        for (int q = 0; q < R; ++q) zr[q] = src[lane + 64 * q];
    };
    int n = cbase + wave;
    if (usable(n)) fetch(n);
    for (int r = 0; r < nround; ++r, n += kXW) {
        const bool live = usable(n);
        if (n < cend && !live) {
            if (lane < 4) a.chan[((int64_t)s * a.nchan + n) * 4 + lane] = 0.0;
            if (usable(n + kXW)) fetch(n + kXW);
        }
        if (live) {
            const int64_t crow = (int64_t)s * a.nchan + n;
            double2 x[R];
#pragma unroll
            for (int q = 0; q < R; ++q) x[q] = cmk((double)zr[q].x, (double)zr[q].y);
            if (usable(n + kXW)) fetch(n + kXW);       // next row in flight during this FFT
            wfft::fft_row<LOG2N>(x, buf, a.T, lane);

            // real-FFT post-pass on pairs (k, N-k), k = lane + 64 i < N/2; lane
            // 0 also owns k = N/2.  Pass 1: power sums (noise, Sd); pass 2
            // recomputes D from the LDS spectrum.
            auto dpair = [&](int i, double2 w, double2 &Dlo, double2 &Dhi) {
                const int k = lane + 64 * i;
                const double2 zk = buf[wfft::pad<LOG2N>(k)];
                const double2 zn = buf[k == 0 ? 0 : wfft::pad<LOG2N>(N - k)];
                const double2 e = cmk(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y));
                const double2 o = cmk(0.5 * (zk.x - zn.x), 0.5 * (zk.y + zn.y));
                const double2 wo = cmul(w, o);
                Dlo = cmk(e.x + wo.y, e.y - wo.x);
                Dhi = cmk(e.x - wo.y, -(e.y + wo.x));
            };
            auto dmid = [&]() {
                const double2 zm = buf[wfft::pad<LOG2N>(N / 2)];
                return cmk(zm.x, -zm.y);
            };
            double pn = 0.0, pd = 0.0;
            {
                double2 w = w_seed;
#pragma unroll
                for (int i = 0; i < NP; ++i) {
                    const int klo = lane + 64 * i, khi = N - klo;
                    double2 Dlo, Dhi;
                    dpair(i, w, Dlo, Dhi);
                    w = cmul(w, w_step);
                    const double p0 = cabs2(Dlo), p1 = cabs2(Dhi);
                    if (klo >= a.kc) pn += p0;
                    if (khi >= a.kc) pn += p1;
                    if (klo >= 1) pd += p0;
                    pd += p1;
                    SCHED_CUT();
                }
            }
            if (lane == 0) {
                const double p = cabs2(dmid());
                if (N / 2 >= a.kc) pn += p;
                pd += p;
            }
            pn = wave_sum(pn);
            pd = wave_sum(pd);
            double errs_FT;
            if (a.errs) errs_FT = a.errs[crow] * sqrtN;
            else errs_FT = sqrt(pn / (double)(NH - a.kc) / (double)(2 * N)) * sqrtN;
            const double inv_e2 = 1.0 / (errs_FT * errs_FT);

            const double2 *Mrow = a.Mft + ((int64_t)mi * a.nchan + n) * NH;
            double2 *Xrow = a.X + crow * NH;
            double wn = 0.0;
            double2 E = cmk(1.0, 0.0), W = cmk(1.0, 0.0), EN = cmk(1.0, 0.0), Em = cmk(1.0, 0.0);
            if constexpr (GUESS) {
                // phasor seeds in a region of their own: the sincos
                // temporaries must not interleave with the post-pass
                __builtin_amdgcn_sched_barrier(0);
                wn = a.guess_weights[crow];
                const double fn = fr[n];
                const double phg = Dg * (1.0 / (fn * fn) - nu_mean_m2);
                E = cexp2pi((double)lane * phg);
                __builtin_amdgcn_sched_barrier(0);
                W = cexp2pi(64.0 * phg);
                // exp(2 pi i N/2 phg) = W^(N/128), exp(2 pi i N phg) = W^(N/64)
                Em = W;
#pragma unroll
                for (int t = 128; t < N; t <<= 1) Em = cmul(Em, Em);
                EN = cmul(Em, Em);
                wsum += wn;
                wcnt += 1.0;
                __builtin_amdgcn_sched_barrier(0);
            }
            // GUESS: the contribution w_n D_k exp(2 pi i k phi_n) overwrites the
            // spectrum slot it was computed from (pad(k) for 0 < k < N, slot 0
            // for k = N; k = 0 is not used by the guess).  No lane reads a slot
            // another lane has already overwritten: iteration i reads only
            // pad(lane + 64 i) and pad(N - lane - 64 i).
            double mp = 0.0;
            double2 Dm = cmk(0.0, 0.0);
            if (lane == 0) Dm = dmid();
            {
                double2 w = w_seed;
#pragma unroll
                for (int i = 0; i < NP; ++i) {
                    const int klo = lane + 64 * i, khi = N - klo;
                    double2 Dlo, Dhi;
                    dpair(i, w, Dlo, Dhi);
                    w = cmul(w, w_step);
                    const double2 Mlo = Mrow[klo], Mhi = Mrow[khi];
                    if (klo >= 1) mp += cabs2(Mlo);
                    mp += cabs2(Mhi);
                    Xrow[klo] = (klo == 0) ? cmk(0.0, 0.0) : cscale(cmulc(Dlo, Mlo), inv_e2);
                    Xrow[khi] = cscale(cmulc(Dhi, Mhi), inv_e2);
                    if constexpr (GUESS) {
                        // exp(2 pi i (N - k) phg) = EN conj(E_k)
                        const double2 chi = cscale(cmul(Dhi, cmul(EN, cconj(E))), wn);
                        if (klo != 0) {
                            buf[wfft::pad<LOG2N>(klo)] = cscale(cmul(Dlo, E), wn);
                            buf[wfft::pad<LOG2N>(khi)] = chi;
                        } else {
                            buf[0] = chi;
                        }
                        E = cmul(E, W);
                    }
                    SCHED_CUT();
                }
            }
            if (lane == 0) {
                const double2 Mm = Mrow[N / 2];
                mp += cabs2(Mm);
                Xrow[N / 2] = cscale(cmulc(Dm, Mm), inv_e2);
                if constexpr (GUESS) buf[wfft::pad<LOG2N>(N / 2)] = cscale(cmul(Dm, Em), wn);
            }
            mp = wave_sum(mp);
            if (lane == 0) {
                double *chan = a.chan + crow * 4;
                chan[0] = errs_FT;
                chan[1] = inv_e2;
                chan[2] = pd * inv_e2;        // Sd_n
                chan[3] = mp * inv_e2;        // S_n at tau = 0
            }
            wfft::wave_sync();
        } else if (GUESS) {
            for (int k = lane; k < SL; k += 64) buf[k] = cmk(0.0, 0.0);
        }
        if constexpr (GUESS) {
            // block accumulation of this round's rows in wave order
            // (deterministic, independent of timing)
            __syncthreads();
            for (int k = tid + 1; k < NH; k += 64 * kXW) {
                const int slot = (k == N) ? 0 : wfft::pad<LOG2N>(k);
                double2 acc = racc[k];
#pragma unroll
                for (int w = 0; w < kXW; ++w) acc = cadd(acc, lds[w * SL + slot]);
                racc[k] = acc;
            }
            __syncthreads();
        }
    }
    if constexpr (GUESS) {
        if (lane == 0) {
            tail[2 * wave] = wsum;
            tail[2 * wave + 1] = wcnt;
        }
        __syncthreads();
        const int64_t base = ((int64_t)s * a.nblk + cb) * NH;
        for (int k = tid; k < NH; k += 64 * kXW) a.gR[base + k] = racc[k];
        if (tid == 0) {
            double ws = 0.0, wc = 0.0;
            for (int w = 0; w < kXW; ++w) { ws += tail[2 * w]; wc += tail[2 * w + 1]; }
            a.gw[((int64_t)s * a.nblk + cb) * 2 + 0] = ws;
            a.gw[((int64_t)s * a.nblk + cb) * 2 + 1] = wc;
        }
    }
}

// sum_n M[model][n][k] over all channels, fixed order (mean model spectrum of
// the GetTOAs guess; k_guess removes the masked channels)
__global__ void k_model_sum(const double2 *Mft, int nchan, int nharm, int nmodel, double2 *out) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = blockIdx.y;
    if (k >= nharm || m >= nmodel) return;
    const double2 *M = Mft + (int64_t)m * nchan * nharm;
    double2 acc = cmk(0.0, 0.0);
    for (int n = 0; n < nchan; ++n) acc = cadd(acc, M[(int64_t)n * nharm + k]);
    out[(int64_t)m * nharm + k] = acc;
}

template <int L2, int DT>
static void launch_w(const XspecArgs &a, hipStream_t st) {
    constexpr int N = 1 << L2;
    const size_t lds = ((size_t)kXW * wfft::buf_slots<L2>() + (a.guess ? N + 1 + kXW : 0)) *
                       sizeof(double2);
    dim3 g((unsigned)((int64_t)a.nsub * a.nblk)), b(64 * kXW);
    if (a.guess) hipLaunchKernelGGL((k_xspec_w<L2, DT, true>), g, b, lds, st, a);
    else hipLaunchKernelGGL((k_xspec_w<L2, DT, false>), g, b, lds, st, a);
}

bool xspec_wave_supported(int log2N, int cb) {
    return log2N >= 7 && log2N <= 10 && cb % kXW == 0;
}

hipError_t launch_xspec_wave(const XspecArgs &a, hipStream_t st) {
    switch (a.log2N * 2 + a.dtype) {
        case 14: launch_w<7, 0>(a, st); break;
        case 15: launch_w<7, 1>(a, st); break;
        case 16: launch_w<8, 0>(a, st); break;
        case 17: launch_w<8, 1>(a, st); break;
        case 18: launch_w<9, 0>(a, st); break;
        case 19: launch_w<9, 1>(a, st); break;
        case 20: launch_w<10, 0>(a, st); break;
        case 21: launch_w<10, 1>(a, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_model_sum(const double2 *Mft, int nchan, int nharm, int nmodel, double2 *out,
                            hipStream_t st) {
    dim3 g((unsigned)((nharm + 255) / 256), (unsigned)nmodel);
    hipLaunchKernelGGL(k_model_sum, g, dim3(256), 0, st, Mft, nchan, nharm, nmodel, out);
    return hipGetLastError();
}

}  // namespace ppf
