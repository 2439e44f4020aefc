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
#include "ppf_device.hpp"
#include "ppf_internal.hpp"

namespace ppf {

// ===========================================================================
// common row loading: z_j = x_{2j} + i x_{2j+1}
// ===========================================================================
__device__ __forceinline__ void load_row(double2 *buf, const void *src, int dtype, int64_t row,
                                         int nbin) {
    const int N = nbin >> 1;
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
__global__ __launch_bounds__(kBlock) void k_rfft_rows(RfftArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int N = a.nbin >> 1;
    const int64_t row = blockIdx.x;
    load_row(lds, a.in, a.dtype, row, a.nbin);
    __syncthreads();
    lds_fft(lds, a.log2N, a.T, false);
    double2 *o = a.out + row * (int64_t)(N + 1);
    for (int k = threadIdx.x; k <= N; k += kBlock) o[k] = rfft_bin(lds, N, a.T2, k);
}

// ===========================================================================
// k_xspec: one workgroup per (sub-integration, block of channels)
// ===========================================================================
template <int KMAX>
__global__ __launch_bounds__(kBlock) void k_xspec(XspecArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double red[kWaves * 4];
    const int N = a.nbin >> 1, nharm = N + 1;
    const int s = blockIdx.x / a.nblk, cb = blockIdx.x % a.nblk;
    const int c0 = cb * a.cb, c1 = min(a.nchan, c0 + a.cb);
    const int tid = threadIdx.x;
    const int mi = a.model_index ? a.model_index[s] : 0;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double *fr = a.freqs + (int64_t)s * a.nchan;
    const double sqrt_half_nbin = sqrt((double)a.nbin / 2.0);

    // guess stage: dedispersion phase of each channel, relative to the mean
    // frequency of the usable channels (pptoas.py:439,462-464)
    double Dg = 0.0, nu_mean_m2 = 0.0;
    if (a.guess) {
        double v[2] = {0.0, 0.0};
        for (int n = tid; n < a.nchan; n += kBlock)
            if (!mask || mask[n]) { v[0] += fr[n]; v[1] += 1.0; }
        block_sum<2>(v, red);
        double nu_mean = v[0] / v[1];
        Dg = kDconst * a.guess_DM[s] / a.P[s];
        nu_mean_m2 = pow(nu_mean, -2.0);
    }
    // per-thread guess accumulators for harmonics k = tid + kBlock*i
    double2 R[KMAX], Mb[KMAX];
    if (a.guess) {
#pragma unroll
        for (int i = 0; i < KMAX; ++i) { R[i] = cmk(0, 0); Mb[i] = cmk(0, 0); }
    }
    double wsum = 0.0, wcnt = 0.0;

    for (int n = c0; n < c1; ++n) {
        const int64_t crow = (int64_t)s * a.nchan + n;
        double *chan = a.chan + crow * 4;
        if (mask && !mask[n]) {
            if (tid == 0) { chan[0] = 0.0; chan[1] = 0.0; chan[2] = 0.0; chan[3] = 0.0; }
            continue;
        }
        load_row(lds, a.data, a.dtype, crow, a.nbin);
        __syncthreads();
        lds_fft(lds, a.log2N, a.T, false);
        // D_k for my harmonics, noise power over k >= kc, data power k >= 1
        double2 Dk[KMAX];
        double acc[2] = {0.0, 0.0};
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
            int k = tid + i * kBlock;
            if (k <= N) {
                Dk[i] = rfft_bin(lds, N, a.T2, k);
                double p2 = cabs2(Dk[i]);
                if (k >= a.kc) acc[0] += p2;
                if (k >= 1) acc[1] += p2;
            }
        }
        block_sum<2>(acc, red);   // (also orders the LDS reads before reuse)
        double errs_FT;
        if (a.errs) errs_FT = a.errs[crow] * sqrt_half_nbin;
        else errs_FT = sqrt(acc[0] / (double)(nharm - a.kc) / (double)a.nbin) * sqrt_half_nbin;
        const double inv_e2 = 1.0 / (errs_FT * errs_FT);
        // cross spectrum and model power
        const double2 *Mrow = a.Mft + ((int64_t)mi * a.nchan + n) * nharm;
        double2 *Xrow = a.X + crow * nharm;
        double mpow[1] = {0.0};
        double2 Eg = cmk(1, 0), Wg = cmk(1, 0);
        double wn = 0.0;
        if (a.guess) {
            double phg = Dg * (pow(fr[n], -2.0) - nu_mean_m2);
            Eg = cexp2pi((double)tid * phg);
            Wg = cexp2pi((double)kBlock * phg);
            wn = a.guess_weights[crow];
        }
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
            int k = tid + i * kBlock;
            if (k <= N) {
                double2 M = Mrow[k];
                if (k == 0) {
                    Xrow[0] = cmk(0.0, 0.0);       // F0_fact = 0 (pplib.py:82)
                } else {
                    mpow[0] += cabs2(M);
                    Xrow[k] = cscale(cmulc(Dk[i], M), inv_e2);
                }
                if (a.guess) {
                    R[i] = cadd(R[i], cscale(cmul(Dk[i], Eg), wn));
                    Mb[i] = cadd(Mb[i], M);
                    Eg = cmul(Eg, Wg);
                }
            }
        }
        block_sum<1>(mpow, red);
        if (tid == 0) {
            chan[0] = errs_FT;
            chan[1] = inv_e2;
            chan[2] = acc[1] * inv_e2;     // Sd_n
            chan[3] = mpow[0] * inv_e2;    // S_n at tau = 0
        }
        wsum += wn;
        wcnt += 1.0;
    }
    if (a.guess) {
        const int64_t base = ((int64_t)s * a.nblk + cb) * nharm;
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
            int k = tid + i * kBlock;
            if (k <= N) { a.gR[base + k] = R[i]; a.gM[base + k] = Mb[i]; }
        }
        if (tid == 0) {
            a.gw[((int64_t)s * a.nblk + cb) * 2 + 0] = wsum;
            a.gw[((int64_t)s * a.nblk + cb) * 2 + 1] = wcnt;
        }
    }
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
__device__ double brute_fmin(const double2 *xm, int nharm, double inv_err2, int Ns, double lo,
                             double hi, double *sh /*LDS >= 2*Ns+8*/, double *fval, int *nfev) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double step = (Ns != 1) ? (hi - lo) / (double)(Ns - 1) : 1.0;
    for (int j = wave; j < Ns; j += kWaves) {
        double ph = (double)j * step + lo;
        double f = wave_fps_eval(xm, nharm, ph, inv_err2);
        if (lane == 0) sh[j] = f;
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
        while (nf < 200 && iters < 200) {
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
// k_guess: GetTOAs initial phase (pptoas.py:461-499): FFTFIT of the weighted,
// dedispersed mean profile against the mean model profile, then
// phase_transform to nu_fit_DM (pplib.py:2688-2712).
// ===========================================================================
__global__ __launch_bounds__(kBlock) void k_guess(GuessArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];   // xm[N+1] | sh[Ns+8]
    __shared__ double red[kWaves * 4];
    const int N = a.nbin >> 1, nharm = N + 1, s = blockIdx.x, tid = threadIdx.x;
    double *sh = reinterpret_cast<double *>(lds + nharm + 1);
    double ws[2] = {0.0, 0.0};
    if (tid == 0) {
        for (int b = 0; b < a.nblk; ++b) {
            ws[0] += a.gw[((int64_t)s * a.nblk + b) * 2 + 0];
            ws[1] += a.gw[((int64_t)s * a.nblk + b) * 2 + 1];
        }
        sh[0] = ws[0]; sh[1] = ws[1];
    }
    __syncthreads();
    const double wsum = sh[0], cnt = sh[1];
    __syncthreads();
    double pw[1] = {0.0};
    for (int k = tid; k <= N; k += kBlock) {
        double2 R = cmk(0, 0), M = cmk(0, 0);
        for (int b = 0; b < a.nblk; ++b) {
            int64_t o = ((int64_t)s * a.nblk + b) * nharm + k;
            R = cadd(R, a.gR[o]);
            M = cadd(M, a.gM[o]);
        }
        R = cscale(R, 1.0 / wsum);
        M = cscale(M, 1.0 / cnt);
        if (a.guess_tau && a.guess_tau[s] != 0.0) {   // scattered model profile
            double u = kTwoPi * (double)k * a.guess_tau[s];
            double dd = 1.0 / fma(u, u, 1.0);
            M = cmul(M, cmk(dd, -u * dd));
        }
        if (k == N) R.y = 0.0;   // irfft drops the imaginary Nyquist part
        if (k >= a.kc) pw[0] += cabs2(R);
        lds[k] = (k == 0) ? cmk(0.0, 0.0) : cmulc(R, M);
    }
    block_sum<1>(pw, red);
    const double sig = sqrt(pw[0] / (double)(nharm - a.kc) / (double)a.nbin);
    const double err = sig * sqrt((double)a.nbin / 2.0);
    const double phase = brute_fmin(lds, nharm, 1.0 / (err * err), a.Ns, -0.5, 0.5, sh, nullptr,
                                    nullptr);
    if (tid == 0) {
        // nu_mean of the usable channels
        const double *fr = a.freqs + (int64_t)s * a.nchan;
        const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
        double sum = 0.0, c = 0.0;
        for (int n = 0; n < a.nchan; ++n)
            if (!mask || mask[n]) { sum += fr[n]; c += 1.0; }
        double nu_mean = sum / c;
        double nu_fit = a.nu_fits[(int64_t)s * 3 + 0];
        if (nu_fit != nu_fit) nu_fit = nu_mean;
        double DM = a.guess_DM[s], P = a.P[s];
        double out = phase + kDconst * DM * pow(P, -1.0) * (pow(nu_fit, -2.0) - pow(nu_mean, -2.0));
        if (fabs(out) >= 0.5) out = out - floor(out);   // python % 1
        if (out >= 0.5) out -= 1.0;
        a.x0[(int64_t)s * 8 + 0] = out;
    }
}

// ===========================================================================
// per-channel likelihood terms (pptoaslib.py:195-561)
// stats: 0 C, 1 C', 2 C'', 3 Q1, 4 Q1', 5 Q2, 6 S, 7 S1, 8 S2a, 9 S2b
// (all already normalised by sigma~_n^2)
// ===========================================================================
struct Fac {
    double dphi[3];   // d phi_n / d(phi, DM, GM)
    double t[2];      // (d tau_n / d theta_j) / tau_n for j = tau, alpha
    double u[3];      // (d2 tau_n / d theta_i d theta_j) / tau_n: tt, ta, aa
    bool br_tt, br_ta, br_aa;   // reference bracket gates (pptoaslib.py:371-379)
};

__device__ __forceinline__ void chan_derivs(const double *st, const Fac &fc, double dC[5],
                                            double dS[5], double d2C[5][5], double d2S[5][5]) {
    const double Cp = st[1], Cpp = st[2], Q1 = st[3], Q1p = st[4], Q2 = st[5];
    const double S1 = st[7], S2a = st[8], S2b = st[9];
    for (int i = 0; i < 3; ++i) { dC[i] = Cp * fc.dphi[i]; dS[i] = 0.0; }
    for (int j = 0; j < 2; ++j) { dC[3 + j] = Q1 * fc.t[j]; dS[3 + j] = S1 * fc.t[j]; }
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) { d2C[i][j] = Cpp * fc.dphi[i] * fc.dphi[j]; d2S[i][j] = 0.0; }
        for (int j = 0; j < 2; ++j) {
            d2C[i][3 + j] = d2C[3 + j][i] = fc.dphi[i] * fc.t[j] * Q1p;
            d2S[i][3 + j] = d2S[3 + j][i] = 0.0;
        }
    }
    const bool br[3] = {fc.br_tt, fc.br_ta, fc.br_aa};
    const int ii[3] = {0, 0, 1}, jj[3] = {0, 1, 1};
    for (int q = 0; q < 3; ++q) {
        double tt = fc.t[ii[q]] * fc.t[jj[q]];
        double c2, s2;
        if (br[q]) {
            c2 = 2.0 * tt * Q2 + fc.u[q] * Q1;
            s2 = tt * S2a + 2.0 * tt * S2b + fc.u[q] * S1;
        } else {
            c2 = tt * Q1;
            s2 = tt * S2a + tt * S1;
        }
        d2C[3 + ii[q]][3 + jj[q]] = d2C[3 + jj[q]][3 + ii[q]] = c2;
        d2S[3 + ii[q]][3 + jj[q]] = d2S[3 + jj[q]][3 + ii[q]] = s2;
    }
}

// per-channel profiled Hessian H_n (pptoaslib.py:662-671, no division by C)
__device__ __forceinline__ void chan_hess(const double *st, const Fac &fc, double H[5][5]) {
    double dC[5], dS[5], d2C[5][5], d2S[5][5];
    chan_derivs(st, fc, dC, dS, d2C, d2S);
    const double C = st[0], S = st[6];
    const double iS = 1.0 / S, iS2 = iS * iS, iS3 = iS2 * iS, C2 = C * C;
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j)
            H[i][j] = -2.0 * (C * d2C[i][j] * iS - 0.5 * C2 * d2S[i][j] * iS2 + dC[i] * dC[j] * iS +
                              C2 * dS[i] * dS[j] * iS3 - C * (dC[i] * dS[j] + dS[i] * dC[j]) * iS2);
}

struct FitGeom {           // per-sub-integration reference frequencies etc.
    double P, nu_DM, nu_GM, nu_tau, tau_lin;  // tau_lin: linear tau at nu_tau
    int log10_tau;
    bool g_sum, g_tau, g_alpha;    // taus.sum(), dtau.sum(), dalpha.sum() != 0
};

__device__ __forceinline__ Fac make_fac(double nu, const FitGeom &g, double alpha) {
    Fac f;
    const double P = g.P;
    f.dphi[0] = 1.0;
    f.dphi[1] = kDconst * (pow(nu, -2.0) - pow(g.nu_DM, -2.0)) / P;
    f.dphi[2] = kDconst * kDconst * (pow(nu, -4.0) - pow(g.nu_GM, -4.0)) / P;
    const double lnf = log(nu / g.nu_tau);
    if (!g.g_sum) {
        f.t[0] = f.t[1] = 0.0;
        f.u[0] = f.u[1] = f.u[2] = 0.0;
    } else if (g.log10_tau) {
        f.t[0] = kLn10;
        f.t[1] = lnf;
        f.u[0] = kLn10 * kLn10;
        f.u[1] = kLn10 * lnf;
        f.u[2] = lnf * lnf;
    } else {
        f.t[0] = 1.0 / g.tau_lin;
        f.t[1] = lnf;
        f.u[0] = 0.0;
        f.u[1] = lnf / g.tau_lin;
        f.u[2] = lnf * lnf;
    }
    (void)alpha;
    f.br_tt = g.g_tau;
    f.br_aa = g.g_alpha;
    f.br_ta = g.g_alpha && g.g_tau;
    return f;
}

// ===========================================================================
// k_solve: one workgroup per sub-integration
// ===========================================================================
struct SubView {
    const double2 *X;      // [nchan][nharm]
    const double2 *M;      // model spectra [nchan][nharm]
    const double *chan;    // [nchan][4]
    const double *fr;
    const uint8_t *mask;
    double *stats;         // [2][nchan][10]
    int nchan, nharm;
};

// One streaming pass over X at theta: per-channel stats -> slot, and the
// block-reduced objective f, gradient g[5], Hessian H (upper 15) -> out[21]
// (valid in every thread).  SCAT: scattering kernel B_nk != 1.
template <bool SCAT>
__device__ void eval_pass(const SubView &v, const double *th, const FitGeom &g0, int flagmask,
                          int slot, double *red, double *out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    FitGeom g = g0;
    double tau_lin = th[3];
    if (g.log10_tau) tau_lin = pow(10.0, th[3]);
    const double alpha = th[4];
    g.tau_lin = tau_lin;
    if (SCAT) {
        // reference gates: taus.sum(), dtau.sum(), dalpha.sum() (unmasked chans)
        double sm[3] = {0.0, 0.0, 0.0};
        for (int n = threadIdx.x; n < v.nchan; n += kBlock) {
            if (v.mask && !v.mask[n]) continue;
            double tn = tau_lin * pow(v.fr[n] / g.nu_tau, alpha);
            sm[0] += tn;
            sm[1] += g.log10_tau ? kLn10 * tn : tn / tau_lin;
            sm[2] += log(v.fr[n] / g.nu_tau) * tn;
        }
        block_sum<3>(sm, red);
        g.g_sum = sm[0] != 0.0;
        g.g_tau = g.g_sum && (sm[1] != 0.0);
        g.g_alpha = sm[2] != 0.0;
    } else {
        g.g_sum = g.g_tau = g.g_alpha = false;
    }
    double acc[21];
#pragma unroll
    for (int i = 0; i < 21; ++i) acc[i] = 0.0;
    // waves own contiguous channel ranges; channels processed in chunks of 64
    const int cpw = (v.nchan + kWaves - 1) / kWaves;
    const int cbeg = wave * cpw, cend = min(v.nchan, cbeg + cpw);
    for (int chunk = cbeg; chunk < cend; chunk += 64) {
        double my[10];
#pragma unroll
        for (int q = 0; q < 10; ++q) my[q] = 0.0;
        const int clim = min(cend, chunk + 64);
        for (int n = chunk; n < clim; ++n) {
            if (v.mask && !v.mask[n]) continue;
            const double nu = v.fr[n];
            const double phin = th[0] + kDconst * th[1] * (pow(nu, -2.0) - pow(g.nu_DM, -2.0)) / g.P +
                                kDconst * kDconst * th[2] * (pow(nu, -4.0) - pow(g.nu_GM, -4.0)) / g.P;
            double2 E = cexp2pi((double)lane * phin);
            const double2 W = cexp2pi(64.0 * phin);
            const double2 *Xr = v.X + (int64_t)n * v.nharm;
            double a0 = 0.0, a1 = 0.0, a2 = 0.0;
            double q1 = 0.0, q1p = 0.0, q2 = 0.0, s0 = 0.0, s1 = 0.0, s2a = 0.0, s2b = 0.0;
            double aa = 0.0, inv_e2 = 0.0;
            const double2 *Mr = nullptr;
            if (SCAT) {
                const double taun = tau_lin * pow(nu / g.nu_tau, alpha);
                aa = kTwoPi * taun;
                inv_e2 = v.chan[n * 4 + 1];
                Mr = v.M + (int64_t)n * v.nharm;
            }
            for (int k = lane; k < v.nharm; k += 64) {
                const double2 x = Xr[k];
                const double2 y = cmul(x, E);      // X E
                const double kk = (double)k;
                if (!SCAT) {
                    a0 += y.x;
                    a1 = fma(kk, y.y, a1);
                    a2 = fma(kk * kk, y.x, a2);
                } else {
                    const double uu = aa * kk;
                    const double d = 1.0 / fma(uu, uu, 1.0);
                    const double2 B = cmk(d, -uu * d);                 // 1/(1+iu)
                    const double2 Bm1 = cmk(d - 1.0, -uu * d);
                    const double2 be = cmul(B, Bm1);                   // B(B-1)
                    const double2 be2 = cmul(be, Bm1);                 // B(B-1)^2
                    const double2 cy = cmulc(y, B);                    // conj(B) Y
                    const double2 qy = cmulc(y, be);
                    a0 += cy.x;
                    a1 = fma(kk, cy.y, a1);
                    a2 = fma(kk * kk, cy.x, a2);
                    q1 += qy.x;
                    q1p = fma(kk, qy.y, q1p);
                    q2 += fma(y.x, be2.x, y.y * be2.y);
                    if (k > 0) {
                        const double Pk = cabs2(Mr[k]) * inv_e2;
                        s0 = fma(d, Pk, s0);
                        s1 = fma(2.0 * fma(B.x, be.x, B.y * be.y), Pk, s1);
                        s2a = fma(2.0 * cabs2(be), Pk, s2a);
                        s2b = fma(2.0 * fma(B.x, be2.x, B.y * be2.y), Pk, s2b);
                    }
                }
                E = cmul(E, W);
            }
            double r[10];
            r[0] = wave_sum(a0);
            r[1] = -kTwoPi * wave_sum(a1);
            r[2] = -kTwoPi * kTwoPi * wave_sum(a2);
            if (SCAT) {
                r[3] = wave_sum(q1);
                r[4] = -kTwoPi * wave_sum(q1p);
                r[5] = wave_sum(q2);
                r[6] = wave_sum(s0);
                r[7] = wave_sum(s1);
                r[8] = wave_sum(s2a);
                r[9] = wave_sum(s2b);
            } else {
                r[3] = r[4] = r[5] = 0.0;
                r[6] = v.chan[n * 4 + 3];
                r[7] = r[8] = r[9] = 0.0;
            }
            if (lane == n - chunk) {
#pragma unroll
                for (int q = 0; q < 10; ++q) my[q] = r[q];
            }
        }
        // lane l now owns channel chunk + l
        const int n = chunk + lane;
        if (n < clim && (!v.mask || v.mask[n])) {
            double *dst = v.stats + ((int64_t)slot * v.nchan + n) * 10;
#pragma unroll
            for (int q = 0; q < 10; ++q) dst[q] = my[q];
            Fac fc = make_fac(v.fr[n], g, alpha);
            double dC[5], dS[5], d2C[5][5], d2S[5][5];
            chan_derivs(my, fc, dC, dS, d2C, d2S);
            const double C = my[0], S = my[6];
            const double iS = 1.0 / S, iS2 = iS * iS, iS3 = iS2 * iS, C2 = C * C;
            acc[0] += -C2 * iS;
            int o = 6;
            for (int i = 0; i < 5; ++i) {
                if (flagmask >> i & 1) acc[1 + i] += -(2.0 * C * dC[i] * iS - C2 * dS[i] * iS2);
                for (int j = i; j < 5; ++j) {
                    if ((flagmask >> i & 1) && (flagmask >> j & 1))
                        acc[o] += -2.0 * (C * d2C[i][j] * iS - 0.5 * C2 * d2S[i][j] * iS2 +
                                          dC[i] * dC[j] * iS + C2 * dS[i] * dS[j] * iS3 -
                                          C * (dC[i] * dS[j] + dS[i] * dC[j]) * iS2);
                    ++o;
                }
            }
        }
    }
    block_sum<21>(acc, red);
#pragma unroll
    for (int i = 0; i < 21; ++i) out[i] = acc[i];
}

__device__ __forceinline__ void unpack_model(const double *o, int flagmask, const int *idx, int nf,
                                             TRModel &m) {
    m.f = o[0];
    double H[5][5];
    int q = 6;
    for (int i = 0; i < 5; ++i)
        for (int j = i; j < 5; ++j) { H[i][j] = H[j][i] = o[q]; ++q; }
    for (int a = 0; a < nf; ++a) {
        m.g[a] = o[1 + idx[a]];
        for (int b = 0; b < nf; ++b) m.H[a][b] = H[idx[a]][idx[b]];
    }
    (void)flagmask;
}

// nu_zero-case accumulation slots
enum { NZ_MAX = 16 };

template <bool SCAT>
__global__ __launch_bounds__(kBlock) void k_solve(SolveArgs a) {
    __shared__ double red[kWaves * 32];
    __shared__ double sh_theta[8];
    __shared__ int sh_cmd;
    __shared__ double sh_x[8];
    __shared__ double sh_Xinv[25];
    __shared__ double sh_misc[16];
    const int s = blockIdx.x, tid = threadIdx.x;
    const int nharm = (a.nbin >> 1) + 1;
    SubView v;
    v.X = a.X + (int64_t)s * a.nchan * nharm;
    v.M = a.Mft + (int64_t)(a.model_index ? a.model_index[s] : 0) * a.nchan * nharm;
    v.chan = a.chan + (int64_t)s * a.nchan * 4;
    v.fr = a.freqs + (int64_t)s * a.nchan;
    v.mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    v.stats = a.stats + (int64_t)s * 2 * a.nchan * 10;
    v.nchan = a.nchan;
    v.nharm = nharm;
    ppf_result *res = a.results + s;

    // ---- prologue: usable channels, mean frequency, flags --------------------
    double pr[4] = {0.0, 0.0, 0.0, 0.0};
    for (int n = tid; n < a.nchan; n += kBlock)
        if (!v.mask || v.mask[n]) { pr[0] += v.fr[n]; pr[1] += 1.0; pr[2] += v.chan[n * 4 + 2]; }
    block_sum<4>(pr, red);
    const double nu_mean = pr[0] / pr[1];
    const int nchanx = (int)pr[1];
    const double Sd = pr[2];
    int flagmask = 0;
    for (int i = 0; i < 5; ++i)
        if (a.fit_flags[(int64_t)s * 5 + i]) flagmask |= 1 << i;
    int idx[5], nf = 0;
    for (int i = 0; i < 5; ++i)
        if (flagmask >> i & 1) idx[nf++] = i;
    FitGeom g;
    g.P = a.P[s];
    double nu_fit[3];
    for (int i = 0; i < 3; ++i) {
        nu_fit[i] = a.nu_fits[(int64_t)s * 3 + i];
        if (nu_fit[i] != nu_fit[i]) nu_fit[i] = nu_mean;
    }
    g.nu_DM = nu_fit[0];
    g.nu_GM = nu_fit[1];
    g.nu_tau = nu_fit[2];
    g.log10_tau = a.log10_tau;
    g.tau_lin = 0.0;
    g.g_sum = g.g_tau = g.g_alpha = false;
    double x[5];
    for (int i = 0; i < 5; ++i) x[i] = a.init[(int64_t)s * 5 + i];
    if (a.guess) x[0] = a.x0[(int64_t)s * 8 + 0];
    const double phi_guess = x[0];
    // scattering kernel active if tau is fit or held at a nonzero value
    const double tau0 = a.log10_tau ? pow(10.0, x[3]) : x[3];
    const bool scat = (flagmask & 0x18) || tau0 != 0.0;
    if (scat != SCAT) return;     // the other instantiation owns this sub-int
    const double dof = (double)nchanx * a.nbin - (double)(nf + nchanx);

    if (nf == 0 || nchanx == 0) {
        if (tid == 0) {
            for (int i = 0; i < 32; ++i) reinterpret_cast<double *>(res)[i] = 0.0;
            res->status = PPF_ST_NOFIT;
            res->phi_guess = phi_guess;
        }
        return;
    }

    // ---- trust-region minimisation ---------------------------------------------
    int slot = 0;
    double o[21];
    eval_pass<SCAT>(v, x, g, flagmask, slot, red, o);
    TRModel m, mp;
    double radius = 1.0, p[5];
    int k = 0, status = PPF_ST_CONVERGED, nfev = 1;
    if (tid == 0) {
        unpack_model(o, flagmask, idx, nf, m);
        if (!(m.f == m.f)) status = PPF_ST_NONFINITE;
    }
    const int maxiter = a.max_iter > 0 ? a.max_iter : 200 * 5;
    while (true) {
        if (tid == 0) {
            int cmd = 0;
            if (status == PPF_ST_CONVERGED) {
                double jm = sqrt(dotn(m.g, m.g, nf));
                bool hb = cg_steihaug(m, jm, radius, p, nf);
                double pv = model_value(m, p, nf);
                if (m.f - pv <= 0.0) {
                    cmd = 0;              // scipy warnflag 2
                } else {
                    for (int i = 0; i < 5; ++i) sh_theta[i] = x[i];
                    for (int q = 0; q < nf; ++q) sh_theta[idx[q]] = x[idx[q]] + p[q];
                    sh_misc[0] = pv;
                    sh_misc[1] = hb ? 1.0 : 0.0;
                    cmd = 1;
                }
            }
            sh_cmd = cmd;
        }
        __syncthreads();
        if (sh_cmd == 0) break;
        double th[5];
        for (int i = 0; i < 5; ++i) th[i] = sh_theta[i];
        __syncthreads();
        eval_pass<SCAT>(v, th, g, flagmask, slot ^ 1, red, o);
        if (tid == 0) {
            ++nfev;
            unpack_model(o, flagmask, idx, nf, mp);
            double pv = sh_misc[0];
            bool hb = sh_misc[1] != 0.0;
            double actual = m.f - mp.f, pred = m.f - pv;
            double rho = actual / pred;
            if (rho < 0.25) radius *= 0.25;
            else if (rho > 0.75 && hb) radius = fmin(2.0 * radius, 1000.0);
            if (rho > 0.15) {
                for (int i = 0; i < 5; ++i) x[i] = th[i];
                m = mp;
                sh_misc[2] = 1.0;
            } else {
                sh_misc[2] = 0.0;
            }
            ++k;
            if (!(mp.f == mp.f) && rho != rho) { status = PPF_ST_NONFINITE; }
            if (k >= maxiter) status = PPF_ST_MAXITER;
        }
        __syncthreads();
        if (sh_misc[2] != 0.0) slot ^= 1;
        __syncthreads();
    }
    if (tid == 0) {
        for (int i = 0; i < 5; ++i) sh_x[i] = x[i];
        sh_x[5] = m.f;
        sh_x[6] = (double)status;
        sh_x[7] = (double)nfev + 1000.0 * k;
    }
    __syncthreads();
    for (int i = 0; i < 5; ++i) x[i] = sh_x[i];
    const double fun = sh_x[5];
    status = (int)sh_x[6];
    nfev = (int)fmod(sh_x[7], 1000.0);
    k = (int)(sh_x[7] / 1000.0);
    __syncthreads();
    const double *st_fit = v.stats + (int64_t)slot * v.nchan * 10;

    // ---- gates at the fit point ---------------------------------------------------
    const double tau_fit_lin = a.log10_tau ? pow(10.0, x[3]) : x[3];
    auto gates = [&](FitGeom &gg, double taulin, double alpha) {
        gg.tau_lin = taulin;
        if (!scat) { gg.g_sum = gg.g_tau = gg.g_alpha = false; return; }
        double sm[3] = {0.0, 0.0, 0.0};
        for (int n = tid; n < v.nchan; n += kBlock) {
            if (v.mask && !v.mask[n]) continue;
            double tn = taulin * pow(v.fr[n] / gg.nu_tau, alpha);
            sm[0] += tn;
            sm[1] += gg.log10_tau ? kLn10 * tn : tn / taulin;
            sm[2] += log(v.fr[n] / gg.nu_tau) * tn;
        }
        block_sum<3>(sm, red);
        gg.g_sum = sm[0] != 0.0;
        gg.g_tau = gg.g_sum && sm[1] != 0.0;
        gg.g_alpha = sm[2] != 0.0;
    };
    gates(g, tau_fit_lin, x[4]);

    // ---- zero-covariance frequencies (pptoaslib.py:776-950) -------------------------
    double nu_out[3];
    bool need_nz = false;
    for (int i = 0; i < 3; ++i) {
        nu_out[i] = a.nu_outs[(int64_t)s * 3 + i];
        if (!(nu_out[i] == nu_out[i]) || nu_out[i] == 0.0) need_nz = true;
    }
    int nzcase = flagmask;
    if (a.mode == PPF_MODE_LEGACY2) nzcase = 0x3;
    if (nzcase == 0x1f) nzcase = 0x1b;   // [1,1,1,1,1] -> [1,1,0,1,1]
    double nz[3] = {g.nu_DM, g.nu_GM, g.nu_tau};
    bool no_root = false;
    const bool closed = (nzcase == 0x3 || nzcase == 0x5 || nzcase == 0x18 || nzcase == 0xb ||
                         nzcase == 0x7 || nzcase == 0x1b || nzcase == 0xf);
    if (need_nz && closed) {
        double accv[NZ_MAX + 8];
        for (int i = 0; i < NZ_MAX + 8; ++i) accv[i] = 0.0;
        const double cD = kDconst / g.P, cG = kDconst * kDconst / g.P;
        for (int n = tid; n < v.nchan; n += kBlock) {
            if (v.mask && !v.mask[n]) continue;
            const double *st = st_fit + (int64_t)n * 10;
            const double nu = v.fr[n];
            Fac fc = make_fac(nu, g, x[4]);
            double H[5][5], Hd[5][5], Hg[5][5], Ha[5][5];
            chan_hess(st, fc, H);
            Fac f1 = fc; f1.dphi[1] = 1.0; chan_hess(st, f1, Hd);
            Fac f2 = fc; f2.dphi[2] = 1.0; chan_hess(st, f2, Hg);
            double rd[5], rg[5], ra[5];
            for (int b = 0; b < 5; ++b) { rd[b] = Hd[1][b]; rg[b] = Hg[2][b]; }
            rd[1] = Hd[1][1] * fc.dphi[1];
            rg[2] = Hg[2][2] * fc.dphi[2];
            if (nzcase == 0x18 || nzcase == 0x1b) {
                Fac f3 = fc;
                if (fc.t[1] != 0.0) {
                    f3.u[1] = fc.u[1] / fc.t[1];
                    f3.u[2] = fc.u[2] / fc.t[1];
                }
                f3.t[1] = 1.0;
                chan_hess(st, f3, Ha);
                for (int b = 0; b < 5; ++b) ra[b] = Ha[4][b];
            }
            const double w2 = pow(nu, -2.0), w4 = pow(nu, -4.0), wl = log(nu);
            double *c = accv;
            switch (nzcase) {
                case 0x3: c[0] += w2 * rd[0]; c[1] += rd[0]; break;
                case 0x5: c[0] += w4 * rg[0]; c[1] += rg[0]; break;
                case 0x18: c[0] += wl * ra[3]; c[1] += ra[3]; break;
                case 0xb:
                    c[0] += w2 * rd[3]; c[1] += w2 * rd[0]; c[2] += rd[3]; c[3] += rd[0];
                    c[16] += H[3][0]; c[17] += H[3][3];
                    break;
                case 0x7:
                    if (a.option == 0) {
                        c[0] += w4 * rg[0]; c[1] += rg[0]; c[2] += w2 * rd[2]; c[3] += rd[2];
                        c[4] += w4 * rg[2]; c[5] += rg[2]; c[6] += w2 * rd[0]; c[7] += rd[0];
                    } else {
                        c[0] += w4 * rd[0]; c[1] += rd[0]; c[2] += w2 * rg[1]; c[3] += rg[1];
                        c[4] += w4 * rd[1]; c[5] += rd[1]; c[6] += w2 * rg[0]; c[7] += rg[0];
                    }
                    break;
                case 0x1b:
                    c[0] += w2 * rd[0]; c[1] += w2 * rd[3]; c[2] += w2 * rd[4];
                    c[3] += rd[0]; c[4] += rd[3]; c[5] += rd[4];
                    c[6] += wl * ra[0]; c[7] += wl * ra[1]; c[8] += wl * ra[3];
                    c[9] += ra[0]; c[10] += ra[1]; c[11] += ra[3];
                    {   // totals over (phi, DM, tau, alpha): 10 unique
                        const int r4[4] = {0, 1, 3, 4};
                        int q = 12;
                        for (int i = 0; i < 4; ++i)
                            for (int j = i; j < 4; ++j) c[q++] += H[r4[i]][r4[j]];
                    }
                    break;
                case 0xf: {
                    double d0 = rd[0] * cD, d1 = rd[1] * cD, d2 = rd[2] * cD, d3 = rd[3] * cD;
                    double e0 = rg[0] * cG, e1 = rg[1] * cG, e2 = rg[2] * cG, e3 = rg[3] * cG;
                    if (a.option == 0) {
                        c[0] += w4 * e3; c[1] += e3; c[2] += w2 * d0; c[3] += d0;
                        c[4] += w4 * e0; c[5] += e0; c[6] += w2 * d2; c[7] += d2;
                        c[8] += w4 * e2; c[9] += e2; c[10] += w2 * d3; c[11] += d3;
                    } else {
                        c[0] += w2 * d3; c[1] += d3; c[2] += w4 * e0; c[3] += e0;
                        c[4] += w2 * d0; c[5] += d0; c[6] += w4 * e1; c[7] += e1;
                        c[8] += w2 * d1; c[9] += d1; c[10] += w4 * e3; c[11] += e3;
                    }
                    c[16] += H[3][0]; c[17] += H[3][3];
                    break;
                }
                default: break;
            }
        }
        block_sum<NZ_MAX + 8>(accv, red);
        if (tid == 0) {
            const double *c = accv;
            double num, den;
            switch (nzcase) {
                case 0x3: nz[0] = pow(c[0] / c[1], -0.5); break;
                case 0x5: nz[1] = pow(c[0] / c[1], -0.25); break;
                case 0x18: nz[2] = exp(c[0] / c[1]); break;
                case 0xb: {
                    double H13 = c[16], H33 = c[17];
                    num = H13 * c[0] - H33 * c[1];
                    den = H13 * c[2] - H33 * c[3];
                    nz[0] = pow(num / den, -0.5);
                    break;
                }
                case 0x7: {
                    if (a.option == 0 || a.option == 1) {
                        double A = c[0], B = c[1], C = c[2], D = c[3], E = c[4], F = c[5], G = c[6],
                               H = c[7];
                        double co[7] = {A * C - E * G, 0.0, E * H - A * D, 0.0, F * G - B * C, 0.0,
                                        B * D - F * H};
                        double roots[8];
                        int nr = poly_real_roots(co, 6, roots);
                        double best = 0.0, bd = 1e300;
                        bool any = false;
                        for (int i = 0; i < nr; ++i)
                            if (roots[i] > 0.0 && fabs(nu_mean - roots[i]) < bd) {
                                bd = fabs(nu_mean - roots[i]); best = roots[i]; any = true;
                            }
                        if (any) { nz[0] = nz[1] = best; } else no_root = true;
                    }
                    break;
                }
                case 0x1b: {
                    double T[4][4];
                    int q = 12;
                    for (int i = 0; i < 4; ++i)
                        for (int j = i; j < 4; ++j) { T[i][j] = T[j][i] = c[q]; ++q; }
                    double H11 = T[0][0], H22 = T[1][1], H33 = T[2][2], H44 = T[3][3];
                    double H12 = T[0][1], H13 = T[0][2], H14 = T[0][3], H23 = T[1][2],
                           H34 = T[2][3];
                    num = (H34 * H34 - H33 * H44) * c[0] + (H13 * H44 - H14 * H34) * c[1] +
                          (H14 * H33 - H13 * H34) * c[2];
                    den = (H34 * H34 - H33 * H44) * c[3] + (H13 * H44 - H14 * H34) * c[4] +
                          (H14 * H33 - H13 * H34) * c[5];
                    nz[0] = pow(num / den, -0.5);
                    num = (H13 * H22 - H12 * H23) * c[6] + (H11 * H23 - H12 * H13) * c[7] +
                          (H12 * H12 - H11 * H22) * c[8];
                    den = (H13 * H22 - H12 * H23) * c[9] + (H11 * H23 - H12 * H13) * c[10] +
                          (H12 * H12 - H11 * H22) * c[11];
                    nz[2] = exp(num / den);
                    break;
                }
                case 0xf: {
                    if (a.option == 0 || a.option == 1) {
                        double H14 = c[16], H44 = c[17];
                        double A = c[0], aa = c[1], B = c[2], b = c[3], C = c[4], cc = c[5],
                               D = c[6], d = c[7], E = c[8], e = c[9], F = c[10], f = c[11];
                        double co[6];
                        int deg;
                        if (a.option == 0) {
                            co[0] = A * A * B + H44 * C * D + H14 * E * F - H44 * B * E - A * C * F -
                                    H14 * A * D;
                            co[1] = -A * A * b - H44 * C * d - H14 * E * f + H44 * b * E + A * C * f +
                                    H14 * A * d;
                            co[2] = -2 * A * aa * B - H44 * cc * D - H14 * e * F + H44 * B * e +
                                    (A * cc + aa * C) * F + H14 * aa * D;
                            co[3] = 2 * A * aa * b + H44 * cc * d + H14 * e * f - H44 * b * e -
                                    (A * cc + aa * C) * f - H14 * aa * d;
                            co[4] = aa * aa * B - aa * cc * F;
                            co[5] = -aa * aa * b + aa * cc * f;
                            deg = 5;
                        } else {
                            co[0] = A * A * B + H44 * C * D + H14 * E * F - H44 * B * E - A * C * F -
                                    H14 * A * D;
                            co[1] = -2 * A * aa * B - H44 * cc * D - H14 * e * F + H44 * B * e +
                                    (A * cc + aa * C) * F + H14 * aa * D;
                            co[2] = -(A * A * b - aa * aa * B) - H44 * C * d - H14 * E * f +
                                    H44 * b * E + (A * C * f - aa * cc * F) + H14 * A * d;
                            co[3] = 2 * A * aa * b + H44 * cc * d + H14 * e * f - H44 * b * e -
                                    (A * cc + aa * C) * f - H14 * aa * d;
                            co[4] = -aa * aa * b + aa * cc * f;
                            deg = 4;
                        }
                        double roots[8];
                        int nr = poly_real_roots(co, deg, roots);
                        double best = 0.0, bd = 1e300;
                        bool any = false;
                        for (int i = 0; i < nr; ++i)
                            if (roots[i] > 0.0) {
                                double rr = sqrt(roots[i]);
                                if (fabs(nu_mean - rr) < bd) { bd = fabs(nu_mean - rr); best = rr; any = true; }
                            }
                        if (any) { nz[0] = nz[1] = best; } else no_root = true;
                    }
                    break;
                }
                default: break;
            }
            sh_misc[4] = nz[0]; sh_misc[5] = nz[1]; sh_misc[6] = nz[2];
            sh_misc[7] = no_root ? 1.0 : 0.0;
        }
        __syncthreads();
        nz[0] = sh_misc[4]; nz[1] = sh_misc[5]; nz[2] = sh_misc[6];
        no_root = sh_misc[7] != 0.0;
        __syncthreads();
    }
    if (need_nz)
        for (int i = 0; i < 3; ++i)
            if (!(nu_out[i] == nu_out[i]) || nu_out[i] == 0.0) nu_out[i] = nz[i];
    if (a.mode == PPF_MODE_LEGACY2) { nu_out[1] = nu_out[0]; nu_out[2] = g.nu_tau; }
    if (a.is_toa) {
        if (flagmask & 2) nu_out[1] = nu_out[0];
        else if (flagmask & 4) nu_out[0] = nu_out[1];
    }

    // ---- output transform (pptoaslib.py:1100-1114) -----------------------------------
    const double P = g.P;
    double phi_inf = x[0] + kDconst * x[1] * (0.0 - pow(g.nu_DM, -2.0)) / P +
                     kDconst * kDconst * x[2] * (0.0 - pow(g.nu_GM, -4.0)) / P;
    double phi_out = phi_inf + (kDconst / P) * x[1] * pow(nu_out[0], -2.0) +
                     (kDconst * kDconst / P) * x[2] * pow(nu_out[1], -4.0);
    if (fabs(phi_out) >= 0.5) phi_out = phi_out - floor(phi_out);
    if (phi_out >= 0.5) phi_out -= 1.0;
    double tau_out_lin = tau_fit_lin * pow(nu_out[2] / g.nu_tau, x[4]);
    double tau_out = a.log10_tau ? log10(tau_out_lin) : tau_out_lin;

    // ---- covariance at the output reference frequencies (Schur complement of
    //      fit_portrait_full_function_2deriv_with_scales, pptoaslib.py:687-773)
    FitGeom go = g;
    go.nu_DM = nu_out[0];
    go.nu_GM = nu_out[1];
    go.nu_tau = nu_out[2];
    gates(go, tau_out_lin, x[4]);
    double cv[31];
    for (int i = 0; i < 31; ++i) cv[i] = 0.0;
    for (int n = tid; n < v.nchan; n += kBlock) {
        if (v.mask && !v.mask[n]) continue;
        const double *st = st_fit + (int64_t)n * 10;
        Fac fc = make_fac(v.fr[n], go, x[4]);
        double dC[5], dS[5], d2C[5][5], d2S[5][5];
        chan_derivs(st, fc, dC, dS, d2C, d2S);
        const double C = st[0], S = st[6], an = C / S;
        double U[5];
        for (int i = 0; i < 5; ++i) U[i] = (flagmask >> i & 1) ? -2.0 * (dC[i] - an * dS[i]) : 0.0;
        const double cinv = 1.0 / (2.0 * S);
        int q = 0;
        for (int i = 0; i < 5; ++i)
            for (int j = i; j < 5; ++j) {
                if ((flagmask >> i & 1) && (flagmask >> j & 1)) {
                    cv[q] += -2.0 * (C * d2C[i][j] / S - 0.5 * C * C * d2S[i][j] / (S * S));
                    cv[15 + q] += U[i] * U[j] * cinv;
                }
                ++q;
            }
    }
    block_sum<31>(cv, red);
    int sing = 0;
    if (tid == 0) {
        double Xm[5][5], Xi[5][5];
        double full[5][5];
        int q = 0;
        for (int i = 0; i < 5; ++i)
            for (int j = i; j < 5; ++j) { full[i][j] = full[j][i] = cv[q] - cv[15 + q]; ++q; }
        for (int i2 = 0; i2 < nf; ++i2)
            for (int j2 = 0; j2 < nf; ++j2) Xm[i2][j2] = full[idx[i2]][idx[j2]];
        if (!invert_small(Xm, Xi, nf)) sing = 1;
        for (int i2 = 0; i2 < 25; ++i2) sh_Xinv[i2] = 0.0;
        for (int i2 = 0; i2 < nf; ++i2)
            for (int j2 = 0; j2 < nf; ++j2) sh_Xinv[i2 * 5 + j2] = Xi[i2][j2];
        sh_misc[8] = (double)sing;
    }
    __syncthreads();
    sing = (int)sh_misc[8];
    double Xinv[5][5];
    for (int i2 = 0; i2 < 5; ++i2)
        for (int j2 = 0; j2 < 5; ++j2) Xinv[i2][j2] = sh_Xinv[i2 * 5 + j2];
    // per-channel scales, scale errors, channel S/N
    double sn[1] = {0.0};
    for (int n = tid; n < v.nchan; n += kBlock) {
        const int64_t o2 = (int64_t)s * a.nchan + n;
        if (v.mask && !v.mask[n]) {
            a.scales[o2] = 0.0; a.scale_errs[o2] = 0.0; a.channel_snrs[o2] = 0.0;
            continue;
        }
        const double *st = st_fit + (int64_t)n * 10;
        Fac fc = make_fac(v.fr[n], go, x[4]);
        double dC[5], dS[5], d2C[5][5], d2S[5][5];
        chan_derivs(st, fc, dC, dS, d2C, d2S);
        const double C = st[0], S = st[6], an = C / S;
        double U[5];
        for (int i2 = 0; i2 < nf; ++i2) U[i2] = -2.0 * (dC[idx[i2]] - an * dS[idx[i2]]);
        double quad = 0.0;
        for (int i2 = 0; i2 < nf; ++i2)
            for (int j2 = 0; j2 < nf; ++j2) quad += U[i2] * Xinv[i2][j2] * U[j2];
        const double cinv = 1.0 / (2.0 * S);
        double var = 2.0 * (cinv + quad * cinv * cinv);
        double serr = (a.mode == PPF_MODE_LEGACY2) ? pow(S, -0.5) : sqrt(var);
        double csnr = an * sqrt(S);
        a.scales[o2] = an;
        a.scale_errs[o2] = serr;
        a.channel_snrs[o2] = csnr;
        sn[0] += csnr * csnr;
    }
    block_sum<1>(sn, red);
    if (tid == 0) {
        double pe[5] = {0, 0, 0, 0, 0};
        double *cov = a.covariance + (int64_t)s * 25;
        for (int i2 = 0; i2 < 25; ++i2) cov[i2] = 0.0;
        for (int i2 = 0; i2 < nf; ++i2) {
            for (int j2 = 0; j2 < nf; ++j2) cov[i2 * 5 + j2] = 2.0 * Xinv[i2][j2];
            pe[idx[i2]] = sqrt(2.0 * Xinv[i2][i2]);
        }
        double params[5] = {phi_out, x[1], x[2], tau_out, x[4]};
        for (int i2 = 0; i2 < 5; ++i2) { res->params[i2] = params[i2]; res->param_errs[i2] = pe[i2]; }
        for (int i2 = 0; i2 < 3; ++i2) res->nu_out[i2] = nu_out[i2];
        res->nu_fit[0] = g.nu_DM; res->nu_fit[1] = g.nu_GM; res->nu_fit[2] = g.nu_tau;
        res->chi2 = Sd + fun;
        res->red_chi2 = (Sd + fun) / dof;
        res->snr = sqrt(sn[0]);
        res->fun = fun;
        res->Sd = Sd;
        res->phi_guess = phi_guess;
        res->nfeval = (double)nfev;
        int st2 = status;
        if (no_root) st2 |= PPF_ST_NO_ROOT;
        if (sing) st2 |= PPF_ST_SINGULAR;
        if (!(fun == fun)) st2 |= PPF_ST_NONFINITE;
        res->status = (double)st2;
        res->niter = (double)k;
        res->dof = dof;
        res->nchanx = (double)nchanx;
        res->x_fit_phi = x[0];
        res->x_fit_tau = x[3];
        res->reserved[0] = res->reserved[1] = res->reserved[2] = 0.0;
    }
}

// ===========================================================================
// k_rotate: out = irfft(rfft(in) * exp(2 pi i k phase_row))
// ===========================================================================
template <int KMAX>
__global__ __launch_bounds__(kBlock) void k_rotate(RotateArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int N = a.nbin >> 1;
    const int64_t row = blockIdx.x;
    load_row(lds, a.in, a.dtype, row, a.nbin);
    __syncthreads();
    lds_fft(lds, a.log2N, a.T, false);
    double2 Xk[KMAX], Xn[KMAX];
    const double ph = a.phases[row];
    // harmonics handled by this thread: k = tid + 256 i, k < N (pre-pass pairs k, N-k)
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        int k = threadIdx.x + i * kBlock;
        if (k < N) {
            double2 X1 = rfft_bin(lds, N, a.T2, k);
            double2 X2 = rfft_bin(lds, N, a.T2, N - k);
            X1 = cmul(X1, cexp2pi((double)k * ph));
            X2 = cmul(X2, cexp2pi((double)(N - k) * ph));
            if (k == 0) { X1.y = 0.0; X2.y = 0.0; }   // DC and Nyquist: real parts only
            Xk[i] = X1;
            Xn[i] = X2;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        int k = threadIdx.x + i * kBlock;
        if (k < N) lds[k] = irfft_prebin(Xk[i], Xn[i], a.T2[k]);
    }
    __syncthreads();
    lds_fft(lds, a.log2N, a.T, true);
    const double sc = 1.0 / (double)N;
    double2 *o = reinterpret_cast<double2 *>(a.out) + row * (int64_t)N;
    for (int j = threadIdx.x; j < N; j += kBlock) o[j] = cscale(lds[j], sc);
}

// ===========================================================================
// k_noise: get_noise_PS per row
// ===========================================================================
__global__ __launch_bounds__(kBlock) void k_noise(NoiseArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    __shared__ double red[kWaves * 2];
    const int N = a.nbin >> 1;
    const int64_t row = blockIdx.x;
    load_row(lds, a.in, a.dtype, row, a.nbin);
    __syncthreads();
    lds_fft(lds, a.log2N, a.T, false);
    double acc[1] = {0.0};
    for (int k = threadIdx.x + a.kc; k <= N; k += kBlock) acc[0] += cabs2(rfft_bin(lds, N, a.T2, k));
    block_sum<1>(acc, red);
    if (threadIdx.x == 0) a.out[row] = sqrt(acc[0] / (double)a.nbin / (double)(N + 1 - a.kc));
}

// ===========================================================================
// k_phase_shift: pplib.fit_phase_shift per profile
// ===========================================================================
__global__ __launch_bounds__(kBlock) void k_phase_shift(PhaseShiftArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];   // [N] fft | [N+1] xm | sh
    __shared__ double red[kWaves * 4];
    const int N = a.nbin >> 1, nharm = N + 1;
    double *sh = reinterpret_cast<double *>(lds + 2 * N + 2);
    const int64_t prof = blockIdx.x;
    double2 *fbuf = lds, *xm = lds + N;
    // model spectrum first (into xm as M_k)
    const int mi = a.model_index ? a.model_index[prof] : 0;
    load_row(fbuf, a.model, 1, mi, a.nbin);
    __syncthreads();
    lds_fft(fbuf, a.log2N, a.T, false);
    double pp[1] = {0.0};
    for (int k = threadIdx.x; k <= N; k += kBlock) {
        double2 M = rfft_bin(fbuf, N, a.T2, k);
        xm[k] = M;
        if (k >= 1) pp[0] += cabs2(M);
    }
    __syncthreads();
    load_row(fbuf, a.data, a.dtype, prof, a.nbin);
    __syncthreads();
    lds_fft(fbuf, a.log2N, a.T, false);
    double acc[3] = {0.0, 0.0, pp[0]};
    for (int k = threadIdx.x; k <= N; k += kBlock) {
        double2 D = rfft_bin(fbuf, N, a.T2, k);
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

__global__ __launch_bounds__(kBlock) void k_synth(SynthArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int N = a.nbin >> 1;
    const int s = blockIdx.x / a.nchan, n = blockIdx.x % a.nchan;
    const double2 *Mrow = a.Mft + (int64_t)n * (N + 1);
    // phase of this row: rotate_data(model, -phi, -DM, P, freq, nu_ref)
    const double D = kDconst * (-a.DM[s]) / a.P[s];
    const double ph = -a.phi[s] + D * (pow(a.freqs[n], -2.0) - pow(a.nu_ref, -2.0));
    for (int k = threadIdx.x; k < N; k += kBlock) {
        double2 X1 = cmul(Mrow[k], cexp2pi((double)k * ph));
        double2 X2 = cmul(Mrow[N - k], cexp2pi((double)(N - k) * ph));
        if (k == 0) { X1.y = 0.0; X2.y = 0.0; }
        lds[k] = irfft_prebin(X1, X2, a.T2[k]);
    }
    __syncthreads();
    lds_fft(lds, a.log2N, a.T, true);
    const double sc = 1.0 / (double)N;
    const int64_t row = (int64_t)s * a.nchan + n;
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
// host-side launchers
// ===========================================================================
static inline int log2i(int n) {
    int l = 0;
    while ((1 << l) < n) ++l;
    return l;
}

hipError_t launch_twiddles(int N, double2 *T, double2 *T2, hipStream_t st) {
    hipLaunchKernelGGL(k_twiddles, dim3((N + 255) / 256), dim3(256), 0, st, N, T, T2);
    return hipGetLastError();
}
hipError_t launch_rfft_rows(const RfftArgs &a, int64_t nrows, hipStream_t st) {
    size_t lds = (size_t)(a.nbin / 2) * sizeof(double2);
    hipLaunchKernelGGL(k_rfft_rows, dim3((unsigned)nrows), dim3(kBlock), lds, st, a);
    return hipGetLastError();
}
static inline int kmax_for(int N) { return (N + 1 + kBlock - 1) / kBlock; }

hipError_t launch_xspec(const XspecArgs &a, hipStream_t st) {
    size_t lds = (size_t)(a.nbin / 2) * sizeof(double2);
    dim3 g((unsigned)((int64_t)a.nsub * a.nblk)), b(kBlock);
    switch (kmax_for(a.nbin / 2)) {
        case 1: hipLaunchKernelGGL(k_xspec<1>, g, b, lds, st, a); break;
        case 2: hipLaunchKernelGGL(k_xspec<2>, g, b, lds, st, a); break;
        case 3: hipLaunchKernelGGL(k_xspec<3>, g, b, lds, st, a); break;
        case 5: hipLaunchKernelGGL(k_xspec<5>, g, b, lds, st, a); break;
        case 9: hipLaunchKernelGGL(k_xspec<9>, g, b, lds, st, a); break;
        case 17: hipLaunchKernelGGL(k_xspec<17>, g, b, lds, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_guess(const GuessArgs &a, hipStream_t st) {
    size_t lds = (size_t)(a.nbin / 2 + 2) * sizeof(double2) + (size_t)(a.Ns + 8) * sizeof(double);
    hipLaunchKernelGGL(k_guess, dim3((unsigned)a.nsub), dim3(kBlock), lds, st, a);
    return hipGetLastError();
}
hipError_t launch_solve(const SolveArgs &a, hipStream_t st) {
    if (a.any_plain) hipLaunchKernelGGL(k_solve<false>, dim3((unsigned)a.nsub), dim3(kBlock), 0, st, a);
    if (a.any_scat) hipLaunchKernelGGL(k_solve<true>, dim3((unsigned)a.nsub), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_rotate(const RotateArgs &a, int64_t nrows, hipStream_t st) {
    size_t lds = (size_t)(a.nbin / 2) * sizeof(double2);
    dim3 g((unsigned)nrows), b(kBlock);
    switch ((a.nbin / 2 + kBlock - 1) / kBlock) {
        case 1: hipLaunchKernelGGL(k_rotate<1>, g, b, lds, st, a); break;
        case 2: hipLaunchKernelGGL(k_rotate<2>, g, b, lds, st, a); break;
        case 4: hipLaunchKernelGGL(k_rotate<4>, g, b, lds, st, a); break;
        case 8: hipLaunchKernelGGL(k_rotate<8>, g, b, lds, st, a); break;
        case 16: hipLaunchKernelGGL(k_rotate<16>, g, b, lds, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_noise(const NoiseArgs &a, int64_t nrows, hipStream_t st) {
    size_t lds = (size_t)(a.nbin / 2) * sizeof(double2);
    hipLaunchKernelGGL(k_noise, dim3((unsigned)nrows), dim3(kBlock), lds, st, a);
    return hipGetLastError();
}
hipError_t launch_phase_shift(const PhaseShiftArgs &a, int nprof, hipStream_t st) {
    size_t lds = (size_t)(a.nbin + 2) * sizeof(double2) + (size_t)(a.Ns + 8) * sizeof(double);
    hipLaunchKernelGGL(k_phase_shift, dim3((unsigned)nprof), dim3(kBlock), lds, st, a);
    return hipGetLastError();
}
hipError_t launch_synth(const SynthArgs &a, hipStream_t st) {
    size_t lds = (size_t)(a.nbin / 2) * sizeof(double2);
    hipLaunchKernelGGL(k_synth, dim3((unsigned)(a.nsub * a.nchan)), dim3(kBlock), lds, st, a);
    return hipGetLastError();
}

}  // namespace ppf
