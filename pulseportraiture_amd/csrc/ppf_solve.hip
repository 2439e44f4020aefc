// ppf_solve.hip -- the batched wideband solver (pptoaslib.py:564-1144).
//
// One ppf_fit_batch call runs, after k_xspec / k_guess:
//   k_tr_init                     per sub-int: prologue (usable channels,
//                                 nu_fit defaults, Sd, dof, start point)
//   repeat { k_pass ; k_tr_step } until every sub-int has stopped
//     k_pass<SCAT,U>              grid (sub-int x block of 64 channels): one
//                                 streaming pass over the cross spectrum at
//                                 the point each sub-int wants evaluated ->
//                                 per-channel C, C', C'' (+ scattering sums)
//                                 and the block's share of f, g, H
//     k_tr_step                   one wave per sub-int: fixed-order reduction
//                                 of the block partials, then one iteration
//                                 of the scipy trust-ncg replica (accept /
//                                 reject, radius, CG-Steihaug subproblem)
//   k_postfit                     one workgroup per sub-int: zero-covariance
//                                 frequencies, output transform, Schur
//                                 covariance, scales, channel S/N, chi2
// Splitting the cold trust-region / post-fit code out of the streaming pass
// keeps the pass at <= 128 VGPRs (>= 4 waves/SIMD) with every harmonic load
// of a channel row in flight.
#include "ppf_device.hpp"
#include "ppf_internal.hpp"
#include "ppf_state.hpp"

namespace ppf {

// Newton trust region also for the moment-expansion fits (phase / DM / GM
// without scattering; C4: 1.04 instead of 2.34 data passes per fit);
// 0 builds them with scipy's trust-ncg path only
#ifndef PPF_NEWTON_MOM
#define PPF_NEWTON_MOM 1
#endif
// channel-subset warm start of the Newton scattering fits (0: every
// evaluation on every channel)
#ifndef PPF_NEWTON_SUBSET
#define PPF_NEWTON_SUBSET 1
#endif

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

// reference gates (taus.sum(), dtau.sum(), dalpha.sum()) at (tau_lin, alpha)
// over the usable channels; wave-level (all 64 lanes of the calling wave).
// The reference's gates taus.sum(), dtau.sum(), dalpha.sum() != 0
// (pptoaslib.py:271-276, 351-355, 368-382).  lnr[n] = ln(nu_n / nu_tau) is
// cached per channel by k_tr_init (only the exact-zero outcome matters, so
// tau_n = tau exp(alpha lnr) instead of the fit's pow form is equivalent).
__device__ void wave_gates(const double *lnr, const uint8_t *mask, int nchan, double tau_lin,
                           double alpha, int log10_tau, int &g_sum, int &g_tau, int &g_alpha) {
    const int lane = threadIdx.x & 63;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int n = lane; n < nchan; n += 64) {
        if (mask && !mask[n]) continue;
        const double l = lnr[n];
        const double tn = tau_lin * exp(alpha * l);
        s0 += tn;
        s1 += log10_tau ? kLn10 * tn : tn / tau_lin;
        s2 += l * tn;
    }
    s0 = wave_sum(s0); s1 = wave_sum(s1); s2 = wave_sum(s2);
    g_sum = s0 != 0.0;
    g_tau = g_sum && s1 != 0.0;
    g_alpha = s2 != 0.0;
}

// k_classify: which sub-ints need the cross spectrum X in HBM (scattering
// fits, which k_pass streams; every fit when the moments are taken from X,
// i.e. off the fused k_xmom_g path), and X's slot for each of them: the
// slots are the order of those sub-ints (one workgroup, a running
// exclusive scan), so the workspace holds X only for the sub-ints that use
// it.  Past the caller's xcap: slot -2, and k_tr_init fails the fit with
// PPF_ST_NOSPACE.  Same scattering test as k_tr_init's `scat`.
constexpr int kClassifyBlock = 1024;
__global__ __launch_bounds__(kClassifyBlock) void k_classify(int nsub, const int32_t *fit_flags,
                                                             const double *init, int log10_tau,
                                                             int fused, int xcap, uint8_t *needx,
                                                             int32_t *xslot) {
    __shared__ int wtot[kClassifyBlock / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int base_slot = 0;
    for (int s0 = 0; s0 < nsub; s0 += kClassifyBlock) {
        const int s = s0 + tid;
        int need = 0;
        if (s < nsub) {
            const double x3 = init[(int64_t)s * 5 + 3];
            const double tau0 = log10_tau ? pow(10.0, x3) : x3;
            const bool scat =
                fit_flags[(int64_t)s * 5 + 3] || fit_flags[(int64_t)s * 5 + 4] || tau0 != 0.0;
            need = (!fused || scat) ? 1 : 0;
        }
        const unsigned long long bal = __ballot(need);
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[wave] = __popcll(bal);
        __syncthreads();
        int off = base_slot;
        for (int w = 0; w < wave; ++w) off += wtot[w];
        int chunk = 0;
        for (int w = 0; w < kClassifyBlock / 64; ++w) chunk += wtot[w];
        if (s < nsub) {
            const int slot = off + below;
            needx[s] = (need && slot < xcap) ? 1 : 0;
            xslot[s] = need ? (slot < xcap ? slot : -2) : -1;
        }
        base_slot += chunk;
        __syncthreads();
    }
}

// k_gflag: the sub-ints whose GetTOAs guess spectrum k_xspec_w accumulates
// (ppf_xspec.hip, GS): those it streams (needx) whose mean model has no
// harmonic above the fused range (max_n KC[model][n] <= klim, the FFTFIT sums
// of k_guess stop at that cutoff); the others take k_dsum.
__global__ __launch_bounds__(kBlock) void k_gflag(int nsub, int nchan, const uint8_t *needx,
                                                  const int32_t *KC, const int32_t *model_index,
                                                  int klim, uint8_t *gflag) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= nsub) return;
    int ok = 0;
    if (!needx || needx[s]) {
        const int64_t m = model_index ? model_index[s] : 0;
        int mx = 0;
        for (int n = 0; n < nchan; ++n) mx = max(mx, KC[m * nchan + n]);
        ok = mx <= klim ? 1 : 0;
    }
    gflag[s] = (uint8_t)ok;
}

hipError_t launch_gflag(int nsub, int nchan, const uint8_t *needx, const int32_t *KC,
                        const int32_t *model_index, int klim, uint8_t *gflag, hipStream_t st) {
    hipLaunchKernelGGL(k_gflag, dim3((unsigned)((nsub + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       nsub, nchan, needx, KC, model_index, klim, gflag);
    return hipGetLastError();
}

#ifndef PPF_TRINIT_ZERO
#define PPF_TRINIT_ZERO 0   // 1: k_tr_init zeroes the moment fits' stats slots
#endif
// ===========================================================================
// k_tr_init: one wave per sub-integration (4 per workgroup)
// ===========================================================================
__global__ __launch_bounds__(kBlock) void k_tr_init(SolveArgs a) {
    const int lane = threadIdx.x & 63;
    const int s = blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (s >= a.nsub) return;
    const double *fr = a.freqs + (int64_t)s * a.nchan;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    // (runs before the spectrum kernels: nothing here reads chan[])
    double sf = 0.0, cnt = 0.0;
    for (int n = lane; n < a.nchan; n += 64)
        if (!mask || mask[n]) { sf += fr[n]; cnt += 1.0; }
    sf = wave_sum(sf); cnt = wave_sum(cnt);
    TRState &S = a.state[s];
    int flagmask = 0, nf = 0;
    for (int i = 0; i < 5; ++i)
        if (a.fit_flags[(int64_t)s * 5 + i]) { flagmask |= 1 << i; ++nf; }
    double x[5];
    for (int i = 0; i < 5; ++i) x[i] = a.init[(int64_t)s * 5 + i];
    if (a.guess) x[0] = a.x0[(int64_t)s * 8 + 0];
    // method='TNC' box (NaN: no bound): scipy's TNC starts from x0 clipped
    // into it
    double lo[5], hi[5];
    int bnd = 0;
    for (int i = 0; i < 5; ++i) {
        lo[i] = -INFINITY;
        hi[i] = INFINITY;
        if (a.bounds) {
            const double l = a.bounds[((int64_t)s * 5 + i) * 2], u = a.bounds[((int64_t)s * 5 + i) * 2 + 1];
            if (l == l) lo[i] = l;
            if (u == u) hi[i] = u;
        }
        x[i] = fmin(fmax(x[i], lo[i]), hi[i]);
        if ((flagmask >> i & 1) && (lo[i] > -INFINITY || hi[i] < INFINITY)) bnd = 1;
    }
    const double tau0 = a.log10_tau ? pow(10.0, x[3]) : x[3];
    const int scat = ((flagmask & 0x18) || tau0 != 0.0) ? 1 : 0;
    const double nu_mean = sf / cnt;
    double nu_fit[3];
    for (int i = 0; i < 3; ++i) {
        nu_fit[i] = a.nu_fits[(int64_t)s * 3 + i];
        if (nu_fit[i] != nu_fit[i]) nu_fit[i] = nu_mean;
    }
    int gs = 0, gt = 0, ga = 0;
    if (scat) {
        // ln(nu_n / nu_tau) for the gates (the moment path's dphi slot is
        // free for scattering fits)
        double *lnr = a.dphi + (int64_t)s * a.nchan * 2;
        for (int n = lane; n < a.nchan; n += 64) lnr[n] = log(fr[n] / nu_fit[2]);
        wave_lds_sync();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        wave_gates(lnr, mask, a.nchan, tau0, x[4], a.log10_tau, gs, gt, ga);
    }
    if (lane == 0) {
        for (int i = 0; i < 5; ++i) { S.x[i] = x[i]; S.th[i] = x[i]; S.g[i] = 0.0; }
        S.f = 0.0;
        for (int i = 0; i < 15; ++i) S.H[i] = 0.0;
        // scattering fits without bounds take the Newton trust region
        // (tr_update_newton) unless the caller asked for scipy's path
        S.newton = (a.newton && (scat || PPF_NEWTON_MOM) && !bnd) ? 1 : 0;
        S.radius = S.newton ? kNewtonR0 : 1.0;   // scipy initial_trust_radius = 1
        // channel-subset warm start of the scattering fits (every sub-th
        // group of 64 channels, at least two groups; PPF_NEWTON_SUBSET)
        int sub = 1;
        if (PPF_NEWTON_SUBSET && S.newton && scat) {
            const int ng = (a.nchan + 63) / 64;
            while (sub * 2 <= kSubsetMaxStride && sub * 2 <= ng / 2) sub *= 2;
        }
        S.sub = sub;
        S.sub0 = sub;
        S.nsubev = 0;
        S.pnorm = 0.0;
        S.pred = 0.0;
        for (int i = 0; i < 3; ++i) S.nu_fit[i] = nu_fit[i];
        S.nu_mean = nu_mean;
        S.Sd = 0.0;                     // summed from chan[] in k_postfit
        S.dof = cnt * (double)a.nbin - (double)(nf + (int)cnt);
        S.phi_guess = x[0];
        S.k = 0;
        S.status = PPF_ST_CONVERGED;
        S.nfev = 0;
        S.slot_cur = 0;
        S.slot_eval = 0;
        S.flagmask = flagmask;
        S.nchanx = (int)cnt;
        S.scat = scat;
        S.hb = 0;
        S.g_sum = gs; S.g_tau = gt; S.g_alpha = ga;
        for (int i = 0; i < 5; ++i) { S.lo[i] = lo[i]; S.hi[i] = hi[i]; }
        S.bnd = bnd;
        if (nf == 0 || cnt == 0.0) {
            S.phase = PH_DONE;
            S.status = PPF_ST_NOFIT;
        } else if (a.xslot && a.xslot[s] == -2) {
            S.phase = PH_DONE;               // needs X, but the workspace has no slot
            S.status = PPF_ST_NOSPACE;
        } else {
            S.phase = PH_INIT;
        }
    }
    // moment mode: phase-only channel model (no scattering), the objective
    // and its derivatives from per-channel Taylor moments (ppf_moments)
    const int mmode = (a.moments && !scat && nf > 0 && cnt > 0.0) ? 1 : 0;
    if (lane == 0) {
        S.mmode = mmode;
        S.mom16 = (mmode && a.mom16) ? 1 : 0;
        S.need_mom = mmode;
        S.mtarget = 0;
        S.macc = 0;
        S.meval = 0;
        S.nmom = 0;
        S.mvalid[0] = mmode;
        S.mvalid[1] = 0;
        for (int i = 0; i < 3; ++i) { S.mc[0][i] = x[i]; S.mc[1][i] = x[i]; }
        // which iteration kernels the call needs at all (the host skips the
        // others)
        if (a.kinds && S.phase == PH_INIT) atomicAdd(a.kinds + (mmode ? 0 : 1), 1u);
    }
    if (mmode) {
        const double P = a.P[s];
        const double nuDM2 = pow(nu_fit[0], -2.0), nuGM4 = pow(nu_fit[1], -4.0);
        double *dp = a.dphi + (int64_t)s * a.nchan * 2;
        double *st = a.stats + (int64_t)s * 2 * a.nchan * 10;
        for (int n = lane; n < a.nchan; n += 64) {
            const double nu = fr[n];
            dp[2 * n + 0] = kDconst * (pow(nu, -2.0) - nuDM2) / P;
            dp[2 * n + 1] = kDconst * kDconst * (pow(nu, -4.0) - nuGM4) / P;
            // S_n (slot 6) is stored with C, C', C'' by k_tr_mom, and (round
            // 6) the scattering slots' zeros with them: zeroing both slots
            // here wrote nsub x nchan x 160 B (840 MB, 0.3 ms at C2)
            if (PPF_TRINIT_ZERO)
                for (int q = 0; q < 2; ++q) {
                    double *d = st + ((int64_t)q * a.nchan + n) * 10;
                    for (int j = 0; j < 10; ++j) d[j] = 0.0;
                }
        }
    }
}

// ===========================================================================
// k_pass: one streaming pass over X for the sub-ints that asked for one
// grid = nsub * nblk; workgroup = 4 waves; thread t owns channel
// blk * kPassChans + t and runs its whole harmonic sum (X is harmonic-major,
// so a wave's loads of one harmonic are 64 consecutive channels, 1 KiB):
// no cross-lane reduction per channel, the per-channel setup (phase, the
// scattering time, exact phasor seeds every 64 harmonics) amortised over the
// row, one fixed-order block reduction of f, g, H per workgroup.
// ===========================================================================
constexpr int kPassChans = kBlock;             // channels per workgroup

#ifndef PPF_PASS_WPE
#define PPF_PASS_WPE 3
#endif
#ifndef PPF_PASS_SPLIT
#define PPF_PASS_SPLIT 1
#endif
#ifndef PPF_PASS_NT
#define PPF_PASS_NT PPF_NT
#endif
template <bool SCAT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PPF_PASS_WPE))) void k_pass(SolveArgs a) {
    __shared__ double red[kWaves * 21];
    const int nblk = (a.nchan + kPassChans - 1) / kPassChans;
    // channel-block-major order: the workgroups resident together share one
    // block of |M|^2 (nharm x 256 channels, read by every sub-int's pass)
    // instead of each streaming its own.  With nblk a multiple of 8 the
    // blocks of one XCD (workgroups b = x mod 8) take nblk / 8 channel blocks
    // for all sub-ints, so that XCD's L2 holds its |M|^2 share.
    int s, blk;
    if (nblk % 8 == 0) {
        const int x = blockIdx.x & 7, r = blockIdx.x >> 3;
        blk = x * (nblk >> 3) + r / a.nsub;
        s = r % a.nsub;
    } else {
        blk = blockIdx.x / a.nsub;
        s = blockIdx.x % a.nsub;
    }
    const TRState &S = a.state[s];
    if (S.phase == PH_DONE || S.scat != (SCAT ? 1 : 0) || S.mmode) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nharm = (a.nbin >> 1) + 1;
    const double *fr = a.freqs + (int64_t)s * a.nchan;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double *chan = a.chan + (int64_t)s * a.nchan * 4;
    const int mi = a.model_index ? a.model_index[s] : 0;
    double *stats = a.stats + ((int64_t)s * 2 + S.slot_eval) * a.nchan * 10;
    double th[5];
    for (int i = 0; i < 5; ++i) th[i] = S.th[i];
    const int flagmask = S.flagmask;
    FitGeom g;
    g.P = a.P[s];
    g.nu_DM = S.nu_fit[0];
    g.nu_GM = S.nu_fit[1];
    g.nu_tau = S.nu_fit[2];
    g.log10_tau = a.log10_tau;
    const double tau_lin = a.log10_tau ? pow(10.0, th[3]) : th[3];
    const double alpha = th[4];
    g.tau_lin = tau_lin;
    g.g_sum = S.g_sum; g.g_tau = S.g_tau; g.g_alpha = S.g_alpha;
    const double nuDM2 = pow(g.nu_DM, -2.0), nuGM4 = pow(g.nu_GM, -4.0);

    // Newton warm start: only every S.sub-th group of 64 channels (a wave).
    // With a stride of four groups or more a workgroup holds at most one such
    // group, its first; then all four waves take that group's 64 channels and
    // split its harmonics (split: workgroup-uniform), so a subset pass is not
    // one wave's serial harmonic loop per 256 channels while the other three
    // idle (C5: 16 of 256 groups per sub-int)
    const bool split = PPF_PASS_SPLIT && S.sub >= kWaves;
    const int n = blk * kPassChans + (split ? lane : (int)threadIdx.x);
    const bool in_sub = S.sub <= 1 || ((n >> 6) % S.sub) == 0;
    const bool use_n = in_sub && n < a.nchan && (!mask || mask[n]);
    // harmonics the wave sums: up to the largest cutoff of its channels
    // (k_model_cut; wave-uniform so the loads stay coalesced); split: the
    // wave's quarter of them, in whole 64-harmonic phasor-seed spans
    const int kend = (int)wave_max(use_n ? (double)a.KC[(int64_t)mi * a.nchan + n] : 1.0);
    int kb0 = 0, kb1 = kend;
    if (split) {
        const int Q = ((kend + 64 * kWaves - 1) / (64 * kWaves)) * 64;
        kb0 = min(kend, wave * Q);
        kb1 = min(kend, kb0 + Q);
    }
    double nu = 0.0, aa = 0.0, inv_e2 = 0.0;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    double q1 = 0.0, q1p = 0.0, q2 = 0.0, s0 = 0.0, t1 = 0.0, t2 = 0.0;
    if (use_n) {
        nu = fr[n];
        const double phin = th[0] + kDconst * th[1] * (pow(nu, -2.0) - nuDM2) / g.P +
                            kDconst * kDconst * th[2] * (pow(nu, -4.0) - nuGM4) / g.P;
        const double2 W = cexp2pi(phin);
        const double2 *Xc = a.X + (int64_t)(a.xslot ? a.xslot[s] : s) * nharm * a.nchan + n;
        const double *Pc = a.MP + (int64_t)mi * nharm * a.nchan + n;
        const int64_t xs = a.nchan;
        if (SCAT) {
            aa = kTwoPi * tau_lin * pow(nu / g.nu_tau, alpha);
            inv_e2 = chan[n * 4 + 1];
        }
        // Scattering terms in closed form (pptoaslib.py:344-455 restated):
        // with u = 2 pi k tau_n, d = 1 / (1 + u^2), w = conj(B) = d (1 + iu),
        //   B - 1 = -iu B, so dB ~ B (B - 1) = -iu B^2, d2B ~ -u^2 B^3 and
        //   y conj(B) = y w = z1,  y conj(B (B-1)) = iu z2 (z2 = z1 w),
        //   y conj(B (B-1)^2) = -u^2 z1 w^2 w,
        //   |B|^2 = d, Re B conj(B(B-1)) = -u^2 d^2, |B(B-1)|^2 = u^2 d^2,
        //   Re B conj(B(B-1)^2) = -u^2 d^3 (1 - u^2):
        // the S sums need only the real t1 = sum u^2 d^2 P, t2 = sum
        // u^2 d^3 (1 - u^2) P.
        // harmonics in groups of KB: the next group's loads are issued before
        // the current group is summed (software pipeline, one memory wait per
        // group)
#ifndef PPF_PASS_KB
// harmonics per load group.  Round 6: 3 instead of 4 -- at three waves per
// SIMD the 4-harmonic body spilled 40 B (168 VGPRs), the 3-harmonic one
// fits in 154: C3 +0.8 %, C5 +2 % (profiles/r06/ab_kb_status.txt)
#define PPF_PASS_KB 3
#endif
        constexpr int KB = PPF_PASS_KB;
        // two buffers, loads one group ahead of the sums.  The loop is
        // unrolled by two so each buffer keeps its registers (rotating them
        // with moves would make each iteration wait for all its loads).
        // Loads are unconditional (the index clamped into the row) and terms
        // past the last harmonic are zeroed where they are SUMMED: a select
        // on a freshly loaded value would also force that wait.
        double2 xa[KB], xb[KB];
        double pa[KB], pb[KB];
        auto ldg = [&](int kb, double2 (&xo)[KB], double (&po)[KB]) {
#pragma unroll
            for (int u = 0; u < KB; ++u) {
                const int k = min(kb + u, kend - 1);
#if PPF_PASS_NT
                // X streamed past the L2, which keeps |M|^2 (ld_stream)
                xo[u] = ld_stream(Xc + k * xs);
#else
                xo[u] = Xc[k * xs];
#endif
                if (SCAT) po[u] = Pc[k * xs];
            }
        };
        double2 E = cmk(1.0, 0.0);
        auto sum_group = [&](int kb, const double2 (&xv)[KB], const double (&pv)[KB]) {
            // exact seed at the first group of every 64 harmonics (KB need
            // not divide 64; with KB = 4 this is kb % 64 == 0 as before)
            if ((kb & 63) < KB) E = cexp2pi((double)kb * phin);
#pragma unroll
            for (int u = 0; u < KB; ++u) {
                const double kk = (double)(kb + u);
                const bool in = kb + u < kb1;
                const double2 y = in ? cmul(xv[u], E) : cmk(0.0, 0.0);
                if (!SCAT) {
                    a0 += y.x;
                    a1 = fma(kk, y.y, a1);
                    a2 = fma(kk * kk, y.x, a2);
                } else {
                    const double uu = aa * kk, u2 = uu * uu;
                    const double den = 1.0 + u2;
                    // 1 / den: hardware reciprocal + two Newton steps (den in
                    // [1, inf): no scaling or special cases needed)
                    double d = __builtin_amdgcn_rcp(den);
                    d = fma(d, fma(-den, d, 1.0), d);
                    d = fma(d, fma(-den, d, 1.0), d);
                    const double ud = uu * d;
                    const double2 z1 = cmk(fma(y.x, d, -y.y * ud), fma(y.y, d, y.x * ud));
                    const double2 z2 = cmk(fma(z1.x, d, -z1.y * ud), fma(z1.y, d, z1.x * ud));
                    const double z3 = fma(z2.x, d, -z2.y * ud);
                    a0 += z1.x;
                    a1 = fma(kk, z1.y, a1);
                    a2 = fma(kk * kk, z1.x, a2);
                    q1 = fma(-uu, z2.y, q1);
                    q1p = fma(kk * uu, z2.x, q1p);
                    q2 = fma(-u2, z3, q2);
                    const double Pk = (in ? pv[u] : 0.0) * inv_e2;
                    s0 = fma(d, Pk, s0);
                    const double tp = u2 * d * d * Pk;
                    t1 += tp;
                    t2 = fma(tp * d, 1.0 - u2, t2);
                }
                E = cmul(E, W);
            }
        };
        ldg(kb0, xa, pa);
        // (no early exit: a trailing group may sum zeros, which keeps one
        // straight-line body and its load/wait schedule.  Whole iterations
        // below kb1 without the end-of-row selects, 8.6 % fewer VALU
        // instructions per harmonic, measured no faster: C3 1.315-1.375 vs
        // 1.353-1.399 ms, C5 2.47-2.48 vs 2.45-2.49 ms per launch in one call)
        for (int kb = kb0; kb < kb1; kb += 2 * KB) {
            ldg(kb + KB, xb, pb);
            sum_group(kb, xa, pa);
            ldg(kb + 2 * KB, xa, pa);
            sum_group(kb + KB, xb, pb);
        }
    }
    if (split) {
        // the four waves' partial sums of the same 64 channels, added in wave
        // order (fixed: bitwise reproducible)
        __shared__ double sp[kWaves - 1][9][64];
        if (wave > 0) {
            double *o = &sp[wave - 1][0][lane];
            o[0] = a0; o[64] = a1; o[128] = a2; o[192] = q1; o[256] = q1p;
            o[320] = q2; o[384] = s0; o[448] = t1; o[512] = t2;
        }
        __syncthreads();
        if (wave == 0) {
            for (int w = 0; w < kWaves - 1; ++w) {
                const double *o = &sp[w][0][lane];
                a0 += o[0]; a1 += o[64]; a2 += o[128]; q1 += o[192]; q1p += o[256];
                q2 += o[320]; s0 += o[384]; t1 += o[448]; t2 += o[512];
            }
        }
    }
    // (the 21 sums come to life only after the harmonic loop)
    double acc[21];
#pragma unroll
    for (int i = 0; i < 21; ++i) acc[i] = 0.0;
    if (use_n && (!split || wave == 0)) {
        double my[10];
        my[0] = a0; my[1] = -kTwoPi * a1; my[2] = -kTwoPi * kTwoPi * a2;
        if (SCAT) {
            my[3] = q1; my[4] = -kTwoPi * q1p; my[5] = q2;
            my[6] = s0; my[7] = -2.0 * t1; my[8] = 2.0 * t1; my[9] = -2.0 * t2;
        } else {
            my[3] = my[4] = my[5] = my[7] = my[8] = my[9] = 0.0;
            my[6] = chan[n * 4 + 3];
        }
        double *dst = stats + (int64_t)n * 10;
#pragma unroll
        for (int q = 0; q < 10; ++q) dst[q] = my[q];
        const double C = my[0], Sn = my[6], iS = 1.0 / Sn;
        if (!SCAT) {
            const double dph[3] = {1.0, kDconst * (pow(nu, -2.0) - nuDM2) / g.P,
                                   kDconst * kDconst * (pow(nu, -4.0) - nuGM4) / g.P};
            const double Cp = my[1], Cpp = my[2];
            const double hn = -2.0 * (C * Cpp + Cp * Cp) * iS;
            acc[0] = -C * C * iS;
            for (int i = 0; i < 3; ++i) {
                if (!(flagmask >> i & 1)) continue;
                acc[1 + i] = -2.0 * C * Cp * dph[i] * iS;
                for (int j = i; j < 3; ++j)
                    if (flagmask >> j & 1) acc[6 + uidx(i, j)] = hn * dph[i] * dph[j];
            }
        } else {
            Fac fc = make_fac(nu, g, alpha);
            double dC[5], dS[5], d2C[5][5], d2S[5][5];
            chan_derivs(my, fc, dC, dS, d2C, d2S);
            const double iS2 = iS * iS, iS3 = iS2 * iS, C2 = C * C;
            acc[0] = -C2 * iS;
            for (int i = 0; i < 5; ++i) {
                if (!(flagmask >> i & 1)) continue;
                acc[1 + i] = -(2.0 * C * dC[i] * iS - C2 * dS[i] * iS2);
                for (int j = i; j < 5; ++j)
                    if (flagmask >> j & 1)
                        acc[6 + uidx(i, j)] =
                            -2.0 * (C * d2C[i][j] * iS - 0.5 * C2 * d2S[i][j] * iS2 +
                                    dC[i] * dC[j] * iS + C2 * dS[i] * dS[j] * iS3 -
                                    C * (dC[i] * dS[j] + dS[i] * dC[j]) * iS2);
            }
        }
    }
    // fixed-order reduction: lanes (channel order) -> waves -> block partial
#pragma unroll
    for (int i = 0; i < 21; ++i) acc[i] = wave_sum(acc[i]);
    if (lane == 0)
        for (int i = 0; i < 21; ++i) red[wave * 21 + i] = acc[i];
    __syncthreads();
    if (threadIdx.x < 21) {
        double v = 0.0;
        for (int w = 0; w < kWaves; ++w) v += red[w * 21 + threadIdx.x];
        a.partials[((int64_t)s * nblk + blk) * 21 + threadIdx.x] = v;
    }
}

// ===========================================================================
// method='TNC' box bounds (pptoas.py:503-513, pptoaslib.py:1041-1053): the
// trust-region step projected onto the box.  Fitted parameters sitting at a
// bound whose descent direction (or CG step) leaves the box are held there;
// the CG-Steihaug step over the others is cut at the first bound it crosses.
// The fit then stops, as the unbounded one does, when no step predicts a
// decrease: at the bounded stationary point TNC converges to.
// ===========================================================================
template <int NF>
__device__ __forceinline__ void tr_box_step(const TRState &S, TRModel &m, const int (&idx)[5],
                                            double *p, double *pv, int *hbo) {
    // held: a bit per subspace parameter; its gradient entry and Hessian
    // row/column are replaced by (0, unit) in place, which leaves the model
    // value of a step that does not move it unchanged
    int held = 0;
#pragma unroll
    for (int q = 0; q < NF; ++q) {
        const double x = S.x[idx[q]];
        if ((x <= S.lo[idx[q]] && m.g[q] > 0.0) || (x >= S.hi[idx[q]] && m.g[q] < 0.0)) held |= 1 << q;
    }
    bool hb = false;
    for (int pass = 0; pass <= NF; ++pass) {
#pragma unroll
        for (int q = 0; q < NF; ++q) {
            if (!(held >> q & 1)) continue;
            m.g[q] = 0.0;
#pragma unroll
            for (int r = 0; r < NF; ++r) m.H[q][r] = m.H[r][q] = (q == r ? 1.0 : 0.0);
        }
        hb = cg_steihaug<NF>(m, sqrt(dotn<NF>(m.g, m.g)), S.radius, p);
        int more = 0;
#pragma unroll
        for (int q = 0; q < NF; ++q) {
            const double x = S.x[idx[q]];
            if (!(held >> q & 1) && ((x <= S.lo[idx[q]] && p[q] < 0.0) || (x >= S.hi[idx[q]] && p[q] > 0.0)))
                more |= 1 << q;
        }
        if (!more) break;
        held |= more;
    }
    double t = 1.0;
#pragma unroll
    for (int q = 0; q < NF; ++q) {
        if (held >> q & 1) p[q] = 0.0;
        const double x = S.x[idx[q]];
        if (p[q] < 0.0 && x + p[q] < S.lo[idx[q]]) t = fmin(t, (S.lo[idx[q]] - x) / p[q]);
        if (p[q] > 0.0 && x + p[q] > S.hi[idx[q]]) t = fmin(t, (S.hi[idx[q]] - x) / p[q]);
    }
#pragma unroll
    for (int q = 0; q < NF; ++q) p[q] *= t;
    *pv = model_value<NF>(m, p);
    *hbo = hb ? 1 : 0;
}

// ===========================================================================
// one iteration of scipy _minimize_trust_region (scipy/optimize/_trustregion.py)
// with CGSteihaugSubproblem (_trustregion_ncg.py): consume the evaluation o
// (f, g[5], H[15]) of S.th, accept/reject, then propose the next point.
// gtol = -1 (pptoaslib.py:1047-1048), eta 0.15, initial radius 1, max radius
// 1000, maxiter 200 * len(x0).  Returns 1 when a new proposal is pending.
// ===========================================================================
template <int NF, bool BOX>
__device__ int tr_update_t(TRState &S, const double *o, int max_iter, const int (&idx)[5]) {
    const int phase = S.phase;
    const int maxiter = max_iter > 0 ? max_iter : 200 * 5;
    TRModel m;
    bool done = false;
    int cmd = 0;
    if (phase == PH_INIT) {
        S.nfev = 1;
        S.f = o[0];
        for (int i = 0; i < 5; ++i) S.g[i] = o[1 + i];
        for (int i = 0; i < 15; ++i) S.H[i] = o[6 + i];
        if (!(o[0] == o[0])) { S.status = PPF_ST_NONFINITE; done = true; }
        S.macc = S.meval;
    } else {
        S.nfev += 1;
        const double fp = o[0];
        const double actual = S.f - fp, pred = S.f - S.pred;
        const double rho = actual / pred;
        if (rho < 0.25) S.radius *= 0.25;
        else if (rho > 0.75 && S.hb) S.radius = fmin(2.0 * S.radius, 1000.0);
        if (rho > 0.15) {
            for (int i = 0; i < 5; ++i) S.x[i] = S.th[i];
            S.f = fp;
            for (int i = 0; i < 5; ++i) S.g[i] = o[1 + i];
            for (int i = 0; i < 15; ++i) S.H[i] = o[6 + i];
            S.slot_cur = S.slot_eval;
            S.macc = S.meval;
        }
        S.k += 1;
        if (!(fp == fp)) { S.status = PPF_ST_NONFINITE; done = true; }
        if (S.k >= maxiter) { S.status = PPF_ST_MAXITER; done = true; }
    }
    if (!done) {
        m.f = S.f;
#pragma unroll
        for (int q = 0; q < NF; ++q) {
            m.g[q] = S.g[idx[q]];
#pragma unroll
            for (int r = 0; r < NF; ++r) {
                int i = min(idx[q], idx[r]), j = max(idx[q], idx[r]);
                m.H[q][r] = S.H[uidx(i, j)];
            }
        }
        double p[5], pv;
        bool hb;
        if (BOX && S.bnd) {
            int h;
            tr_box_step<NF>(S, m, idx, p, &pv, &h);
            hb = h != 0;
        } else {
            const double jm = sqrt(dotn<NF>(m.g, m.g));
            hb = cg_steihaug<NF>(m, jm, S.radius, p);
            pv = model_value<NF>(m, p);
        }
        if (m.f - pv <= 0.0) {
            done = true;                 // warnflag 2: no predicted improvement
        } else {
            for (int i = 0; i < 5; ++i) S.th[i] = S.x[i];
#pragma unroll
            for (int q = 0; q < NF; ++q) {
                const double v = S.x[idx[q]] + p[q];
                S.th[idx[q]] = (BOX && S.bnd) ? fmin(fmax(v, S.lo[idx[q]]), S.hi[idx[q]]) : v;
            }
            S.pred = pv;
            S.hb = hb ? 1 : 0;
            S.slot_eval = S.slot_cur ^ 1;
            cmd = 1;
        }
    }
    S.phase = done ? PH_DONE : PH_PROPOSAL;
    return cmd;
}
// ===========================================================================
// Newton trust region (the default for scattering fits; PPF_OPT_SCIPY_TR
// selects the scipy replica above).  It minimises the same objective
// (pptoaslib.py:564-684) to the same stationary point, in fewer evaluations,
// each of which is a pass over the cross spectrum:
//   - the step is taken in Jacobi-scaled coordinates z_i = sqrt|H_ii| x_i,
//     where a unit step moves the objective by O(1) (about 1 sigma) in every
//     parameter: scipy's radius is in raw units (rotations, pc cm^-3, log10 s)
//     and its CG-Steihaug solve stops at the loose tolerance
//     min(0.5, sqrt|g|) |g|, so on these badly conditioned 5-parameter
//     problems it alternates short boundary and inexact-Newton steps
//     (27-52 evaluations against 7-22 here, tools/tr_probe.py);
//   - the subproblem is solved exactly (tr_exact: eigendecomposition and the
//     secular equation), so an interior step is the full Newton step;
//   - radius: initial kNewtonR0, x4 on a boundary step with rho > 0.75,
//     0.25 |p| when rho < 0.25, accept when rho > 0.15 (scipy's eta);
//   - stop when the step's predicted reduction is <= kNewtonTol: the point is
//     then within ~sqrt(kNewtonTol) sigma of the stationary point, where the
//     reference's own trust-ncg ends at its rounding floor (~5e-5 sigma).
// ===========================================================================
template <int NF>
__device__ int tr_update_newton(TRState &S, const double *o, int max_iter, const int (&idx)[5]) {
    const int maxiter = max_iter > 0 ? max_iter : 200 * 5;
    bool done = false;
    int cmd = 0;
    if (S.sub > 1) S.nsubev += 1;        // o is a channel-subset evaluation
    if (S.phase == PH_INIT || S.phase == PH_RESTART) {
        // first evaluation, or the point x evaluated again on every channel
        S.nfev = S.phase == PH_INIT ? 1 : S.nfev + 1;
        S.f = o[0];
        for (int i = 0; i < 5; ++i) S.g[i] = o[1 + i];
        for (int i = 0; i < 15; ++i) S.H[i] = o[6 + i];
        if (!(o[0] == o[0])) { S.status = PPF_ST_NONFINITE; done = true; }
        S.slot_cur = S.slot_eval;
        S.macc = S.meval;
    } else {
        S.nfev += 1;
        const double fp = o[0];
        const double rho = (S.f - fp) / S.pred;      // S.pred: predicted reduction
        if (rho < 0.25) S.radius = 0.25 * S.pnorm;
        else if (rho > 0.75 && S.hb) S.radius = fmin(4.0 * S.radius, 1e6);
        if (rho > 0.15) {
            for (int i = 0; i < 5; ++i) S.x[i] = S.th[i];
            S.f = fp;
            for (int i = 0; i < 5; ++i) S.g[i] = o[1 + i];
            for (int i = 0; i < 15; ++i) S.H[i] = o[6 + i];
            S.slot_cur = S.slot_eval;
            S.macc = S.meval;
        }
        S.k += 1;
        if (!(fp == fp)) { S.status = PPF_ST_NONFINITE; done = true; }
        if (S.k >= maxiter) { S.status = PPF_ST_MAXITER; done = true; }
    }
    if (!done) {
        double g[5], H[5][5], d[5], p[5];
#pragma unroll
        for (int q = 0; q < NF; ++q) d[q] = sqrt(fmax(fabs(S.H[uidx(idx[q], idx[q])]), 1e-300));
#pragma unroll
        for (int q = 0; q < NF; ++q) {
            g[q] = S.g[idx[q]] / d[q];
#pragma unroll
            for (int r = 0; r < NF; ++r) {
                const int i = min(idx[q], idx[r]), j = max(idx[q], idx[r]);
                H[q][r] = S.H[uidx(i, j)] / (d[q] * d[r]);
            }
        }
        const bool hb = tr_exact<NF>(H, g, S.radius, p);
        double gp = 0.0, pHp = 0.0, pn = 0.0;
#pragma unroll
        for (int q = 0; q < NF; ++q) {
            double s = 0.0;
#pragma unroll
            for (int r = 0; r < NF; ++r) s += H[q][r] * p[r];
            gp += g[q] * p[q];
            pHp += p[q] * s;
            pn += p[q] * p[q];
        }
        const double pred = -(gp + 0.5 * pHp);
        if (S.sub > 1 && !hb && pred < kSubsetSwitch) {
            done = true;                 // the subset's basin is found: switch below
        } else if (!(pred > kNewtonTol)) {
            done = true;                 // converged (scipy's warnflag 2 status)
        } else {
            for (int i = 0; i < 5; ++i) S.th[i] = S.x[i];
#pragma unroll
            for (int q = 0; q < NF; ++q) S.th[idx[q]] = S.x[idx[q]] + p[q] / d[q];
            S.pred = pred;
            S.pnorm = sqrt(pn);
            S.hb = hb ? 1 : 0;
            S.slot_eval = S.slot_cur ^ 1;
            cmd = 1;
        }
    }
    if (done && S.sub > 1 && S.status != PPF_ST_NONFINITE) {
        // leave the channel subset: evaluate x on every channel and go on
        // from there (a fit never ends on a subset evaluation, so k_postfit
        // always reads complete per-channel terms)
        S.sub = 1;
        for (int i = 0; i < 5; ++i) S.th[i] = S.x[i];
        S.slot_eval = S.slot_cur ^ 1;
        S.phase = PH_RESTART;
        return 1;
    }
    S.phase = done ? PH_DONE : PH_PROPOSAL;
    return cmd;
}

template <int MAXNF = 5>
__device__ int tr_update_newton_n(TRState &S, const double *o, int max_iter) {
    int idx[5] = {0, 0, 0, 0, 0}, nf = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i)
        if (S.flagmask >> i & 1) idx[nf++] = i;
    switch (nf) {
        case 1: return tr_update_newton<1>(S, o, max_iter, idx);
        case 2: return tr_update_newton<2>(S, o, max_iter, idx);
        default:
            if constexpr (MAXNF <= 3) return tr_update_newton<3>(S, o, max_iter, idx);
            else {
                if (nf == 3) return tr_update_newton<3>(S, o, max_iter, idx);
                if (nf == 4) return tr_update_newton<4>(S, o, max_iter, idx);
                return tr_update_newton<5>(S, o, max_iter, idx);
            }
    }
}

// MAXNF: the largest subspace the caller can meet (3 for the moment path,
// which never fits tau/alpha; instantiating only those keeps its registers
// down).  BOX: the instantiation also handles method='TNC' bounds.
template <int MAXNF = 5, bool BOX = true>
__device__ int tr_update(TRState &S, const double *o, int max_iter) {
    const int flagmask = S.flagmask;
    int idx[5] = {0, 0, 0, 0, 0}, nf = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i)
        if (flagmask >> i & 1) idx[nf++] = i;
    switch (nf) {
        case 1: return tr_update_t<1, BOX>(S, o, max_iter, idx);
        case 2: return tr_update_t<2, BOX>(S, o, max_iter, idx);
        default:
            if constexpr (MAXNF <= 3) return tr_update_t<3, BOX>(S, o, max_iter, idx);
            else {
                if (nf == 3) return tr_update_t<3, BOX>(S, o, max_iter, idx);
                if (nf == 4) return tr_update_t<4, BOX>(S, o, max_iter, idx);
                return tr_update_t<5, BOX>(S, o, max_iter, idx);
            }
    }
}

// ===========================================================================
// k_tr_step: one wave per sub-integration; scipy _minimize_trust_region
// (scipy/optimize/_trustregion.py) with CGSteihaugSubproblem
// (_trustregion_ncg.py), gtol = -1 (pptoaslib.py:1047-1048), eta 0.15,
// initial radius 1, max radius 1000, maxiter 200 * len(x0).
// ===========================================================================
// BOX: the bounded (method='TNC') instantiation, launched only when the call
// has bounds, so the unbounded one keeps its 3 waves per SIMD
template <bool BOX>
__global__ __launch_bounds__(kBlock) void k_tr_step(SolveArgs a) {
    __shared__ double thb[kWaves][8];
    // the trust-region update runs on lane 0 against an LDS copy of the
    // sub-int's state: on the global TRState every one of its serial field
    // accesses was a dependent L2 round trip (~170 us per launch at C5)
    __shared__ TRState Ls[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int s = blockIdx.x * kWaves + wave;
    if (s >= a.nsub) return;
    TRState &G = a.state[s];
    const int phase = G.phase;
    if (phase == PH_DONE || G.mmode) return;
    static_assert(sizeof(TRState) % 8 == 0, "TRState copy");
    constexpr int NW = (int)(sizeof(TRState) / 8);
    TRState &S = Ls[wave];
    for (int i = lane; i < NW; i += 64)
        reinterpret_cast<double *>(&S)[i] = reinterpret_cast<const double *>(&G)[i];
    const int nblk = (a.nchan + kPassChans - 1) / kPassChans;
    double o[21];
#pragma unroll
    for (int i = 0; i < 21; ++i) o[i] = 0.0;
    for (int b = lane; b < nblk; b += 64) {
        const double *p = a.partials + ((int64_t)s * nblk + b) * 21;
#pragma unroll
        for (int i = 0; i < 21; ++i) o[i] += p[i];
    }
#pragma unroll
    for (int i = 0; i < 21; ++i) o[i] = wave_sum(o[i]);
    wave_lds_sync();                                   // every lane's copy of the state has landed
    int cmd = 0;
    if (lane == 0) {
        cmd = S.newton ? tr_update_newton_n<5>(S, o, a.max_iter) : tr_update<5, BOX>(S, o, a.max_iter);
        for (int i = 0; i < 5; ++i) thb[wave][i] = S.th[i];
        thb[wave][5] = (double)cmd;
    }
    cmd = __shfl(cmd, 0, 64);
    if (cmd) {
        if (lane == 0) atomicAdd(a.active, 1u);
        if (S.scat) {
            // reference gates at the proposal (taus.sum(), dtau.sum(), dalpha.sum())
            const double t3 = __shfl(lane == 0 ? S.th[3] : 0.0, 0, 64);
            const double t4 = __shfl(lane == 0 ? S.th[4] : 0.0, 0, 64);
            const double tl = a.log10_tau ? pow(10.0, t3) : t3;
            int gs, gt, ga;
            wave_gates(a.dphi + (int64_t)s * a.nchan * 2, a.mask ? a.mask + (int64_t)s * a.nchan : nullptr,
                       a.nchan, tl, t4, a.log10_tau, gs, gt, ga);
            if (lane == 0) { S.g_sum = gs; S.g_tau = gt; S.g_alpha = ga; }
        }
    }
    wave_lds_sync();                                   // lane 0's updates are visible to the wave
    for (int i = lane; i < NW; i += 64)
        reinterpret_cast<double *>(&G)[i] = reinterpret_cast<const double *>(&S)[i];
}

// The sum k_tr_step forms from nblk block partials p[b * stride], in ONE
// lane: lane b of its wave adds blocks b, b + 64, ... in order, and wave_sum
// adds the 64 lane values as a balanced pairwise tree (DPP xor 1, xor 2,
// half-row and row mirrors, then rows (r0 + r1) + (r2 + r3); IEEE addition
// commutes, so each node is left + right).  Lanes past nblk hold 0 and an
// all-zero subtree passes its sibling through unchanged, so the tree over
// the first L = 2^ceil(log2 min(nblk, 64)) leaves gives the same bits.  A
// binary-counter stack builds exactly that tree.
__device__ __forceinline__ double tree_sum64(const double *p, int nblk, int stride) {
    const int nl = nblk < 64 ? nblk : 64;
    int L = 1;
    while (L < nl) L <<= 1;
    double st[7];
    for (int b = 0; b < L; ++b) {
        double v = 0.0;
        for (int j = b; j < nblk; j += 64) v += p[(int64_t)j * stride];
        int lvl = 0;
        for (; (b >> lvl) & 1; ++lvl) v = st[lvl] + v;
        st[lvl] = v;
    }
    int top = 0;
    while ((1 << top) < L) ++top;
    return st[top];
}

// k_tr_step_l: the same update with one LANE per sub-int (64 sub-ints per
// single-wave workgroup, their states in LDS): the serial trust-region update
// (eigen / secular-equation subproblem, a few thousand dependent f64
// operations) of 64 sub-ints runs in one wave's lanes instead of one lane of
// 64 waves.  The block partials are summed in k_tr_step's order
// (tree_sum64), so a sub-int's fit does not depend on which of the two
// kernels its batch size selects.  The scattering gates at the
// new proposal need a pass over the channels: k_tr_gates, a wave per flagged
// sub-int, follows.  It pays where there are many narrow sub-ints (C3, 10k
// x 512 channels: 68.4-70.2 vs 71.3-71.7 ms per step) and not for a few wide
// ones (C5, 500 x 16384: 87.5-88.2 vs 83.6-85.3 ms; 8 waves on the chip and
// 64 block partials per lane), tools/g33.sh.  PPF_TRSTEP_LANE: 1 = by shape
// (nsub >= 2048 and nchan <= 2048; default), 2 = always (the whole GPU suite
// passed so), 0 = never.
#ifndef PPF_TRSTEP_LANE
#define PPF_TRSTEP_LANE 1
#endif
template <bool BOX>
__global__ __launch_bounds__(64) void k_tr_step_l(SolveArgs a) {
    extern __shared__ __attribute__((aligned(16))) double tsl[];
    TRState *Ls = reinterpret_cast<TRState *>(tsl);
    constexpr int NW = (int)(sizeof(TRState) / 8);
    const int lane = threadIdx.x;
    const int n0 = blockIdx.x * 64, cnt = min(64, a.nsub - n0);
    if (cnt <= 0) return;
    const double *gsrc = reinterpret_cast<const double *>(a.state + n0);
    for (int i = lane; i < cnt * NW; i += 64) tsl[i] = gsrc[i];
    __syncthreads();
    const int s = n0 + lane;
    TRState &S = Ls[lane < cnt ? lane : 0];
    const bool act = lane < cnt && S.phase != PH_DONE && !S.mmode;
    if (act) {
        const int nblk = (a.nchan + kPassChans - 1) / kPassChans;
        const double *ps = a.partials + (int64_t)s * nblk * 21;
        double o[21];
        for (int i = 0; i < 21; ++i) o[i] = tree_sum64(ps + i, nblk, 21);
        const int cmd = S.newton ? tr_update_newton_n<5>(S, o, a.max_iter) : tr_update<5, BOX>(S, o, a.max_iter);
        S.step_cmd = cmd;
        if (cmd) atomicAdd(a.active, 1u);
    } else if (lane < cnt) {
        S.step_cmd = 0;
    }
    __syncthreads();
    double *gdst = reinterpret_cast<double *>(a.state + n0);
    for (int i = lane; i < cnt * NW; i += 64) gdst[i] = tsl[i];
}

// the reference gates (taus.sum(), dtau.sum(), dalpha.sum()) at the proposal
// of every scattering sub-int whose k_tr_step_l update asked for a pass
__global__ __launch_bounds__(kBlock) void k_tr_gates(SolveArgs a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int s = blockIdx.x * kWaves + wave;
    if (s >= a.nsub) return;
    TRState &G = a.state[s];
    if (!G.step_cmd || !G.scat || G.mmode) return;
    const double t3 = G.th[3], t4 = G.th[4];
    const double tl = a.log10_tau ? pow(10.0, t3) : t3;
    int gs, gt, ga;
    wave_gates(a.dphi + (int64_t)s * a.nchan * 2, a.mask ? a.mask + (int64_t)s * a.nchan : nullptr,
               a.nchan, tl, t4, a.log10_tau, gs, gt, ga);
    if (lane == 0) { G.g_sum = gs; G.g_tau = gt; G.g_alpha = ga; }
}

// ===========================================================================
// Moment-expansion evaluation (fits without scattering).
//
// With tau = 0 every channel enters only through its phase phi_n(theta) =
// phi + DM dphi1_n + GM dphi2_n, and C_n(phi_n) = Re sum_k X_nk e^{2 pi i k
// phi_n}.  Around a centre phi_c (Y_k = X_k e^{2 pi i k phi_c}), with h = N/2,
// u_k = (k - h)/h in [-1, 1] and x = 2 pi h Delta:
//   sum_k Y_k e^{2 pi i k Delta} = e^{i x} sum_m (i x)^m / m! mu_m,
//   mu_m = sum_k Y_k u_k^m,  and k = h (1 + u) gives the k- and k^2-weighted
// sums (C', C'') from mu_m + mu_{m+1} and mu_m + 2 mu_{m+1} + mu_{m+2}.
// kMoments = 32 moments and |x| <= 4.5 bound the truncation of the
// second-derivative series by 4.5^30 / 30! < 1.6e-13 of sum_k |Y_k| (the
// largest term x^m / m! is 17, so rounding adds < 4e-15), so every
// trust-region evaluation inside that radius costs O(nchan) instead of a pass
// over the cross spectrum; a point outside it re-centres (k_moments /
// k_xmom_g).  (3.2 until round 2: 5e-18, but ppalign fits against a sharp
// template then re-centred 3.2 times per fit instead of 2.3.)
// Delta_n includes the per-channel centre residual mres (k_xmom_g rounds the
// centre to a whole bin, |residual| <= 1/(2 nbin), i.e. |x| <= pi/4).
// ===========================================================================
constexpr double kXMax = 4.5;
// Below |x| = 2.3 the first 24 moments hold the same bound (2.3^22 / 22! <
// 1.6e-13): the evaluation then skips the last quarter of the moments.
constexpr double kX24 = 2.3;
// 16 moments (mom16): x^14 / 14! < 1.6e-13 for |x| <= 0.73, with x = 2 pi h_n
// Delta and h_n the centre of the channel band's harmonics (k_moments)
constexpr double kX16 = 0.73;
// fewer of the 16 (k_tr_mom, PPF_TRMOM_ADAPT): x^10 / 10! and x^6 / 6! <
// 1.6e-13 for |x| <= 0.2368 (12 moments) and 0.0220 (8)
constexpr double kX12 = 0.2368;
constexpr double kX8 = 0.0220;
#ifndef PPF_TRMOM_ADAPT
#define PPF_TRMOM_ADAPT 1
#endif
constexpr int kMomChans = 64;                    // channels per k_moments workgroup
typedef double f64x4 __attribute__((ext_vector_type(4)));

// k_moments: mu[s][q][n][m] for the sub-ints that asked for a (re)centre.
// MFMA f64 16x16x4: A = Y (16 channels x 4 harmonics; one wave = 16
// channels), B = u^m (4 harmonics x 16 moments), two B tiles (m < 16, m >=
// 16) and separate real / imaginary A.  The harmonic sum is the MFMA K loop.
#ifndef PPF_MOM_WPE
#define PPF_MOM_WPE 3
#endif
// (measured, C2 per 10k sub-ints, same call: KU = 8 6.12 vs 5.76 ms; the
// loop unrolled by two over two buffers, so that no batch waits for loads it
// has just issued, 5.77 at KU = 4 and 5.91 at KU = 2: no latency to hide.
// Round 5, with the loads unconditional: KU = 2 / 8 5.61-5.77 / 5.70-5.97
// vs 5.68-5.83 ms; the first two batches requested before the dphi / cutoff
// loads, 5.83-5.85 vs 5.61-5.65 ms, and with the mask / dphi / cutoff loads
// issued together before them (one round trip), 5.56-5.58 vs 5.54-5.55 ms:
// not kept.  The same one-round-trip prologue for k_pass, and unconditional
// loads in the scattering-gate and k_tr_init channel loops, measured within
// the noise at C3 / C5 (profiles/r05/ab_ps1_status.txt, ab_gt1_status.txt))
#ifndef PPF_MOM_KU
#define PPF_MOM_KU 4
#endif
// PPF_MOM_ILP (round 6, measured and not kept): the batch's phasors from
// its base phasor and two accumulator pairs -- k_moments 5.83 vs 5.72-5.76
// ms per 10k at C2 (profiles/r06/ab_r6a_status.txt): the kernel is not
// bound by its dependency chains, and the 164 VGPRs cost a wave per SIMD
#ifndef PPF_MOM_ILP
#define PPF_MOM_ILP 0
#endif
// M16: the call's moment count (a.mom16: 16 on the moments-from-X path, 32
// otherwise), a template argument so the MFMA loop carries no branch
template <bool M16>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PPF_MOM_WPE))) void k_moments(SolveArgs a) {
    const int nblk = (a.nchan + kMomChans - 1) / kMomChans;
    const int s = blockIdx.x / nblk, blk = blockIdx.x % nblk;
    const TRState &S = a.state[s];
    if (!S.mmode || !S.need_mom) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = S.mtarget;
    const double c0 = S.mc[q][0], c1 = S.mc[q][1], c2 = S.mc[q][2];
    const int nharm = (a.nbin >> 1) + 1;
    const double h = 0.5 * (double)(nharm - 1);
    const int ci = lane & 15, kk = lane >> 4;
    const int nbase = blk * kMomChans + wave * 16;
    const int n = nbase + ci;
    const bool valid = n < a.nchan && (!a.mask || a.mask[(int64_t)s * a.nchan + n]);
    double phin = 0.0;
    if (valid) {
        const double *dp = a.dphi + ((int64_t)s * a.nchan + n) * 2;
        phin = c0 + c1 * dp[0] + c2 * dp[1];
        if (kk == 0) a.mres[((int64_t)s * 2 + q) * a.nchan + n] = 0.0;   // exact centre
    }
    const double2 *Xr = a.X + (int64_t)(a.xslot ? a.xslot[s] : s) * nharm * a.nchan +
                         (valid ? n : 0);   // X[slot][k][n]
    // harmonic cutoff of the wave's 16 channels (k_model_cut; they lie in one
    // aligned 64-channel group): X past it carries |M_k| < 1e-14 of the
    // channel's peak, and k_xspec_w writes X only below the group's largest
    // cutoff
    int kend = nharm;
    if (a.KC) {
        const int mi = a.model_index ? a.model_index[s] : 0;
        const int nn = min(n, a.nchan - 1);
        kend = (int)wave_max((double)a.KC[(int64_t)mi * a.nchan + nn]);
    }
    // mom16: 16 moments in u = (k - hw) / hw, hw = kend / 2 the centre of
    // the band the wave sums (|u| <= 1 there), one B tile; h_n recorded
    // for k_tr_mom
    constexpr bool m16 = M16;
    const double hw = m16 ? 0.5 * (double)(kend > 2 ? kend : 2) : h, ihw = 1.0 / hw;
    if (m16 && valid && kk == 0) a.hcen[((int64_t)s * 2 + q) * a.nchan + n] = hw;
    const double2 W4 = cexp2pi(4.0 * phin);
    f64x4 dre0 = {0.0, 0.0, 0.0, 0.0}, dre1 = dre0, dim0 = dre0, dim1 = dre0;
    double2 E = cmk(1.0, 0.0);
    // batches of 4 K-steps (16 harmonics), software-pipelined: the next
    // batch's loads are in flight while this one's MFMAs run
    constexpr int KU = PPF_MOM_KU;
#if PPF_MOM_ILP
    // Round 6: no serial chains through a batch.  The K-step phasors are
    // Eb W4^t from the batch's base phasor Eb (one product each, all
    // independent; Eb itself advances by W4^KU once per batch), and the
    // m < 16 contraction runs on two accumulator pairs (even / odd K-steps,
    // summed at the end), so consecutive MFMAs do not wait for each other:
    // the kernel waited on instruction dependencies 63 % of its wave cycles
    // (profiles/r05/sq_c2_r5a.txt) at half the HBM rate
    double2 Wt[KU];
    Wt[0] = cmk(1.0, 0.0);
#pragma unroll
    for (int t = 1; t < KU; ++t) Wt[t] = cmul(Wt[t - 1], W4);
    const double2 WB = cmul(Wt[KU - 1], W4);
    f64x4 dre0b = dre0, dim0b = dre0;
#endif
    double2 xa[KU], xb[KU];
    // The loads are unconditional (clamped to a valid harmonic; values past
    // the cutoff or of a masked channel are replaced by 0 after the load):
    // under a lane-divergent branch the compiler cannot count the loads in
    // flight and waited for all of them (vmcnt(0)) -- the next batch's
    // included -- before every batch's MFMAs, so nothing was pipelined.
    auto ld = [&](double2 (&xv)[KU], int kb) {
#pragma unroll
        for (int t = 0; t < KU; ++t) {
            const int k = kb + 4 * t + kk;
            // (past the end: the last needed harmonic again, an L2 hit)
            const int kc = k < kend ? k : kend - 1;
            xv[t] = ld_stream(Xr + (int64_t)kc * a.nchan);
        }
    };
    auto keep = [&](int k) { return valid && k < kend; };
    auto mm = [&](const double2 (&xv)[KU], int kb) {
#if PPF_MOM_ILP
        // base phasor of the batch (k = kb + kk), re-seeded exactly every
        // 64 harmonics (kb is a multiple of 4 KU)
        if ((kb & 63) == 0) E = cexp2pi((double)(kb + kk) * phin);
        else E = cmul(E, WB);
#endif
#pragma unroll
        for (int t = 0; t < KU; ++t) {
            const int k = kb + 4 * t + kk;
#if PPF_MOM_ILP
            const double2 Et = t == 0 ? E : cmul(E, Wt[t]);
#else
            // phasor by recurrence, re-seeded exactly every 64 harmonics
            // (kb is a multiple of 16: only t = 0 can re-seed)
            if (t == 0 && (kb & 63) == 0) E = cexp2pi((double)k * phin);
            else E = cmul(E, W4);
            const double2 Et = E;
#endif
            const double2 xk = keep(k) ? xv[t] : cmk(0.0, 0.0);
            const double2 y = cmul(xk, Et);
            const double u = ((double)k - hw) * ihw;
            const double u2 = u * u, u4 = u2 * u2, u8 = u4 * u4, u16 = u8 * u8;
            const double uj = ((ci & 1) ? u : 1.0) * ((ci & 2) ? u2 : 1.0) *
                              ((ci & 4) ? u4 : 1.0) * ((ci & 8) ? u8 : 1.0);
#if PPF_MOM_ILP
            // (32 moments: dre1 / dim1 already make four chains)
            if (m16 && (t & 1)) {
                dre0b = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, uj, dre0b, 0, 0, 0);
                dim0b = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, uj, dim0b, 0, 0, 0);
            } else
#endif
            {
                dre0 = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, uj, dre0, 0, 0, 0);
                dim0 = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, uj, dim0, 0, 0, 0);
            }
            if constexpr (!m16) {
                const double ujh = uj * u16;
                dre1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, ujh, dre1, 0, 0, 0);
                dim1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, ujh, dim1, 0, 0, 0);
            }
        }
    };
    // two batches in flight, the buffers alternating (no register copy, so
    // no wait for the batch just issued)
    ld(xa, 0);
    ld(xb, 4 * KU);
    for (int kb = 0; kb < kend; kb += 8 * KU) {
        mm(xa, kb);
        ld(xa, kb + 8 * KU);
        if (kb + 4 * KU < kend) mm(xb, kb + 4 * KU);    // (uniform)
        ld(xb, kb + 12 * KU);
    }
#if PPF_MOM_ILP
    if constexpr (m16) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            dre0[r] += dre0b[r];
            dim0[r] += dim0b[r];
        }
    }
#endif
    // D[row][col]: col = lane & 15 = moment, row = (lane >> 4) + 4 r = channel
    double2 *M = a.mom + ((int64_t)s * 2 + q) * a.nchan * kMoments;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int ch = nbase + kk + 4 * r;
        if (ch < a.nchan) {
            M[(int64_t)ch * kMoments + ci] = cmk(dre0[r], dim0[r]);
            if constexpr (!m16) M[(int64_t)ch * kMoments + 16 + ci] = cmk(dre1[r], dim1[r]);
        }
    }
}

// rotate by i^P (compile time) and scale: r * i^P * z
template <int P>
__device__ __forceinline__ double2 rot_scale(double2 z, double r) {
    if constexpr ((P & 3) == 0) return cmk(r * z.x, r * z.y);
    else if constexpr ((P & 3) == 1) return cmk(-r * z.y, r * z.x);
    else if constexpr ((P & 3) == 2) return cmk(-r * z.x, -r * z.y);
    else return cmk(r * z.y, -r * z.x);
}
// G_j += i^(m-j) x^(m-j)/(m-j)! mu_m for j = 0, 1, 2; r0, r1, r2 hold
// x^m/m!, x^(m-1)/(m-1)!, x^(m-2)/(m-2)! (sliding window, no array)
template <int M>
__device__ __forceinline__ void taylor_acc(const double2 *mu, double x, double r0, double r1,
                                           double r2, double2 &G0, double2 &G1, double2 &G2) {
    if constexpr (M < kMoments) {
        const double2 v = mu[M];
        G0 = cadd(G0, rot_scale<M>(v, r0));
        if constexpr (M >= 1) G1 = cadd(G1, rot_scale<M - 1>(v, r1));
        if constexpr (M >= 2) G2 = cadd(G2, rot_scale<M - 2>(v, r2));
        taylor_acc<M + 1>(mu, x, r0 * x * (1.0 / (double)(M + 1)), r0, r1, G0, G1, G2);
    }
}

// moments [M, M1) from registers (mu[m - M0], SZ >= M1 - M0); the window
// r0..r2 and the partial sums carry over between segments
template <int M, int M1, int M0, int SZ>
__device__ __forceinline__ void taylor_seg(const double2 (&mu)[SZ], double x, double &r0,
                                           double &r1, double &r2, double2 &G0, double2 &G1,
                                           double2 &G2) {
    if constexpr (M < M1) {
        const double2 v = mu[M - M0];
        G0 = cadd(G0, rot_scale<M>(v, r0));
        if constexpr (M >= 1) G1 = cadd(G1, rot_scale<M - 1>(v, r1));
        if constexpr (M >= 2) G2 = cadd(G2, rot_scale<M - 2>(v, r2));
        r2 = r1;
        r1 = r0;
        r0 = r0 * x * (1.0 / (double)(M + 1));
        taylor_seg<M + 1, M1, M0, SZ>(mu, x, r0, r1, r2, G0, G1, G2);
    }
}

#ifndef PPF_TRMOM_WPE
#define PPF_TRMOM_WPE 2
#endif
#ifdef PPF_TM_PROF
// section cycle counters of k_tr_mom, thread 0 of each workgroup (profiling
// builds only: tools/tprof.py)
__device__ unsigned long long g_tprof[8];
#define TP_INIT() unsigned long long tp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long tp_t = __builtin_amdgcn_s_memtime()
#define TP(i) do { const unsigned long long tp_n = __builtin_amdgcn_s_memtime(); tp_acc[i] += tp_n - tp_t; tp_t = tp_n; } while (0)
#define TP_DONE() do { if (tid == 0) for (int ti = 0; ti < 8; ++ti) atomicAdd(&g_tprof[ti], tp_acc[ti]); } while (0)
#else
#define TP_INIT()
#define TP(i)
#define TP_DONE()
#endif
// k_tr_mom: one workgroup per moment-mode sub-integration; runs trust-region
// iterations back to back, every evaluation from the moments, until the fit
// stops or a point leaves the expansion radius of both moment sets (then it
// asks for a new centre and exits).  Thread t owns channels t + 256 j; each
// evaluation is one pass over them (moments of the next channel half in
// flight while the current half is summed), a fixed-order block reduction
// of f, g, H and the scipy trust-ncg update on thread 0.
template <int TB>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(PPF_TRMOM_WPE))) void k_tr_mom(SolveArgs a) {
    __shared__ TRState L;
    __shared__ double red[kWaves * 10];
    __shared__ int cmdb;
    const int tid = threadIdx.x;
    const int s = blockIdx.x;
    if (s >= a.nsub) return;
    TRState &G = a.state[s];
    if (!G.mmode || G.phase == PH_DONE) return;          // uniform per workgroup
    TP_INIT();
    static_assert(sizeof(TRState) % 8 == 0, "TRState copy");
    constexpr int NW = (int)(sizeof(TRState) / 8);
    for (int i = tid; i < NW; i += TB)
        reinterpret_cast<double *>(&L)[i] = reinterpret_cast<const double *>(&G)[i];
    __syncthreads();
    const int nharm = (a.nbin >> 1) + 1;
    const double h = 0.5 * (double)(nharm - 1);
    const double *dp = a.dphi + (int64_t)s * a.nchan * 2;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    // mask bytes are loaded unconditionally (no per-channel branch between
    // the loads): without a mask from any valid address and ignored
    const bool use_mask = mask != nullptr;
    const uint8_t *mk = use_mask ? mask : reinterpret_cast<const uint8_t *>(a.dphi);
    const double *chan = a.chan + (int64_t)s * a.nchan * 4;
    const double2 *MOM = a.mom + (int64_t)s * 2 * a.nchan * kMoments;
    const double *MRES = a.mres + (int64_t)s * 2 * a.nchan;
    // mom16: per-channel expansion centres h_n and 16 moments (radius kX16)
    const bool m16 = L.mom16 != 0;
    const double *HC = m16 ? a.hcen + (int64_t)s * 2 * a.nchan : MRES;
    const double xmax = m16 ? kX16 : kXMax;
    double *stats = a.stats + (int64_t)s * 2 * a.nchan * 10;
    const int flagmask = L.flagmask;
    const int nit = (a.nchan + TB - 1) / TB;
    __syncthreads();
    if (tid == 0) L.need_mom = 0;
    const int cap = (a.max_iter > 0 ? a.max_iter : 1000) + 4;
    TP(0);
    for (int it = 0; it < cap; ++it) {
        __syncthreads();
        const double t0 = L.th[0], t1 = L.th[1], t2 = L.th[2];
        // moment set whose centre is within the expansion radius for every channel
        int qsel = -1;
        double xsel = 0.0;
        for (int t = 0; t < 2 && qsel < 0; ++t) {
            const int cand = t == 0 ? L.macc : 1 - L.macc;
            if (!L.mvalid[cand]) continue;
            const double e0 = t0 - L.mc[cand][0], e1 = t1 - L.mc[cand][1], e2 = t2 - L.mc[cand][2];
            const double *rc = MRES + (int64_t)cand * a.nchan;
            const double *hc = HC + (int64_t)cand * a.nchan;
            double xm[1] = {0.0};          // max_n h_n |Delta_n|
            for (int n0 = 0; n0 < a.nchan; n0 += 4 * TB) {   // 4 channels' loads, then use
                double v1[4], v2[4], vr[4], vh[4];
                bool ok[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int n = n0 + tid + TB * j, nc = min(n, a.nchan - 1);
                    v1[j] = dp[2 * nc]; v2[j] = dp[2 * nc + 1]; vr[j] = rc[nc];
                    vh[j] = m16 ? hc[nc] : h;
                    ok[j] = n < a.nchan && (!use_mask || mk[nc] != 0);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (ok[j]) xm[0] = fmax(xm[0], vh[j] * fabs(e0 + e1 * v1[j] + e2 * v2[j] + vr[j]));
            }
            blk_max<1, TB>(xm, red);
            if (kTwoPi * xm[0] <= xmax) {
                qsel = cand;
                xsel = kTwoPi * xm[0];
            }
        }
        TP(1);
        if (qsel < 0) {
            if (tid == 0) {
                const int tgt = L.mvalid[L.macc] ? 1 - L.macc : L.macc;
                L.mtarget = tgt;
                L.mc[tgt][0] = t0; L.mc[tgt][1] = t1; L.mc[tgt][2] = t2;
                L.mvalid[tgt] = 1;
                L.need_mom = 1;
                L.nmom += 1;
                atomicAdd(a.active, 1u);
                if (a.rc_list) a.rc_list[atomicAdd(a.rc_count, 1u)] = s;
            }
            break;
        }
        const double e0 = t0 - L.mc[qsel][0], e1 = t1 - L.mc[qsel][1], e2 = t2 - L.mc[qsel][2];
        const double2 *Mq = MOM + (int64_t)qsel * a.nchan * kMoments;
        const double *rq = MRES + (int64_t)qsel * a.nchan;
        const double *hq = HC + (int64_t)qsel * a.nchan;
        double *st = stats + (int64_t)L.slot_eval * a.nchan * 10;
        double acc[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) acc[i] = 0.0;
        // channel n = tid + 256 i; its 32 moments come in quarters of 8
        // (8 x 16 B loads), two buffers rotating so that the next quarter is
        // in flight while the current one is summed
        constexpr int KQ = kMoments / 4;
        double2 qa[KQ], qb[KQ];
        double c_d1, c_d2, c_rq, c_S, c_h;      // channel scalars, prefetched with quarter 0
        int c_ok;
        auto ldq = [&](int i, int quarter, double2 (&b)[KQ]) {
            const int n = min(tid + TB * i, a.nchan - 1);
            const double2 *p = Mq + (int64_t)n * kMoments + KQ * quarter;
#pragma unroll
            for (int m = 0; m < KQ; ++m) b[m] = p[m];
        };
        auto ldc = [&](int i) {
            const int n = min(tid + TB * i, a.nchan - 1);
            c_d1 = dp[2 * n]; c_d2 = dp[2 * n + 1]; c_rq = rq[n]; c_S = chan[n * 4 + 3];
            c_h = m16 ? hq[n] : h;
            c_ok = mk[n];
        };
        const bool q4 = !m16 && xsel > kX24;   // uniform: all 32 moments needed
#if PPF_TRMOM_ADAPT
        // mom16 (round 6): only the moments the step needs.  The second
        // derivative's series truncated after M moments errs by at most
        // x^(M-2) / (M-2)! of sum |Y| (|u| <= 1), so with x = max_n 2 pi h_n
        // |Delta_n| (xsel): M = 8 for x <= kX8 -- every fit's first
        // evaluation, at the centre itself (x = 0) --, 12 for x <= kX12,
        // else 16: the same 1.6e-13 bound as kX16, 128 / 192 instead of 256
        // B of moments per channel read per evaluation
        const int mq = !m16 ? 2 : (xsel <= kX8 ? 0 : (xsel <= kX12 ? 1 : 2));
        auto ldq4 = [&](int i, double2 (&b)[KQ]) {
            const int n = min(tid + TB * i, a.nchan - 1);
            const double2 *p = Mq + (int64_t)n * kMoments + KQ;
#pragma unroll
            for (int m = 0; m < 4; ++m) b[m] = p[m];
        };
#else
        constexpr int mq = 2;
        auto ldq4 = [&](int, double2 (&)[KQ]) {};
#endif
        ldq(0, 0, qa);
        ldc(0);
        for (int i = 0; i < nit; ++i) {
            const int n = tid + TB * i;
            if (mq == 2) ldq(i, 1, qb);
            else if (mq == 1) ldq4(i, qb);
            const bool valid = n < a.nchan && (!use_mask || c_ok != 0);
            const double d1 = c_d1, d2 = c_d2, Sn = c_S, hn_ = c_h;
            const double del = e0 + e1 * d1 + e2 * d2 + c_rq;
            const double x = kTwoPi * hn_ * del;
            double2 G0 = cmk(0.0, 0.0), G1 = G0, G2 = G0;
            double r0 = 1.0, r1 = 0.0, r2 = 0.0;
            taylor_seg<0, KQ, 0, KQ>(qa, x, r0, r1, r2, G0, G1, G2);
            if (m16) {
                // 16 moments: the next channel's first quarter is in flight
                // while the second is summed
                if (i + 1 < nit) {
                    ldq(i + 1, 0, qa);
                    ldc(i + 1);
                }
                if (mq == 2) taylor_seg<KQ, 2 * KQ, KQ, KQ>(qb, x, r0, r1, r2, G0, G1, G2);
                else if (mq == 1) taylor_seg<KQ, KQ + 4, KQ, KQ>(qb, x, r0, r1, r2, G0, G1, G2);
            } else {
                ldq(i, 2, qa);
                taylor_seg<KQ, 2 * KQ, KQ, KQ>(qb, x, r0, r1, r2, G0, G1, G2);
                if (q4) ldq(i, 3, qb);
                taylor_seg<2 * KQ, 3 * KQ, 2 * KQ, KQ>(qa, x, r0, r1, r2, G0, G1, G2);
                if (i + 1 < nit) {
                    ldq(i + 1, 0, qa);
                    ldc(i + 1);
                }
                if (q4) taylor_seg<3 * KQ, kMoments, 3 * KQ, KQ>(qb, x, r0, r1, r2, G0, G1, G2);
            }
            if (!valid) continue;
            const double2 eix = cexp2pi(hn_ * del);
            const double2 F = cmul(eix, G0);
            const double2 K1 = cscale(cmul(eix, cadd(G0, G1)), hn_);
            const double2 K2 = cscale(cmul(eix, cadd(cadd(G0, G2), cscale(G1, 2.0))), hn_ * hn_);
            const double C = F.x, Cp = -kTwoPi * K1.y, Cpp = -kTwoPi * kTwoPi * K2.x;
            double *sn = st + (int64_t)n * 10;
            sn[0] = C; sn[1] = Cp; sn[2] = Cpp; sn[6] = Sn;
            if (!PPF_TRINIT_ZERO) sn[3] = sn[4] = sn[5] = sn[7] = sn[8] = sn[9] = 0.0;
            const double iS = 1.0 / Sn;
            const double dph[3] = {1.0, d1, d2};
            const double hn = -2.0 * (C * Cpp + Cp * Cp) * iS;
            // acc: f, g(phi, DM, GM), H upper triangle 00 01 02 11 12 22
            acc[0] += -C * C * iS;
#pragma unroll
            for (int q = 0; q < 3; ++q)
                if (flagmask >> q & 1) acc[1 + q] += -2.0 * C * Cp * dph[q] * iS;
            constexpr int hi[6] = {0, 0, 0, 1, 1, 2}, hj[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
            for (int e = 0; e < 6; ++e)
                if ((flagmask >> hi[e] & 1) && (flagmask >> hj[e] & 1))
                    acc[4 + e] += hn * dph[hi[e]] * dph[hj[e]];
        }
        TP(2);
        blk_sum<10, TB>(acc, red);
        TP(3);
        if (tid == 0) {
            double o[21];
#pragma unroll
            for (int i = 0; i < 21; ++i) o[i] = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = acc[i];
            constexpr int hi[6] = {0, 0, 0, 1, 1, 2}, hj[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
            for (int e = 0; e < 6; ++e) o[6 + uidx(hi[e], hj[e])] = acc[4 + e];
            L.meval = qsel;
#if PPF_NEWTON_MOM
            cmdb = L.newton ? tr_update_newton_n<3>(L, o, a.max_iter) : tr_update<3>(L, o, a.max_iter);
#else
            cmdb = tr_update<3>(L, o, a.max_iter);
#endif
        }
        TP(4);
        __syncthreads();
        TP(5);
        if (!cmdb) break;
    }
    __syncthreads();
    for (int i = tid; i < NW; i += TB)
        reinterpret_cast<double *>(&G)[i] = reinterpret_cast<const double *>(&L)[i];
    TP(6);
    TP_DONE();
}

// nu_zero-case accumulation slots
enum { NZ_MAX = 16 };

// ===========================================================================
// k_postfit: one workgroup per sub-integration
// ===========================================================================
// zero-covariance frequencies from the channel sums c[] (thread 0 of
// k_postfit): the closed forms and np.roots cases of get_nu_zeros
// (pptoaslib.py:776-950).  Out of line so that its root-finder locals do not
// weigh on k_postfit's per-channel loops.
__device__ __noinline__ void nz_solve(const double *c, int nzcase, int option, double nu_mean,
                                      double *nz, int *no_root_out) {
    double num, den;
    bool no_root = false;
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
            if (option == 0 || option == 1) {
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
            if (option == 0 || option == 1) {
                double H14 = c[16], H44 = c[17];
                double A = c[0], aa = c[1], B = c[2], b = c[3], C = c[4], cc = c[5],
                       D = c[6], d = c[7], E = c[8], e = c[9], F = c[10], f = c[11];
                double co[6];
                int deg;
                if (option == 0) {
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
    *no_root_out = no_root ? 1 : 0;
}

#ifdef PPF_POSTFIT_WPE
#define PPF_POSTFIT_ATTR __attribute__((amdgpu_waves_per_eu(PPF_POSTFIT_WPE)))
#else
#define PPF_POSTFIT_ATTR
#endif
// PB threads per sub-int.  64 (one wave) lets four sub-ints share a CU at
// the kernel's one wave per SIMD, so the serial parts (the zero-covariance
// root finding, the covariance inversion by thread 0) of four sub-ints
// overlap instead of one: C2 264.0k -> 269.6k fits/s, C3 73.8-74.3 ->
// 71.7-71.9 ms per step in one call (tools/g27.sh).  Wide sub-ints keep 256
// (C5, 16384 channels in 500 sub-ints: 85.0-86.0 vs 86.2-86.7 ms with 64).
// PPF_POSTFIT_PB forces one of them.
template <int PB>
__global__ __launch_bounds__(PB) PPF_POSTFIT_ATTR void k_postfit(SolveArgs a) {
    __shared__ double red[kWaves * 32];
    __shared__ double sh_Xinv[25];
    __shared__ double sh_misc[16];
    __shared__ double sh_acc[NZ_MAX + 8];
    const int s = blockIdx.x, tid = threadIdx.x;
    const TRState &S = a.state[s];
    ppf_result *res = a.results + s;
    if (S.status == PPF_ST_NOFIT || S.status == PPF_ST_NOSPACE) {
        if (tid == 0) {
            for (int i = 0; i < 32; ++i) reinterpret_cast<double *>(res)[i] = 0.0;
            res->status = S.status;
            res->phi_guess = S.phi_guess;
        }
        for (int n = tid; n < a.nchan; n += PB) {
            const int64_t o2 = (int64_t)s * a.nchan + n;
            a.scales[o2] = 0.0; a.scale_errs[o2] = 0.0; a.channel_snrs[o2] = 0.0;
        }
        return;
    }
    struct { const double *fr; const uint8_t *mask; int nchan; } v;
    v.fr = a.freqs + (int64_t)s * a.nchan;
    v.mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    v.nchan = a.nchan;
    const int flagmask = S.flagmask;
    int idx[5], nf = 0;
    for (int i = 0; i < 5; ++i)
        if (flagmask >> i & 1) idx[nf++] = i;
    double x[5];
    for (int i = 0; i < 5; ++i) x[i] = S.x[i];
    const double fun = S.f;
    const int status = S.status, nfev = S.nfev, k = S.k;
    const bool scat = S.scat != 0;
    const double nu_mean = S.nu_mean, dof = S.dof, phi_guess = S.phi_guess;
    // Sd = sum_n |D_n|^2 / sigma~_n^2 over the usable channels
    // (pptoaslib.py:1031), from the spectrum kernels' chan[]
    double sdv[1] = {0.0};
    {
        const double *chan = a.chan + (int64_t)s * a.nchan * 4;
        const uint8_t *mk = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
        for (int n = tid; n < a.nchan; n += PB)
            if (!mk || mk[n]) sdv[0] += chan[n * 4 + 2];
    }
    blk_sum<1, PB>(sdv, red);
    const double Sd = sdv[0];
    const int nchanx = S.nchanx;
    FitGeom g;
    g.P = a.P[s];
    g.nu_DM = S.nu_fit[0];
    g.nu_GM = S.nu_fit[1];
    g.nu_tau = S.nu_fit[2];
    g.log10_tau = a.log10_tau;
    g.tau_lin = 0.0;
    g.g_sum = g.g_tau = g.g_alpha = false;
    const double *st_fit = a.stats + ((int64_t)s * 2 + S.slot_cur) * a.nchan * 10;

    // ---- gates at the fit point ---------------------------------------------------
    const double tau_fit_lin = a.log10_tau ? pow(10.0, x[3]) : x[3];
    auto gates = [&](FitGeom &gg, double taulin, double alpha) {
        gg.tau_lin = taulin;
        if (!scat) { gg.g_sum = gg.g_tau = gg.g_alpha = false; return; }
        double sm[3] = {0.0, 0.0, 0.0};
        for (int n = tid; n < v.nchan; n += PB) {
            if (v.mask && !v.mask[n]) continue;
            double tn = taulin * pow(v.fr[n] / gg.nu_tau, alpha);
            sm[0] += tn;
            sm[1] += gg.log10_tau ? kLn10 * tn : tn / taulin;
            sm[2] += log(v.fr[n] / gg.nu_tau) * tn;
        }
        blk_sum<3, PB>(sm, red);
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
        for (int n = tid; n < v.nchan; n += PB) {
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
        blk_sum<NZ_MAX + 8, PB>(accv, red);
        if (tid == 0) {
            for (int i = 0; i < NZ_MAX + 8; ++i) sh_acc[i] = accv[i];
            int nr_flag = 0;
            nz_solve(sh_acc, nzcase, a.option, nu_mean, nz, &nr_flag);
            no_root = nr_flag != 0;
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
    for (int n = tid; n < v.nchan; n += PB) {
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
    blk_sum<31, PB>(cv, red);
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
        // scattered to parameter positions (zeros for fixed parameters), so
        // the per-channel loops below index it with compile-time constants
        for (int i2 = 0; i2 < 25; ++i2) sh_Xinv[i2] = 0.0;
        for (int i2 = 0; i2 < nf; ++i2)
            for (int j2 = 0; j2 < nf; ++j2) sh_Xinv[idx[i2] * 5 + idx[j2]] = Xi[i2][j2];
        sh_misc[8] = (double)sing;
    }
    __syncthreads();
    sing = (int)sh_misc[8];
    double Xinv[5][5];
    for (int i2 = 0; i2 < 5; ++i2)
        for (int j2 = 0; j2 < 5; ++j2) Xinv[i2][j2] = sh_Xinv[i2 * 5 + j2];
    // per-channel scales, scale errors, channel S/N
    double sn[1] = {0.0};
    for (int n = tid; n < v.nchan; n += PB) {
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
        // U X^-1 U over the fitted parameters in order (fixed ones add
        // exact zeros)
        double U[5];
#pragma unroll
        for (int i2 = 0; i2 < 5; ++i2) U[i2] = (flagmask >> i2 & 1) ? -2.0 * (dC[i2] - an * dS[i2]) : 0.0;
        double quad = 0.0;
#pragma unroll
        for (int i2 = 0; i2 < 5; ++i2)
#pragma unroll
            for (int j2 = 0; j2 < 5; ++j2)
                if ((flagmask >> i2 & 1) && (flagmask >> j2 & 1)) quad += U[i2] * Xinv[i2][j2] * U[j2];
        const double cinv = 1.0 / (2.0 * S);
        double var = 2.0 * (cinv + quad * cinv * cinv);
        double serr = (a.mode == PPF_MODE_LEGACY2) ? pow(S, -0.5) : sqrt(var);
        double csnr = an * sqrt(S);
        a.scales[o2] = an;
        a.scale_errs[o2] = serr;
        a.channel_snrs[o2] = csnr;
        sn[0] += csnr * csnr;
    }
    blk_sum<1, PB>(sn, red);
    if (tid == 0) {
        double pe[5] = {0, 0, 0, 0, 0};
        double *cov = a.covariance + (int64_t)s * 25;
        for (int i2 = 0; i2 < 25; ++i2) cov[i2] = 0.0;
        for (int i2 = 0; i2 < nf; ++i2) {
            for (int j2 = 0; j2 < nf; ++j2) cov[i2 * 5 + j2] = 2.0 * sh_Xinv[idx[i2] * 5 + idx[j2]];
            pe[idx[i2]] = sqrt(2.0 * sh_Xinv[idx[i2] * 5 + idx[i2]]);
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
        // full passes over X: one per evaluation (k_pass) or one per moment
        // (re)centre (k_moments)
        // passes over X: subset evaluations count their fraction of the
        // channel groups
        double npass = S.mmode ? (double)S.nmom + 1.0 : (double)nfev;
        if (!S.mmode && S.nsubev > 0) {
            const int ng = (a.nchan + 63) / 64, nsel = (ng + S.sub0 - 1) / S.sub0;
            npass -= (double)S.nsubev * (1.0 - (double)nsel / (double)ng);
        }
        res->npass = npass;
        res->reserved[0] = res->reserved[1] = 0.0;
    }
}

// ===========================================================================
// launchers
// ===========================================================================
hipError_t launch_classify(int nsub, const int32_t *fit_flags, const double *init, int log10_tau,
                           int fused, int xcap, uint8_t *needx, int32_t *xslot, hipStream_t st) {
    hipLaunchKernelGGL(k_classify, dim3(1), dim3(kClassifyBlock), 0, st, nsub, fit_flags, init,
                       log10_tau, fused, xcap, needx, xslot);
    return hipGetLastError();
}

hipError_t launch_tr_init(const SolveArgs &a, hipStream_t st) {
    hipLaunchKernelGGL(k_tr_init, dim3((unsigned)((a.nsub + kWaves - 1) / kWaves)), dim3(kBlock), 0,
                       st, a);
    return hipGetLastError();
}

template <bool SCAT>
static void launch_pass_t(const SolveArgs &a, hipStream_t st, dim3 g) {
    hipLaunchKernelGGL((k_pass<SCAT>), g, dim3(kBlock), 0, st, a);
}

hipError_t launch_pass(const SolveArgs &a, hipStream_t st) {
    const int nblk = (a.nchan + kPassChans - 1) / kPassChans;
    dim3 g((unsigned)((int64_t)a.nsub * nblk));
    if (a.any_plain) launch_pass_t<false>(a, st, g);
    if (a.any_scat) launch_pass_t<true>(a, st, g);
    return hipGetLastError();
}

hipError_t launch_tr_step(const SolveArgs &a, hipStream_t st) {
    const dim3 g((unsigned)((a.nsub + kWaves - 1) / kWaves));
    const bool lane = PPF_TRSTEP_LANE == 2 || (PPF_TRSTEP_LANE == 1 && a.nsub >= 2048 && a.nchan <= 2048);
    if (lane) {
        const dim3 gl((unsigned)((a.nsub + 63) / 64));
        const size_t lds = 64 * sizeof(TRState);
        if (a.bounds) hipLaunchKernelGGL(k_tr_step_l<true>, gl, dim3(64), lds, st, a);
        else hipLaunchKernelGGL(k_tr_step_l<false>, gl, dim3(64), lds, st, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (a.any_scat) hipLaunchKernelGGL(k_tr_gates, g, dim3(kBlock), 0, st, a);
        return hipGetLastError();
    }
    if (a.bounds)
        hipLaunchKernelGGL(k_tr_step<true>, g, dim3(kBlock), 0, st, a);
    else
        hipLaunchKernelGGL(k_tr_step<false>, g, dim3(kBlock), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_moments(const SolveArgs &a, hipStream_t st) {
    const int nblk = (a.nchan + kMomChans - 1) / kMomChans;
    if (a.mom16) hipLaunchKernelGGL(k_moments<true>, dim3((unsigned)((int64_t)a.nsub * nblk)), dim3(kBlock), 0, st, a);
    else hipLaunchKernelGGL(k_moments<false>, dim3((unsigned)((int64_t)a.nsub * nblk)), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_tr_mom(const SolveArgs &a, hipStream_t st) {
    // (one wave per sub-int, as k_postfit, measured slower here: C2 solve
    // stage 815 vs 777 ms per 24 calls, C4 305-332k vs 338-339k
    // archive-iterations/s: the evaluation pass, not the thread-0 update,
    // is most of a launch.  Round 5: a variant with thread = channel and the
    // moment set resident in registers for the whole launch (no per-
    // evaluation re-reads) was slower too, C2 224 vs 168 ms of k_tr_mom per
    // 120 calls, C4 unchanged: with the thread-0 update's registers on top
    // of 64 resident ones it spills (256 VGPRs + 324 B scratch) and holds
    // one 512-thread workgroup per CU, so the serial updates no longer
    // overlap other workgroups' evaluations; capped at three waves per SIMD
    // it spills 670 B and takes 247 ms).  Also measured in round 5 and not
    // kept: the expansion-radius test folded into the evaluation pass
    // (evaluate from the first valid moment set, one block reduction for
    // the sums and the radius max, the two-set test only when that fails):
    // the evaluation as a lambda with two call sites raised the spills from
    // 30 to 70 VGPRs, 229-232 ms vs 168 ms per 120 C2 calls (with the test
    // off, the same structure took 209 ms), C4 299-311k vs 330k)
    // Round 5: 128-thread workgroups (two waves, four channels per thread at
    // 512 channels; four sub-ints per CU instead of two, so more thread-0
    // updates overlap other workgroups' evaluation passes): C2 k_tr_mom 163
    // vs 171 ms per 120 calls, C4 332.8-338.6k vs 322.7-330.6k
    // archive-iterations/s in one call (profiles/r05/ab_tb1_status.txt)
#ifdef PPF_TRMOM_TB
    const int tb = PPF_TRMOM_TB;
#else
    const int tb = 128;
#endif
    if (tb == 64) hipLaunchKernelGGL(k_tr_mom<64>, dim3((unsigned)a.nsub), dim3(64), 0, st, a);
    else if (tb == 128) hipLaunchKernelGGL(k_tr_mom<128>, dim3((unsigned)a.nsub), dim3(128), 0, st, a);
    else hipLaunchKernelGGL(k_tr_mom<256>, dim3((unsigned)a.nsub), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_postfit(const SolveArgs &a, hipStream_t st) {
#ifdef PPF_POSTFIT_PB
    const int pb = PPF_POSTFIT_PB;
#else
    const int pb = a.nchan <= 2048 ? 64 : 256;
#endif
    // (128 threads measured slower in round 5: C2 285.3-286.5k vs 287.6-288.2k, C3
    // 145.0-146.5k vs 147.7-148.1k, profiles/r05/ab_pf1_status.txt)
    if (pb == 64) hipLaunchKernelGGL(k_postfit<64>, dim3((unsigned)a.nsub), dim3(64), 0, st, a);
    else hipLaunchKernelGGL(k_postfit<256>, dim3((unsigned)a.nsub), dim3(256), 0, st, a);
    return hipGetLastError();
}

size_t tr_state_bytes() { return sizeof(TRState); }
int pass_blocks(int nchan) { return (nchan + kPassChans - 1) / kPassChans; }

}  // namespace ppf

#ifdef PPF_TM_PROF
extern "C" int ppf_debug_tprof(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ppf::g_tprof), sizeof(unsigned long long) * 8) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(ppf::g_tprof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
