// ppf_internal.hpp -- kernel argument blocks and launchers (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ppfit.h"

namespace ppf {

struct RfftArgs {
    int nbin, log2N, dtype;
    const void *in;
    const double2 *T, *T2;
    double2 *out;      // [rows][N+1]
};

struct XspecArgs {
    int nsub, nchan, nbin, log2N, kc, nblk, cb, dtype, xcd_swizzle;
    const void *data;
    const double2 *Mft;          // [nmodel][nchan][N+1]
    const int32_t *model_index;
    const uint8_t *mask;
    const double *errs;          // [nsub][nchan] or null
    const double *freqs, *P;
    const double2 *T, *T2;
    double2 *X;                  // [nsub][N+1][nchan] (harmonic-major)
    double *chan;                // [nsub][nchan][4]
    const double2 *spec;         // k_xspec_spec: the rows' rFFTs [nsub][nchan][N+1] (long rows)
    // wave path: model row power sum_{k>=1} |M_nk|^2 ([nmodel][nchan]) and
    // the per-sub-int "write X" flag (null: every sub-int).  Sub-ints whose
    // fit runs on moments (k_xmom) are skipped.
    const double *Mpow;
    const uint8_t *needx;        // [nsub]
    const int32_t *KC;           // [nmodel][nchan] harmonic cutoff (k_model_cut) or null: X is
                                 // written only below the cutoff of each 64-channel group
    const int32_t *xslot;        // [nsub] X slot of each sub-int (k_classify), or null: slot = s
    // GetTOAs guess spectrum fused into the wave pass (gflag[s] set, see
    // k_gflag): sum_n w_n D_nk exp(2 pi i k dphi_n(DM_guess)) of the block's
    // rows for the harmonics guess_pairs() covers, per (sub-int, block)
    const uint8_t *gflag;        // [nsub] or null (no fused guess)
    double2 *gpart;              // [nsub][nblk][guess_slots(log2N)]
    double *gw;                  // [nsub][nblk][3] (sum w, count, sum w^2 errs_FT^2)
    const double *guess_weights, *guess_DM, *nu_fits;
    int guess_ref;
};

// Fused guess harmonics of an N = 2^log2N point wave FFT: k < 64 guess_npl
// (the FFTFIT sums stop at the mean model's cutoff; a sub-int whose cutoff
// is higher takes the time-domain pass, k_dsum)
__host__ __device__ constexpr int guess_npl(int log2N) { return log2N >= 10 ? 7 : (log2N == 9 ? 3 : (log2N == 8 ? 2 : 1)); }
__host__ __device__ constexpr int guess_slots(int log2N) { return 64 * guess_npl(log2N); }

// k_dsum: GetTOAs guess profile, time-domain dedispersion (pptoas.py:461-464)
struct DsumArgs {
    int nsub, nchan, nbin, dtype, cbd, nblkd;
    int guess_ref;               // 1: dedisperse at nu_fits[s][0] (ppalign), 0: at the mean freq
    const double *nu_fits;       // [nsub][3]
    const void *data;
    const uint8_t *mask;
    const double *freqs, *P, *guess_DM, *guess_weights;
    double *gP;                  // [nsub][nblkd][nbin] partial profiles
    double *gw;                  // [nsub][nblkd][2] (sum w, count)
    const uint8_t *gflag;        // [nsub]: 1 = fused into k_xspec_w (skip), or null
    double *nuref;               // [nsub] nu_ref^-2 per sub-int (k_nu_ref), or null:
                                 // every workgroup reduces the frequencies itself
};

// k_xmom: fused re-FFT + cross spectrum + Taylor moments (no X in HBM)
struct XmomArgs {
    int nsub, nchan, nbin, log2N, nblk, cb, dtype, xcd_swizzle, nmodel;
    const void *data;
    const double2 *Mft;
    const int32_t *model_index;
    const uint8_t *mask;
    double *chan;                // [nsub][nchan][4] (written: noise, Sd, S)
    const double *dphi;          // [nsub][nchan][2]
    const double2 *T, *T2;
    const void *state;           // TRState[nsub]
    double *mom;                 // [nsub][2][nchan][kMoments] (double2)
    const double *Bt;            // [N/2][16] folded-moment B tile (k_btab)
    int kc;                      // get_noise_PS cut
    const double *errs;          // [nsub][nchan] or null
    const double *Mpow;          // [nmodel][nchan]
    double *mres;                // [nsub][2][nchan] centre residual phi_c,n - s_n/nbin
    const int32_t *KC;           // [nchan] harmonic cutoff of the (single) model, or null
    // re-centring launches (FULL = false): the sub-ints of rc_list[0..*rc_count)
    // packed eight to a workgroup; null: every sub-int whose need_mom is set
    const unsigned *rc_count;
    const int32_t *rc_list;
};

struct GuessArgs {
    int nsub, nchan, nbin, log2N, kc, nblkd, Ns;
    int guess_ref;               // 1: the profile is already at nu_fit (no phase_transform)
    const uint8_t *mask;
    const double *freqs, *P, *guess_DM, *guess_tau, *nu_fits;
    const double *gP;            // [nsub][nblkd][nbin] (k_dsum)
    const double *gw;            // [nsub][nblkd][2]
    const double2 *T, *T2;
    double *x0;                  // [nsub][8]
    // mean model = (Msum - masked rows) / count
    const double2 *Msum;         // [nmodel][N+1]
    const double2 *Mft;
    const int32_t *model_index;
    const int32_t *KC;           // [nmodel][nchan] harmonic cutoff (k_model_cut) or null
    // fused guess spectrum (k_xspec_w) for the sub-ints with gflag set
    const uint8_t *gflag;        // [nsub] or null
    const double2 *gpart;        // [nsub][nblk][guess_slots(log2N)]
    const double *gwx;           // [nsub][nblk][3]
    int nblk;
    // brute grid of a whole turn (Ns >= 512, ppalign's Ns = nbin) as a
    // chirp z-transform (round 6): czB = FFT_P of the chirp kernel of each of
    // the czQ output chunks of czJ points (scaled by 1/P), czT its P-point
    // twiddles; null: the direct sums
    const double2 *czB, *czT;
    int czP, czJ, czQ, czK;
    // long rows (round 6): the guess profiles' rFFTs [nsub][N+1], taken on
    // the long transforms, replace the LDS transform of the profile
    const double2 *gspec;
    // long rows whose brute grid does not fit next to the spectrum in LDS
    // (ppalign: Ns = nbin): the grid in global memory, [nsub][Ns + 8]
    double *gsh;
};

// chirp z-transform plan of a whole-turn brute grid (k_guess): Kmax
// harmonics, Ns points over [lo, lo + 1], outputs in Q chunks of J points,
// P-point transforms (P = pow2 >= Kmax + 255, J = P - Kmax + 1)
struct CzPlan {
    int Ns, K, P, J, Q;
};
hipError_t launch_cz_table(const CzPlan &c, double2 *B, const double2 *T, hipStream_t st);

struct TRState;

struct SolveArgs {
    int nsub, nchan, nbin;
    const double2 *X, *Mft;
    const double *MP;            // [nmodel][N+1][nchan] |M_nk|^2 (k = 0: 0)
    const int32_t *KC;           // [nmodel][nchan] harmonics that matter (k_model_cut)
    const int32_t *model_index;
    const double *chan;
    const double *freqs, *P;
    const uint8_t *mask;
    const double *init;
    const int32_t *fit_flags;
    const double *nu_fits, *nu_outs;
    const double *bounds;        // [nsub][5][2] (NaN: none) or null
    int log10_tau, option, is_toa, mode, max_iter, guess;
    int newton;                  // 1: scattering fits use the Newton trust region (not PPF_OPT_SCIPY_TR)
    const double *x0;
    double *stats;               // [nsub][2][nchan][10]
    ppf_result *results;
    double *scales, *scale_errs, *channel_snrs, *covariance;
    int any_plain, any_scat;
    TRState *state;              // [nsub]
    double *partials;            // [nsub][pass_blocks(nchan)][21]
    unsigned *active;            // sub-ints still iterating (k_tr_step)
    unsigned *kinds;             // k_tr_init: [0] moment-mode fits, [1] streaming-pass fits
    // moment-expansion solver for fits without scattering (ppf_moments)
    int moments;                 // 1: enabled
    double2 *mom;                // [nsub][2][nchan][kMoments]
    double *dphi;                // [nsub][nchan][2]: d phi_n / d(DM, GM)
    double *mres;                // [nsub][2][nchan]: moment-centre residual per channel
    // PPF_OPT_MOM_X: 16 moments per channel, expanded in u = (k - h_n) / h_n
    // about the centre h_n of the wave's harmonic band [0, cutoff)
    int mom16;
    double *hcen;                // [nsub][2][nchan]: h_n of each moment set (mom16)
    const int32_t *xslot;        // [nsub] X slot (k_classify; -1 none, -2 no room) or null
    unsigned *rc_count;          // sub-ints k_tr_mom sent back for a new moment centre
    int32_t *rc_list;            // [nsub] their indices (slot order of the atomic)
};

struct RotateArgs {
    int nbin, log2N, dtype;
    const void *in;
    const double *phases;
    const double2 *T, *T2;
    double *out;
    // ref_len (odd nbin only): the reference's length-less irfft
    // (pplib.py:2466, 2508-2512, 2550, 2652): nbin - 1 samples per row from
    // X_0..X_{nbin/2}, the last as the Nyquist term; out rows of nbin - 1;
    // Te / T2e the twiddles of nbin - 1
    int ref_len;
    const double2 *Te, *T2e;
};

// ppalign accumulation (ppalign.py:236-247): per channel, sum_s w_sn *
// rotate(x_sn, phase_sn), done in the frequency domain
struct AlignArgs {
    int nsub, nchan, nbin, log2N, dtype, ngroup;
    const void *in;              // [nsub][nchan][nbin]
    const double *phases;        // [nsub][nchan]
    const double *weights;       // [nsub][nchan]
    const double2 *T, *T2;
    double2 *part;               // [ngroup][nchan][N+1] partial spectra
    double *wpart;               // [ngroup][nchan] partial weight sums
    double *out;                 // [nchan][nbin] (accumulated into)
    double *wsum;                // [nchan]      (accumulated into)
};
int align_groups(int nsub, int nchan);
hipError_t launch_align(const AlignArgs &a, hipStream_t st);
bool align_wave_supported(int log2N);                                   // nbin 256..2048
hipError_t launch_align_part_w(const AlignArgs &a, hipStream_t st);
hipError_t launch_align_phases(int nsub, int nchan, const double *results, const double *freqs, const double *P,
                               const uint8_t *mask, const double *scales, const double *errs, double *phases,
                               double *weights, hipStream_t st);     // wave-per-row partials

// per-row reduced chi^2 of (rotated data - scale * model) (the channel test
// of pptoas.get_channels_to_zap, pptoas.py:1266-1343 via show_fit 1375-1480)
struct ResidArgs {
    int nbin, log2N, dtype;
    const void *in;              // [nrows][nbin]
    const double *phases;        // [nrows]
    const double *model;         // [nmodelrows][nbin]
    const int32_t *model_row;    // [nrows]
    const double *scales, *errs; // [nrows]
    double dof;
    const double2 *T, *T2;
    double *out;                 // [nrows]
};
hipError_t launch_resid_chi2(const ResidArgs &a, int64_t nrows, hipStream_t st);

struct NoiseArgs {
    int nbin, log2N, dtype, kc;
    const void *in;
    const double2 *T, *T2;
    double *out;
};

// get_noise_PS of long rows (ppf_longfft.hip): the plan of one call
struct LongNoiseArgs {
    int64_t nbin;               // real samples per row
    int64_t n;                  // complex transform length (rfft_len)
    int64_t M, M1, M2;          // four-step size M = M1 M2 (powers of two)
    int log2M, log2M1;
    int packed;                 // even nbin: two samples per complex point
    int bluestein;              // n not a power of two >= 64: chirp z-transform
    int64_t nharm, kc;          // rfft bins nbin / 2 + 1, noise cut
    int in_dtype;
    const void *in;
    int64_t row0;               // first row of this launch
};
// ppf_rotate_long: the forward (f: nbin) and inverse (b: output) Bluestein
// plans of one call
struct LongRotArgs {
    LongNoiseArgs f, b;
    int out_even;               // output of even length 2 b.n (packed inverse)
    int64_t nout;               // output samples per row
    const double *phases;       // [nrows], or null: no rotation
    // [nrows] scattering tau_n (rotations per harmonic): the spectrum times
    // 1 / (1 + 2 pi i k tau_n) (the long rows' scattered Gaussian
    // portraits); null: none
    const double *taus;
    double *out;                // [nrows][nout]
};
struct LongPassArgs {
    int64_t nbatch;
    int len, log2len;
    int64_t in_stride, in_bstride, out_stride, out_bstride, row_elems, M;
    int twiddle, inverse;
    const double2 *in;
    double2 *out;
    const double2 *T;
};

struct PhaseShiftArgs {
    int nbin, log2N, dtype, kc, Ns;
    double lo, hi;
    const void *data;
    const double *model;
    const int32_t *model_index;
    const double *noise;
    const double2 *T, *T2;
    double *out;
    // long rows (round 6): the profiles' and model rows' rFFTs ([nprof] /
    // [nmodel][N+1]) taken beforehand on the long transforms; null: LDS FFTs
    const double2 *Dspec, *Mspec;
    // their brute grid in global memory ([nprof][Ns + 8]) when it does not
    // fit next to the spectrum in LDS; null: in LDS
    double *gsh;
};

struct SynthArgs {
    int nsub, nchan, nbin, log2N, dtype;
    const double2 *Mft;          // [nchan][N+1]
    const double *freqs, *phi, *DM, *P;
    double nu_ref, noise;
    uint64_t seed;
    int64_t first;
    const double2 *T, *T2;
    void *out;
};

// pptoaslib.get_scales_full (pptoaslib.py:953-971) per (sub-int, channel) row
struct ScalesArgs {
    int nsub, nchan, nharm, log10_tau;
    const double2 *D;            // [nsub][nchan][nharm] data spectra
    const double2 *M;            // [nmodel][nchan][nharm] model spectra
    const int32_t *model_index;  // [nsub] or null (model 0)
    const double *errs_FT;       // [nsub][nchan] or null (no division)
    const double *params;        // [nsub][5]
    const double *P;             // [nsub]
    const double *freqs;         // [nsub][nchan]
    const double *nus;           // [nsub][3] nu_DM, nu_GM, nu_tau
    double *out;                 // [nsub][nchan]
};
hipError_t launch_scales(const ScalesArgs &a, hipStream_t st);

// PSRFITS fast path (ppf_psrfits.hip): raw SUBINT DATA bytes -> float32
// total-intensity rows, baseline window, per-row statistics
struct UnpackArgs {
    int nsub, npol, nchan, nbin;
    int elem;                    // 0 big-endian int16, 1 uint8, 2 big-endian float32
    int pol_mode;                // 0: pol 0 (npol 1, IQUV); 1: AA + BB
    int rm_baseline, win;        // subtract the off-pulse mean; window bins
    const uint8_t *raw;          // [nsub] blocks of sub_stride bytes
    int64_t sub_stride;
    const float *scl, *offs;     // [nsub][npol * nchan]
    const float *wts;            // [nsub][nchan] or null
    float *out;                  // [nsub][nchan][nbin]
    double *part;                // [nsub][nblk][nbin] workspace
    double *total;               // [nsub][nbin]
    int32_t *wstart;             // [nsub]
    double *stats;               // [nsub][nchan][3]: off mean, off sigma, S/N
};
hipError_t launch_unpack(const UnpackArgs &a, hipStream_t st);
hipError_t launch_copy_host(const void *src_dev, void *dst, int64_t nbytes, hipStream_t st);
size_t unpack_partials(int nsub, int nchan, int nbin);

// pplib.gen_gaussian_portrait (pplib.py:886-963) per (portrait, channel) row
struct GaussArgs {
    int nport, nchan, nbin, log2N, ngauss, npar;
    int code[3];                 // evolution code per (loc, wid, amp): 0 power law, 1 linear
    const double *params;        // [nport][npar]: dc, tau [bin], ngauss x (loc, mloc, wid, mwid, amp, mamp)
    const double *scat_index;    // [nport]
    const double *freqs;         // [nport][nchan]
    const double *nu_ref;        // [nport]
    const double2 *T, *T2;
    const double2 *Te, *T2e;     // odd nbin: the twiddles of nbin - 1 (the scattered rows' irfft)
    double *out;                 // [nport][nchan][nbin] (odd nbin, tau != 0: nbin - 1 bins, then 0)
    // long rows: the unscattered rows, and each row's tau_n here for the
    // convolution on the long transforms (0: unscattered); null: in LDS
    double *taus_out;
};
hipError_t launch_gauss_port(const GaussArgs &a, hipStream_t st);

// pplib.gen_spline_portrait (pplib.py:966-990): per (portrait, channel) row,
// splev of the B-spline curve tck at the channel frequency (FITPACK splev /
// fpbspl, ext = 0), the eigenvector expansion plus the mean profile, and
// (nbin != nbin_model) scipy.signal.resample to nbin followed by the
// half-bin rotate_portrait of the reference
struct SplineArgs {
    int nport, nchan, nbin_model, nbin, ncomp, nknots, degree;
    int log2N0, log2N1;          // log2 of the half lengths (model, output)
    const double *mean_prof;     // [nbin_model]
    const double *eigvec;        // [nbin_model][ncomp]
    const double *knots;         // [nknots]
    const double *coefs;         // [ncomp][nknots]  (splprep c, zero-padded)
    const double *freqs;         // [nport][nchan]
    const double2 *T0, *T20;     // twiddles of nbin_model
    const double2 *T1, *T21;     // twiddles of nbin
    double *out;                 // [nport][nchan][nbin]
};
constexpr int kSplineMaxComp = 64;
constexpr int kSplineMaxDeg = 5;
hipError_t launch_spline_port(const SplineArgs &a, hipStream_t st);

hipError_t launch_twiddles(int N, double2 *T, double2 *T2, hipStream_t st);
hipError_t launch_rfft_rows(const RfftArgs &a, int64_t nrows, hipStream_t st);
hipError_t launch_xspec(const XspecArgs &a, hipStream_t st);
hipError_t launch_guess(const GuessArgs &a, hipStream_t st);
hipError_t launch_gflag(int nsub, int nchan, const uint8_t *needx, const int32_t *KC,
                        const int32_t *model_index, int klim, uint8_t *gflag, hipStream_t st);
hipError_t launch_dsum(const DsumArgs &a, hipStream_t st);
bool xspec_wave_supported(int log2N, int cb);
// wave-per-row mixed-radix spectrum pass (k_xspec_wm): nbin / 2 not a power
// of two, <= 1024 (prime factors above 7 on the generic-radix stage)
bool xspec_wm_supported(int nbin);
// the spectrum pass accumulates the GetTOAs guess at this FFT size (k_gflag)
bool xspec_guess_fused_n(int log2N);
hipError_t launch_xspec_wm(const XspecArgs &a, hipStream_t st);
hipError_t launch_xspec_wave(const XspecArgs &a, hipStream_t st);
hipError_t launch_xmom(const XmomArgs &a, bool full, hipStream_t st);
hipError_t launch_btab(int N, double *Bt, hipStream_t st);
hipError_t launch_classify(int nsub, const int32_t *fit_flags, const double *init, int log10_tau,
                           int fused, int xcap, uint8_t *needx, int32_t *xslot, hipStream_t st);
hipError_t launch_model_pow(const double2 *Mft, int nchan, int nharm, int nmodel, double *out,
                            hipStream_t st);
hipError_t launch_model_sum(const double2 *Mft, int nchan, int nharm, int nmodel, double2 *out,
                            hipStream_t st);
hipError_t launch_tr_init(const SolveArgs &a, hipStream_t st);
hipError_t launch_pass(const SolveArgs &a, hipStream_t st);
hipError_t launch_tr_step(const SolveArgs &a, hipStream_t st);
hipError_t launch_moments(const SolveArgs &a, hipStream_t st);
hipError_t launch_tr_mom(const SolveArgs &a, hipStream_t st);
constexpr int kMoments = 32;     // Taylor moments per channel
// Newton trust region of the scattering fits (ppf_solve.hip tr_update_newton):
// initial radius in Jacobi-scaled units (~sigma), and the predicted reduction
// of the objective (chi^2 units) below which the fit has converged
constexpr double kNewtonR0 = 10.0;
constexpr double kNewtonTol = 1e-12;
// its warm start on a channel subset (every sub-th group of 64 channels;
// scattering fits with >= 256 channels): leave it for every channel once an
// interior step predicts less than kSubsetSwitch (chi^2 units of the subset)
constexpr double kSubsetSwitch = 1.0;
constexpr int kSubsetMaxStride = 16;
hipError_t launch_postfit(const SolveArgs &a, hipStream_t st);
size_t tr_state_bytes();
int pass_blocks(int nchan);
hipError_t launch_rotate(const RotateArgs &a, int64_t nrows, hipStream_t st);
hipError_t launch_noise(const NoiseArgs &a, int64_t nrows, hipStream_t st);
int lf_pow_blocks(const LongNoiseArgs &a);
hipError_t launch_chirp_ft(const LongNoiseArgs &a, double2 *Bf, double2 *Bs, const double2 *T1,
                           const double2 *T2, hipStream_t st);
hipError_t launch_rfft_long(const LongNoiseArgs &f, int64_t nrows, double2 *A, double2 *Y, const double2 *Bf,
                            double2 *out, const double2 *T1, const double2 *T2, hipStream_t st);
hipError_t launch_xspec_spec(const XspecArgs &a, hipStream_t st);
hipError_t launch_gsum(int nsub, int nblkd, int nbin, const double *gP, double *prof, hipStream_t st);
hipError_t launch_rotate_long(const LongRotArgs &r, int64_t nrows, double2 *A, double2 *Y, const double2 *Bff,
                              const double2 *Bfb, const double2 *T1f, const double2 *T2f, const double2 *T1b,
                              const double2 *T2b, hipStream_t st);
hipError_t launch_noise_long(const LongNoiseArgs &a, int64_t nrows, double2 *A, double2 *Y,
                             const double2 *Bf, double *part, double *out, const double2 *T1,
                             const double2 *T2, hipStream_t st);
// wave-per-row noise (k_noise_w) for N = nbin/2 = 128..1024
bool noise_wave_supported(int log2N);
hipError_t launch_noise_wave(const NoiseArgs &a, int64_t nrows, hipStream_t st);
hipError_t launch_phase_shift(const PhaseShiftArgs &a, int nprof, hipStream_t st);
hipError_t launch_synth(const SynthArgs &a, hipStream_t st);
// per (model, channel): 1 + the last harmonic with |M_k|^2 > kCutRel max_k |M_k|^2
constexpr double kCutRel = 1e-28;   // |M_k| < 1e-14 max|M|: below the template's own FFT rounding floor
hipError_t launch_model_cut(const double *MP, int nchan, int nharm, int nmodel, bool off,
                            int32_t *KC, hipStream_t st);
hipError_t launch_model_pow_t(const double2 *Mft, int nchan, int nharm, int nmodel, double *MP,
                              hipStream_t st);

}  // namespace ppf
