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
    double2 *X;                  // [nsub][nchan][N+1]
    double *chan;                // [nsub][nchan][4]
    int guess;
    const double *guess_weights, *guess_DM;
    double2 *gR, *gM;            // [nsub][nblk][N+1]
    double *gw;                  // [nsub][nblk][2]
};

struct GuessArgs {
    int nsub, nchan, nbin, kc, nblk, Ns;
    const uint8_t *mask;
    const double *freqs, *P, *guess_DM, *guess_tau, *nu_fits;
    const double2 *gR, *gM;
    const double *gw;
    double *x0;                  // [nsub][8]
    // wave xspec path: mean model = (Msum - masked rows) / count
    const double2 *Msum;         // [nmodel][N+1] or null (use gM partials)
    const double2 *Mft;
    const int32_t *model_index;
};

struct TRState;

struct SolveArgs {
    int nsub, nchan, nbin;
    const double2 *X, *Mft;
    const int32_t *model_index;
    const double *chan;
    const double *freqs, *P;
    const uint8_t *mask;
    const double *init;
    const int32_t *fit_flags;
    const double *nu_fits, *nu_outs;
    int log10_tau, option, is_toa, mode, max_iter, guess;
    const double *x0;
    double *stats;               // [nsub][2][nchan][10]
    ppf_result *results;
    double *scales, *scale_errs, *channel_snrs, *covariance;
    int any_plain, any_scat;
    TRState *state;              // [nsub]
    double *partials;            // [nsub][pass_blocks(nchan)][21]
    unsigned *active;            // sub-ints still iterating (k_tr_step)
    // moment-expansion solver for fits without scattering (ppf_moments)
    int moments;                 // 1: enabled
    double2 *mom;                // [nsub][2][nchan][kMoments]
    double *dphi;                // [nsub][nchan][2]: d phi_n / d(DM, GM)
};

struct RotateArgs {
    int nbin, log2N, dtype;
    const void *in;
    const double *phases;
    const double2 *T, *T2;
    double *out;
};

struct NoiseArgs {
    int nbin, log2N, dtype, kc;
    const void *in;
    const double2 *T, *T2;
    double *out;
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

hipError_t launch_twiddles(int N, double2 *T, double2 *T2, hipStream_t st);
hipError_t launch_rfft_rows(const RfftArgs &a, int64_t nrows, hipStream_t st);
hipError_t launch_xspec(const XspecArgs &a, hipStream_t st);
hipError_t launch_guess(const GuessArgs &a, hipStream_t st);
bool xspec_wave_supported(int log2N, int cb);
hipError_t launch_xspec_wave(const XspecArgs &a, hipStream_t st);
hipError_t launch_model_sum(const double2 *Mft, int nchan, int nharm, int nmodel, double2 *out,
                            hipStream_t st);
hipError_t launch_tr_init(const SolveArgs &a, hipStream_t st);
hipError_t launch_pass(const SolveArgs &a, hipStream_t st);
hipError_t launch_tr_step(const SolveArgs &a, hipStream_t st);
hipError_t launch_moments(const SolveArgs &a, hipStream_t st);
hipError_t launch_tr_mom(const SolveArgs &a, hipStream_t st);
constexpr int kMoments = 32;     // Taylor moments per channel
hipError_t launch_postfit(const SolveArgs &a, hipStream_t st);
size_t tr_state_bytes();
int pass_blocks(int nchan);
hipError_t launch_rotate(const RotateArgs &a, int64_t nrows, hipStream_t st);
hipError_t launch_noise(const NoiseArgs &a, int64_t nrows, hipStream_t st);
hipError_t launch_phase_shift(const PhaseShiftArgs &a, int nprof, hipStream_t st);
hipError_t launch_synth(const SynthArgs &a, hipStream_t st);

}  // namespace ppf
