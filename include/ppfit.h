/*
 * ppfit.h -- C ABI of libppfit, the MI355X (gfx950) wideband FFTFIT engine.
 *
 * Drop-in boundary for the PulsePortraiture hot path.
 * The reference has no FFI: each entry point below replaces a Python/NumPy
 * routine of the reference and is bound from Python with ctypes
 * (pulseportraiture_amd/_lib.py; see INTEGRATION.md for the binding a
 * PulsePortraiture maintainer would add).
 *
 * Conventions
 *   - Every array pointer is a DEVICE pointer (hipMalloc / torch.cuda memory)
 *     unless stated otherwise; arrays are C-contiguous.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  All
 *     calls are asynchronous on that stream; they never synchronise the
 *     device and never allocate device memory except the per-context
 *     twiddle-table cache (created on first use of an nbin).
 *   - Return value: PPF_OK (0) or a negative PPF_E* code; ppf_last_error()
 *     gives the message.  Per-sub-integration numerical outcomes are reported
 *     in ppf_result.status, never by aborting the batch.
 *   - nbin: even 32..8192 or odd 33..4095 (nbin/2 not a power of two: the
 *     mixed-radix LDS FFT, a generic-radix stage for prime factors above 7;
 *     odd nbin: the row transformed as nbin complex points on the same
 *     stages); other nbin returns PPF_EUNSUP.  Powers of two
 *     in [256, 2048] take the wave-per-row kernels.
 *   - Threads: ppf_fit_batch / ppf_fit2_batch must not run concurrently on
 *     the same context (they share its profiling event ring and pinned
 *     iteration counter); any other entry point may run on another host
 *     thread beside them (GetTOAs builds templates with
 *     ppf_gauss_portrait_batch while a worker thread fits).  The twiddle
 *     cache and the error message are guarded; ppf_last_error returns the
 *     message as last set by any thread, copied for the calling thread.
 */
#ifndef PPFIT_H
#define PPFIT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 4 (round 5): the options PPF_OPT_MOM_X / PPF_OPT_FUSED_MOM, elem = 3
 * of ppf_unpack_psrfits_batch, PPF_EIO, ppf_read_rows and
 * ppf_copy_from_pinned (added in round 4 without a bump), and
 * ppf_kernel_ms_history slot 0 = the first moment pass of either kind;
 * ppf_solver_ms_history, ppf_host_copy. */
/* ABI 5 (round 6): ppf_rotate_batch_ref. */
/* ABI 6 (round 6): ppf_noise_long, ppf_rotate_long (+ their workspace
 * queries), ppf_align_phases, PPF_OPT_SPIN_WAIT; ppf_fit_batch /
 * ppf_gauss_portrait_batch / ppf_phase_shift_batch accept nbin past the LDS
 * transforms (even > 8192, odd > 4095) on the long transforms. */
#define PPF_ABI_VERSION 6

enum ppf_error {
    PPF_OK = 0,
    PPF_EINVAL = -1,   /* bad argument / shape */
    PPF_EHIP = -2,     /* HIP runtime error */
    PPF_ENOMEM = -3,   /* workspace too small */
    PPF_EUNSUP = -4,   /* unsupported configuration (e.g. nbin) */
    PPF_EIO = -5       /* file read failed or came up short */
};

enum ppf_dtype { PPF_F32 = 0, PPF_F64 = 1 };

/* ppf_result.status values (low byte = scipy trust-region warnflag) */
enum ppf_status {
    PPF_ST_SUCCESS = 0,      /* gradient test met (never, gtol = -1)        */
    PPF_ST_MAXITER = 1,      /* iteration cap reached                        */
    PPF_ST_CONVERGED = 2,    /* predicted reduction <= 0 (the usual stop)    */
    PPF_ST_LINALG = 3,       /* subproblem failure                           */
    PPF_ST_NO_ROOT = 0x100,  /* no positive real zero-covariance root:
                                the reference raises ValueError here         */
    PPF_ST_SINGULAR = 0x200, /* singular covariance (LinAlgError)            */
    PPF_ST_NONFINITE = 0x400,/* non-finite objective encountered             */
    PPF_ST_NOFIT = 0x800,    /* no parameter to fit / no usable channel      */
    PPF_ST_NOSPACE = 0x1000  /* the fit streams the cross spectrum but the
                                workspace holds fewer X slots (x_subints)    */
};

/* ppf_fit_desc.options bits */
enum ppf_option {
    PPF_OPT_NO_HCUT = 1,     /* sum every harmonic: no per-channel cutoff of
                                the harmonics whose template power is below
                                1e-28 of the channel's peak */
    PPF_OPT_NO_X = 2,        /* the caller has checked that no sub-int
                                streams the cross spectrum (no scattering
                                flag, zero initial tau): on the fused
                                phase+DM path no X slot is reserved and the
                                cross-spectrum pass is not launched (a
                                sub-int that would need X ends with
                                PPF_ST_NOSPACE) */
    PPF_OPT_SCIPY_TR = 4,    /* the fits follow scipy's trust-ncg path
                                step by step (pptoaslib.py:1055-1060:
                                radius 1 in raw parameter units,
                                CG-Steihaug subproblem).  Default: the
                                Newton trust region (Jacobi-scaled
                                coordinates, exact subproblem), which stops
                                at the same stationary point, closer (the
                                reference's Newton decrement at its end
                                point reaches 6e-6, this one's 1e-20), in
                                fewer evaluations: scattering fits 3x fewer
                                passes over the cross spectrum, ppalign
                                fits half the data passes.
                                Bounded (method='TNC') fits always take the
                                scipy path with projected steps. */
    PPF_OPT_MOM_X = 8,       /* phase/DM/GM fits on the wave-FFT shapes take
                                their Taylor moments from the cross spectrum
                                X (one spectrum pass writing X below the
                                harmonic cutoff, then k_moments: 16 moments
                                about the centre of each channel band's
                                harmonics), instead of the fused pass that
                                re-FFTs the data rows for every moment
                                centre (k_xmom_g): every sub-int then holds
                                an X slot (x_subints and PPF_OPT_NO_X are
                                overridden: nsub * nchan * (nbin/2 + 1) * 16
                                bytes of workspace, 8.4 MB per 512 x 2048
                                sub-int; ppf_fit_workspace_bytes includes
                                it).  Default (neither this nor
                                PPF_OPT_FUSED_MOM) where the GetTOAs guess
                                rides along in the spectrum pass: guess != 0
                                and nbin = 2048 */
    PPF_OPT_FUSED_MOM = 16,  /* force the fused k_xmom_g pass (no X for the
                                phase/DM/GM fits) */
    PPF_OPT_SPIN_WAIT = 32   /* (ABI 6) the call's read-backs of the count
                                of fits still iterating are polled on the
                                host instead of waited for with
                                hipStreamSynchronize: 30-70 us less per
                                read-back, for a caller with no host threads
                                of its own competing for the cores (ppalign:
                                C4 +2-3 %; GetTOAs' readers and stagers lost
                                up to 20 % to it) */
};

enum ppf_mode {
    PPF_MODE_FULL = 0,    /* pptoaslib.fit_portrait_full semantics */
    PPF_MODE_LEGACY2 = 1  /* pplib.fit_portrait semantics (phase + DM)  */
};

/* One fixed-size record per sub-integration (all doubles, 32 of them). */
typedef struct ppf_result {
    double params[5];      /* phi_out, DM, GM, tau_out, alpha               */
    double param_errs[5];
    double nu_out[3];      /* nu_DM, nu_GM, nu_tau of the reported params   */
    double nu_fit[3];      /* reference frequencies used inside the fit     */
    double chi2, red_chi2, snr;
    double fun;            /* objective at the fit (chi2 - Sd)              */
    double Sd;             /* data power term                               */
    double phi_guess;      /* initial phase actually used                   */
    double nfeval;         /* objective evaluations (scipy nfev)            */
    double status;         /* ppf_status bits                               */
    double niter;          /* trust-region iterations                       */
    double dof;
    double nchanx;         /* channels used                                 */
    double x_fit_phi;      /* phi at nu_fit (before output transform)      */
    double x_fit_tau;      /* tau parameter at nu_fit                       */
    double npass;          /* streaming passes over the cross spectrum      */
    double reserved[2];
} ppf_result;

/* Batched wideband fit: replaces pptoaslib.fit_portrait_full
 * (pptoaslib.py:974-1144) per sub-integration, plus -- when guess != 0 --
 * the initial-phase stage of pptoas.GetTOAs.get_TOAs (pptoas.py:461-499),
 * and with mode == PPF_MODE_LEGACY2 pplib.fit_portrait (pplib.py:2185-2287). */
typedef struct ppf_fit_desc {
    int32_t nsub, nchan, nbin;
    int32_t data_dtype;           /* PPF_F32 or PPF_F64                        */
    const void *data;             /* [nsub][nchan][nbin]                       */
    const double *model;          /* [nmodel][nchan][nbin]                     */
    int32_t nmodel;
    const int32_t *model_index;   /* [nsub] or NULL (all use model 0)          */
    const uint8_t *chan_mask;     /* [nsub][nchan], 1 = use; NULL = all        */
    const double *freqs;          /* [nsub][nchan] MHz                         */
    const double *P;              /* [nsub] s                                  */
    const double *errs;           /* [nsub][nchan] time-domain sigma, or NULL:
                                     estimated as pplib.get_noise_PS           */
    const double *init;           /* [nsub][5] initial params                  */
    const int32_t *fit_flags;     /* [nsub][5]                                 */
    const double *nu_fits;        /* [nsub][3]; NaN -> mean(freqs)             */
    const double *nu_outs;        /* [nsub][3]; NaN -> zero-covariance freq    */
    int32_t log10_tau;
    int32_t option;               /* get_nu_zeros option (GM cases)            */
    int32_t is_toa;
    int32_t mode;                 /* ppf_mode                                  */
    int32_t max_iter;             /* <= 0: reference default 200 * 5           */
    /* optional initial-phase stage (GetTOAs): phi_guess from the weighted,
       DM-dedispersed mean profile (brute grid of guess_Ns points + fmin) */
    int32_t guess;
    const double *guess_weights;  /* [nsub][nchan]                             */
    const double *guess_DM;       /* [nsub] DM used to dedisperse              */
    const double *guess_tau;      /* [nsub] scattering time [rot] applied to the
                                     mean model profile (pptoas.py:484-489), or
                                     NULL for none                             */
    int32_t guess_Ns;
    /* outputs */
    ppf_result *results;          /* [nsub]                                    */
    double *scales;               /* [nsub][nchan] (0 for masked channels)     */
    double *scale_errs;           /* [nsub][nchan]                             */
    double *channel_snrs;         /* [nsub][nchan]                             */
    double *covariance;           /* [nsub][5][5], fit block in leading corner */
    void *workspace;
    size_t workspace_bytes;
    /* ABI 2 */
    int32_t x_subints;            /* cross-spectrum (X) slots the workspace
                                     holds: the number of sub-ints whose fit
                                     streams X (scattering fits: fit_flags[3]
                                     or [4] set, or a nonzero initial tau).
                                     <= 0: nsub.  Sub-ints past it end with
                                     PPF_ST_NOSPACE.  Off the fused phase+DM
                                     path (nbin outside 256..2048) every
                                     sub-int streams X and nsub slots are
                                     always reserved. */
    int32_t options;              /* ppf_option bits                           */
    int32_t guess_ref;            /* frame of the guess stage's dedispersed
                                     mean profile: 0 = the mean usable
                                     frequency, phase then moved to nu_fit
                                     (GetTOAs, pptoas.py:461-499); 1 = nu_fit
                                     itself (ppalign, ppalign.py:214-219) */
    /* ABI 3 */
    const double *bounds;         /* [nsub][5][2] lower, upper bound of each
                                     parameter (NaN: none), or NULL for an
                                     unbounded fit.  method='TNC' of
                                     fit_portrait_full / get_TOAs
                                     (pptoaslib.py:1041-1053, pptoas.py:503-513):
                                     the initial point is clipped into the box
                                     and the trust-region steps are projected
                                     (parameters at a bound whose descent
                                     direction leaves the box are held there,
                                     the step over the others is cut at the
                                     first bound it crosses), so the fit ends
                                     at the bounded stationary point. */
} ppf_fit_desc;

int ppf_abi_version(void);
/* sizeof(ppf_fit_desc) / sizeof(ppf_result) as compiled, for FFI layout checks */
size_t ppf_sizeof_fit_desc(void);
size_t ppf_sizeof_result(void);

/* context: one per device; owns twiddle tables and the error string */
typedef struct ppf_ctx ppf_ctx;
int ppf_create(int device, ppf_ctx **out);
void ppf_destroy(ppf_ctx *ctx);
const char *ppf_last_error(const ppf_ctx *ctx);

/* Stage timing with HIP events recorded on the caller's stream around each
 * kernel of ppf_fit_batch (model rfft, xspec, guess, solve).  Off by
 * default; ppf_last_stage_ms waits for the last call's events and returns
 * the four stage durations in milliseconds (0 for a skipped stage). */
int ppf_set_profiling(ppf_ctx *ctx, int enable);
int ppf_last_stage_ms(ppf_ctx *ctx, double *ms4);
/* The stage times of the last n (<= 256) profiled ppf_fit_batch calls,
 * oldest first, into ms[n][4]; returns the number written.  Events are kept
 * in a ring, so a timed loop records without synchronising. */
int ppf_stage_ms_history(ppf_ctx *ctx, int n, double *ms);
/* Single-kernel times of the last n profiled ppf_fit_batch calls into
 * ms[n][2]: [0] the call's first moment pass over every moment-mode sub-int
 * -- the fused k_xmom_g over the data rows, or, on the moments-from-X path
 * (PPF_OPT_MOM_X, and the GetTOAs default at nbin 2048), k_moments over the
 * stored cross spectrum; 0 if the call had none -- and [1] the separate
 * guess-profile pass (k_dsum_w; 0 without a guess or when the guess rides in
 * the spectrum pass).  The spectrum pass itself (k_xspec_w) is stage [1] of
 * ppf_stage_ms_history.  Same event ring as ppf_stage_ms_history. */
int ppf_kernel_ms_history(ppf_ctx *ctx, int n, double *ms);
/* The streaming passes (k_pass: one trust-region evaluation of every
 * scattering fit still iterating) of the last n profiled ppf_fit_batch calls
 * into ms[n][2]: [0] their summed duration in ms (HIP events around each
 * launch), [1] the number of launches. */
int ppf_pass_ms_history(ppf_ctx *ctx, int n, double *ms);
/* The solver kernels of the last n profiled ppf_fit_batch calls into
 * ms[n][6] (ABI 4): summed ms and launch count of k_tr_mom (the moment-path
 * trust-region iterations), of k_tr_step (+ k_tr_gates; the scattering
 * path's update), and of k_postfit (zero-covariance frequencies, output
 * transform, covariance, scales), each launch bracketed by HIP events. */
int ppf_solver_ms_history(ppf_ctx *ctx, int n, double *ms);

/* Workspace needed by ppf_fit_batch for `desc` (only sizes/flags are read). */
size_t ppf_fit_workspace_bytes(const ppf_fit_desc *desc);

/* pptoaslib.fit_portrait_full (pptoaslib.py:974) / pptoas.get_TOAs inner loop
 * (pptoas.py:384-533) / pplib.fit_portrait (pplib.py:2185). */
int ppf_fit_batch(ppf_ctx *ctx, const ppf_fit_desc *desc, void *stream);

/* Same as ppf_fit_batch with desc->mode forced to PPF_MODE_LEGACY2:
 * pplib.fit_portrait (pplib.py:2185-2287). */
int ppf_fit2_batch(ppf_ctx *ctx, const ppf_fit_desc *desc, void *stream);

/* Rotate rows: out_r = irfft(rfft(in_r) * exp(2 pi i k phase_r)).
 * Replaces the FFT core of pplib.rotate_data (pplib.py:2427-2515),
 * pplib.rotate_portrait (2518-2550), pplib.rotate_profile (2641-2652) and
 * pptoaslib.rotate_portrait_full (pptoaslib.py:61-90); the host computes the
 * per-row phase phase + Dconst*DM/P*(nu**-2 - nu_ref**-2) exactly as those
 * routines do.  in: [nrows][nbin] of in_dtype; phases: [nrows] double;
 * out: [nrows][nbin] double. */
int ppf_rotate_batch(ppf_ctx *ctx, int64_t nrows, int32_t nbin,
                     int32_t in_dtype, const void *in, const double *phases,
                     double *out, void *stream);

/* ppf_rotate_batch with the reference's output length (ABI 5): the public
 * rotate routines call numpy's irfft WITHOUT a length (pplib.py:2466,
 * 2508-2512, 2550, 2652; pptoaslib.py:89), which at odd nbin returns
 * nbin - 1 samples: the inverse of length nbin - 1 of X_0..X_{nbin/2}, the
 * last harmonic taken as the Nyquist term (its imaginary part dropped).
 * out: [nrows][nbin] at even nbin (identical to ppf_rotate_batch),
 * [nrows][nbin - 1] at odd nbin. */
int ppf_rotate_batch_ref(ppf_ctx *ctx, int64_t nrows, int32_t nbin,
                         int32_t in_dtype, const void *in, const double *phases,
                         double *out, void *stream);

/* ppalign.align_archives accumulation (ppalign.py:236-247, the inner
 * "aligned_port += weights * rotate_data(...)" / "total_weights += weights"
 * over every sub-integration of every archive):
 *   out[n][:] += sum_s w[s][n] * irfft(rfft(in[s][n]) * exp(2 pi i k ph[s][n]))
 *   wsum[n]   += sum_s w[s][n]
 * Rows with w == 0 are skipped.  in: [nsub][nchan][nbin] (in_dtype);
 * phases, weights: [nsub][nchan]; out: [nchan][nbin] f64; wsum: [nchan].
 * The sum over sub-ints is taken in a fixed order (bitwise reproducible).
 * workspace: device scratch of ppf_align_workspace_bytes() bytes. */
size_t ppf_align_workspace_bytes(int32_t nsub, int32_t nchan, int32_t nbin);
int ppf_align_accum(ppf_ctx *ctx, int32_t nsub, int32_t nchan, int32_t nbin,
                    int32_t in_dtype, const void *in, const double *phases,
                    const double *weights, double *out, double *wsum,
                    void *workspace, size_t workspace_bytes, void *stream);

/* ppalign's per-row rotation phases and weights from a fit (ppalign.py:
 * 222-247; round 6, ABI 6): for sub-int s, channel n with mask[s][n] != 0
 *   phases[s][n]  = phi_s + Dconst DM_s / P_s (freqs[s][n]^-2 - nu_DM,s^-2)
 *   weights[s][n] = scales[s][n] / errs[s][n]^2
 * and 0 where masked; phi, DM, nu_DM from results[s] (ppf_result: params[0],
 * params[1], nu_out[0]).  One launch instead of the dozen elementwise
 * operations it replaces in each ppalign iteration.  results: [nsub]
 * ppf_result; freqs, scales, errs, phases, weights: [nsub][nchan]; P:
 * [nsub]; mask: [nsub][nchan] or NULL (all used). */
int ppf_align_phases(ppf_ctx *ctx, int32_t nsub, int32_t nchan, const double *results,
                     const double *freqs, const double *P, const uint8_t *mask,
                     const double *scales, const double *errs, double *phases,
                     double *weights, void *stream);

/* Channel reduced chi^2 of a fit (pptoas.get_channels_to_zap,
 * pptoas.py:1266-1343, through show_fit 1375-1480 and get_red_chi2
 * pplib.py:754-779): for each row r,
 *   out[r] = sum_t (rot(in[r], phases[r])[t] - scales[r] model[model_row[r]][t])^2
 *            / errs[r]^2 / dof
 * with rot the rfft-phasor-irfft rotation of ppf_rotate_batch.
 * in: [nrows][nbin]; model: [*][nbin] f64; phases, scales, errs, out: [nrows]. */
int ppf_resid_chi2_batch(ppf_ctx *ctx, int64_t nrows, int32_t nbin, int32_t in_dtype,
                         const void *in, const double *phases, const double *model,
                         const int32_t *model_row, const double *scales,
                         const double *errs, double dof, double *out, void *stream);

/* Per-row power-spectrum noise: pplib.get_noise_PS(chans=True)
 * (pplib.py:2312-2332): sqrt(mean(|rfft(x)|^2/nbin over k >= int((1-1/frac)
 * * nharm))).  in: [nrows][nbin]; out: [nrows]. */
int ppf_noise_batch(ppf_ctx *ctx, int64_t nrows, int32_t nbin,
                    int32_t in_dtype, const void *in, int32_t frac,
                    double *out, void *stream);

/* Power-spectrum noise of rows of ANY length (round 6, ABI 6):
 * pplib.get_noise_PS (pplib.py:2312-2338) where ppf_noise_batch's LDS
 * transforms do not reach -- chans=False ravels a whole portrait into one
 * row of nchan * nbin samples (2^20 at 512 x 2048), and rows past 8192 (even)
 * / 4095 (odd) samples.  The rFFT is a four-step transform of block LDS FFTs
 * (transform length a power of two) or Bluestein's chirp z-transform on one
 * (any other length), up to 2^24 complex points (2^25 samples for a
 * power-of-two row, 2^24 otherwise; PPF_EUNSUP past that).
 * in: [nrows][nbin] (in_dtype); out: [nrows] device doubles; workspace:
 * device scratch of ppf_noise_long_workspace_bytes(nrows, nbin) bytes
 * (0: nbin unsupported). */
size_t ppf_noise_long_workspace_bytes(int64_t nrows, int64_t nbin);
int ppf_noise_long(ppf_ctx *ctx, int64_t nrows, int64_t nbin, int32_t in_dtype,
                   const void *in, int32_t frac, double *out, void *workspace,
                   size_t workspace_bytes, void *stream);

/* rotate_data's rotation of rows of ANY length (round 6, ABI 6): rows the
 * LDS transforms of ppf_rotate_batch do not take (even nbin > 8192, odd
 * nbin > 4095), as Bluestein transforms both ways (up to 2^23 complex
 * points).  out[r] = irfft(rfft(in[r]) * exp(2 pi i k phases[r])), nbin
 * samples, or nbin - 1 at odd nbin with ref_len != 0 (the reference's
 * length-less irfft, as ppf_rotate_batch_ref).  in: [nrows][nbin]
 * (in_dtype); phases: [nrows]; out: [nrows][nout] f64; workspace: device
 * scratch of ppf_rotate_long_workspace_bytes(nrows, nbin, ref_len) bytes
 * (0: unsupported). */
size_t ppf_rotate_long_workspace_bytes(int64_t nrows, int64_t nbin, int32_t ref_len);
int ppf_rotate_long(ppf_ctx *ctx, int64_t nrows, int64_t nbin, int32_t in_dtype,
                    const void *in, const double *phases, double *out, int32_t ref_len,
                    void *workspace, size_t workspace_bytes, void *stream);

/* Batched 1-D FFTFIT: pplib.fit_phase_shift (pplib.py:2136-2182): brute
 * force over Ns points of [lo, hi] then Nelder-Mead (scipy fmin) polish.
 * data: [nprof][nbin] (in_dtype); model: [nmodel_prof][nbin] double with
 * model_index[nprof] (NULL -> 0); noise: [nprof] time-domain sigma or NULL
 * (estimated); out: [nprof][8] = phase, phase_err, scale, scale_err, snr,
 * red_chi2, nfev, status. */
int ppf_phase_shift_batch(ppf_ctx *ctx, int32_t nprof, int32_t nbin,
                          int32_t in_dtype, const void *data,
                          const double *model, const int32_t *model_index,
                          const double *noise, int32_t Ns, double lo,
                          double hi, double *out, void *stream);

/* Maximum-likelihood channel amplitudes at given parameters:
 * pptoaslib.get_scales_full (pptoaslib.py:953-971), a_n = C_n / S_n with
 * S_n = sum_k |B_nk|^2 |M_nk|^2 / e_n^2 (Sbp) and
 * C_n = Re sum_k D_nk conj(M_nk) conj(B_nk) exp(2 pi i k phi_n) / e_n^2 (Cdbp),
 * phi_n = phase_shifts(phi, DM, GM, nu_n, nu_DM, nu_GM, P), B the one-sided
 * exponential scattering FT at tau_n = tau (nu_n / nu_tau)^alpha
 * (10**tau with log10_tau).  D: [nsub][nchan][nharm] complex (re, im pairs);
 * M: [nmodel][nchan][nharm] complex with model_index[nsub] (NULL -> 0);
 * errs_FT: [nsub][nchan] or NULL; params: [nsub][5]; P: [nsub];
 * freqs: [nsub][nchan]; nus: [nsub][3] = nu_DM, nu_GM, nu_tau;
 * out: [nsub][nchan]. */
int ppf_scales_batch(ppf_ctx *ctx, int32_t nsub, int32_t nchan, int32_t nharm, const double *D,
                     const double *M, const int32_t *model_index, const double *errs_FT,
                     const double *params, const double *P, const double *freqs, const double *nus,
                     int32_t log10_tau, double *out, void *stream);

/* PSRCHIVE-free PSRFITS fast path (pulseportraiture_amd/psrfits.py; replaces
 * the unpacking, baseline removal, pscrunch and per-profile statistics of
 * pplib.load_data, pplib.py:2749-2915, for fold-mode PSRFITS): raw SUBINT
 * DATA bytes as stored in the file (big-endian; elem 0 = int16, 1 = uint8,
 * 2 = float32; 3 = native little-endian float32 rows, load_data's second
 * statistics pass over dedispersed / tscrunched rows), one block of sub_stride bytes per sub-int holding
 * [npol][nchan][nbin] samples (at least the pols used: 1, or 2 with
 * pol_mode 1; scl / offs still index all npol), become float32 rows
 *   out[s][n][b] = sum_p (DATA * DAT_SCL + DAT_OFFS)   (float32 arithmetic)
 * over p = pol 0 (pol_mode 0: npol 1 or IQUV's I) or pols 0 + 1 (pol_mode 1:
 * AA+BB / AABBCRCI).  The baseline window of each sub-int is the circular
 * window of rint(0.15 nbin) bins with the smallest sum of the weighted
 * total profile (PSRCHIVE's default BaselineWindow); with rm_baseline its
 * mean is subtracted from every row.  scl, offs: float32 [nsub][npol*nchan];
 * wts: float32 [nsub][nchan] or NULL; stats: [nsub][nchan][3] = off-pulse
 * mean, off-pulse sigma, S/N (on-pulse sum / (sigma sqrt(n_on)));
 * total: [nsub][nbin] weighted total profiles; wstart: int32 [nsub] window
 * starts.  Any nbin >= 2.  workspace: ppf_unpack_workspace_bytes(). */
size_t ppf_unpack_workspace_bytes(int32_t nsub, int32_t nchan, int32_t nbin);
int ppf_unpack_psrfits_batch(ppf_ctx *ctx, int32_t nsub, int32_t npol, int32_t nchan, int32_t nbin,
                             int32_t elem, const void *raw, int64_t sub_stride, const float *scl,
                             const float *offs, const float *wts, int32_t pol_mode,
                             int32_t rm_baseline, float *out, double *stats, double *total,
                             int32_t *wstart, void *workspace, size_t workspace_bytes,
                             void *stream);

/* nbytes from page-locked host memory src (a pinned buffer: hipHostMalloc /
 * torch pin_memory) to device memory dst, read by a kernel over PCIe on
 * stream instead of by a copy engine.  GetTOAs stages each archive's fit
 * inputs (engine._stage_host: the per-sub-int arrays of the reference's
 * fit_portrait_full calls, pptoas.py:530-533) this way, so they never wait
 * behind the archive uploads the copy engines are busy with.  Both pointers
 * 16-byte aligned; src must stay untouched until the stream has passed the
 * copy. */
int ppf_copy_from_pinned(ppf_ctx *ctx, void *dst, const void *src, int64_t nbytes, void *stream);

/* Positioned reads of the PSRFITS DATA column into host memory (the file
 * side of the fast path above; psrfits.PSRFITS.read_data_into): for each of
 * nrows rows, nbytes bytes at file offset offset + r * row_stride go to
 * dst + r * dst_stride.  The rows are cut into pieces of at most 4 MiB that
 * nthreads threads (1..64) take in turn with pread(2); the call returns when
 * every piece is in (dst is typically a page-locked upload buffer).  No
 * device and no context: PPF_OK, PPF_EINVAL (bad arguments) or PPF_EIO (a
 * read failed or hit end of file). */
int ppf_read_rows(int32_t fd, int64_t offset, int64_t row_stride, int64_t nbytes,
                  int64_t nrows, void *dst, int64_t dst_stride, int32_t nthreads);

/* Parallel host memcpy (ABI 4): nbytes from src to dst in 4-MiB pieces taken
 * in turn by nthreads threads (1..64).  GetTOAs stages in-memory archives
 * (pageable numpy rows) into its page-locked upload buffers with it
 * (pptoas._Stager; the reference hands the rows to fit_portrait_full
 * directly, pptoas.py:530-533).  Host memory only: PPF_OK or PPF_EINVAL. */
int ppf_host_copy(void *dst, const void *src, int64_t nbytes, int32_t nthreads);

/* Gaussian-component model portraits: pplib.gen_gaussian_portrait
 * (pplib.py:886-963, join_ichans = []) as called by pplib.read_model
 * (pplib.py:2971-3057) for every sub-integration of GetTOAs.get_TOAs
 * (pptoas.py:392-419) and get_narrowband_TOAs.  One launch builds nport
 * portraits (one per distinct frequency set), each row by
 * gen_gaussian_profile / gaussian_profile (pplib.py:801-883) and, when
 * tau != 0, convolved with scattering_portrait_FT (pplib.py:4245-4260).
 * model_code: 3 chars '0' (power law) / '1' (linear) for loc, wid, amp
 * (anything else: PPF_EINVAL, the reference's KeyError).  params:
 * [nport][2 + 6*ngauss] = DC, tau [bin], then per component loc, m_loc,
 * wid, m_wid, amp, m_amp; scattering_index, nu_ref: [nport];
 * freqs: [nport][nchan]; out: [nport][nchan][nbin] f64 (device).
 * Rows past the LDS transforms (even nbin > 8192, odd > 4095; nbin ≤
 * 19,200, the row in LDS): built per bin, a scattered model's convolution
 * then on the long transforms (synchronous; PPF_EUNSUP for a scattered
 * model at odd nbin there). */
int ppf_gauss_portrait_batch(ppf_ctx *ctx, int32_t nport, int32_t nchan, int32_t nbin,
                             int32_t ngauss, const char *model_code, const double *params,
                             const double *scattering_index, const double *freqs,
                             const double *nu_ref, double *out, void *stream);

/* Spline (PCA + B-spline) model portraits: pplib.gen_spline_portrait
 * (pplib.py:966-990) as called by pplib.read_spline_model (pplib.py:3060-3096)
 * from pptoas.GetTOAs.get_TOAs (pptoas.py:416-419) for make_spline_model
 * templates.  Per (portrait, channel): the B-spline curve (knots[nknots],
 * coefs[ncomp][nknots] -- splprep's c arrays, zero-padded --, degree
 * <= 5) evaluated at freqs[p][n] as FITPACK splev (ext = 0), expanded on
 * eigvec [nbin_model][ncomp] plus mean_prof [nbin_model]; ncomp = 0 tiles
 * mean_prof.  nbin != nbin_model: scipy.signal.resample to nbin, then the
 * reference's half-bin rotate_portrait.  nbin == nbin_model: any length;
 * resampled: both even in [32, 8192] on the LDS transforms (round 6: any
 * such length, was powers of two; else PPF_EUNSUP); ncomp <= 64.
 * out: [nport][nchan][nbin] f64 (device). */
int ppf_spline_portrait_batch(ppf_ctx *ctx, int32_t nport, int32_t nchan, int32_t nbin_model,
                              int32_t nbin, int32_t ncomp, int32_t nknots, int32_t degree,
                              const double *mean_prof, const double *eigvec,
                              const double *knots, const double *coefs, const double *freqs,
                              double *out, void *stream);

/* Synthetic sub-integrations for benchmarks/tests (make_fake_pulsar minus
 * PSRCHIVE, pplib.py:3355-3493): out[s][n] = rotate(model[n], -phi[s],
 * -DM[s], P[s], freqs[n], nu_ref) + N(0, noise) with a counter-based RNG
 * keyed by (seed, first_sub + s, n), so a sub-integration's data do not
 * depend on how a job is sharded.  model: [nchan][nbin]; out: [nsub][nchan][nbin]
 * in out_dtype. */
int ppf_synth_batch(ppf_ctx *ctx, int32_t nsub, int32_t nchan, int32_t nbin,
                    const double *model, const double *freqs,
                    const double *phi, const double *DM, const double *P,
                    double nu_ref, double noise, uint64_t seed,
                    int64_t first_sub, int32_t out_dtype, void *out,
                    void *stream);

/* Host-side (CPU) helper: real roots of a degree <= 8 polynomial, highest
 * power first, with np.roots semantics (companion-matrix eigenvalues with an
 * exactly zero imaginary part; pptoaslib.py:834-836, 902-904).  Returns the
 * root count or a negative value on failure.  The same code runs on the
 * device inside ppf_fit_batch; this export exists for CPU tests. */
int ppf_poly_real_roots_host(const double *coeffs, int deg, double *out);

/* Host-side (CPU) helper: the exact trust-region subproblem of the Newton
 * solver, min g.p + p.H p / 2 over |p| <= R for a symmetric n x n H
 * (row-major, n <= 5).  Writes p[n]; returns 1 if the step is on the
 * boundary, 0 if interior, negative on a bad argument.  The same code runs
 * on the device; this export exists for CPU tests. */
int ppf_tr_subproblem_host(const double *H, const double *g, int n, double R, double *p);

#ifdef __cplusplus
}
#endif
#endif /* PPFIT_H */
