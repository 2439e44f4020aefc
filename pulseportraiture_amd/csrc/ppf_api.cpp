// ppf_api.cpp -- C ABI of libppfit (include/ppfit.h): validation, workspace
// carving, twiddle-table cache and kernel sequencing.  No compute here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/ppfit.h"
#include "ppf_internal.hpp"
#include "ppf_device.hpp"

struct ppf_ctx {
    int device;
    std::string err;               // last error message, guarded by err_mu
    mutable std::mutex err_mu;
    std::map<int, double2 *> tw;   // nbin -> [T (N) | T2 (N)]
    std::map<std::pair<int, int>, double2 *> cz;   // (Ns, Kmax) -> chirp z-transform tables
    std::mutex tw_mu;              // guards tw and cz (calls from several host threads)
    bool prof = false;
    static constexpr int kRing = 256;
    // [0..4]: stage boundaries; [5, 6]: the first moment pass (k_xmom_g,
    // FULL); [7, 8]: the guess-profile pass (k_dsum_w)
    static constexpr int kEv = 9;
    hipEvent_t ring[kRing][kEv] = {};
    bool ran[kRing][6] = {};
    // every streaming pass (k_pass) of a call: its (start, end) event pairs,
    // the pool grown on demand and reused by the ring slot
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pass_ev[kRing];
    int npass[kRing] = {};
    // the solver kernels of a call (kind 0 k_tr_mom, 1 k_tr_step (+ gates),
    // 2 k_postfit): (start, end) pairs, as pass_ev
    std::vector<std::pair<hipEvent_t, hipEvent_t>> solv_ev[kRing];
    std::vector<int> solv_kind[kRing];
    int nsolv[kRing] = {};
    long ncalls = 0;
    unsigned *host_active = nullptr;   // pinned, for the iteration loop
    // device scratch of the long-row FFTFIT (ppf_phase_shift_batch past the
    // LDS transforms; grown on demand, held for the whole synchronous call)
    void *lscr = nullptr;
    size_t lscr_bytes = 0;
    std::mutex lscr_mu;
};

namespace {

int fail(ppf_ctx *ctx, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) {
        std::lock_guard<std::mutex> lk(ctx->err_mu);
        ctx->err = buf;
    }
    return code;
}

int hip_fail(ppf_ctx *ctx, hipError_t e, const char *where) {
    return fail(ctx, PPF_EHIP, "%s: %s", where, hipGetErrorString(e));
}

bool pow2_in_range(int nbin) {
    return nbin >= 32 && nbin <= 8192 && (nbin & (nbin - 1)) == 0;
}

// nbin the FFT kernels take: even 32..8192 and odd 33..4095 (power-of-two
// nbin on the register / radix-4 paths, the others on the mixed-radix LDS
// FFT, whose generic-radix stage takes prime factors above 7; odd nbin as a
// full-length complex transform of the row, ppf::rfft_len)
bool nbin_supported(int nbin) {
    return nbin >= 32 && nbin <= 8192 && ppf::fft_len_supported(ppf::rfft_len(nbin));
}

// log2 of a power-of-two FFT length, 0 otherwise (the kernels' "not a power
// of two" marker: no wave-FFT path, mixed-radix LDS FFT)
int fft_log2(int n) {
    if (n < 1 || (n & (n - 1))) return 0;
    int l = 0;
    while ((1 << l) < n) ++l;
    return l;
}

// fft_log2 of the real-row transform: 0 (mixed-radix LDS FFT) for odd nbin
int rfft_log2(int nbin) { return (nbin & 1) ? 0 : fft_log2(nbin / 2); }

int ilog2(int n) {
    int l = 0;
    while ((1 << l) < n) ++l;
    return l;
}

// get_noise_PS cut: int((1 - frac**-1) * nharm)  (pplib.py:2330)
int noise_kc(int nharm, int frac) {
    return (int)((1.0 - std::pow((double)frac, -1.0)) * (double)nharm);
}

int twiddles(ppf_ctx *ctx, int nbin, hipStream_t st, const double2 **T, const double2 **T2) {
    std::lock_guard<std::mutex> lock(ctx->tw_mu);
    auto it = ctx->tw.find(nbin);
    if (it == ctx->tw.end()) {
        const int N = ppf::rfft_len(nbin);
        double2 *p = nullptr;
        hipError_t e = hipMalloc(&p, sizeof(double2) * 2 * (size_t)N);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc(twiddles)");
        e = ppf::launch_twiddles(N, p, p + N, st);
        if (e != hipSuccess) return hip_fail(ctx, e, "k_twiddles");
        // the table is cached for calls on ANY stream: finish it before it
        // is published (one-time cost per nbin)
        e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize(twiddles)");
        it = ctx->tw.emplace(nbin, p).first;
    }
    *T = it->second;
    *T2 = it->second + ppf::rfft_len(nbin);
    return PPF_OK;
}

// A small device -> pinned-host read-back the iteration loop waits on (round
// 6).  hipStreamSynchronize wakes the host 30-70 us after the copy lands
// (C4's kernel trace: the gaps before the re-centring k_xmom_g and before
// k_postfit); with PPF_OPT_SPIN_WAIT the words are instead preset to a
// sentinel no count takes and polled until the copy has overwritten them,
// with the stream synchronisation as the fallback after 2 s.  Opt-in: on
// GetTOAs' threaded host pipeline the polling cost 20 % of the PSRFITS rate
// even yielding the core (profiles/r06/ab_gtspin_status.txt).
#ifndef PPF_SPIN_WAIT
#define PPF_SPIN_WAIT 1
#endif
constexpr unsigned kUnset = 0xFFFFFFFFu;
int read_back(ppf_ctx *ctx, unsigned *host, const unsigned *dev, int n, hipStream_t st, bool spin) {
    volatile unsigned *h = host;
    for (int i = 0; i < n; ++i) h[i] = kUnset;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipError_t e = hipMemcpyAsync(host, dev, n * sizeof(unsigned), hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipMemcpyAsync");
    if (PPF_SPIN_WAIT && spin) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            bool done = true;
            for (int i = 0; i < n; ++i) done = done && h[i] != kUnset;
            if (done) {
                std::atomic_thread_fence(std::memory_order_seq_cst);
                return PPF_OK;
            }
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::seconds(2)) break;
            // past the first 50 us the core is offered to other host threads
            // between polls (GetTOAs' readers and stagers share the CPUs)
            if (dt > std::chrono::microseconds(50)) std::this_thread::yield();
            else __builtin_ia32_pause();
        }
    }
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
    return PPF_OK;
}

// The guess's brute grid of a whole turn with Ns >= 512 points (ppalign:
// Ns = nbin) as a chirp z-transform (k_guess, round 6): the plan and its
// cached kernel tables.  Returns false (direct sums) where it does not apply.
// (Round 6, first build: P was taken >= 2K - 1 = 1025, i.e. 2048, which
// cz_fft refuses, so the A/B of ab_czc4_status.txt ran the direct sums on
// both sides.)
#ifndef PPF_GUESS_CZ
#define PPF_GUESS_CZ 1
#endif
bool cz_plan(int Ns, int K, ppf::CzPlan &c) {
    if (!PPF_GUESS_CZ || Ns < 2 * ppf::kBlock || K < 2) return false;
    // P >= K + J - 1 with chunks of J >= 256 outputs (nbin 1024: K = 513,
    // P = 1024, two chunks of 512)
    int P = 64;
    while (P < K + 255) P *= 2;
    if (P < 512 || P > 2048) return false;       // k_guess's instantiations (nbin 512-2048)
    c.Ns = Ns; c.K = K; c.P = P; c.J = P - K + 1; c.Q = (Ns + c.J - 1) / c.J;
    return true;
}
int cz_tables(ppf_ctx *ctx, const ppf::CzPlan &c, hipStream_t st, const double2 **B, const double2 **T) {
    const double2 *T2;
    int rc = twiddles(ctx, 2 * c.P, st, T, &T2);
    if (rc) return rc;
    std::lock_guard<std::mutex> lock(ctx->tw_mu);
    const auto key = std::make_pair(c.Ns, c.K);
    auto it = ctx->cz.find(key);
    if (it == ctx->cz.end()) {
        double2 *p = nullptr;
        hipError_t e = hipMalloc(&p, sizeof(double2) * (size_t)c.Q * c.P);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc(cz)");
        e = ppf::launch_cz_table(c, p, *T, st);
        if (e != hipSuccess) return hip_fail(ctx, e, "k_cz_table");
        // cached for calls on any stream (as the twiddles)
        e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize(cz)");
        it = ctx->cz.emplace(key, p).first;
    }
    *B = it->second;
    return PPF_OK;
}

// 16-moment sets on the non-power-of-two shapes too (their moments always
// come from X): nbin 1000 278-280k -> 293-294k, 1536 178-179k -> 183k fits/s
// in one call (profiles/r05/ab_m16_status.txt)
#ifndef PPF_MOM16_BLOCK
#define PPF_MOM16_BLOCK 1
#endif
struct FitLayout {
    size_t M, X, chan, stats, x0, gP, gw, nuref, Msum, gpart, gwx, gflag, state, partials, active, mom, dphi,
        mres, hcen, Mpow, MP, KC, needx, xslot, rclist, Bt, total;
    // rows past the LDS transforms (round 6): their rFFTs (data spectra,
    // long-transform chirp tables and work rows, rows per chunk)
    int lng;
    size_t spec, lchirp, lA, lY, gprof, gspec, gsh;
    int64_t lrows;
    int nblk, cb, cbd, nblkd;
    int fused;    // phase+DM fits on the fused moment pass (k_xmom_g), X only for scattering fits
    int momx;     // wave shapes, PPF_OPT_MOM_X: every fit's moments from X (k_xspec_w + k_moments)
    int xcap;     // X slots
};

// 16 moments about each wave's band centre where the moments come from a
// stored X and that was measured to pay (ab_m16_status.txt): the wave
// shapes' MOM_X path and (PPF_MOM16_BLOCK) the non-power-of-two nbin.
// Power-of-two nbin off the wave shapes (32-128, 4096, 8192) and block sizes
// the wave kernels refuse keep 32 moments about the global centre (radius
// 4.5 instead of 0.73, so fewer re-centring passes).
static bool mom16_layout(const FitLayout &L, int nbin) {
    return L.momx || (!L.fused && PPF_MOM16_BLOCK && !ppf::is_pow2(ppf::rfft_len(nbin)));
}


size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

bool bluestein_plan(int64_t nbin, int64_t n, bool packed, ppf::LongNoiseArgs &a);

// fits at nbin past the LDS transforms (even > 8192, odd > 4095): the rows'
// rFFTs on the long transforms, then the X-based fit.  With the GetTOAs
// guess the profile's spectrum (N + 1 harmonics) sits in one workgroup's
// LDS (nbin up to ~19,000); its brute grid too where it fits, else in
// global memory (grid_gsh: ppalign's Ns = nbin)
//
// grid_gsh: whether the FFTFIT brute grid of Ns points leaves the LDS for
// global memory ([rows][Ns + 8] doubles): the spectrum (N + 2 bins), the
// rFFT buffer of the LDS transforms (none for long rows, whose spectra come
// from the long transforms) and the grid past 150 KB.  ppalign at nbin 8192
// (Ns = nbin: 197 KB) and past.
bool grid_gsh(int nbin, int Ns, bool lng) {
    const size_t fb = lng ? 0 : (size_t)ppf::rfft_len(nbin) * sizeof(double2);
    return fb + ((size_t)nbin / 2 + 2) * sizeof(double2) + (size_t)(Ns + 8) * sizeof(double) > 150u * 1024u;
}
bool long_fit_ok(const ppf_fit_desc *d) {
    ppf::LongNoiseArgs f;
    if (d->guess && ((size_t)d->nbin / 2 + 2) * sizeof(double2) > 150u * 1024u) return false;
    return !nbin_supported(d->nbin) && d->nbin > 4095 &&
           bluestein_plan(d->nbin, (d->nbin & 1) ? d->nbin : d->nbin / 2, !(d->nbin & 1), f);
}

FitLayout fit_layout(const ppf_fit_desc *d) {
    FitLayout L{};
    const size_t nharm = (size_t)d->nbin / 2 + 1;
    const size_t nsub = (size_t)d->nsub, nchan = (size_t)d->nchan;
    L.cb = d->nchan < 32 ? d->nchan : 32;
    L.nblk = (d->nchan + L.cb - 1) / L.cb;
    L.fused = ppf::xspec_wave_supported(rfft_log2(d->nbin), L.cb) ? 1 : 0;
    // moments from X: on request, or by default where the GetTOAs guess is
    // fused into the spectrum pass (1024-point rows): there the X pass
    // replaces both the guess pass (k_dsum) and k_xmom_g's re-FFT
    const bool mom_auto = d->guess && rfft_log2(d->nbin) == 10;
    L.momx = (L.fused && !(d->options & PPF_OPT_FUSED_MOM) &&
              ((d->options & PPF_OPT_MOM_X) || mom_auto)) ? 1 : 0;
    L.xcap = (L.fused && d->x_subints > 0 && d->x_subints < d->nsub) ? d->x_subints : d->nsub;
    if (L.fused && (d->options & PPF_OPT_NO_X)) L.xcap = 0;
    if (L.momx) L.xcap = d->nsub;
    L.cbd = d->nchan < 128 ? d->nchan : 128;          // k_dsum channel block
    L.nblkd = (d->nchan + L.cbd - 1) / L.cbd;
    size_t o = 0;
    L.M = o;     o += align256(sizeof(double2) * (size_t)(d->nmodel > 0 ? d->nmodel : 1) * nchan * nharm);
    L.X = o;     o += align256(sizeof(double2) * (size_t)L.xcap * nchan * nharm);
    L.chan = o;  o += align256(sizeof(double) * nsub * nchan * 4);
    L.stats = o; o += align256(sizeof(double) * nsub * 2 * nchan * 10);
    L.x0 = o;    o += align256(sizeof(double) * nsub * 8);
    L.state = o; o += align256(ppf::tr_state_bytes() * nsub);
    L.partials = o; o += align256(sizeof(double) * nsub * (size_t)ppf::pass_blocks(d->nchan) * 21);
    L.active = o; o += 256;
    L.mom = o;   o += align256(sizeof(double2) * nsub * 2 * nchan * (size_t)ppf::kMoments);
    L.dphi = o;  o += align256(sizeof(double) * nsub * nchan * 2);
    L.mres = o;  o += align256(sizeof(double) * nsub * 2 * nchan);
    L.hcen = o;  o += mom16_layout(L, d->nbin) ? align256(sizeof(double) * nsub * 2 * nchan) : 0;
    L.Mpow = o;  o += align256(sizeof(double) * (size_t)(d->nmodel > 0 ? d->nmodel : 1) * nchan);
    L.MP = o;    o += align256(sizeof(double) * (size_t)(d->nmodel > 0 ? d->nmodel : 1) * nchan * nharm);
    L.KC = o;    o += align256(sizeof(int32_t) * (size_t)(d->nmodel > 0 ? d->nmodel : 1) * nchan);
    L.needx = o; o += align256(nsub);
    L.xslot = o; o += align256(sizeof(int32_t) * nsub);
    L.rclist = o; o += align256(sizeof(int32_t) * nsub);
    L.Bt = o;    o += align256(sizeof(double) * (nharm - 1) / 2 * 16);
    if (d->guess) {
        L.gP = o; o += align256(sizeof(double) * nsub * (size_t)L.nblkd * (size_t)d->nbin);
        L.gw = o; o += align256(sizeof(double) * nsub * (size_t)L.nblkd * 2);
        L.nuref = o; o += align256(sizeof(double) * nsub);
        L.Msum = o; o += align256(sizeof(double2) * (size_t)(d->nmodel > 0 ? d->nmodel : 1) * nharm);
        if (L.fused) {   // guess spectrum fused into k_xspec_w (k_gflag)
            const size_t ng = (size_t)ppf::guess_slots(rfft_log2(d->nbin));
            L.gpart = o; o += align256(sizeof(double2) * nsub * (size_t)L.nblk * ng);
            L.gwx = o;   o += align256(sizeof(double) * nsub * (size_t)L.nblk * 3);
            L.gflag = o; o += align256(nsub);
        }
    }
    L.lng = long_fit_ok(d) ? 1 : 0;
    if (L.lng) {
        ppf::LongNoiseArgs f;
        bluestein_plan(d->nbin, (d->nbin & 1) ? d->nbin : d->nbin / 2, !(d->nbin & 1), f);
        const size_t row_b = (size_t)f.M * sizeof(double2);
        const int64_t rows = (int64_t)(nsub > (size_t)(d->nmodel > 0 ? d->nmodel : 1) ? nsub
                                       : (size_t)(d->nmodel > 0 ? d->nmodel : 1)) * (int64_t)nchan;
        int64_t rc = (int64_t)((size_t)(256u << 20) / (2 * row_b));
        if (rc < 1) rc = 1;
        L.lrows = rows < rc ? rows : rc;
        L.spec = o;   o += align256(sizeof(double2) * nsub * nchan * nharm);
        if (d->guess) {
            L.gprof = o; o += align256(sizeof(double) * nsub * (size_t)d->nbin);
            L.gspec = o; o += align256(sizeof(double2) * nsub * nharm);
        }
        L.lchirp = o; o += align256(2 * row_b);
        L.lA = o;     o += align256((size_t)L.lrows * row_b);
        L.lY = o;     o += align256((size_t)L.lrows * row_b);
    }
    if (d->guess && grid_gsh(d->nbin, d->guess_Ns, L.lng)) {
        L.gsh = o; o += align256(sizeof(double) * nsub * ((size_t)d->guess_Ns + 8));
    }
    L.total = o;
    return L;
}

// the rFFTs of nrows real rows of nbin samples on the long transforms into
// out[row][k], k <= nbin / 2 (Bluestein; the chirp table once per call)
int long_rfft_rows(ppf_ctx *ctx, const FitLayout &L, char *ws, int64_t nbin, int64_t nrows, int dtype,
                   const void *in, double2 *out, bool chirp_ready, hipStream_t st) {
    ppf::LongNoiseArgs f;
    if (!bluestein_plan(nbin, (nbin & 1) ? nbin : nbin / 2, !(nbin & 1), f))
        return fail(ctx, PPF_EUNSUP, "nbin=%lld", (long long)nbin);
    const double2 *T1, *T2, *unused;
    int rc;
    if ((rc = twiddles(ctx, (int)(2 * f.M1), st, &T1, &unused))) return rc;
    if ((rc = twiddles(ctx, (int)(2 * f.M2), st, &T2, &unused))) return rc;
    double2 *Bf = (double2 *)(ws + L.lchirp);
    hipError_t e;
    if (!chirp_ready && (e = ppf::launch_chirp_ft(f, Bf, Bf + f.M, T1, T2, st)) != hipSuccess)
        return hip_fail(ctx, e, "k_lf_chirp");
    f.in_dtype = dtype;
    f.in = in;
    for (int64_t r0 = 0; r0 < nrows; r0 += L.lrows) {
        f.row0 = r0;
        const int64_t nr = nrows - r0 < L.lrows ? nrows - r0 : L.lrows;
        if ((e = ppf::launch_rfft_long(f, nr, (double2 *)(ws + L.lA), (double2 *)(ws + L.lY), Bf, out, T1, T2,
                                       st)) != hipSuccess)
            return hip_fail(ctx, e, "k_lr_spec");
    }
    return PPF_OK;
}

int check_fit_desc(ppf_ctx *ctx, const ppf_fit_desc *d) {
    if (!d) return fail(ctx, PPF_EINVAL, "null descriptor");
    if (d->nsub < 1 || d->nchan < 1) return fail(ctx, PPF_EINVAL, "nsub=%d nchan=%d", d->nsub, d->nchan);
    if (!nbin_supported(d->nbin) && !long_fit_ok(d))
        return fail(ctx, PPF_EUNSUP,
                    "nbin=%d: must be even in [32, 8192] or odd in [33, 4095], or longer without the "
                    "GetTOAs guess (up to 2^23 transform points)", d->nbin);
    if (d->data_dtype != PPF_F32 && d->data_dtype != PPF_F64)
        return fail(ctx, PPF_EINVAL, "data_dtype=%d", d->data_dtype);
    if (d->nmodel < 1) return fail(ctx, PPF_EINVAL, "nmodel=%d", d->nmodel);
    if (!d->data || !d->model || !d->freqs || !d->P || !d->init || !d->fit_flags || !d->nu_fits ||
        !d->nu_outs || !d->results || !d->scales || !d->scale_errs || !d->channel_snrs ||
        !d->covariance)
        return fail(ctx, PPF_EINVAL, "required pointer is NULL");
    if (d->mode != PPF_MODE_FULL && d->mode != PPF_MODE_LEGACY2)
        return fail(ctx, PPF_EINVAL, "mode=%d", d->mode);
    if (d->guess) {
        if (!d->guess_weights || !d->guess_DM) return fail(ctx, PPF_EINVAL, "guess needs weights and DM");
        if (d->guess_Ns < 1 || d->guess_Ns > 65536) return fail(ctx, PPF_EINVAL, "guess_Ns=%d", d->guess_Ns);
    }
    if (!d->workspace) return fail(ctx, PPF_EINVAL, "workspace is NULL");
    FitLayout L = fit_layout(d);
    if (d->workspace_bytes < L.total)
        return fail(ctx, PPF_ENOMEM, "workspace %zu < %zu bytes", d->workspace_bytes, L.total);
    return PPF_OK;
}

}  // namespace

extern "C" {

int ppf_abi_version(void) { return PPF_ABI_VERSION; }
size_t ppf_sizeof_fit_desc(void) { return sizeof(ppf_fit_desc); }
size_t ppf_sizeof_result(void) { return sizeof(ppf_result); }

int ppf_create(int device, ppf_ctx **out) {
    if (!out) return PPF_EINVAL;
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return PPF_EHIP;
    if (device < 0 || device >= n) return PPF_EINVAL;
    ppf_ctx *c = new ppf_ctx();
    c->device = device;
    *out = c;
    return PPF_OK;
}

void ppf_destroy(ppf_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    for (auto &kv : ctx->tw) (void)hipFree(kv.second);
    for (auto &kv : ctx->cz) (void)hipFree(kv.second);
    for (auto &set : ctx->ring)
        for (auto &e : set)
            if (e) (void)hipEventDestroy(e);
    for (auto &v : ctx->pass_ev)
        for (auto &pr : v) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    for (auto &v : ctx->solv_ev)
        for (auto &pr : v) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    if (ctx->host_active) (void)hipHostFree(ctx->host_active);
    if (ctx->lscr) (void)hipFree(ctx->lscr);
    delete ctx;
}

int ppf_set_profiling(ppf_ctx *ctx, int enable) {
    if (!ctx) return PPF_EINVAL;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    if (enable && !ctx->ring[0][0])
        for (auto &set : ctx->ring)
            for (auto &ev : set)
                if ((e = hipEventCreate(&ev)) != hipSuccess) return hip_fail(ctx, e, "hipEventCreate");
    ctx->prof = enable != 0;
    ctx->ncalls = 0;
    return PPF_OK;
}

int ppf_stage_ms_history(ppf_ctx *ctx, int n, double *ms) {
    if (!ctx || !ms || n < 0) return PPF_EINVAL;
    if (!ctx->prof) return fail(ctx, PPF_EINVAL, "profiling is off");
    long avail = ctx->ncalls < ppf_ctx::kRing ? ctx->ncalls : ppf_ctx::kRing;
    if (n > avail) n = (int)avail;
    for (int c = 0; c < n; ++c) {
        int slot = (int)((ctx->ncalls - n + c) % ppf_ctx::kRing);
        hipError_t e = hipEventSynchronize(ctx->ring[slot][4]);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipEventSynchronize");
        for (int i = 0; i < 4; ++i) {
            float t = 0.f;
            if (ctx->ran[slot][i]) {
                e = hipEventElapsedTime(&t, ctx->ring[slot][i], ctx->ring[slot][i + 1]);
                if (e != hipSuccess) return hip_fail(ctx, e, "hipEventElapsedTime");
            }
            ms[c * 4 + i] = (double)t;
        }
    }
    return n;
}

int ppf_kernel_ms_history(ppf_ctx *ctx, int n, double *ms) {
    if (!ctx || !ms || n < 0) return PPF_EINVAL;
    if (!ctx->prof) return fail(ctx, PPF_EINVAL, "profiling is off");
    long avail = ctx->ncalls < ppf_ctx::kRing ? ctx->ncalls : ppf_ctx::kRing;
    if (n > avail) n = (int)avail;
    for (int c = 0; c < n; ++c) {
        int slot = (int)((ctx->ncalls - n + c) % ppf_ctx::kRing);
        hipError_t e = hipEventSynchronize(ctx->ring[slot][4]);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipEventSynchronize");
        for (int i = 0; i < 2; ++i) {
            float t = 0.f;
            if (ctx->ran[slot][4 + i]) {
                e = hipEventElapsedTime(&t, ctx->ring[slot][5 + 2 * i], ctx->ring[slot][6 + 2 * i]);
                if (e != hipSuccess) return hip_fail(ctx, e, "hipEventElapsedTime");
            }
            ms[c * 2 + i] = (double)t;
        }
    }
    return n;
}

int ppf_pass_ms_history(ppf_ctx *ctx, int n, double *ms) {
    if (!ctx || !ms || n < 0) return PPF_EINVAL;
    if (!ctx->prof) return fail(ctx, PPF_EINVAL, "profiling is off");
    long avail = ctx->ncalls < ppf_ctx::kRing ? ctx->ncalls : ppf_ctx::kRing;
    if (n > avail) n = (int)avail;
    for (int c = 0; c < n; ++c) {
        int slot = (int)((ctx->ncalls - n + c) % ppf_ctx::kRing);
        double tot = 0.0;
        for (int i = 0; i < ctx->npass[slot]; ++i) {
            const auto &pr = ctx->pass_ev[slot][i];
            hipError_t e = hipEventSynchronize(pr.second);
            if (e != hipSuccess) return hip_fail(ctx, e, "hipEventSynchronize");
            float t = 0.f;
            e = hipEventElapsedTime(&t, pr.first, pr.second);
            if (e != hipSuccess) return hip_fail(ctx, e, "hipEventElapsedTime");
            tot += (double)t;
        }
        ms[c * 2 + 0] = tot;
        ms[c * 2 + 1] = (double)ctx->npass[slot];
    }
    return n;
}

int ppf_solver_ms_history(ppf_ctx *ctx, int n, double *ms) {
    if (!ctx || !ms || n < 0) return PPF_EINVAL;
    if (!ctx->prof) return fail(ctx, PPF_EINVAL, "profiling is off");
    long avail = ctx->ncalls < ppf_ctx::kRing ? ctx->ncalls : ppf_ctx::kRing;
    if (n > avail) n = (int)avail;
    for (int c = 0; c < n; ++c) {
        int slot = (int)((ctx->ncalls - n + c) % ppf_ctx::kRing);
        double *o = ms + c * 6;
        for (int i = 0; i < 6; ++i) o[i] = 0.0;
        for (int i = 0; i < ctx->nsolv[slot]; ++i) {
            const auto &pr = ctx->solv_ev[slot][i];
            hipError_t e = hipEventSynchronize(pr.second);
            if (e != hipSuccess) return hip_fail(ctx, e, "hipEventSynchronize");
            float t = 0.f;
            e = hipEventElapsedTime(&t, pr.first, pr.second);
            if (e != hipSuccess) return hip_fail(ctx, e, "hipEventElapsedTime");
            const int k = ctx->solv_kind[slot][i];
            o[2 * k] += (double)t;
            o[2 * k + 1] += 1.0;
        }
    }
    return n;
}

int ppf_last_stage_ms(ppf_ctx *ctx, double *ms4) {
    int n = ppf_stage_ms_history(ctx, 1, ms4);
    if (n < 0) return n;
    return n == 1 ? PPF_OK : fail(ctx, PPF_EINVAL, "no profiled call yet");
}

const char *ppf_last_error(const ppf_ctx *ctx) {
    if (!ctx) return "null context";
    // a copy per calling thread: another thread's failure cannot rewrite the
    // buffer this pointer refers to
    thread_local std::string copy;
    std::lock_guard<std::mutex> lk(ctx->err_mu);
    copy = ctx->err;
    return copy.c_str();
}

size_t ppf_fit_workspace_bytes(const ppf_fit_desc *desc) {
    if (!desc || desc->nsub < 1 || desc->nchan < 1 || (!nbin_supported(desc->nbin) && !long_fit_ok(desc)))
        return 0;
    return fit_layout(desc).total;
}

int ppf_fit_batch(ppf_ctx *ctx, const ppf_fit_desc *d, void *stream) {
    if (!ctx) return PPF_EINVAL;
    int rc = check_fit_desc(ctx, d);
    if (rc) return rc;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    const FitLayout L = fit_layout(d);
    // (long rows: no LDS transform runs, so no twiddle table of nbin)
    const double2 *T = nullptr, *T2 = nullptr;
    if (!L.lng && (rc = twiddles(ctx, d->nbin, st, &T, &T2))) return rc;
    char *ws = (char *)d->workspace;
    double2 *Mft = (double2 *)(ws + L.M);
    const int nharm = d->nbin / 2 + 1;
    const int kc = noise_kc(nharm, 4);

    const int slot = (int)(ctx->ncalls % ppf_ctx::kRing);
    auto mark = [&](int i) {
        if (ctx->prof) (void)hipEventRecord(ctx->ring[slot][i], st);
    };
    for (int i = 0; i < 4; ++i) ctx->ran[slot][i] = true;
    ctx->npass[slot] = 0;
    ctx->nsolv[slot] = 0;
    // events around one solver launch (profiling only)
    auto solv_begin = [&](int kind) -> std::pair<hipEvent_t, hipEvent_t> * {
        if (!ctx->prof) return nullptr;
        auto &v = ctx->solv_ev[slot];
        auto &kv = ctx->solv_kind[slot];
        if ((int)v.size() <= ctx->nsolv[slot]) {
            std::pair<hipEvent_t, hipEvent_t> pr{};
            if (hipEventCreate(&pr.first) != hipSuccess) return nullptr;
            if (hipEventCreate(&pr.second) != hipSuccess) {
                (void)hipEventDestroy(pr.first);
                return nullptr;
            }
            v.push_back(pr);
            kv.push_back(0);
        }
        kv[ctx->nsolv[slot]] = kind;
        auto *pe = &v[ctx->nsolv[slot]++];
        (void)hipEventRecord(pe->first, st);
        return pe;
    };
    auto solv_end = [&](std::pair<hipEvent_t, hipEvent_t> *pe) {
        if (pe) (void)hipEventRecord(pe->second, st);
    };
    ctx->ran[slot][2] = d->guess != 0;
    ctx->ran[slot][4] = ctx->ran[slot][5] = false;
    mark(0);
    if (L.lng) {
        if ((rc = long_rfft_rows(ctx, L, ws, d->nbin, (int64_t)d->nmodel * d->nchan, PPF_F64, d->model, Mft,
                                 false, st)))
            return rc;
    } else {
        ppf::RfftArgs ra{d->nbin, rfft_log2(d->nbin), PPF_F64, d->model, T, T2, Mft};
        if ((e = ppf::launch_rfft_rows(ra, (int64_t)d->nmodel * d->nchan, st)) != hipSuccess)
            return hip_fail(ctx, e, "k_rfft_rows");
    }
    double *Mpow = (double *)(ws + L.Mpow);
    if ((e = ppf::launch_model_pow_t(Mft, d->nchan, nharm, d->nmodel, (double *)(ws + L.MP), st)) !=
        hipSuccess)
        return hip_fail(ctx, e, "k_model_pow_t");
    if ((e = ppf::launch_model_cut((const double *)(ws + L.MP), d->nchan, nharm, d->nmodel,
                                   (d->options & PPF_OPT_NO_HCUT) != 0, (int32_t *)(ws + L.KC),
                                   st)) != hipSuccess)
        return hip_fail(ctx, e, "k_model_cut");
    if ((e = ppf::launch_model_pow(Mft, d->nchan, nharm, d->nmodel, Mpow, st)) != hipSuccess)
        return hip_fail(ctx, e, "k_model_pow");
    // moment-mode sub-ints (no scattering) on the fused path never need the
    // cross spectrum in HBM: k_xmom_g re-FFTs their rows; k_classify marks
    // the others and gives each an X slot
    const int use_moments = 1;
    uint8_t *needx = (uint8_t *)(ws + L.needx);
    int32_t *xslot = (int32_t *)(ws + L.xslot);
    if ((e = ppf::launch_classify(d->nsub, d->fit_flags, d->init, d->log10_tau, L.fused && !L.momx, L.xcap,
                                  needx, xslot, st)) != hipSuccess)
        return hip_fail(ctx, e, "k_classify");
    // fused guess: the sub-ints k_xspec_w streams whose mean-model cutoff
    // fits its guess harmonics accumulate the guess spectrum there
    uint8_t *gflag = nullptr;
    if (d->guess && L.fused && ppf::xspec_guess_fused_n(rfft_log2(d->nbin))) {
        gflag = (uint8_t *)(ws + L.gflag);
        const int klim = 64 * ppf::guess_npl(rfft_log2(d->nbin));
        if ((e = ppf::launch_gflag(d->nsub, d->nchan, needx, (const int32_t *)(ws + L.KC),
                                   d->model_index, klim, gflag, st)) != hipSuccess)
            return hip_fail(ctx, e, "k_gflag");
    }
    mark(1);

    ppf::XspecArgs xa{};
    xa.nsub = d->nsub; xa.nchan = d->nchan; xa.nbin = d->nbin; xa.log2N = rfft_log2(d->nbin);
    xa.kc = kc; xa.nblk = L.nblk; xa.cb = L.cb; xa.dtype = d->data_dtype;
    // k_xspec_w: channel-block-major (mode 2) when the model spectra
    // outgrow the L2s, sub-int-major otherwise; k_xmom_g stages its model
    // row in LDS per workgroup and keeps mode 1
#ifndef PPF_XSPEC_ORDER2_BYTES
#define PPF_XSPEC_ORDER2_BYTES (32ll << 20)
#endif
    const long long model_bytes = (long long)d->nchan * (d->nbin / 2 + 1) * 16;
    const int xcd1 = (L.nblk % 8 == 0) ? 1 : 0;
    xa.xcd_swizzle = (xcd1 && model_bytes > PPF_XSPEC_ORDER2_BYTES) ? 2 : xcd1;
    xa.data = d->data; xa.Mft = Mft; xa.model_index = d->model_index; xa.mask = d->chan_mask;
    xa.errs = d->errs; xa.freqs = d->freqs; xa.P = d->P; xa.T = T; xa.T2 = T2;
    xa.X = (double2 *)(ws + L.X); xa.chan = (double *)(ws + L.chan);
    xa.Mpow = Mpow;
    xa.xslot = xslot;
    xa.gflag = gflag;
    if (gflag) {
        xa.gpart = (double2 *)(ws + L.gpart);
        xa.gw = (double *)(ws + L.gwx);
        xa.guess_weights = d->guess_weights;
        xa.guess_DM = d->guess_DM;
        xa.nu_fits = d->nu_fits;
        xa.guess_ref = d->guess_ref;
    }
    const bool wave = L.fused != 0;
    // fused moment pass (k_xmom) only on the wave-FFT shapes; elsewhere the
    // moments are taken from X (k_moments)
    const bool fused = wave && use_moments && !L.momx;
    xa.needx = (fused || L.momx) ? needx : nullptr;
    // fused: only k_pass reads X, and only below its channels' cutoffs;
    // momx: k_moments reads it below the same cutoffs
    // block-FFT path: only k_xspec_wm (the smooth non-power-of-two lengths)
    // uses it, writing X below the same cutoffs its readers stop at
    xa.KC = (fused || L.momx || !wave) ? (const int32_t *)(ws + L.KC) : nullptr;
    if (wave) {
        // (nothing to do when the caller has ruled out X: every sub-int is
        // fitted from k_xmom_g's moments)
        if (!(fused && L.xcap == 0) &&
            (e = ppf::launch_xspec_wave(xa, st)) != hipSuccess)
            return hip_fail(ctx, e, "k_xspec_w");
    } else if (L.lng) {
        double2 *spec = (double2 *)(ws + L.spec);
        if ((rc = long_rfft_rows(ctx, L, ws, d->nbin, (int64_t)d->nsub * d->nchan, d->data_dtype, d->data, spec,
                                 true, st)))
            return rc;
        xa.spec = spec;
        if ((e = ppf::launch_xspec_spec(xa, st)) != hipSuccess) return hip_fail(ctx, e, "k_xspec_spec");
    } else {
        if ((e = ppf::launch_xspec(xa, st)) != hipSuccess) return hip_fail(ctx, e, "k_xspec");
    }
    mark(2);

    if (d->guess) {
        // guess profile: time-domain dedispersion (k_dsum), then FFTFIT
        // against the mean model (k_guess)
        ppf::DsumArgs da{};
        da.nsub = d->nsub; da.nchan = d->nchan; da.nbin = d->nbin; da.dtype = d->data_dtype;
        da.cbd = L.cbd; da.nblkd = L.nblkd; da.data = d->data; da.mask = d->chan_mask;
        da.freqs = d->freqs; da.P = d->P; da.guess_DM = d->guess_DM;
        da.guess_weights = d->guess_weights;
        da.guess_ref = d->guess_ref; da.nu_fits = d->nu_fits;
        da.gP = (double *)(ws + L.gP); da.gw = (double *)(ws + L.gw);
        da.nuref = (double *)(ws + L.nuref);
        da.gflag = gflag;
        mark(7);
        if ((e = ppf::launch_dsum(da, st)) != hipSuccess) return hip_fail(ctx, e, "k_dsum");
        mark(8);
        ctx->ran[slot][5] = true;
        double2 *msum = (double2 *)(ws + L.Msum);
        if ((e = ppf::launch_model_sum(Mft, d->nchan, nharm, d->nmodel, msum, st)) != hipSuccess)
            return hip_fail(ctx, e, "k_model_sum");
        ppf::GuessArgs ga{};
        ga.nsub = d->nsub; ga.nchan = d->nchan; ga.nbin = d->nbin; ga.log2N = rfft_log2(d->nbin);
        ga.kc = kc; ga.nblkd = L.nblkd; ga.Ns = d->guess_Ns; ga.mask = d->chan_mask;
        ga.guess_ref = d->guess_ref;
        ga.freqs = d->freqs; ga.P = d->P; ga.guess_DM = d->guess_DM; ga.guess_tau = d->guess_tau;
        ga.nu_fits = d->nu_fits; ga.gP = da.gP; ga.gw = da.gw; ga.T = T; ga.T2 = T2;
        ga.KC = (const int32_t *)(ws + L.KC);
        ga.x0 = (double *)(ws + L.x0); ga.Msum = msum; ga.Mft = Mft;
        ga.model_index = d->model_index;
        ga.gflag = gflag;
        ga.gpart = xa.gpart;
        ga.gwx = xa.gw;
        ga.nblk = L.nblk;
        if (L.lng) {
            // the profiles' rFFTs on the long transforms (same plan as the rows)
            double *prof = (double *)(ws + L.gprof);
            double2 *gspec = (double2 *)(ws + L.gspec);
            if ((e = ppf::launch_gsum(d->nsub, L.nblkd, d->nbin, da.gP, prof, st)) != hipSuccess)
                return hip_fail(ctx, e, "k_gsum");
            if ((rc = long_rfft_rows(ctx, L, ws, d->nbin, d->nsub, PPF_F64, prof, gspec, true, st))) return rc;
            ga.gspec = gspec;
        }
        if (grid_gsh(d->nbin, ga.Ns, L.lng)) ga.gsh = (double *)(ws + L.gsh);
        ppf::CzPlan cz{};
        if (cz_plan(ga.Ns, d->nbin / 2 + 1, cz)) {
            if ((rc = cz_tables(ctx, cz, st, &ga.czB, &ga.czT))) return rc;
            ga.czP = cz.P; ga.czJ = cz.J; ga.czQ = cz.Q; ga.czK = cz.K;
        }
        if ((e = ppf::launch_guess(ga, st)) != hipSuccess) return hip_fail(ctx, e, "k_guess");
    }
    mark(3);

    ppf::SolveArgs sa{};
    sa.nsub = d->nsub; sa.nchan = d->nchan; sa.nbin = d->nbin;
    sa.X = xa.X; sa.Mft = Mft; sa.model_index = d->model_index; sa.chan = xa.chan;
    sa.MP = (const double *)(ws + L.MP);
    sa.KC = (const int32_t *)(ws + L.KC);
    sa.freqs = d->freqs; sa.P = d->P; sa.mask = d->chan_mask; sa.init = d->init;
    sa.fit_flags = d->fit_flags; sa.nu_fits = d->nu_fits; sa.nu_outs = d->nu_outs;
    sa.bounds = d->bounds;
    sa.log10_tau = d->log10_tau; sa.option = d->option; sa.is_toa = d->is_toa; sa.mode = d->mode;
    sa.max_iter = d->max_iter; sa.guess = d->guess; sa.x0 = (double *)(ws + L.x0);
    sa.newton = (d->options & PPF_OPT_SCIPY_TR) ? 0 : 1;
    sa.stats = (double *)(ws + L.stats); sa.results = d->results; sa.scales = d->scales;
    sa.scale_errs = d->scale_errs; sa.channel_snrs = d->channel_snrs; sa.covariance = d->covariance;
    sa.any_plain = 1;
    sa.any_scat = 1;
    sa.state = (ppf::TRState *)(ws + L.state);
    sa.partials = (double *)(ws + L.partials);
    sa.active = (unsigned *)(ws + L.active);
    sa.rc_count = sa.active + 1;             // reset together with active
    sa.rc_list = (int32_t *)(ws + L.rclist);
    sa.kinds = (unsigned *)(ws + L.active + 16);
    if (!ctx->host_active) {
        e = hipHostMalloc((void **)&ctx->host_active, 4 * sizeof(unsigned));
        if (e != hipSuccess) return hip_fail(ctx, e, "hipHostMalloc");
    }
    if ((e = hipMemsetAsync(sa.kinds, 0, 2 * sizeof(unsigned), st)) != hipSuccess)
        return hip_fail(ctx, e, "hipMemsetAsync");
    sa.moments = use_moments;
    sa.mom = (double2 *)(ws + L.mom);
    sa.dphi = (double *)(ws + L.dphi);
    sa.mres = (double *)(ws + L.mres);
    // 16 moments about each wave's band centre (mom16_layout)
    const bool m16 = mom16_layout(L, d->nbin);
    sa.mom16 = m16;
    sa.hcen = m16 ? (double *)(ws + L.hcen) : nullptr;
    sa.xslot = xslot;
    if (sa.moments) sa.any_plain = 0;      // plain fits go through the moments
    if ((e = ppf::launch_tr_init(sa, st)) != hipSuccess) return hip_fail(ctx, e, "k_tr_init");
    // how many fits iterate on the moments and how many on streaming passes:
    // the iteration loop launches only the kernels some fit needs.  With
    // PPF_OPT_NO_X the caller has ruled out every streaming fit (no X slot
    // exists), so the answer is known without the read-back and its stream
    // synchronisation (round 6: one host round trip less per call, a few
    // percent of a ppalign iteration); the moment kernels of a batch with
    // nothing left to fit exit at once
    bool any_mom = true, any_pass = false;
    if (!((d->options & PPF_OPT_NO_X) && sa.moments)) {
        if ((rc = read_back(ctx, ctx->host_active + 1, sa.kinds, 2, st, d->options & PPF_OPT_SPIN_WAIT))) return rc;
        any_mom = ctx->host_active[1] != 0;
        any_pass = ctx->host_active[2] != 0;
    }
    ppf::XmomArgs ma{};
    ma.nsub = d->nsub; ma.nchan = d->nchan; ma.nbin = d->nbin; ma.log2N = xa.log2N;
    ma.nblk = L.nblk; ma.cb = L.cb; ma.dtype = d->data_dtype; ma.xcd_swizzle = xcd1;
    ma.data = d->data; ma.Mft = Mft; ma.model_index = d->model_index; ma.mask = d->chan_mask;
    ma.chan = xa.chan; ma.dphi = sa.dphi; ma.T = T; ma.T2 = T2; ma.state = sa.state;
    ma.mom = (double *)sa.mom;
    ma.Bt = (const double *)(ws + L.Bt);
    ma.kc = kc; ma.errs = d->errs; ma.Mpow = Mpow; ma.mres = sa.mres; ma.nmodel = d->nmodel;
    ma.rc_count = sa.rc_count; ma.rc_list = sa.rc_list;
    ma.KC = (const int32_t *)(ws + L.KC);
    if (fused && (e = ppf::launch_btab(d->nbin / 2, (double *)(ws + L.Bt), st)) != hipSuccess)
        return hip_fail(ctx, e, "k_btab");
    // trust-region iterations.  Scattering fits: each iteration = one
    // streaming pass (k_pass) + one step (k_tr_step).  Other fits: k_moments
    // (re)centres the moment sets of the sub-ints that asked, k_tr_mom runs
    // iterations until the fit stops or leaves the expansion radius.  Groups
    // of rounds are queued without host synchronisation; the count of
    // sub-ints still needing work is read back between groups.
    const int maxiter = d->max_iter > 0 ? d->max_iter : 200 * 5;
    int iter = 0;
    // Moment-only batches read the counter after the first round: most
    // phase+DM fits finish inside it (C2: 1.0 data passes per fit), so the
    // empty re-centring launches that a longer first group would queue
    // are not worth the one synchronisation they save.
    for (int group = (sa.moments && !any_pass) ? 1 : (sa.moments ? 3 : 6); any_mom || any_pass;
         group = sa.moments ? 2 : 4) {
        for (int g = 0; g < group; ++g) {
            if (any_pass) {
                std::pair<hipEvent_t, hipEvent_t> *pe = nullptr;
                if (ctx->prof) {
                    auto &v = ctx->pass_ev[slot];
                    if ((int)v.size() <= ctx->npass[slot]) {
                        std::pair<hipEvent_t, hipEvent_t> pr{};
                        if ((e = hipEventCreate(&pr.first)) != hipSuccess)
                            return hip_fail(ctx, e, "hipEventCreate");
                        if ((e = hipEventCreate(&pr.second)) != hipSuccess) {
                            (void)hipEventDestroy(pr.first);
                            return hip_fail(ctx, e, "hipEventCreate");
                        }
                        v.push_back(pr);
                    }
                    pe = &v[ctx->npass[slot]++];
                    (void)hipEventRecord(pe->first, st);
                }
                if ((e = ppf::launch_pass(sa, st)) != hipSuccess) return hip_fail(ctx, e, "k_pass");
                if (pe) (void)hipEventRecord(pe->second, st);
            }
            if (sa.moments && any_mom) {
                const bool full = iter == 0 && g == 0;
                if (full) mark(5);
                if (fused && !full) {
                    // re-centring passes: usually few sub-ints, so 8-channel
                    // blocks (4x the workgroups, a quarter of the rounds
                    // each) keep more CUs busy; a channel's moments do not
                    // depend on its block
                    ppf::XmomArgs mr = ma;
                    if (mr.cb > 8) {
                        mr.cb = 8;
                        mr.nblk = (d->nchan + 7) / 8;
                        mr.xcd_swizzle = (mr.nblk % 8 == 0) ? 1 : 0;
                    }
                    e = ppf::launch_xmom(mr, false, st);
                } else {
                    e = fused ? ppf::launch_xmom(ma, full, st) : ppf::launch_moments(sa, st);
                }
                if (e != hipSuccess) return hip_fail(ctx, e, fused ? "k_xmom" : "k_moments");
                if (full) {
                    mark(6);
                    ctx->ran[slot][4] = true;
                }
            }
            if ((e = hipMemsetAsync(sa.active, 0, 2 * sizeof(unsigned), st)) != hipSuccess)
                return hip_fail(ctx, e, "hipMemsetAsync");
            if (any_pass) {
                auto *pe = solv_begin(1);
                if ((e = ppf::launch_tr_step(sa, st)) != hipSuccess) return hip_fail(ctx, e, "k_tr_step");
                solv_end(pe);
            }
            if (sa.moments && any_mom) {
                auto *pe = solv_begin(0);
                if ((e = ppf::launch_tr_mom(sa, st)) != hipSuccess) return hip_fail(ctx, e, "k_tr_mom");
                solv_end(pe);
            }
        }
        iter += group;
        if ((rc = read_back(ctx, ctx->host_active, sa.active, 1, st, d->options & PPF_OPT_SPIN_WAIT))) return rc;
        if (*ctx->host_active == 0 || iter > maxiter + 2) break;
    }
    {
        auto *pe = solv_begin(2);
        if ((e = ppf::launch_postfit(sa, st)) != hipSuccess) return hip_fail(ctx, e, "k_postfit");
        solv_end(pe);
    }
    mark(4);
    if (ctx->prof) ++ctx->ncalls;
    return PPF_OK;
}

int ppf_fit2_batch(ppf_ctx *ctx, const ppf_fit_desc *desc, void *stream) {
    if (!desc) return fail(ctx, PPF_EINVAL, "null descriptor");
    ppf_fit_desc d = *desc;
    d.mode = PPF_MODE_LEGACY2;
    return ppf_fit_batch(ctx, &d, stream);
}

static int rotate_batch(ppf_ctx *ctx, int64_t nrows, int32_t nbin, int32_t in_dtype, const void *in,
                        const double *phases, double *out, void *stream, bool ref_len) {
    if (!ctx) return PPF_EINVAL;
    if (!nbin_supported(nbin)) return fail(ctx, PPF_EUNSUP, "nbin=%d unsupported", nbin);
    if (nrows < 0 || (nrows > 0 && (!in || !phases || !out)))
        return fail(ctx, PPF_EINVAL, "bad rotate arguments");
    if (in_dtype != PPF_F32 && in_dtype != PPF_F64) return fail(ctx, PPF_EINVAL, "in_dtype");
    if (nrows == 0) return PPF_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    const double2 *T, *T2;
    int rc = twiddles(ctx, nbin, st, &T, &T2);
    if (rc) return rc;
    ppf::RotateArgs a{nbin, rfft_log2(nbin), in_dtype, in, phases, T, T2, out, 0, T, T2};
    if (ref_len && (nbin & 1)) {
        a.ref_len = 1;
        if ((rc = twiddles(ctx, nbin - 1, st, &a.Te, &a.T2e))) return rc;
    }
    if ((e = ppf::launch_rotate(a, nrows, st)) != hipSuccess) return hip_fail(ctx, e, "k_rotate");
    return PPF_OK;
}

int ppf_rotate_batch(ppf_ctx *ctx, int64_t nrows, int32_t nbin, int32_t in_dtype, const void *in,
                     const double *phases, double *out, void *stream) {
    return rotate_batch(ctx, nrows, nbin, in_dtype, in, phases, out, stream, false);
}

int ppf_rotate_batch_ref(ppf_ctx *ctx, int64_t nrows, int32_t nbin, int32_t in_dtype, const void *in,
                         const double *phases, double *out, void *stream) {
    return rotate_batch(ctx, nrows, nbin, in_dtype, in, phases, out, stream, true);
}

size_t ppf_align_workspace_bytes(int32_t nsub, int32_t nchan, int32_t nbin) {
    if (nsub <= 0 || nchan <= 0 || nbin <= 0) return 0;
    const size_t g = (size_t)ppf::align_groups(nsub, nchan);
    return align256(g * nchan * (size_t)(nbin / 2 + 1) * sizeof(double2)) +
           align256(g * nchan * sizeof(double));
}

int ppf_align_phases(ppf_ctx *ctx, int32_t nsub, int32_t nchan, const double *results, const double *freqs,
                     const double *P, const uint8_t *mask, const double *scales, const double *errs,
                     double *phases, double *weights, void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (nsub < 0 || nchan <= 0) return fail(ctx, PPF_EINVAL, "bad align shape");
    if (nsub == 0) return PPF_OK;
    if (!results || !freqs || !P || !scales || !errs || !phases || !weights)
        return fail(ctx, PPF_EINVAL, "null align_phases argument");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    if ((e = ppf::launch_align_phases(nsub, nchan, results, freqs, P, mask, scales, errs, phases, weights,
                                      (hipStream_t)stream)) != hipSuccess)
        return hip_fail(ctx, e, "k_align_phases");
    return PPF_OK;
}

int ppf_align_accum(ppf_ctx *ctx, int32_t nsub, int32_t nchan, int32_t nbin, int32_t in_dtype,
                    const void *in, const double *phases, const double *weights, double *out,
                    double *wsum, void *workspace, size_t workspace_bytes, void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (!nbin_supported(nbin)) return fail(ctx, PPF_EUNSUP, "nbin=%d unsupported", nbin);
    if (nsub < 0 || nchan <= 0) return fail(ctx, PPF_EINVAL, "bad align shape");
    if (in_dtype != PPF_F32 && in_dtype != PPF_F64) return fail(ctx, PPF_EINVAL, "in_dtype");
    if (nsub == 0) return PPF_OK;
    if (!in || !phases || !weights || !out || !wsum || !workspace)
        return fail(ctx, PPF_EINVAL, "null align argument");
    const size_t need = ppf_align_workspace_bytes(nsub, nchan, nbin);
    if (workspace_bytes < need)
        return fail(ctx, PPF_ENOMEM, "align workspace %zu < %zu bytes", workspace_bytes, need);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    const double2 *T, *T2;
    int rc = twiddles(ctx, nbin, st, &T, &T2);
    if (rc) return rc;
    ppf::AlignArgs a{};
    a.nsub = nsub; a.nchan = nchan; a.nbin = nbin; a.log2N = rfft_log2(nbin); a.dtype = in_dtype;
    a.ngroup = ppf::align_groups(nsub, nchan);
    a.in = in; a.phases = phases; a.weights = weights; a.T = T; a.T2 = T2;
    char *ws = (char *)workspace;
    a.part = (double2 *)ws;
    a.wpart = (double *)(ws + align256((size_t)a.ngroup * nchan * (size_t)(nbin / 2 + 1) *
                                        sizeof(double2)));
    a.out = out; a.wsum = wsum;
    if ((e = ppf::launch_align(a, st)) != hipSuccess) return hip_fail(ctx, e, "k_align");
    return PPF_OK;
}

int ppf_resid_chi2_batch(ppf_ctx *ctx, int64_t nrows, int32_t nbin, int32_t in_dtype,
                         const void *in, const double *phases, const double *model,
                         const int32_t *model_row, const double *scales, const double *errs,
                         double dof, double *out, void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (!nbin_supported(nbin)) return fail(ctx, PPF_EUNSUP, "nbin=%d unsupported", nbin);
    if (nrows < 0 || (nrows > 0 && (!in || !phases || !model || !model_row || !scales || !errs ||
                                    !out)))
        return fail(ctx, PPF_EINVAL, "bad resid_chi2 arguments");
    if (in_dtype != PPF_F32 && in_dtype != PPF_F64) return fail(ctx, PPF_EINVAL, "in_dtype");
    if (nrows == 0) return PPF_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    const double2 *T, *T2;
    int rc = twiddles(ctx, nbin, st, &T, &T2);
    if (rc) return rc;
    ppf::ResidArgs a{nbin, rfft_log2(nbin), in_dtype, in, phases, model, model_row, scales, errs,
                     dof, T, T2, out};
    if ((e = ppf::launch_resid_chi2(a, nrows, st)) != hipSuccess) return hip_fail(ctx, e, "k_resid_chi2");
    return PPF_OK;
}

int ppf_noise_batch(ppf_ctx *ctx, int64_t nrows, int32_t nbin, int32_t in_dtype, const void *in,
                    int32_t frac, double *out, void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (!nbin_supported(nbin)) return fail(ctx, PPF_EUNSUP, "nbin=%d unsupported", nbin);
    if (nrows < 0 || frac < 1 || (nrows > 0 && (!in || !out)))
        return fail(ctx, PPF_EINVAL, "bad noise arguments");
    if (in_dtype != PPF_F32 && in_dtype != PPF_F64) return fail(ctx, PPF_EINVAL, "in_dtype");
    if (nrows == 0) return PPF_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    const double2 *T, *T2;
    int rc = twiddles(ctx, nbin, st, &T, &T2);
    if (rc) return rc;
    ppf::NoiseArgs a{nbin, rfft_log2(nbin), in_dtype, noise_kc(nbin / 2 + 1, frac), in, T, T2, out};
    if (ppf::noise_wave_supported(a.log2N)) {
        if ((e = ppf::launch_noise_wave(a, nrows, st)) != hipSuccess) return hip_fail(ctx, e, "k_noise_w");
    } else if ((e = ppf::launch_noise(a, nrows, st)) != hipSuccess) {
        return hip_fail(ctx, e, "k_noise");
    }
    return PPF_OK;
}

// ppf_noise_long's plan and workspace (ppf_longfft.hip): rows in chunks of
// at most 256 MB of complex work buffers
namespace {
struct LongPlan {
    ppf::LongNoiseArgs a;
    int64_t rows_c;
    size_t off_A, off_Y, off_part, bytes;
};
bool long_plan(int64_t nrows, int64_t nbin, int frac, LongPlan &p) {
    if (nrows < 0 || nbin < 1 || frac < 1) return false;
    ppf::LongNoiseArgs &a = p.a;
    a = ppf::LongNoiseArgs{};
    a.nbin = nbin;
    a.packed = (nbin % 2 == 0) ? 1 : 0;
    a.n = a.packed ? nbin / 2 : nbin;
    a.nharm = nbin / 2 + 1;
    a.kc = (int64_t)((1.0 - std::pow((double)frac, -1.0)) * (double)a.nharm);
    const bool pow2 = (a.n & (a.n - 1)) == 0;
    a.bluestein = (pow2 && a.n >= 64) ? 0 : 1;
    int64_t M = 64;
    const int64_t need = a.bluestein ? 2 * a.n - 1 : a.n;
    while (M < need) M *= 2;
    int m = 0;
    while (((int64_t)1 << m) < M) ++m;
    if (m > 24) return false;             // M1, M2 <= 4096 (the block LDS FFT)
    a.M = M;
    a.log2M = m;
    a.log2M1 = (m + 1) / 2;
    a.M1 = (int64_t)1 << a.log2M1;
    a.M2 = M / a.M1;
    const size_t row_b = (size_t)M * sizeof(double2);
    int64_t rc = (int64_t)((size_t)(256u << 20) / (2 * row_b));
    if (rc < 1) rc = 1;
    p.rows_c = nrows < rc ? (nrows > 0 ? nrows : 1) : rc;
    size_t off = a.bluestein ? align256(2 * row_b) : 0;
    p.off_A = off;
    off += align256((size_t)p.rows_c * row_b);
    p.off_Y = off;
    off += align256((size_t)p.rows_c * row_b);
    p.off_part = off;
    off += align256((size_t)p.rows_c * 256 * sizeof(double));
    p.bytes = off;
    return true;
}
}  // namespace

size_t ppf_noise_long_workspace_bytes(int64_t nrows, int64_t nbin) {
    LongPlan p;
    return long_plan(nrows, nbin, 4, p) ? p.bytes : 0;
}

int ppf_noise_long(ppf_ctx *ctx, int64_t nrows, int64_t nbin, int32_t in_dtype, const void *in,
                   int32_t frac, double *out, void *workspace, size_t workspace_bytes, void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (nrows < 0 || nbin < 1 || frac < 1 || (nrows > 0 && (!in || !out)))
        return fail(ctx, PPF_EINVAL, "bad noise arguments");
    if (in_dtype != PPF_F32 && in_dtype != PPF_F64) return fail(ctx, PPF_EINVAL, "in_dtype");
    LongPlan p;
    if (!long_plan(nrows, nbin, frac, p))
        return fail(ctx, PPF_EUNSUP, "nbin=%lld: transform longer than 2^24 points", (long long)nbin);
    if (nrows == 0) return PPF_OK;
    if (!workspace || workspace_bytes < p.bytes)
        return fail(ctx, PPF_EINVAL, "workspace %zu < %zu bytes", workspace_bytes, p.bytes);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    const double2 *T1, *T2, *unused;
    int rc = twiddles(ctx, (int)(2 * p.a.M1), st, &T1, &unused);
    if (rc) return rc;
    if ((rc = twiddles(ctx, (int)(2 * p.a.M2), st, &T2, &unused))) return rc;
    char *ws = (char *)workspace;
    double2 *Bf = (double2 *)ws;
    if (p.a.bluestein && (e = ppf::launch_chirp_ft(p.a, Bf, Bf + p.a.M, T1, T2, st)) != hipSuccess)
        return hip_fail(ctx, e, "k_lf_chirp");
    p.a.in_dtype = in_dtype;
    p.a.in = in;
    for (int64_t r0 = 0; r0 < nrows; r0 += p.rows_c) {
        p.a.row0 = r0;
        const int64_t nr = nrows - r0 < p.rows_c ? nrows - r0 : p.rows_c;
        e = ppf::launch_noise_long(p.a, nr, (double2 *)(ws + p.off_A), (double2 *)(ws + p.off_Y), Bf,
                                   (double *)(ws + p.off_part), out, T1, T2, st);
        if (e != hipSuccess) return hip_fail(ctx, e, "k_lf");
    }
    return PPF_OK;
}

// ppf_rotate_long's plans and workspace: Bluestein transforms both ways
namespace {
bool bluestein_plan(int64_t nbin, int64_t n, bool packed, ppf::LongNoiseArgs &a) {
    a = ppf::LongNoiseArgs{};
    a.nbin = nbin; a.n = n; a.packed = packed ? 1 : 0; a.bluestein = 1;
    int64_t M = 64;
    while (M < 2 * n - 1) M *= 2;
    int m = 0;
    while (((int64_t)1 << m) < M) ++m;
    if (m > 24) return false;
    a.M = M; a.log2M = m; a.log2M1 = (m + 1) / 2;
    a.M1 = (int64_t)1 << a.log2M1; a.M2 = M / a.M1;
    return true;
}
struct RotPlan {
    ppf::LongRotArgs r;
    int64_t rows_c;
    size_t off_Bf, off_Bb, off_A, off_Y, bytes;
};
bool rot_plan(int64_t nrows, int64_t nbin, bool ref_len, RotPlan &p) {
    if (nrows < 0 || nbin < 2) return false;
    const bool odd = nbin & 1;
    if (!bluestein_plan(nbin, odd ? nbin : nbin / 2, !odd, p.r.f)) return false;
    const bool out_even = !odd || ref_len;
    const int64_t nout = odd && ref_len ? nbin - 1 : nbin;
    if (!bluestein_plan(nbin, out_even ? nout / 2 : nout, false, p.r.b)) return false;
    p.r.out_even = out_even ? 1 : 0;
    p.r.nout = nout;
    const size_t row_b = (size_t)p.r.f.M * sizeof(double2);     // b.M <= f.M
    int64_t rc = (int64_t)((size_t)(256u << 20) / (2 * row_b));
    if (rc < 1) rc = 1;
    p.rows_c = nrows < rc ? (nrows > 0 ? nrows : 1) : rc;
    size_t off = 0;
    p.off_Bf = off; off += align256(2 * row_b);
    p.off_Bb = off; off += align256(2 * (size_t)p.r.b.M * sizeof(double2));
    p.off_A = off; off += align256((size_t)p.rows_c * row_b);
    p.off_Y = off; off += align256((size_t)p.rows_c * row_b);
    p.bytes = off;
    return true;
}
}  // namespace

size_t ppf_rotate_long_workspace_bytes(int64_t nrows, int64_t nbin, int32_t ref_len) {
    RotPlan p;
    return rot_plan(nrows, nbin, ref_len != 0, p) ? p.bytes : 0;
}

static int rotate_long_run(ppf_ctx *ctx, RotPlan &p, int64_t nrows, int32_t in_dtype, const void *in,
                           const double *phases, const double *taus, double *out, char *ws, hipStream_t st);

int ppf_rotate_long(ppf_ctx *ctx, int64_t nrows, int64_t nbin, int32_t in_dtype, const void *in,
                    const double *phases, double *out, int32_t ref_len, void *workspace, size_t workspace_bytes,
                    void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (nrows < 0 || nbin < 2 || (nrows > 0 && (!in || !phases || !out)))
        return fail(ctx, PPF_EINVAL, "bad rotate arguments");
    if (in_dtype != PPF_F32 && in_dtype != PPF_F64) return fail(ctx, PPF_EINVAL, "in_dtype");
    RotPlan p;
    if (!rot_plan(nrows, nbin, ref_len != 0, p))
        return fail(ctx, PPF_EUNSUP, "nbin=%lld: transform longer than 2^24 points", (long long)nbin);
    if (nrows == 0) return PPF_OK;
    if (!workspace || workspace_bytes < p.bytes)
        return fail(ctx, PPF_EINVAL, "workspace %zu < %zu bytes", workspace_bytes, p.bytes);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    return rotate_long_run(ctx, p, nrows, in_dtype, in, phases, nullptr, out, (char *)workspace,
                           (hipStream_t)stream);
}

// the long rotation / scattering convolution of nrows rows on a plan whose
// workspace is `ws` (in may be out: each chunk's rows are read before
// they are written)
static int rotate_long_run(ppf_ctx *ctx, RotPlan &p, int64_t nrows, int32_t in_dtype, const void *in,
                           const double *phases, const double *taus, double *out, char *ws, hipStream_t st) {
    hipError_t e;
    const double2 *T1f, *T2f, *T1b, *T2b, *unused;
    int rc;
    if ((rc = twiddles(ctx, (int)(2 * p.r.f.M1), st, &T1f, &unused))) return rc;
    if ((rc = twiddles(ctx, (int)(2 * p.r.f.M2), st, &T2f, &unused))) return rc;
    if ((rc = twiddles(ctx, (int)(2 * p.r.b.M1), st, &T1b, &unused))) return rc;
    if ((rc = twiddles(ctx, (int)(2 * p.r.b.M2), st, &T2b, &unused))) return rc;
    double2 *Bff = (double2 *)(ws + p.off_Bf), *Bfb = (double2 *)(ws + p.off_Bb);
    if ((e = ppf::launch_chirp_ft(p.r.f, Bff, Bff + p.r.f.M, T1f, T2f, st)) != hipSuccess)
        return hip_fail(ctx, e, "k_lf_chirp");
    if ((e = ppf::launch_chirp_ft(p.r.b, Bfb, Bfb + p.r.b.M, T1b, T2b, st)) != hipSuccess)
        return hip_fail(ctx, e, "k_lf_chirp");
    p.r.f.in_dtype = in_dtype;
    p.r.f.in = in;
    p.r.phases = phases;
    p.r.taus = taus;
    p.r.out = out;
    for (int64_t r0 = 0; r0 < nrows; r0 += p.rows_c) {
        p.r.f.row0 = p.r.b.row0 = r0;
        const int64_t nr = nrows - r0 < p.rows_c ? nrows - r0 : p.rows_c;
        e = ppf::launch_rotate_long(p.r, nr, (double2 *)(ws + p.off_A), (double2 *)(ws + p.off_Y), Bff, Bfb,
                                    T1f, T2f, T1b, T2b, st);
        if (e != hipSuccess) return hip_fail(ctx, e, "k_lr");
    }
    return PPF_OK;
}

int ppf_scales_batch(ppf_ctx *ctx, int32_t nsub, int32_t nchan, int32_t nharm, const double *D,
                     const double *M, const int32_t *model_index, const double *errs_FT,
                     const double *params, const double *P, const double *freqs, const double *nus,
                     int32_t log10_tau, double *out, void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (nsub < 0 || nchan < 1 || nharm < 1 ||
        (nsub > 0 && (!D || !M || !params || !P || !freqs || !nus || !out)))
        return fail(ctx, PPF_EINVAL, "bad scales arguments");
    if (nsub == 0) return PPF_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    ppf::ScalesArgs a{nsub, nchan, nharm, log10_tau != 0, (const double2 *)D, (const double2 *)M,
                      model_index, errs_FT, params, P, freqs, nus, out};
    if ((e = ppf::launch_scales(a, (hipStream_t)stream)) != hipSuccess) return hip_fail(ctx, e, "k_scales");
    return PPF_OK;
}

size_t ppf_unpack_workspace_bytes(int32_t nsub, int32_t nchan, int32_t nbin) {
    if (nsub < 0 || nchan < 1 || nbin < 2) return 0;
    return ppf::unpack_partials(nsub, nchan, nbin) * sizeof(double) + 256;
}

int ppf_unpack_psrfits_batch(ppf_ctx *ctx, int32_t nsub, int32_t npol, int32_t nchan, int32_t nbin,
                             int32_t elem, const void *raw, int64_t sub_stride, const float *scl,
                             const float *offs, const float *wts, int32_t pol_mode,
                             int32_t rm_baseline, float *out, double *stats, double *total,
                             int32_t *wstart, void *workspace, size_t workspace_bytes,
                             void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (nsub < 0 || npol < 1 || nchan < 1 || nbin < 2 || elem < 0 || elem > 3 || pol_mode < 0 ||
        pol_mode > 1 || (pol_mode == 1 && npol < 2))
        return fail(ctx, PPF_EINVAL, "bad unpack arguments (npol=%d nchan=%d nbin=%d elem=%d "
                    "pol_mode=%d)", npol, nchan, nbin, elem, pol_mode);
    const int64_t esize = elem == 0 ? 2 : (elem == 1 ? 1 : 4);
    if (sub_stride < (int64_t)(pol_mode == 1 ? 2 : 1) * nchan * nbin * esize)
        return fail(ctx, PPF_EINVAL, "sub_stride %lld < one sub-int's DATA", (long long)sub_stride);
    if (nsub == 0) return PPF_OK;
    if (!raw || !scl || !offs || !out || !stats || !total || !wstart || !workspace)
        return fail(ctx, PPF_EINVAL, "null unpack pointer");
    if (workspace_bytes < ppf_unpack_workspace_bytes(nsub, nchan, nbin))
        return fail(ctx, PPF_ENOMEM, "unpack workspace %zu < %zu", workspace_bytes,
                    ppf_unpack_workspace_bytes(nsub, nchan, nbin));
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    ppf::UnpackArgs a{};
    a.nsub = nsub; a.npol = npol; a.nchan = nchan; a.nbin = nbin; a.elem = elem;
    a.pol_mode = pol_mode; a.rm_baseline = rm_baseline ? 1 : 0;
    a.win = std::min(nbin - 1, std::max(1, (int)std::lrint(0.15 * nbin)));
    a.raw = (const uint8_t *)raw; a.sub_stride = sub_stride;
    a.scl = scl; a.offs = offs; a.wts = wts; a.out = out;
    a.part = (double *)workspace; a.total = total; a.wstart = wstart; a.stats = stats;
    if ((e = ppf::launch_unpack(a, (hipStream_t)stream)) != hipSuccess) return hip_fail(ctx, e, "k_unpack");
    return PPF_OK;
}

int ppf_copy_from_pinned(ppf_ctx *ctx, void *dst, const void *src, int64_t nbytes, void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (nbytes < 0 || (nbytes > 0 && (!dst || !src)))
        return fail(ctx, PPF_EINVAL, "bad copy arguments");
    if (((uintptr_t)dst | (uintptr_t)src) % 16)
        return fail(ctx, PPF_EINVAL, "copy buffers must be 16-byte aligned");
    if (nbytes == 0) return PPF_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    void *src_dev = nullptr;
    if ((e = hipHostGetDevicePointer(&src_dev, const_cast<void *>(src), 0)) != hipSuccess || !src_dev) {
        (void)hipGetLastError();   // not sticky: the next launch must not see it
        return hip_fail(ctx, e != hipSuccess ? e : hipErrorInvalidValue,
                        "hipHostGetDevicePointer (src must be page-locked host memory)");
    }
    if ((e = ppf::launch_copy_host(src_dev, dst, nbytes, (hipStream_t)stream)) != hipSuccess)
        return hip_fail(ctx, e, "k_copy_host");
    return PPF_OK;
}

// grows the context's scratch to at least `bytes` (lscr_mu held)
static int lscr_reserve(ppf_ctx *ctx, size_t bytes) {
    if (ctx->lscr_bytes >= bytes) return PPF_OK;
    hipError_t e;
    if (ctx->lscr) {
        if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(ctx, e, "hipDeviceSynchronize");
        (void)hipFree(ctx->lscr);
        ctx->lscr = nullptr;
        ctx->lscr_bytes = 0;
    }
    if ((e = hipMalloc(&ctx->lscr, bytes)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(scratch)");
    ctx->lscr_bytes = bytes;
    return PPF_OK;
}

int ppf_phase_shift_batch(ppf_ctx *ctx, int32_t nprof, int32_t nbin, int32_t in_dtype,
                          const void *data, const double *model, const int32_t *model_index,
                          const double *noise, int32_t Ns, double lo, double hi, double *out,
                          void *stream) {
    if (!ctx) return PPF_EINVAL;
    // rows past the LDS transforms (round 6): their rFFTs on the long
    // transforms first, the FFTFIT on the stored bins (a synchronous call)
    const bool lng = !nbin_supported(nbin) && nbin > 4095;
    if (!nbin_supported(nbin) && !lng) return fail(ctx, PPF_EUNSUP, "nbin=%d unsupported", nbin);
    if (nprof < 0 || Ns < 1 || Ns > 65536 || (nprof > 0 && (!data || !model || !out)))
        return fail(ctx, PPF_EINVAL, "bad phase-shift arguments");
    if (in_dtype != PPF_F32 && in_dtype != PPF_F64) return fail(ctx, PPF_EINVAL, "in_dtype");
    if (lng && (size_t)(nbin / 2 + 2) * sizeof(double2) > 150u * 1024u)
        return fail(ctx, PPF_EUNSUP, "nbin=%d: the spectrum exceeds one workgroup's LDS", nbin);
    if (nprof == 0) return PPF_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    const double2 *T = nullptr, *T2 = nullptr;
    int rc;
    if (!lng && (rc = twiddles(ctx, nbin, st, &T, &T2))) return rc;
    ppf::PhaseShiftArgs a{};
    a.nbin = nbin; a.log2N = rfft_log2(nbin); a.dtype = in_dtype; a.kc = noise_kc(nbin / 2 + 1, 4);
    a.Ns = Ns; a.lo = lo; a.hi = hi; a.data = data; a.model = model; a.model_index = model_index;
    a.noise = noise; a.T = T; a.T2 = T2; a.out = out;
    if (!lng && !grid_gsh(nbin, Ns, false)) {
        if ((e = ppf::launch_phase_shift(a, nprof, st)) != hipSuccess) return hip_fail(ctx, e, "k_phase_shift");
        return PPF_OK;
    }
    if (!lng) {
        // the brute grid past the LDS (Ns = nbin at 8192): in the context's
        // scratch, held for the whole (synchronous) call
        std::lock_guard<std::mutex> lk(ctx->lscr_mu);
        if ((rc = lscr_reserve(ctx, align256(sizeof(double) * (size_t)nprof * ((size_t)Ns + 8))))) return rc;
        a.gsh = (double *)ctx->lscr;
        if ((e = ppf::launch_phase_shift(a, nprof, st)) != hipSuccess) return hip_fail(ctx, e, "k_phase_shift");
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
        return PPF_OK;
    }
    // model rows in use: 1 + the largest model_index
    int nmodel = 1;
    if (model_index) {
        std::vector<int32_t> mi(nprof);
        if ((e = hipMemcpyAsync(mi.data(), model_index, nprof * sizeof(int32_t), hipMemcpyDeviceToHost, st)) !=
                hipSuccess ||
            (e = hipStreamSynchronize(st)) != hipSuccess)
            return hip_fail(ctx, e, "hipMemcpyAsync(model_index)");
        for (int i = 0; i < nprof; ++i) {
            if (mi[i] < 0) return fail(ctx, PPF_EINVAL, "model_index[%d] = %d", i, mi[i]);
            nmodel = std::max(nmodel, mi[i] + 1);
        }
    }
    ppf::LongNoiseArgs f;
    if (!bluestein_plan(nbin, (nbin & 1) ? nbin : nbin / 2, !(nbin & 1), f))
        return fail(ctx, PPF_EUNSUP, "nbin=%d", nbin);
    const size_t nharm = (size_t)nbin / 2 + 1, row_b = (size_t)f.M * sizeof(double2);
    FitLayout L{};
    const int64_t rows = std::max<int64_t>(nprof, nmodel);
    int64_t rcn = (int64_t)((size_t)(256u << 20) / (2 * row_b));
    L.lrows = rows < rcn ? rows : (rcn < 1 ? 1 : rcn);
    size_t o = 0;
    const size_t oD = o; o += align256(sizeof(double2) * (size_t)nprof * nharm);
    const size_t oM = o; o += align256(sizeof(double2) * (size_t)nmodel * nharm);
    L.lchirp = o; o += align256(2 * row_b);
    L.lA = o; o += align256((size_t)L.lrows * row_b);
    L.lY = o; o += align256((size_t)L.lrows * row_b);
    const bool gs = grid_gsh(nbin, Ns, true);
    const size_t oG = o; o += gs ? align256(sizeof(double) * (size_t)nprof * ((size_t)Ns + 8)) : 0;
    std::lock_guard<std::mutex> lk(ctx->lscr_mu);
    if ((rc = lscr_reserve(ctx, o))) return rc;
    char *ws = (char *)ctx->lscr;
    if ((rc = long_rfft_rows(ctx, L, ws, nbin, nmodel, PPF_F64, model, (double2 *)(ws + oM), false, st))) return rc;
    if ((rc = long_rfft_rows(ctx, L, ws, nbin, nprof, in_dtype, data, (double2 *)(ws + oD), true, st))) return rc;
    a.Mspec = (const double2 *)(ws + oM);
    a.Dspec = (const double2 *)(ws + oD);
    if (gs) a.gsh = (double *)(ws + oG);
    if ((e = ppf::launch_phase_shift(a, nprof, st)) != hipSuccess) return hip_fail(ctx, e, "k_phase_shift");
    // the scratch is reused by the next call (any stream): finish here
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
    return PPF_OK;
}

int ppf_gauss_portrait_batch(ppf_ctx *ctx, int32_t nport, int32_t nchan, int32_t nbin,
                             int32_t ngauss, const char *model_code, const double *params,
                             const double *scattering_index, const double *freqs,
                             const double *nu_ref, double *out, void *stream) {
    if (!ctx) return PPF_EINVAL;
    // rows past the LDS transforms (round 6): the Gaussians are evaluated
    // per bin in LDS (nbin doubles); the scattering convolution of even rows
    // then runs on the long transforms (ppf_rotate_long's pipeline with the
    // 1 / (1 + 2 pi i k tau_n) factor in place of the phasor; a synchronous
    // call with the context's scratch); scattered odd rows are refused
    const bool lng = !nbin_supported(nbin);
    if (lng && (nbin <= 4095 || (size_t)nbin * sizeof(double) > 150u * 1024u))
        return fail(ctx, PPF_EUNSUP, "nbin=%d unsupported", nbin);
    if (nport < 0 || nchan < 1 || ngauss < 0 ||
        (nport > 0 && (!params || !scattering_index || !freqs || !nu_ref || !out)))
        return fail(ctx, PPF_EINVAL, "bad gauss_portrait arguments");
    if (!model_code) return fail(ctx, PPF_EINVAL, "model_code is NULL");
    ppf::GaussArgs a{};
    for (int i = 0; i < 3; ++i) {
        const char c = model_code[i];
        if (c != '0' && c != '1')   // evolve_parameter's KeyError (pplib.py:1082-1084)
            return fail(ctx, PPF_EINVAL, "model_code '%.3s': digit %d must be '0' or '1'",
                        model_code, i);
        a.code[i] = c - '0';
    }
    if (nport == 0) return PPF_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    const double2 *T = nullptr, *T2 = nullptr;
    int rc;
    bool lscat = false;
    if (lng) {
        // the models' tau (params[p][1]) on the host: a scattered one at
        // this length is refused, not half-built (a one-off small copy)
        std::vector<double> prm((size_t)nport * (2 + 6 * ngauss));
        if ((e = hipMemcpyAsync(prm.data(), params, prm.size() * sizeof(double), hipMemcpyDeviceToHost, st)) !=
                hipSuccess ||
            (e = hipStreamSynchronize(st)) != hipSuccess)
            return hip_fail(ctx, e, "hipMemcpyAsync(params)");
        for (int p = 0; p < nport; ++p)
            if (prm[(size_t)p * (2 + 6 * ngauss) + 1] != 0.0) lscat = true;
        if (lscat && (nbin & 1))
            return fail(ctx, PPF_EUNSUP, "scattered model (TAU != 0) at odd nbin=%d past 4095 (the reference's "
                        "nbin - 1-bin irfft rows)", nbin);
    } else if ((rc = twiddles(ctx, nbin, st, &T, &T2))) {
        return rc;
    }
    a.nport = nport; a.nchan = nchan; a.nbin = nbin; a.log2N = rfft_log2(nbin);
    a.ngauss = ngauss; a.npar = 2 + 6 * ngauss;
    a.params = params; a.scat_index = scattering_index; a.freqs = freqs; a.nu_ref = nu_ref;
    a.T = T; a.T2 = T2; a.out = out;
    a.Te = T; a.T2e = T2;
    if (!lng && (nbin & 1) && (rc = twiddles(ctx, nbin - 1, st, &a.Te, &a.T2e))) return rc;
    if (!lscat) {
        if ((e = ppf::launch_gauss_port(a, st)) != hipSuccess) return hip_fail(ctx, e, "k_gauss_port");
        return PPF_OK;
    }
    const int64_t nrows = (int64_t)nport * nchan;
    RotPlan rp;
    if (!rot_plan(nrows, nbin, false, rp)) return fail(ctx, PPF_EUNSUP, "nbin=%d", nbin);
    const size_t oT = align256(rp.bytes);
    std::lock_guard<std::mutex> lk(ctx->lscr_mu);
    if ((rc = lscr_reserve(ctx, oT + align256(sizeof(double) * (size_t)nrows)))) return rc;
    char *ws = (char *)ctx->lscr;
    a.taus_out = (double *)(ws + oT);
    if ((e = ppf::launch_gauss_port(a, st)) != hipSuccess) return hip_fail(ctx, e, "k_gauss_port");
    if ((rc = rotate_long_run(ctx, rp, nrows, PPF_F64, out, nullptr, a.taus_out, out, ws, st))) return rc;
    // the scratch is reused by the next call (any stream): finish here
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
    return PPF_OK;
}

int ppf_spline_portrait_batch(ppf_ctx *ctx, int32_t nport, int32_t nchan, int32_t nbin_model,
                              int32_t nbin, int32_t ncomp, int32_t nknots, int32_t degree,
                              const double *mean_prof, const double *eigvec, const double *knots,
                              const double *coefs, const double *freqs, double *out, void *stream) {
    if (!ctx) return PPF_EINVAL;
    // the model's own length: no transform (any nbin); resampled: two even
    // lengths the LDS transforms take (scipy.signal.resample's Nyquist
    // split as restated in k_spline_port assumes even lengths)
    const bool same = nbin == nbin_model;
    if (same ? nbin < 2
             : !(nbin % 2 == 0 && nbin_model % 2 == 0 && nbin_supported(nbin) && nbin_supported(nbin_model)))
        return fail(ctx, PPF_EUNSUP,
                    "nbin=%d nbin_model=%d: the model's own length, or both even in [32, 8192]", nbin,
                    nbin_model);
    if (nport < 0 || nchan < 1 || ncomp < 0 || ncomp > ppf::kSplineMaxComp || degree < 0 ||
        degree > ppf::kSplineMaxDeg || (ncomp > 0 && nknots < 2 * degree + 2))
        return fail(ctx, PPF_EINVAL, "bad spline model (ncomp=%d nknots=%d degree=%d)", ncomp, nknots,
                    degree);
    if (nport == 0) return PPF_OK;
    if (!mean_prof || !freqs || !out || (ncomp > 0 && (!eigvec || !knots || !coefs)))
        return fail(ctx, PPF_EINVAL, "null spline argument");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    ppf::SplineArgs a{};
    a.nport = nport; a.nchan = nchan; a.nbin_model = nbin_model; a.nbin = nbin; a.ncomp = ncomp;
    a.nknots = nknots; a.degree = degree;
    a.log2N0 = fft_log2(nbin_model / 2); a.log2N1 = rfft_log2(nbin);
    a.mean_prof = mean_prof; a.eigvec = eigvec; a.knots = knots; a.coefs = coefs; a.freqs = freqs;
    a.out = out;
    int rc;
    if (nbin != nbin_model) {
        if ((rc = twiddles(ctx, nbin_model, st, &a.T0, &a.T20))) return rc;
        if ((rc = twiddles(ctx, nbin, st, &a.T1, &a.T21))) return rc;
    }
    if ((e = ppf::launch_spline_port(a, st)) != hipSuccess) return hip_fail(ctx, e, "k_spline_port");
    return PPF_OK;
}

int ppf_synth_batch(ppf_ctx *ctx, int32_t nsub, int32_t nchan, int32_t nbin, const double *model,
                    const double *freqs, const double *phi, const double *DM, const double *P,
                    double nu_ref, double noise, uint64_t seed, int64_t first_sub,
                    int32_t out_dtype, void *out, void *stream) {
    if (!ctx) return PPF_EINVAL;
    if (!nbin_supported(nbin)) return fail(ctx, PPF_EUNSUP, "nbin=%d unsupported", nbin);
    if (nsub < 0 || nchan < 1 || (nsub > 0 && (!model || !freqs || !phi || !DM || !P || !out)))
        return fail(ctx, PPF_EINVAL, "bad synth arguments");
    if (out_dtype != PPF_F32 && out_dtype != PPF_F64) return fail(ctx, PPF_EINVAL, "out_dtype");
    if (nsub == 0) return PPF_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = (hipStream_t)stream;
    const double2 *T, *T2;
    int rc = twiddles(ctx, nbin, st, &T, &T2);
    if (rc) return rc;
    // model spectra into a temporary buffer owned by this call
    double2 *Mft = nullptr;
    const size_t nharm = (size_t)nbin / 2 + 1;
    e = hipMallocAsync((void **)&Mft, sizeof(double2) * nchan * nharm, st);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipMallocAsync(synth)");
    ppf::RfftArgs ra{nbin, rfft_log2(nbin), PPF_F64, model, T, T2, Mft};
    if ((e = ppf::launch_rfft_rows(ra, nchan, st)) != hipSuccess) return hip_fail(ctx, e, "k_rfft_rows");
    ppf::SynthArgs a{};
    a.nsub = nsub; a.nchan = nchan; a.nbin = nbin; a.log2N = rfft_log2(nbin); a.dtype = out_dtype;
    a.Mft = Mft; a.freqs = freqs; a.phi = phi; a.DM = DM; a.P = P; a.nu_ref = nu_ref;
    a.noise = noise; a.seed = seed; a.first = first_sub; a.T = T; a.T2 = T2; a.out = out;
    if ((e = ppf::launch_synth(a, st)) != hipSuccess) return hip_fail(ctx, e, "k_synth");
    (void)hipFreeAsync(Mft, st);
    return PPF_OK;
}

int ppf_poly_real_roots_host(const double *coeffs, int deg, double *out) {
    if (!coeffs || !out || deg < 0 || deg > 8) return -2;
    return ppf::poly_real_roots(coeffs, deg, out);
}

int ppf_tr_subproblem_host(const double *H, const double *g, int n, double R, double *p) {
    if (!H || !g || !p || n < 1 || n > 5 || !(R > 0.0)) return -1;
    double A[5][5];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) A[i][j] = H[i * n + j];
    bool hb = false;
    switch (n) {
        case 1: hb = ppf::tr_exact<1>(A, g, R, p); break;
        case 2: hb = ppf::tr_exact<2>(A, g, R, p); break;
        case 3: hb = ppf::tr_exact<3>(A, g, R, p); break;
        case 4: hb = ppf::tr_exact<4>(A, g, R, p); break;
        default: hb = ppf::tr_exact<5>(A, g, R, p); break;
    }
    return hb ? 1 : 0;
}

}  // extern "C"
