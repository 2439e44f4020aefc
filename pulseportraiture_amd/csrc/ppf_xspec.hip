// ppf_xspec.hip -- wave-per-row spectrum kernels (128 <= nbin/2 <= 1024).
//
// Both kernels give one channel row to one wave: the row is loaded from HBM
// (f32 or f64, prefetched one row ahead), transformed by the wave-private
// register/LDS FFT of ppf_wfft.hpp (no workgroup barrier inside a row) and
// finished by the real-FFT post-pass on (k, N-k) pairs.
//
// k_xspec_w<LOG2N, DT>: the cross spectrum for the sub-ints whose fit
//   streams it (scattering fits, k_pass):
//     get_noise_PS noise (pplib.py:2312-2332), Sd_n, S_n(tau = 0)
//     X_k = D_k conj(M_k) / sigma~_n^2 (pptoaslib.py:1014-1031), k = 0 zeroed
//   Sub-ints fitted from moments (TRState.mmode) are skipped: k_xmom_g
//   produces everything they need without X.
//
// k_xmom_g<LOG2N, DT, SH>: the fused moment pass (fits without scattering).
//   The cross spectrum never reaches HBM: for every sub-int that asks for a
//   moment set (need_mom, centre mc[mtarget]) the workgroup re-reads its
//   block of channel rows and per row forms the noise, Sd_n, S_n (chan[]) and
//     Y_k = D_k conj(M_k) e^{2 pi i k phi_c,n}   (phi_c,n = c0 + c1 dphi1_n
//                                                  + c2 dphi2_n)
//   The moments mu_m = sum_{k=1..N} Y_k u_k^m / sigma~_n^2, u_k = (k - N/2)
//   / (N/2), fold the harmonic pairs (k, N-k), u_{N-k} = -u_k:
//     mu_2j   = sum_{k<N/2} (Y_k + Y_{N-k})       (u_k^2)^j  + [j=0] Y_{N/2}
//     mu_2j+1 = sum_{k<N/2} (Y_k - Y_{N-k}) u_k   (u_k^2)^j
//   so both halves share one B tile (v_k^j, v = u^2, j < 16) and the MFMA
//   K loop runs over N/2 harmonics.  A = 16 rows of v_mfma_f64_16x16x4f64
//   from the 8 wave buffers: 8 sub-ints x {Re, Im}, one MFMA per half.  Each
//   wave takes 1/8 of the folded harmonics; the partial tiles are summed in
//   wave order through LDS (deterministic) and scaled by 1/sigma~_n^2.
//   Output: mu[s][q][n][m] (k_tr_mom consumes it).  HBM traffic per sub-int:
//   the data rows (nchan nbin s_in B) + the moments (nchan 32 16 B).
//   The first launch of a ppf_fit_batch call (FULL) covers every moment-mode
//   sub-int in index order; re-centring launches take the sub-ints k_tr_mom
//   listed (rc_list), packed eight to a workgroup, on 8-channel blocks.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "ppf_internal.hpp"
#include "ppf_state.hpp"
#include "ppf_wfft.hpp"
#include "ppf_wfft2.hpp"

namespace ppf {

constexpr int kXW = 8;                 // waves per k_align_part_w workgroup
// waves (= channel rows per round) per k_xspec_w workgroup: 4 at 1024-point
// rows (two 70 KB workgroups per CU instead of one of 139 KB: a round's
// write-out barrier holds 4 waves, not 8; C3 k_xspec_w 27.7 vs 29.2 ms),
// 8 below (C5, 512-point rows: 29.8 vs 37.0 ms)
template <int LOG2N>
__host__ __device__ constexpr int xsw() {
#ifdef PPF_XSPEC_WAVES
    return PPF_XSPEC_WAVES;
#else
    return LOG2N == 10 ? 4 : 8;
#endif
}
typedef double f64x4 __attribute__((ext_vector_type(4)));
// row elements as native vectors: arrays of HIP_vector_type structs carried
// across the row loop are not promoted to VGPRs
typedef float vf2 __attribute__((ext_vector_type(2)));
typedef double vd2 __attribute__((ext_vector_type(2)));
typedef float vf4 __attribute__((ext_vector_type(4)));
#ifndef PPF_SCHED_CUT
#define PPF_SCHED_CUT 1
#endif
#if PPF_SCHED_CUT
#define SCHED_CUT() __builtin_amdgcn_sched_barrier(0)
#else
#define SCHED_CUT()
#endif
#ifndef PPF_XM_CUT
#define PPF_XM_CUT 0
#endif
#if PPF_XM_CUT
#define XM_CUT() __builtin_amdgcn_sched_barrier(0)
#else
#define XM_CUT()
#endif

// XCD-aware block -> (sub-int, channel block): blocks b and b+8 share an
// XCD, so each XCD keeps only its channel blocks' model rows in its L2.
// Mode 1 walks an XCD's channel blocks sub-int by sub-int (a model larger
// than the L2s is then re-read for every sub-int: 134 MB per C5 sub-int);
// mode 2 walks every sub-int (of nsub) for one channel block before the next,
// so the workgroups resident on an XCD share one block of model rows.
__device__ __forceinline__ void block_map(int xcd_swizzle, int nblk, int &s, int &cb, int nsub = 0) {
    if (xcd_swizzle == 2) {
        const int per = nblk / 8, x = blockIdx.x % 8, r = blockIdx.x / 8;
        cb = x * per + r / nsub;
        s = r % nsub;
    } else if (xcd_swizzle) {
        const int per = nblk / 8, x = blockIdx.x % 8, r = blockIdx.x / 8;
        cb = x * per + r % per;
        s = r / per;
    } else {
        s = blockIdx.x / nblk;
        cb = blockIdx.x % nblk;
    }
}

// real-FFT post-pass of the pair (k, N-k), k = lane + 64 i, from the wave's
// LDS spectrum; w = exp(-i pi k / N)
template <int LOG2N>
__device__ __forceinline__ void rfft_pair(const double2 *buf, int k, double2 w, double2 &Dlo,
                                          double2 &Dhi) {
    constexpr int N = 1 << LOG2N;
    const double2 zk = buf[wfft::pad<LOG2N>(k)];
    const double2 zn = buf[k == 0 ? 0 : wfft::pad<LOG2N>(N - k)];
    const double2 e = cmk(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y));
    const double2 o = cmk(0.5 * (zk.x - zn.x), 0.5 * (zk.y + zn.y));
    const double2 wo = cmul(w, o);
    Dlo = cmk(e.x + wo.y, e.y - wo.x);
    Dhi = cmk(e.x - wo.y, -(e.y + wo.x));
}

// ===========================================================================
// k_xspec_w: cross spectrum X of the sub-ints that stream it
// ===========================================================================
// wave buffer + 2 side slots; with the XOR slot map the buffers start 4
// slots apart mod 16, which makes the eight-channel write-out of k_xspec_w
// conflict-free (tools/lds_conflicts.py)
// largest FFT twiddle index + 1 used by wfft stages >= 1
template <int LOG2N>
__host__ __device__ constexpr int tw_slots() {
    using P = wfft::Plan<LOG2N>;
    return P::NST > 1 ? P::N / P::radix(P::NST - 1) : 1;
}
// Stage twiddles from an LDS copy (default) instead of the global table: the
// wave's next row is already in flight during the FFT, and vmcnt counts in
// order, so a twiddle load issued after that prefetch would wait for it
// (the s_waitcnt vmcnt(0) before every stage's first twiddle use).
#ifndef PPF_TW_LDS
#define PPF_TW_LDS 1
#endif
template <int LOG2N>
__host__ __device__ constexpr int xspec_slw() { return wfft::buf_slots<LOG2N>() + (wfft::use_xor<LOG2N>() ? 4 : 2); }

// GS: the sub-ints with gflag set (k_gflag: every channel's harmonic cutoff
// below NL = 64 guess_npl) also accumulate the GetTOAs guess spectrum
// (pptoas.py:461-464 in the Fourier domain, as rotate_data does it):
// G_k = sum_n w_n D_nk exp(2 pi i k dphi_n), dphi_n = Dconst DM_guess / P
// (nu_n^-2 - nu_ref^-2), for 1 <= k < NL.  No register holds them: pass 2
// of the post-pass stores a row's terms in the wave-buffer slots of the
// harmonics N - k, which X no longer needs (its write-out stops below the
// cutoff), and the write-out phase adds the round's rows to a workgroup sum
// in LDS in wave order (deterministic).  The profile's noise for the
// FFTFIT scale is its expectation from the channels' noise:
// err^2 = sum_n w_n^2 errs_FT,n^2 / W^2.
// minimum waves per SIMD: at 1024 points the LDS admits two 4-wave
// workgroups per CU (two waves per SIMD), and the fused-guess variant must
// keep that register budget (<= 256)
// PPF_GS9: the fused guess at 512 points as well (1: capped at four waves
// per SIMD, spilling; 2: uncapped, two waves per SIMD; 0, default: those
// shapes take k_dsum_w).  Measured (round 5, C5 per 500 sub-ints, one call):
// C5's model reaches harmonic ~430 of 513, above the NL = 192 guess
// harmonics, so k_gflag sets no sub-int and the GS=1 variant only costs its
// registers: k_xspec_w<9> 26.5 vs 22.0 ms, 90.1 vs 84.7 ms per step.
#ifndef PPF_GS9
#define PPF_GS9 0
#endif
template <int LOG2N, bool GS = false>
__host__ __device__ constexpr int xspec_wpe() { return LOG2N == 10 ? 2 : (LOG2N == 9 && GS && PPF_GS9 == 1 ? 4 : 1); }
// the fused guess runs at 1024 points (and 512 with PPF_GS9): below, its
// extra registers cost a wave per SIMD or spill (those shapes take k_dsum)
__host__ __device__ constexpr bool xspec_guess_fused(int log2N) { return log2N == 10 || (log2N == 9 && PPF_GS9 != 0); }
bool xspec_guess_fused_n(int log2N) { return xspec_guess_fused(log2N); }
// one post-pass over the transform (power sums and X together, X scaled at
// the write-out); 0: the two-pass form (sums, then X scaled in the buffer)
#ifndef PPF_XS_ONEPASS
#define PPF_XS_ONEPASS 1
#endif
template <int LOG2N, int DT, bool GS>
__global__ __launch_bounds__(64 * xsw<LOG2N>()) __attribute__((amdgpu_waves_per_eu(xspec_wpe<LOG2N, GS>())))
void k_xspec_w(XspecArgs a) {
    constexpr int kXSW = xsw<LOG2N>();
    using P = wfft::Plan<LOG2N>;
    constexpr int N = P::N, R = P::R, NH = N + 1;
    constexpr int NP = N / 128;                       // (k, N-k) pairs per lane
    constexpr int SL = xspec_slw<LOG2N>();           // padded wave buffer + 2 side slots
    constexpr int XNYQ = SL - 2;                      // X_{N/2} of the row
    constexpr int XIE2 = SL - 1;                      // the row's 1/errs_FT^2 (.x)
    // model pairs loaded ahead in pass 2: at 1024 points the 4-wave
    // workgroups leave VGPRs to spare (LDS caps them at two waves per SIMD:
    // 4 ahead, C3 27.1 -> 25.5 ms); at 512 points k_xspec_w runs four waves
    // per SIMD at <= 128 VGPRs, which one pair ahead keeps (126; C5 29.2 ->
    // 28.6 ms), two would not (132)
#ifndef PPF_XS_MPRE9
#define PPF_XS_MPRE9 1
#endif
#ifdef PPF_XS_MPRE
    constexpr int MD = PPF_XS_MPRE;
#else
    constexpr int MD = LOG2N == 10 ? 4 : (LOG2N == 9 ? (GS && PPF_GS9 == 1 ? 0 : PPF_XS_MPRE9) : 0);
#endif
    using RowT = typename std::conditional<DT == 0, vf2, vd2>::type;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *buf = lds + wave * SL;

    int s, cb;
    block_map(a.xcd_swizzle, a.nblk, s, cb, a.nsub);
    if (a.needx && !a.needx[s]) return;               // uniform: moment-mode sub-int (or no slot)
#if PPF_TW_LDS
    double2 *twl = lds + kXSW * SL;
    for (int i = threadIdx.x; i < tw_slots<LOG2N>(); i += 64 * kXSW) twl[i] = a.T[i];
    __syncthreads();
    const double2 *tw = twl;
#else
    const double2 *tw = a.T;
#endif
    // rounds: in round r wave w takes channel cb*CB + r*kXSW + w
    const int cbase = cb * a.cb, cend = min(a.nchan, cbase + a.cb);
    const int nround = (a.cb + kXSW - 1) / kXSW;
    const int mi = a.model_index ? a.model_index[s] : 0;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double sqrtN = sqrt((double)N);
    const RowT *rows = reinterpret_cast<const RowT *>(a.data);
    // rfft post-pass twiddles w_k = exp(-i pi k / N), k = lane + 64 i, by
    // recurrence from w_lane (T2) with step exp(-i pi 64 / N) = T2[64]
    const double2 w_seed = a.T2[lane], w_step = a.T2[64];
    // X[s][k][n] (harmonic-major: k_pass lanes are channels).  Each round the
    // 8 rows' X are left in the wave buffers and written out together, 8
    // channels x 16 B = one 128-B line per harmonic.
    double2 *Xs = a.X + (int64_t)(a.xslot ? a.xslot[s] : s) * NH * a.nchan;
    // harmonics k_pass reads for this block's channels: the largest cutoff
    // of the aligned 64-channel group (a k_pass wave) containing them
    int kw = NH;
    if (a.KC) {
        const int nn = (cbase & ~63) + lane;
        kw = (int)wave_max(nn < a.nchan ? (double)a.KC[(int64_t)mi * a.nchan + nn] : 1.0);
    }

    // the block's channel mask in lane registers (a.cb <= 64): testing the
    // next channel needs no global load (whose vmcnt wait would also wait
    // for every load issued before it)
    const int mlane = (cbase + lane < cend && (!mask || mask[cbase + lane])) ? 1 : 0;
    auto usable = [&](int n) {
        return n < cend && __builtin_amdgcn_readlane(mlane, n - cbase) != 0;
    };
    // |M|^2 sum and sigma of channel cbase + lane in lane registers, read by
    // readlane per row (round 5, as k_xspec_w2): their global loads in the
    // row loop came after the next row's prefetch, and vmcnt counts in order
    const int nlr = cbase + lane;
    const double ch_mpow = nlr < cend ? a.Mpow[(int64_t)mi * a.nchan + nlr] : 0.0;
    const double ch_err = (a.errs && nlr < cend) ? a.errs[(int64_t)s * a.nchan + nlr] : 0.0;
    // fused guess: per-lane channel weight and dedispersion phase of
    // channel cbase + lane; the workgroup sum G[1..NL) after the twiddles
    constexpr int NL = 64 * guess_npl(LOG2N);
    bool gon = false;
    // the row's weight and dedispersion phase come from wave-uniform loads
    // (guess_weights, freqs) and two uniform scalars (Dg, nu_ref^-2, moved
    // to SGPRs): no VGPRs held across the round loop for them
    double g_Dg = 0.0, g_nrm2 = 0.0, g_w2e2 = 0.0;
    auto g_wn = [&](int nn) {
        return a.guess_weights[(int64_t)s * a.nchan + __builtin_amdgcn_readfirstlane(nn)];
    };
    auto g_dgn = [&](int nn) {
        const double f = a.freqs[(int64_t)s * a.nchan + __builtin_amdgcn_readfirstlane(nn)];
        return g_Dg * (1.0 / (f * f) - g_nrm2);
    };
    double2 *gacc = lds + kXSW * SL + (PPF_TW_LDS ? tw_slots<LOG2N>() : 0);
    if constexpr (GS) {
        gon = a.gflag[s] != 0;                         // uniform
        if (gon) {
            for (int t = threadIdx.x; t < NL; t += 64 * kXSW) gacc[t] = cmk(0.0, 0.0);
            // nu_ref: mean usable frequency of the sub-int (GetTOAs) or
            // nu_fit (ppalign), as k_dsum
            const double *fr = a.freqs + (int64_t)s * a.nchan;
            double v0 = 0.0, v1 = 0.0;
            for (int nn = lane; nn < a.nchan; nn += 64)
                if (!mask || mask[nn]) { v0 += fr[nn]; v1 += 1.0; }
            v0 = wave_sum(v0);
            v1 = wave_sum(v1);
            const double mu = v0 / v1;
            double nu_ref_m2 = 1.0 / (mu * mu);
            if (a.guess_ref) {
                const double nf = a.nu_fits[(int64_t)s * 3];
                if (nf == nf) nu_ref_m2 = 1.0 / (nf * nf);
            }
            g_Dg = readlane_d(kDconst * a.guess_DM[s] / a.P[s], 0);
            g_nrm2 = readlane_d(nu_ref_m2, 0);
            __syncthreads();
        }
    }
    RowT zr[R];
    auto fetch = [&](int n) {
        const RowT *src = rows + ((int64_t)s * a.nchan + n) * N;
#pragma unroll
        for (int q = 0; q < R; ++q) zr[q] = ld_stream(src + lane + 64 * q);
    };
    int n = cbase + wave;
    if (usable(n)) fetch(n);
    for (int r = 0; r < nround; ++r, n += kXSW) {
        const bool live = usable(n);
        if (n < cend && !live) {
            if (lane < 4) a.chan[((int64_t)s * a.nchan + n) * 4 + lane] = 0.0;
            if (usable(n + kXSW)) fetch(n + kXSW);
        }
        if (live) {
            const int64_t crow = (int64_t)s * a.nchan + n;
            double2 x[R];
#pragma unroll
            for (int q = 0; q < R; ++q) x[q] = cmk((double)zr[q].x, (double)zr[q].y);
            const double2 *Mrow = a.Mft + ((int64_t)mi * a.nchan + n) * NH;
            const bool nxt = usable(n + kXSW);
            if (nxt) fetch(n + kXSW);                   // next row in flight during this FFT
            wfft::fft_row<LOG2N>(x, buf, tw, lane);

            // the model pairs of pass 2's first MD iterations, loaded now (the
            // FFT is done, so their wait no longer holds up anything): each
            // pass-2 iteration otherwise waited for its own two L2 loads
            double2 Mq[MD > 0 ? MD : 1][2];
            auto preload_m = [&]() {
#pragma unroll
                for (int i = 0; i < MD; ++i) {
                    Mq[i][0] = Mrow[lane + 64 * i];
                    Mq[i][1] = Mrow[N - lane - 64 * i];
                }
            };
#if PPF_XS_ONEPASS
            // ONE post-pass over the transform: each pair's D_k feeds the
            // power sums (noise, Sd) and leaves the UNSCALED D_k conj(M_k) in
            // the buffer; the row's 1/errs_FT^2 is known once the sums are
            // complete, and the write-out applies it (the same product in
            // the same order, so X is bit-identical to scaling it here).
            // The Nyquist bin leaves pad(N/2) before pair 0 overwrites it.
            double2 Dm = cmk(0.0, 0.0);
            if (lane == 0) {
                const double2 zm = buf[wfft::pad<LOG2N>(N / 2)];
                Dm = cmk(zm.x, -zm.y);
            }
            // guess phasor of this row: El = w e^{2 pi i k dphi} at k = lane
            // + 64 i by recurrence (step e^{2 pi i 64 dphi}: lane 1's phasor
            // squared six times)
            double2 El = cmk(0.0, 0.0), Est = El;
            if (GS && gon) {
                const double dg = g_dgn(n);
                const double2 E1 = cexp2pi((double)lane * dg);
                El = cscale(E1, g_wn(n));
                Est = cmk(readlane_d(E1.x, 1), readlane_d(E1.y, 1));
#pragma unroll
                for (int q = 0; q < 6; ++q) Est = cmul(Est, Est);
            }
            preload_m();
            double pn = 0.0, pd = 0.0;
            {
                double2 w = w_seed;
#pragma unroll
                for (int i = 0; i < NP; ++i) {
                    const int klo = lane + 64 * i, khi = N - klo;
                    double2 Dlo, Dhi;
                    rfft_pair<LOG2N>(buf, klo, w, Dlo, Dhi);
                    w = cmul(w, w_step);
                    const double p0 = cabs2(Dlo), p1 = cabs2(Dhi);
                    if (klo >= a.kc) pn += p0;
                    if (khi >= a.kc) pn += p1;
                    if (klo >= 1) pd += p0;
                    pd += p1;
                    // (fused guess: X stops below NL, past it only the sums)
                    if (!(GS && gon && 64 * i >= NL)) {
                        double2 Mlo, Mhi;
                        if constexpr (MD > 0) {
                            Mlo = Mq[i % MD][0];
                            Mhi = Mq[i % MD][1];
                            if (i + MD < NP) {
                                Mq[i % MD][0] = Mrow[klo + 64 * MD];
                                Mq[i % MD][1] = Mrow[khi - 64 * MD];
                            }
                        } else {
                            Mlo = Mrow[klo];
                            Mhi = Mrow[khi];
                        }
                        buf[wfft::pad<LOG2N>(klo)] = (klo == 0) ? cmk(0.0, 0.0) : cmulc(Dlo, Mlo);
                        if (GS && gon) {
                            // X_{N-k} is past the cutoff: its slot takes the
                            // row's guess term of harmonic k (k = 0: dropped)
                            if (klo != 0) buf[wfft::pad<LOG2N>(khi)] = cmul(Dlo, El);
                            El = cmul(El, Est);
                        } else {
                            buf[klo == 0 ? wfft::pad<LOG2N>(N / 2) : wfft::pad<LOG2N>(khi)] =
                                cmulc(Dhi, Mhi);
                        }
                    }
                    SCHED_CUT();
                }
            }
            if (lane == 0) {
                const double p = cabs2(Dm);
                if (N / 2 >= a.kc) pn += p;
                pd += p;
            }
            pn = wave_sum(pn);
            pd = wave_sum(pd);
            double errs_FT;
            if (a.errs) errs_FT = readlane_d(ch_err, n - cbase) * sqrtN;
            else errs_FT = sqrt(pn / (double)(NH - a.kc) / (double)(2 * N)) * sqrtN;
            const double inv_e2 = 1.0 / (errs_FT * errs_FT);
            if (GS && gon) {
                const double wn = g_wn(n);
                g_w2e2 += wn * wn * errs_FT * errs_FT;
            }
            if (lane == 0) {
                buf[XNYQ] = cmulc(Dm, Mrow[N / 2]);
                reinterpret_cast<double *>(buf + XIE2)[0] = inv_e2;   // for the write-out
                double *chan = a.chan + crow * 4;
                chan[0] = errs_FT;
                chan[1] = inv_e2;
                chan[2] = pd * inv_e2;                                  // Sd_n
                chan[3] = readlane_d(ch_mpow, n - cbase) * inv_e2;     // S_n at tau = 0
            }
#else
            preload_m();
            // pass 1: power sums (noise, Sd); pass 2 recomputes D for X
            double pn = 0.0, pd = 0.0;
            {
                double2 w = w_seed;
#pragma unroll
                for (int i = 0; i < NP; ++i) {
                    const int klo = lane + 64 * i, khi = N - klo;
                    double2 Dlo, Dhi;
                    rfft_pair<LOG2N>(buf, klo, w, Dlo, Dhi);
                    w = cmul(w, w_step);
                    const double p0 = cabs2(Dlo), p1 = cabs2(Dhi);
                    if (klo >= a.kc) pn += p0;
                    if (khi >= a.kc) pn += p1;
                    if (klo >= 1) pd += p0;
                    pd += p1;
                    SCHED_CUT();
                }
            }
            double2 Dm = cmk(0.0, 0.0);
            if (lane == 0) {
                const double2 zm = buf[wfft::pad<LOG2N>(N / 2)];
                Dm = cmk(zm.x, -zm.y);
                const double p = cabs2(Dm);
                if (N / 2 >= a.kc) pn += p;
                pd += p;
            }
            pn = wave_sum(pn);
            pd = wave_sum(pd);
            double errs_FT;
            if (a.errs) errs_FT = readlane_d(ch_err, n - cbase) * sqrtN;
            else errs_FT = sqrt(pn / (double)(NH - a.kc) / (double)(2 * N)) * sqrtN;
            const double inv_e2 = 1.0 / (errs_FT * errs_FT);

            // guess phasor of this row: El = w e^{2 pi i k dphi} at k = lane
            // + 64 i by recurrence (step e^{2 pi i 64 dphi}: lane 1's phasor
            // squared six times)
            double2 El = cmk(0.0, 0.0), Est = El;
            if (GS && gon) {
                const int r = n - cbase;
                const double wn = g_wn(n), dg = g_dgn(n);
                const double2 E1 = cexp2pi((double)lane * dg);
                El = cscale(E1, wn);
                Est = cmk(readlane_d(E1.x, 1), readlane_d(E1.y, 1));
#pragma unroll
                for (int q = 0; q < 6; ++q) Est = cmul(Est, Est);
                g_w2e2 += wn * wn * errs_FT * errs_FT;
            }
            {
                // in place: X_k -> pad(k), X_{N-k} -> pad(N-k); the pair
                // (0, N) keeps X_N in pad(N/2) (read above as Dm).  (Skipping
                // the pairs past the block's cutoff, and X_{N-k} when the
                // cutoff is below N/2, measured slower: C3 k_xspec_w 27.8 ->
                // 28.6 ms, C2 with MOM_X 27.3 -> 28.3 ms)
                double2 w = w_seed;
#pragma unroll
                for (int i = 0; i < NP; ++i) {
                    const int klo = lane + 64 * i, khi = N - klo;
                    if (GS && gon && 64 * i >= NL) break;   // (uniform) beyond the cutoff
                    double2 Dlo, Dhi;
                    rfft_pair<LOG2N>(buf, klo, w, Dlo, Dhi);
                    w = cmul(w, w_step);
                    // (loading these before the next row's prefetch, so their
                    // in-order wait skips it, was measured: the extra
                    // registers cost occupancy, C5 29.7 -> 33.2 ms)
                    double2 Mlo, Mhi;
                    if constexpr (MD > 0) {
                        Mlo = Mq[i % MD][0];
                        Mhi = Mq[i % MD][1];
                        if (i + MD < NP) {
                            Mq[i % MD][0] = Mrow[klo + 64 * MD];
                            Mq[i % MD][1] = Mrow[khi - 64 * MD];
                        }
                    } else {
                        Mlo = Mrow[klo];
                        Mhi = Mrow[khi];
                    }
                    buf[wfft::pad<LOG2N>(klo)] =
                        (klo == 0) ? cmk(0.0, 0.0) : cscale(cmulc(Dlo, Mlo), inv_e2);
                    if (GS && gon) {
                        // X_{N-k} is past the cutoff: its slot takes the
                        // row's guess term of harmonic k (k = 0: dropped)
                        if (klo != 0) buf[wfft::pad<LOG2N>(khi)] = cmul(Dlo, El);
                        El = cmul(El, Est);
                    } else {
                        buf[klo == 0 ? wfft::pad<LOG2N>(N / 2) : wfft::pad<LOG2N>(khi)] =
                            cscale(cmulc(Dhi, Mhi), inv_e2);
                    }
                    SCHED_CUT();
                }
            }
            if (lane == 0) {
                buf[XNYQ] = cscale(cmulc(Dm, Mrow[N / 2]), inv_e2);
                double *chan = a.chan + crow * 4;
                chan[0] = errs_FT;
                chan[1] = inv_e2;
                chan[2] = pd * inv_e2;                                  // Sd_n
                chan[3] = readlane_d(ch_mpow, n - cbase) * inv_e2;     // S_n at tau = 0
            }
#endif
        }
        __syncthreads();
        // write-out: thread t -> channel c = t % 8 of the round, harmonics
        // k = t / 8 + 64 j
        {
            const int c = threadIdx.x % kXSW, n0 = cbase + r * kXSW;
            const int nc = n0 + c;
            if (nc < cend) {
                const bool ok = !mask || mask[nc];
                const double2 *b = lds + c * SL;
#if PPF_XS_ONEPASS
                const double ie2 = ok ? reinterpret_cast<const double *>(b + XIE2)[0] : 0.0;
#endif
                for (int k = threadIdx.x / kXSW; k < kw; k += 64) {
                    const int slot = k == N ? wfft::pad<LOG2N>(N / 2)
                                            : (k == N / 2 ? XNYQ : wfft::pad<LOG2N>(k));
#if PPF_XS_ONEPASS
                    st_stream(Xs + (int64_t)k * a.nchan + nc, ok ? cscale(b[slot], ie2) : cmk(0.0, 0.0));
#else
                    st_stream(Xs + (int64_t)k * a.nchan + nc, ok ? b[slot] : cmk(0.0, 0.0));
#endif
                }
            }
        }
        if (GS && gon) {
            // the round's rows' guess terms, in wave order
            for (int t = threadIdx.x; t < NL; t += 64 * kXSW) {
                if (t == 0) continue;
                double2 acc = gacc[t];
#pragma unroll
                for (int w2 = 0; w2 < kXSW; ++w2)
                    if (usable(cbase + r * kXSW + w2)) acc = cadd(acc, lds[w2 * SL + wfft::pad<LOG2N>(N - t)]);
                gacc[t] = acc;
            }
        }
        __syncthreads();
    }
    if constexpr (GS) {
        if (gon) {
            double2 *gp = a.gpart + ((int64_t)s * a.nblk + cb) * NL;
            for (int t = threadIdx.x; t < NL; t += 64 * kXSW) gp[t] = gacc[t];
            // the block's weight sum and usable-channel count (every wave
            // holds the block's weights in its lanes), and sum w^2 errs_FT^2
            // per wave, added in wave order (buffer slot 0 is free after the
            // last round's barrier)
            const double gwl = mlane ? a.guess_weights[(int64_t)s * a.nchan + cbase + lane] : 0.0;
            const double wsum = wave_sum(gwl), cnt = wave_sum(mlane ? 1.0 : 0.0);
            if (lane == 0) reinterpret_cast<double *>(buf)[0] = g_w2e2;
            __syncthreads();
            if (threadIdx.x == 0) {
                double acc = 0.0;
                for (int w2 = 0; w2 < kXSW; ++w2) acc += reinterpret_cast<const double *>(lds + w2 * SL)[0];
                double *o = a.gw + ((int64_t)s * a.nblk + cb) * 3;
                o[0] = wsum;
                o[1] = cnt;
                o[2] = acc;
            }
        }
    }
}

// ===========================================================================
// k_xmom_g: fused moment pass (see the file header and below)
// ===========================================================================
template <int LOG2N, int XW>
__host__ __device__ constexpr int xmom_slw() {
    // >= 256 slots (the partial tile) + two side slots; consecutive wave
    // buffers start 8 (XW = 8) or 16 (XW = 4) banks apart for the A reads
    return (wfft::buf_slots<LOG2N>() < 272 ? 272 : wfft::buf_slots<LOG2N>()) + (XW == 8 ? 2 : 4);
}


// ===========================================================================
// k_xmom_g: the fused moment pass with the sub-int group layout.
//   Block = (group of 8 sub-ints, block of a.cb <= 64 channels); wave w owns
//   sub-int 8 g + w, and round r processes channel cb a.cb + r for all eight
//   waves.  The round's model row M_n (and sum_k |M_nk|^2) is shared by the
//   eight rows, so it is staged once in LDS instead of being re-read from L2
//   by every row (SH = true: one model per batch).  With several models
//   (SH = false) every wave reads its own model row from L2 with the same
//   arithmetic, so a sub-int's moments do not depend on the batch it is in.
//   The moment centre of each channel is rounded to a whole bin, s_n = rint(nbin phi_c,n) (bin_centre): the phasor e^{2 pi i k s_n /
//   nbin} is then an exact circular shift of the time-domain row, applied by
//   the load indices, and Y_k = D'_k conj(M_k) needs no phasor arithmetic;
//   k_tr_mom adds the residual phi_c,n - s_n/nbin (mres) to every expansion
//   offset.  MFMA A rows = 8 sub-ints x {Re, Im}; B = v_k^j computed in
//   registers.
//   Memory ordering: the only global loads inside the round loop are the
//   prefetches for the NEXT round (model row first, then the data row), so no
//   s_waitcnt inside a round waits for them (vmcnt is in order on gfx950):
//   FFT twiddles live in LDS, and the per-channel inputs (dphi, errs, mask)
//   are read once per block into lane registers and broadcast by readlane.
// ===========================================================================
#ifndef PPF_G_CUT
#define PPF_G_CUT 1
#endif
#if PPF_G_CUT
#define G_CUT() __builtin_amdgcn_sched_barrier(0)
#else
#define G_CUT()
#endif
#ifdef PPF_XM_PROF
// section cycle counters of k_xmom_g (profiling builds only)
__device__ unsigned long long g_xprof[8];
#define XP_INIT() unsigned long long xp_acc[7] = {0, 0, 0, 0, 0, 0, 0}; unsigned long long xp_t = __builtin_amdgcn_s_memtime()
#define XP(i) do { const unsigned long long xp_n = __builtin_amdgcn_s_memtime(); xp_acc[i] += xp_n - xp_t; xp_t = xp_n; } while (0)
#define XP_DONE() do { if (lane == 0) for (int xi = 0; xi < 7; ++xi) atomicAdd(&g_xprof[xi], xp_acc[xi]); } while (0)
#else
#define XP_INIT()
#define XP(i)
#define XP_DONE()
#endif
__device__ __forceinline__ double bin_centre(double phc, int nbin) {
    return rint(phc * (double)nbin);
}
template <int LOG2N>
__host__ __device__ constexpr size_t xmom_g_lds() {
    return ((size_t)8 * xmom_slw<LOG2N, 8>() + (1 << LOG2N) + 2 + tw_slots<LOG2N>()) * sizeof(double2);
}

// FULL = true: the batch's first moment pass (every moment-mode sub-int);
// false: re-centring passes for the few sub-ints that left the expansion
// radius.  Same code; separate instantiations keep the two launch kinds
// apart in kernel traces (the first pass is the one bench.py prices).
template <int LOG2N, int DT, bool SH, bool FULL>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_xmom_g(XmomArgs a) {
    using P = wfft::Plan<LOG2N>;
    constexpr int XW = 8;
    constexpr int N = P::N, R = P::R, NH = N + 1;
    constexpr int NP = N / 128;
    constexpr int SLW = xmom_slw<LOG2N, XW>();
    constexpr int SIDE = SLW - 1;      // Y_{N/2}
    constexpr int SIDE2 = SLW - 2;     // 1/sigma~_n^2 of the row (.x)
    constexpr int KPW = N / 2 / XW;    // folded harmonics (MFMA K) per wave
    constexpr int MPT = (NH + 511) / 512;   // model-row elements per thread
    constexpr int TWN = tw_slots<LOG2N>();
    using ElT = typename std::conditional<DT == 0, float, double>::type;
    // data rows move as 16-B vectors: VE elements per load, NLD loads per lane
    using VecT = typename std::conditional<DT == 0, vf4, vd2>::type;
    constexpr int VE = 16 / (int)sizeof(ElT), NLD = 2 * N / (64 * VE);
    static_assert((2 * N + VE) * sizeof(ElT) <= SLW * sizeof(double2), "row staging fits the buffer");
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double2 *buf = lds + wave * SLW;
    double2 *mrow = lds + XW * SLW;    // model row M_n[0..N], [NH] = (sum |M|^2, 0)
    double2 *tw = mrow + NH + 1;       // FFT twiddles T[0..TWN)

    int g, cb;
    block_map(a.xcd_swizzle, a.nblk, g, cb);
    // wave-uniform in SGPRs (readfirstlane): the row pointers then take the
    // SADDR + 32-bit lane offset load form instead of 64-bit VGPR pointers
    // (at 256 VGPRs those spilled, and every scratch reload waited for all
    // outstanding row prefetches)
    // re-centring launches take the sub-ints k_tr_mom listed, eight to a
    // workgroup (a sub-int's moments do not depend on its group: MFMA rows
    // and the fixed-order partial sums are per sub-int)
    int s = g * XW + wave;
    if (!FULL && a.rc_list) {
        const unsigned cnt = *a.rc_count;
        s = (unsigned)s < cnt ? a.rc_list[s] : a.nsub;
    }
    s = __builtin_amdgcn_readfirstlane(s);
    const TRState *st = reinterpret_cast<const TRState *>(a.state);
    const bool act = s < a.nsub && st[s].mmode && st[s].need_mom;
    if (!__syncthreads_or(act)) return;                  // uniform per workgroup
    const int q = act ? st[s].mtarget : 0;
    // wave-uniform: held in SGPRs
    const double c0 = readfirst_d(act ? st[s].mc[q][0] : 0.0),
                 c1 = readfirst_d(act ? st[s].mc[q][1] : 0.0),
                 c2 = readfirst_d(act ? st[s].mc[q][2] : 0.0);
    const int sv = __builtin_amdgcn_readfirstlane(act ? s : 0);

    const int cbase = cb * a.cb, cend = min(a.nchan, cbase + a.cb);
    const ElT *rows = reinterpret_cast<const ElT *>(a.data) + (int64_t)sv * a.nchan * (2 * N);
    const double2 *Mbase = a.Mft;
    // SH = false: this wave's own model (rows [nchan][NH], powers [nchan])
    const int mi = (!SH && a.model_index) ? a.model_index[sv] : 0;
    const double2 *Mwave = a.Mft + (int64_t)mi * a.nchan * NH;
    const double *Pwave = a.Mpow + (int64_t)mi * a.nchan;
    double *mres = a.mres + ((int64_t)sv * 2 + q) * a.nchan;
    const double2 w_seed = a.T2[lane];
    const double2 w_step = cmk(readfirst_d(a.T2[64].x), readfirst_d(a.T2[64].y));
    const double sqrtN = sqrt((double)N);
    double *mom = a.mom + (((int64_t)sv * 2 + q) * a.nchan) * kMoments * 2;

    // per-lane channel tables: lane l holds channel cbase + l
    double ch_d0 = 0.0, ch_d1 = 0.0, ch_e = 0.0;
    int ch_use = 0;
    // the harmonic cutoff of the block's channels, also per lane: a global
    // load of KC[n] inside the round would wait (vmcnt is in order) for the
    // next round's prefetch
    int ch_kc = NH;
    if (SH && a.KC && lane < cend - cbase) ch_kc = a.KC[cbase + lane];
    if (act && lane < cend - cbase) {
        const int64_t row = (int64_t)sv * a.nchan + cbase + lane;
        ch_d0 = a.dphi[row * 2];
        ch_d1 = a.dphi[row * 2 + 1];
        if (a.errs) ch_e = a.errs[row];
        ch_use = (!a.mask || a.mask[row]) ? 1 : 0;
    }

    const int arow = lane & 15, kk = lane >> 4, bj = lane & 15;
    const double *abase = reinterpret_cast<const double *>(lds + (arow >> 1) * SLW) + (arow & 1);
    constexpr double ih = 2.0 / (double)N;
    const int k0 = wave * KPW;

    vd2 mp[MPT];
    double mpw = 0.0;
    auto mload = [&](int n) {
        if constexpr (!SH) return;
        const int nn = min(n, a.nchan - 1);
        const double2 *src = Mbase + (int64_t)nn * NH;
        int tq = tid;                   // opaque: offsets not kept across rounds
        asm volatile("" : "+v"(tq));
#pragma unroll
        for (int i = 0; i < MPT; ++i) {
            const int k = tq + 512 * i;
            const double2 v = src[k < NH ? k : 0];
            mp[i] = vd2{v.x, v.y};
        }
        if (tid == 0) mpw = a.Mpow[nn];
    };
    auto mstore = [&]() {
        if constexpr (!SH) return;
#pragma unroll
        for (int i = 0; i < MPT; ++i) {
            const int k = tid + 512 * i;
            if (k < NH) mrow[k] = cmk(mp[i][0], mp[i][1]);
        }
        if (tid == 0) mrow[NH] = cmk(mpw, 0.0);
    };
    // The row is fetched unshifted with coalesced 16-B loads (lane l holds
    // elements VE (l + 64 c)), staged through the wave's LDS buffer and read
    // back shifted: z_j = x[(2j + sh) mod 2N] + i x[(2j + 1 + sh) mod 2N].
    // (Per-element 4-B loads with the shift in the address cost 4x the
    // vector-memory issue slots.)
    VecT zr[NLD];
    double nx_r = 0.0;
    int nx_sh = 0;
    auto fetch = [&](int n) {
        const int r = n - cbase;
        const double phc = c0 + c1 * readlane_d(ch_d0, r) + c2 * readlane_d(ch_d1, r);
        const double sb = bin_centre(phc, 2 * N);
        nx_sh = (int)(sb - (double)(2 * N) * floor(sb / (double)(2 * N)));
        nx_r = phc - sb / (double)(2 * N);          // residual centre offset
        const char *x = reinterpret_cast<const char *>(rows + (int64_t)n * (2 * N));
        // the lane's byte offset is re-derived every round (opaque): hoisted,
        // base + offset became a live 64-bit VGPR pointer that spilled
        unsigned off = (unsigned)lane * 16u;
        asm volatile("" : "+v"(off));
#pragma unroll
        for (int c = 0; c < NLD; ++c)
            zr[c] = ld_stream(reinterpret_cast<const VecT *>(x + off + 1024u * (unsigned)c));
    };
    auto usable = [&](int n) {
        return act && n < cend && __builtin_amdgcn_readlane(ch_use, n - cbase) != 0;
    };

    for (int i = tid; i < TWN; i += 512) tw[i] = a.T[i];
    int n = cbase;
    mload(n);
    mstore();
    if (act) fetch(n);
    __syncthreads();
    XP_INIT();
    for (; n < cend; ++n) {
        const bool live = usable(n);
        const double res_in = nx_r;
        const int sh = nx_sh;
        const double errs_in = a.errs ? readlane_d(ch_e, n - cbase) : 0.0;
        // stage: raw row + the first VE elements again past the end (the
        // odd-shift read of element 2N - 1 takes its partner from there)
        ElT *row = reinterpret_cast<ElT *>(buf);
        if (live) {
#pragma unroll
            for (int c = 0; c < NLD; ++c) *reinterpret_cast<VecT *>(row + VE * (lane + 64 * c)) = zr[c];
            if (lane == 0) *reinterpret_cast<VecT *>(row + 2 * N) = zr[0];
        }
        XP(6);
        // next round's model row, then its data row, in flight during this
        // round (the data load is unconditional for active waves: keeps zr[]
        // in VGPRs)
        mload(n + 1);
        if (act) fetch(n + 1 < cend ? n + 1 : n);
        XP(0);
        if (live) {
            const int64_t crow = (int64_t)s * a.nchan + n;
            wfft::wave_sync();
            double2 x[R];
#pragma unroll
            for (int qq = 0; qq < R; ++qq) {
                const int j2 = (2 * (lane + 64 * qq) + sh) & (2 * N - 1);
                x[qq] = cmk((double)row[j2], (double)row[j2 + 1]);
            }
            wfft::wave_sync();
#ifndef G_NOFFT
            wfft::fft_row<LOG2N>(x, buf, tw, lane);
            XP(1);
#else
            for (int qq = 0; qq < R; ++qq) buf[wfft::pad<LOG2N>(lane + 64 * qq)] = x[qq];
#endif
            double2 Dm = cmk(0.0, 0.0);
            if (lane == 0) {
                const double2 zm = buf[wfft::pad<LOG2N>(N / 2)];
                Dm = cmk(zm.x, -zm.y);
            }
            // in place: iteration i reads and rewrites only pad(k) and
            // pad(N - k), k = lane + 64 i (k = 0: the pair (0, N) -> pad(0),
            // pad(N/2), read above as Dm)
            double pn = 0.0, pd = 0.0;
            // the pair's LDS addresses and u_k re-derived from an opaque lane
            // every round: hoisted out of the channel loop they took ~32
            // VGPRs, spilled, and each scratch reload waited for the
            // in-flight row prefetch
            int lpp = lane;
            asm volatile("" : "+v"(lpp));
            auto pair = [&](const double2 *Mr, int i, double2 &w) {
                    const int klo = lpp + 64 * i, khi = N - klo;
                    double2 Dlo, Dhi;
                    rfft_pair<LOG2N>(buf, klo, w, Dlo, Dhi);
                    w = cmul(w, w_step);
                    const double p0 = cabs2(Dlo), p1 = cabs2(Dhi);
                    if (klo >= a.kc) pn += p0;
                    if (khi >= a.kc) pn += p1;
                    if (klo >= 1) pd += p0;
                    pd += p1;
                    const double2 Ylo = klo == 0 ? cmk(0.0, 0.0) : cmulc(Dlo, Mr[klo]);
                    const double2 Yhi = cmulc(Dhi, Mr[khi]);
                    const double uk = (double)(klo - N / 2) * ih;
                    buf[wfft::pad<LOG2N>(klo)] = cadd(Ylo, Yhi);
                    buf[klo == 0 ? wfft::pad<LOG2N>(N / 2) : wfft::pad<LOG2N>(khi)] =
                        cscale(csub(Ylo, Yhi), uk);
            };
            const double2 *Mr = SH ? mrow : Mwave + (int64_t)n * NH;
            double2 w = w_seed;
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                pair(Mr, i, w);
                G_CUT();
            }
            if (lane == 0) buf[SIDE] = cmulc(Dm, Mr[N / 2]);
            const double mpow = SH ? mrow[NH].x : Pwave[n];
            if (lane == 0) {
                const double p = cabs2(Dm);
                if (N / 2 >= a.kc) pn += p;
                pd += p;
            }
            pn = wave_sum(pn);
            pd = wave_sum(pd);
            const double errs_FT = a.errs ? errs_in * sqrtN
                                          : sqrt(pn / (double)(NH - a.kc) / (double)(2 * N)) * sqrtN;
            const double inv_e2 = 1.0 / (errs_FT * errs_FT);
            if (lane == 0) {
                buf[SIDE2] = cmk(inv_e2, 0.0);
                double *chan = a.chan + crow * 4;
                chan[0] = errs_FT;
                chan[1] = inv_e2;
                chan[2] = pd * inv_e2;        // Sd_n
                chan[3] = mpow * inv_e2;      // S_n at tau = 0
                mres[n] = res_in;
            }
        } else if (act && n < cend && lane < 4) {
            unsigned lo = (unsigned)lane;       // opaque: see fetch()
            asm volatile("" : "+v"(lo));
            a.chan[((int64_t)s * a.nchan + n) * 4 + lo] = 0.0;      // masked channel
        }
        XP(2);
        __syncthreads();
        XP(3);
        mstore();                         // this round no longer reads mrow

        f64x4 d0 = {0.0, 0.0, 0.0, 0.0}, d1 = d0;
        // folded pairs (k, N - k) with k >= KC_n hold only harmonics whose
        // model amplitude is below 1e-14 of its peak (k_model_cut): the
        // needed range [0, KC_n) is spread over the eight waves instead
        int kpw = KPW, kw0 = k0;
        if constexpr (SH) {
            const int kn = __builtin_amdgcn_readlane(ch_kc, n - cbase);
            if (kn < N / 2) {
                kpw = min(KPW, ((kn + 4 * XW - 1) / (4 * XW)) * 4);
                kw0 = wave * kpw;
            }
        }
#ifndef G_NOMFMA
#pragma unroll 4
        for (int t = 0; t < KPW / 4; ++t) {
            if (t >= (kpw >> 2)) break;                       // wave-uniform
            const int k = kw0 + 4 * t + kk;
            const int se = wfft::pad<LOG2N>(k);
            const int so = k == 0 ? wfft::pad<LOG2N>(N / 2) : wfft::pad<LOG2N>(N - k);
            // B[k][j] = v_k^j, v = u_k^2 (same arithmetic as k_btab)
            const double u = (double)(k - N / 2) * ih;
            const double v = u * u, v2 = v * v, v4 = v2 * v2, v8 = v4 * v4;
            const double bv = ((bj & 1) ? v : 1.0) * ((bj & 2) ? v2 : 1.0) * ((bj & 4) ? v4 : 1.0) *
                              ((bj & 8) ? v8 : 1.0);
            d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(abase[2 * se], bv, d0, 0, 0, 0);
            d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(abase[2 * so], bv, d1, 0, 0, 0);
        }
#endif
        XP(4);
        // output element tid: this wave's sub-int, moment om = 2 j + set,
        // Re/Im ori
        const int om = (tid >> 1) & 31, ori = tid & 1;
        double val = 0.0;
        if (om == 0) val = reinterpret_cast<const double *>(buf + SIDE)[ori];
        const double ie = reinterpret_cast<const double *>(buf + SIDE2)[0];
        __syncthreads();
        {
            double *sc = reinterpret_cast<double *>(buf);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                sc[rr * 64 + lane] = d0[rr];
                sc[256 + rr * 64 + lane] = d1[rr];
            }
        }
        __syncthreads();
        {
            const int row = 2 * wave + ori;
            const int idx = (om & 1) * 256 + (row >> 2) * 64 + ((row & 3) << 4) + (om >> 1);
#pragma unroll
            for (int w2 = 0; w2 < XW; ++w2) val += reinterpret_cast<const double *>(lds + w2 * SLW)[idx];
            unsigned mo = (unsigned)(om * 2 + ori);     // opaque: see fetch()
            asm volatile("" : "+v"(mo));
            if (live) mom[(int64_t)n * kMoments * 2 + mo] = val * ie;
        }
        __syncthreads();
        XP(5);
    }
    XP_DONE();
}

// folded-moment B table: Bt[k][j] = (u_k^2)^j, u_k = (k - N/2)/(N/2), k < N/2
__global__ void k_btab(int N, double *Bt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N / 2 * 16) return;
    const int k = i >> 4, j = i & 15;
    const double u = (double)(k - N / 2) * (2.0 / (double)N);
    const double v = u * u, v2 = v * v, v4 = v2 * v2, v8 = v4 * v4;
    Bt[i] = ((j & 1) ? v : 1.0) * ((j & 2) ? v2 : 1.0) * ((j & 4) ? v4 : 1.0) * ((j & 8) ? v8 : 1.0);
}

// per model row: sum_{k>=1} |M_nk|^2 (the tau = 0 S_n numerator)
__global__ void k_model_pow(const double2 *Mft, int nrows, int nharm, double *out) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (row >= nrows) return;
    const double2 *M = Mft + (int64_t)row * nharm;
    double acc = 0.0;
    for (int k = lane + 1; k < nharm; k += 64) acc += cabs2(M[k]);
    acc = wave_sum(acc);
    if (lane == 0) out[row] = acc;
}

// sum_n M[model][n][k] over all channels, fixed order (mean model spectrum of
// the GetTOAs guess; k_guess removes the masked channels)
// sum over channels of the model spectra: workgroup = 16 harmonics x 16
// channel groups; each thread sums its group in channel order, then the 16
// group partials are added in group order (deterministic)
__global__ __launch_bounds__(256) void k_model_sum(const double2 *Mft, int nchan, int nharm,
                                                   int nmodel, double2 *out) {
    __shared__ double2 part[16][17];
    const int kl = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int k = blockIdx.x * 16 + kl;
    const int m = blockIdx.y;
    const int per = (nchan + 15) / 16;
    const int n0 = grp * per, n1 = min(nchan, n0 + per);
    double2 acc = cmk(0.0, 0.0);
    if (k < nharm) {
        const double2 *M = Mft + (int64_t)m * nchan * nharm + k;
        // (unrolled: the loads of eight channels in flight, added in the
        // same channel order -- C5's 1,024 channels per thread were one
        // dependent load after another, 0.46 ms per call)
#pragma unroll 8
        for (int n = n0; n < n1; ++n) acc = cadd(acc, M[(int64_t)n * nharm]);
    }
    part[grp][kl] = acc;
    __syncthreads();
    if (grp == 0 && k < nharm) {
        double2 t = part[0][kl];
        for (int g = 1; g < 16; ++g) t = cadd(t, part[g][kl]);
        out[(int64_t)m * nharm + k] = t;
    }
}

// ===========================================================================
// k_xspec_w2: k_xspec_w for 1024-point rows (2048 bins) on the one-exchange
// wave FFT of ppf_wfft2.hpp (round 5).  Same outputs and the same
// workgroup structure (4 waves, a round of 4 channel rows, X written
// harmonic-major after a barrier), but per row:
//   - one LDS exchange inside the FFT instead of three, no natural-order
//     write-back: the real post-pass takes each pair (Z_k, Z_{N-k}) from
//     registers after a v_permlane32_swap (wf2::pairs);
//   - each lane's slot i holds the harmonics k = kA + 64 i and N - k; the
//     lower one (< N/2) is what X and the guess need below their cutoffs,
//     so one model load, one D conj(M) and one LDS store per slot (two only
//     when the group's cutoff passes N/2);
//   - the X staging slots are k + k/64 (k <= N): no special Nyquist slot.
// get_noise_PS (pplib.py:2312-2332), Sd, S(tau = 0) and X = D conj(M) /
// sigma~^2 (pptoaslib.py:1014-1031) as k_xspec_w; the fused GetTOAs guess
// (GS, pptoas.py:461-464) as k_xspec_w, its terms in the slots of N - k.
// PPF_XSPEC2=0 (environment) selects k_xspec_w instead.
// ===========================================================================
// waves per workgroup (= rows per round, channels per X line written:
// 4 -> 64-B segments of the 128-B lines, two workgroups per CU; 8 -> whole
// lines, one workgroup per CU)
#ifndef PPF_X2W
#define PPF_X2W 4
#endif
constexpr int kX2W = PPF_X2W;
constexpr int kX2SL = wf2::kXSlots + wf2::kSpSlots;       // 1072 slots per wave
constexpr int kX2IE = 1041;                               // the row's 1/errs_FT^2 (.x)
__device__ __forceinline__ int x2slot(int k) { return k + (k >> 6); }   // k <= 1024 -> <= 1040
#ifndef PPF_X2_MD
#define PPF_X2_MD 4
#endif
#ifndef PPF_XSPEC2
#define PPF_XSPEC2 1
#endif
#ifndef PPF_X2_NT
#define PPF_X2_NT (PPF_NT ? 3 : 0)   // nontemporal row loads (1), X stores (2): ld/st_stream
#endif
#ifndef PPF_X2_MEARLY
#define PPF_X2_MEARLY 0
#endif
#ifndef PPF_X2_LATEPF
#define PPF_X2_LATEPF 0
#endif
#ifndef PPF_X2_EW
#define PPF_X2_EW 1
#endif
// PPF_X2_DIAG (timing-only builds, results wrong): 1 no X stores, 2 every
// model load from the first model row (L2 hits), 4 no FFT (the row values go
// straight to the post-pass)
#ifndef PPF_X2_DIAG
#define PPF_X2_DIAG 0
#endif
#ifndef PPF_X2_WR
#define PPF_X2_WR 0
#endif

template <int DT, bool GS>
__global__ __launch_bounds__(64 * kX2W) __attribute__((amdgpu_waves_per_eu(2)))
void k_xspec_w2(XspecArgs a) {
    constexpr int N = 1024, NH = N + 1;
    constexpr int MD = PPF_X2_MD;
    using RowT = typename std::conditional<DT == 0, vf2, vd2>::type;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int lane0 = threadIdx.x & 63;
    // (wave-uniform: the row pointers built from it stay in SGPRs, so the
    // loads take the scalar-base + 32-bit-offset form)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double2 *buf = lds + wave * kX2SL;

    int s, cb;
    block_map(a.xcd_swizzle, a.nblk, s, cb, a.nsub);
    if (a.needx && !a.needx[s]) return;               // uniform: moment-mode sub-int (or no slot)
    const int cbase = cb * a.cb, cend = min(a.nchan, cbase + a.cb);
    const int nround = (a.cb + kX2W - 1) / kX2W;
    const int mi = a.model_index ? a.model_index[s] : 0;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double sqrtN = sqrt((double)N);
    const RowT *rows = reinterpret_cast<const RowT *>(a.data);
    const wf2::Seeds sd = wf2::make_seeds(lane0);
    // post-pass twiddle e^{-i pi k / N} of the lane's first pair, step
    // e^{-i pi 64 / N}
    double2 wA0, wstep;
    {
        double sn, cs;
        sincospi(-(double)wf2::pair_k0(lane0) / (double)N, &sn, &cs);
        wA0 = cmk(cs, sn);
        sincospi(-64.0 / (double)N, &sn, &cs);
        wstep = cmk(cs, sn);
    }
    double2 *Xs = a.X + (int64_t)(a.xslot ? a.xslot[s] : s) * NH * a.nchan;
    int kw = NH;
    if (a.KC) {
        const int nn = (cbase & ~63) + lane0;
        kw = (int)wave_max(nn < a.nchan ? (double)a.KC[(int64_t)mi * a.nchan + nn] : 1.0);
    }
    const int mlane = (cbase + lane0 < cend && (!mask || mask[cbase + lane0])) ? 1 : 0;
    auto usable = [&](int n) {
        return n < cend && __builtin_amdgcn_readlane(mlane, n - cbase) != 0;
    };
    constexpr int NL = 64 * guess_npl(10);
    bool gon = false;
    double g_Dg = 0.0, g_nrm2 = 0.0, g_w2e2 = 0.0;
    double2 *gacc = lds + kX2W * kX2SL;
    if constexpr (GS) {
        gon = a.gflag[s] != 0;                         // uniform
        if (gon) {
            for (int t = threadIdx.x; t < NL; t += 64 * kX2W) gacc[t] = cmk(0.0, 0.0);
            const double *fr = a.freqs + (int64_t)s * a.nchan;
            double v0 = 0.0, v1 = 0.0;
            for (int nn = lane0; nn < a.nchan; nn += 64)
                if (!mask || mask[nn]) { v0 += fr[nn]; v1 += 1.0; }
            v0 = wave_sum(v0);
            v1 = wave_sum(v1);
            const double mu = v0 / v1;
            double nu_ref_m2 = 1.0 / (mu * mu);
            if (a.guess_ref) {
                const double nf = a.nu_fits[(int64_t)s * 3];
                if (nf == nf) nu_ref_m2 = 1.0 / (nf * nf);
            }
            g_Dg = readlane_d(kDconst * a.guess_DM[s] / a.P[s], 0);
            g_nrm2 = readlane_d(nu_ref_m2, 0);
            __syncthreads();
        }
    }
    // the block's per-channel scalars in lane registers (lane l: channel
    // cbase + l): a global load of them inside the round loop would wait,
    // vmcnt being in order, for the next row's prefetch
    const int nl = cbase + lane0;
    const bool lin = nl < cend;
    const double ch_mpow = lin ? a.Mpow[(int64_t)mi * a.nchan + nl] : 0.0;
    const double ch_err = (a.errs && lin) ? a.errs[(int64_t)s * a.nchan + nl] : 0.0;
    double ch_wn = 0.0, ch_dg = 0.0;
    if (GS && gon && lin) {
        ch_wn = a.guess_weights[(int64_t)s * a.nchan + nl];
        const double f = a.freqs[(int64_t)s * a.nchan + nl];
        ch_dg = g_Dg * (1.0 / (f * f) - g_nrm2);
    }
    RowT zr[16];
    auto fetch = [&](int n) {
        const RowT *src = rows + ((int64_t)s * a.nchan + n) * N;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
#if PPF_X2_NT & 1
            zr[q] = __builtin_nontemporal_load(src + lane0 + 64 * q);
#else
            zr[q] = src[lane0 + 64 * q];
#endif
        }
    };
#if PPF_X2_EW
    // Round 6: the next row's load is unconditional (a row past the block,
    // or a masked one, is replaced by the block's last row: a valid address
    // whose values are ignored), so the row registers carry no phi between
    // loop paths (that cost two sets of 16 v_mov_b64 per row), and the wait
    // for it is forced at the END of the round (rows_ready), before the
    // round's X stores.  vmcnt counts loads and stores in issue order on
    // gfx950: waited at the top of the next round, as the compiler placed
    // it, the prefetch's wait included every X store of the write-out just
    // issued -- vmcnt(0) on the store acknowledgements once per row.
    auto fetch_c = [&](int m) { fetch(m < cend ? m : cend - 1); };
    auto rows_ready = [&]() {
#pragma unroll
        for (int q = 0; q < 16; ++q) asm volatile("" ::"v"(zr[q].x), "v"(zr[q].y));
    };
    int n = cbase + wave;
    fetch_c(n);
    rows_ready();
#else
    int n = cbase + wave;
    if (usable(n)) fetch(n);
#endif
    XP_INIT();
    for (int r = 0; r < nround; ++r, n += kX2W) {
        const bool live = usable(n);
#if PPF_X2_EW
        if (!PPF_X2_WR && n < cend && !live && lane0 < 4) a.chan[((int64_t)s * a.nchan + n) * 4 + lane0] = 0.0;
        double2 x[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            x[q] = cmk((double)zr[q].x, (double)zr[q].y);
            // (pinned here: sunk into the live branch below, the conversion
            // kept the old row registers alive past the next load, which
            // then took other registers and a copy per row)
            asm volatile("" : "+v"(x[q].x), "+v"(x[q].y));
        }
        // slot i: harmonics k = kA + 64 i and N - k; hl = the lower one
        // (lanes <= 32: k, the others: N - k), D of it in Dl.  Per-lane
        // indices re-derived every row from an opaque lane (hoisted out of
        // the round loop they would hold VGPRs for good)
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        const bool lo = lane <= 32;
        const int kA = wf2::pair_k0(lane);
        const int hl0 = lo ? kA : N - kA, hstep = lo ? 64 : -64;
        const double2 *Mrow = a.Mft + ((int64_t)mi * a.nchan + (n < cend ? n : cend - 1)) * NH;
#if PPF_X2_DIAG & 2
        Mrow = a.Mft;       // (timing-only build: every model load from the first row, L2 hits)
#endif
        // the first MD slots' model values: PPF_X2_MEARLY issues them here,
        // before the next row's prefetch, so that the post-pass's wait for
        // them (vmcnt is in order) does not include the prefetch; else
        // after the FFT.  The loads are unconditional (hl < N/2 is always a
        // valid index): under a lane-divergent branch the compiler cannot
        // count the loads in flight and waits for all of them (vmcnt(0),
        // the next row's prefetch included) at every slot.
        double2 Mq[MD > 0 ? MD : 1];
        auto mpre = [&]() {
#pragma unroll
            for (int i = 0; i < MD; ++i) Mq[i] = Mrow[(unsigned)(hl0 + hstep * i)];
        };
        if (PPF_X2_MEARLY && live) mpre();
        __builtin_amdgcn_sched_barrier(0);
        fetch_c(n + kX2W);                       // next row in flight during this FFT
#else
        if (n < cend && !live) {
            if (lane0 < 4) a.chan[((int64_t)s * a.nchan + n) * 4 + lane0] = 0.0;
            if (usable(n + kX2W)) fetch(n + kX2W);
        }
#endif
        if (live) {
            const int64_t crow = (int64_t)s * a.nchan + n;
#if !PPF_X2_EW
            double2 x[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) x[q] = cmk((double)zr[q].x, (double)zr[q].y);
#endif
            const int rr = n - cbase;
#if !PPF_X2_EW
            int lane = lane0;
            asm volatile("" : "+v"(lane));
            const bool lo = lane <= 32;
            const int kA = wf2::pair_k0(lane);
            const int hl0 = lo ? kA : N - kA, hstep = lo ? 64 : -64;
            const double2 *Mrow = a.Mft + ((int64_t)mi * a.nchan + n) * NH;
            double2 Mq[MD > 0 ? MD : 1];
            auto mpre = [&]() {
#pragma unroll
                for (int i = 0; i < MD; ++i) Mq[i] = Mrow[(unsigned)(hl0 + hstep * i)];
            };
            if (PPF_X2_MEARLY) mpre();
            if (!PPF_X2_LATEPF && usable(n + kX2W)) fetch(n + kX2W);   // next row in flight during this FFT
#endif
            XP(0);
#if !(PPF_X2_DIAG & 4)
            wf2::fft1024(x, buf, lane, sd);
#endif
            XP(1);
            if (PPF_X2_EW) __builtin_amdgcn_sched_barrier(0);
            if (!PPF_X2_MEARLY) mpre();
            if (!PPF_X2_EW && PPF_X2_LATEPF && usable(n + kX2W)) fetch(n + kX2W);
            double2 zm = cmk(0.0, 0.0);
            wf2::pairs(x, buf + wf2::kXSlots, lane, zm);
            XP(2);
            // guess phasor w_n e^{2 pi i hl dphi}, step e^{+-2 pi i 64 dphi}
            double2 El = cmk(0.0, 0.0), Est = El;
            if (GS && gon) {
                const double dg = readlane_d(ch_dg, rr);
                const double2 E1 = cexp2pi((double)hl0 * dg);
                El = cscale(E1, readlane_d(ch_wn, rr));
                // step e^{2 pi i 64 dphi}: lane 1's phasor (hl0 = 1) squared
                // six times
                Est = cmk(readlane_d(E1.x, 1), readlane_d(E1.y, 1));
#pragma unroll
                for (int q = 0; q < 6; ++q) Est = cmul(Est, Est);
                if (!lo) Est = cconj(Est);
            }
            // Per slot (the real-FFT post-pass in doubled form: the 0.5 of
            // e and o dropped, so Dl = 2 D_hl, v = the other harmonic's 2 D
            // up to conjugation; every product below is rescaled by an
            // exact power of two):
            //   e = Z_k + conj Z_{N-k}, o = Z_k - conj Z_{N-k}, wo = w o
            //   lanes <= 32 (sg = +1): 2 D_k = (e.x + wo.y, e.y - wo.x)
            //   the others (sg = -1):  2 D_{N-k} = conj of (e.x - wo.y, e.y + wo.x)
            // u = e + sg (wo.y, -wo.x): Dl = (u.x, sg u.y) is 2 D_hl; v = e -
            // sg (...) has |v| = |2 D_{N - hl}|.
            const double sg = lo ? 1.0 : -1.0;
            const int hcut = N - a.kc;            // N - hl >= kc  <=>  hl <= hcut
            double pn = 0.0, pd = 0.0;
            double2 w = wA0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const double2 zk = x[i], zn = x[i + 8];
                const double ex = zk.x + zn.x, ey = zk.y - zn.y;
                const double ox = zk.x - zn.x, oy = zk.y + zn.y;
                const double wox = fma(w.x, ox, -w.y * oy), woy = fma(w.x, oy, w.y * ox);
                w = cmul(w, wstep);
                const double ux = fma(sg, woy, ex), uy = fma(-sg, wox, ey);
                const double vx = fma(-sg, woy, ex), vy = fma(sg, wox, ey);
                const double2 Dl = cmk(ux, sg * uy);
                const double ph = fma(vx, vx, vy * vy), pl = fma(ux, ux, uy * uy);
                const int hl = hl0 + hstep * i;
                if (hl <= hcut) pn += ph;
                // (lane 0, slot 0: pl = |2 D_0|^2, which Sd leaves out)
                if (i == 0) pd += lane == 0 ? ph : pl + ph;
                else pd += pl + ph;
                double2 Ml;
                if constexpr (MD > 0) {
                    Ml = Mq[i % MD];
                    if (i + MD < 8) Mq[i % MD] = Mrow[(unsigned)(hl + hstep * MD)];
                } else {
                    Ml = Mrow[(unsigned)hl];
                }
                // 2 x the unscaled X of the low harmonic (the write-out
                // applies 1/(2 sigma~^2)); k = 0 zeroed (F0_fact = 0)
                // (k = 0 -- lane 0, slot 0 only -- is zeroed after the loop)
                if (hl < kw) buf[x2slot(hl)] = cmulc(Dl, Ml);
                if (GS && gon) {
                    // 2 x the row's guess term of harmonic hl, in the slot
                    // of N - hl (past X's cutoff: kw <= NL < N/2)
                    if (hl >= 1 && hl < NL) buf[x2slot(N - hl)] = cmul(Dl, El);
                    El = cmul(El, Est);
                } else if (kw > N / 2) {
                    // the group's cutoff passes N/2: the high harmonic too
                    // (2 D_{N - hl} = (vx, -sg vy))
                    const int hh = N - hl;
                    if (hh < kw) buf[x2slot(hh)] = cmulc(cmk(vx, -sg * vy), Mrow[(unsigned)hh]);
                }
            }
            XP(3);
            if (lane == 0) {
                buf[x2slot(0)] = cmk(0.0, 0.0);       // k = 0 (F0_fact = 0)
                // D_{N/2} (pairs: zm = Z_{N/2}), doubled like the rest
                const double2 Dm = cmk(2.0 * zm.x, -2.0 * zm.y);
                const double p = cabs2(Dm);
                if (N / 2 >= a.kc) pn += p;
                pd += p;
                if (N / 2 < kw) buf[x2slot(N / 2)] = cmulc(Dm, Mrow[N / 2]);
            }
            // the doubled sums: exact factor 4
            pn *= 0.25;
            pd *= 0.25;
            pn = wave_sum(pn);
            pd = wave_sum(pd);
            double errs_FT;
            if (a.errs) errs_FT = readlane_d(ch_err, rr) * sqrtN;
            else errs_FT = sqrt(pn / (double)(NH - a.kc) / (double)(2 * N)) * sqrtN;
            const double inv_e2 = 1.0 / (errs_FT * errs_FT);
            if (GS && gon) {
                const double wn = readlane_d(ch_wn, rr);
                g_w2e2 += wn * wn * errs_FT * errs_FT;
            }
            const double mpow = readlane_d(ch_mpow, rr);
            if (lane == 0) {
                // for the write-out: the staged X are doubled
                reinterpret_cast<double *>(buf + kX2IE)[0] = 0.5 * inv_e2;
#if PPF_X2_WR
                // the channel scalars go out with the round's write-out
                buf[kX2IE + 1] = cmk(errs_FT, inv_e2);
                buf[kX2IE + 2] = cmk(pd * inv_e2, mpow * inv_e2);    // Sd_n, S_n at tau = 0
                (void)crow;
#else
                double *chan = a.chan + crow * 4;
                chan[0] = errs_FT;
                chan[1] = inv_e2;
                chan[2] = pd * inv_e2;                                  // Sd_n
                chan[3] = mpow * inv_e2;                                // S_n at tau = 0
#endif
            }
        }
#if PPF_X2_EW
        rows_ready();
#endif
        XP(4);
        __syncthreads();
        XP(5);
#if PPF_X2_WR
        // write-out by ONE wave per round (wave r mod 4, rotating): vmcnt
        // counts stores and loads in issue order, so a wave that stores
        // waits for the acknowledgements at its next load wait; here three
        // of four waves issue no global store in a round.  Lane l: channel
        // l % 4 of the round, harmonics l / 4 + 16 j; lanes < 16 also the
        // round's channel scalars (zero for a zapped channel)
        if (wave == r % kX2W) {
            const int c = lane0 % kX2W, n0 = cbase + r * kX2W;
            const int nc = n0 + c;
            if (nc < cend) {
                const bool ok = !mask || mask[nc];
                const double2 *b = lds + c * kX2SL;
                const double ie2 = ok ? reinterpret_cast<const double *>(b + kX2IE)[0] : 0.0;
                for (int k = lane0 / kX2W; k < kw; k += 64 / kX2W)
                    Xs[(int64_t)k * a.nchan + nc] = ok ? cscale(b[x2slot(k)], ie2) : cmk(0.0, 0.0);
            }
            if (lane0 < 4 * kX2W) {
                const int cc = lane0 >> 2, comp = lane0 & 3, ncc = n0 + cc;
                if (ncc < cend) {
                    const bool okc = !mask || mask[ncc];
                    const double v = reinterpret_cast<const double *>(lds + cc * kX2SL + kX2IE + 1)[comp];
                    a.chan[((int64_t)s * a.nchan + ncc) * 4 + comp] = okc ? v : 0.0;
                }
            }
        }
        if (false)
#endif
        // write-out: thread t -> channel c = t % 4 of the round, harmonics
        // k = t / 4 + 64 j
        {
            const int c = threadIdx.x % kX2W, n0 = cbase + r * kX2W;
            const int nc = n0 + c;
            if (nc < cend) {
                const bool ok = !mask || mask[nc];
                const double2 *b = lds + c * kX2SL;
                const double ie2 = ok ? reinterpret_cast<const double *>(b + kX2IE)[0] : 0.0;
                for (int k = threadIdx.x / kX2W; k < kw; k += 64) {
#if PPF_X2_DIAG & 1
                    if (ie2 == 12345.0)            // (timing-only build: no X stores)
#endif
                    {
#if PPF_X2_NT & 2
                    const double2 v = ok ? cscale(b[x2slot(k)], ie2) : cmk(0.0, 0.0);
                    __builtin_nontemporal_store(vd2{v.x, v.y}, reinterpret_cast<vd2 *>(Xs + (int64_t)k * a.nchan + nc));
#else
                    Xs[(int64_t)k * a.nchan + nc] = ok ? cscale(b[x2slot(k)], ie2) : cmk(0.0, 0.0);
#endif
                    }
                }
            }
        }
        if (GS && gon) {
            // the round's rows' guess terms, in wave order
            for (int t = threadIdx.x; t < NL; t += 64 * kX2W) {
                if (t == 0) continue;
                double2 acc = gacc[t];
#pragma unroll
                for (int w2 = 0; w2 < kX2W; ++w2)
                    if (usable(cbase + r * kX2W + w2)) acc = cadd(acc, lds[w2 * kX2SL + x2slot(N - t)]);
                gacc[t] = acc;
            }
        }
        __syncthreads();
        XP(6);
    }
    {
        const int lane = lane0;
        (void)lane;
        XP_DONE();
    }
    if constexpr (GS) {
        if (gon) {
            double2 *gp = a.gpart + ((int64_t)s * a.nblk + cb) * NL;
            // (the staged guess terms are doubled: exact factor 1/2)
            for (int t = threadIdx.x; t < NL; t += 64 * kX2W) gp[t] = cscale(gacc[t], 0.5);
            const double gwl = mlane ? a.guess_weights[(int64_t)s * a.nchan + cbase + lane0] : 0.0;
            const double wsum = wave_sum(gwl), cnt = wave_sum(mlane ? 1.0 : 0.0);
            if (lane0 == 0) reinterpret_cast<double *>(buf)[0] = g_w2e2;
            __syncthreads();
            if (threadIdx.x == 0) {
                double acc = 0.0;
                for (int w2 = 0; w2 < kX2W; ++w2) acc += reinterpret_cast<const double *>(lds + w2 * kX2SL)[0];
                double *o = a.gw + ((int64_t)s * a.nblk + cb) * 3;
                o[0] = wsum;
                o[1] = cnt;
                o[2] = acc;
            }
        }
    }
}

// ===========================================================================
// k_xspec_wm: the spectrum pass for nbin / 2 not a power of two (1000, 1022,
// 1536, 2000 bins ...), N <= 1024 (round 5).  k_xspec_any gave
// each row to a 256-thread workgroup (a barrier per FFT stage and per
// block sum; 2 points per thread at 1000 bins) and wrote X one channel per
// lane, every harmonic.  Here, as k_xspec_w: a 4-wave workgroup takes a
// block of channels of one sub-int, a round of 4 rows, one row per wave:
// the row's mixed-radix Stockham stages run in the wave's own LDS buffer
// (wave-level ordering only, no workgroup barrier inside a row), the real
// post-pass forms the noise / Sd sums and X = D conj(M) in place, and after
// one barrier the workgroup writes the round's X harmonic-major, below each
// 64-channel group's cutoff (k_model_cut), as k_pass / k_moments read it.
// Same arithmetic as k_xspec_any (lds_fft_mixed's stages, rfft_bin).
// ===========================================================================
constexpr int kWmW = 4;              // waves per workgroup
constexpr int kWmMaxN = 1024;        // largest N (complex points) per wave

// j mod L for j < 8192 with a float reciprocal (L is wave-uniform; an
// integer division by a runtime divisor is a ~40-instruction sequence)
__device__ __forceinline__ int mod_small(int j, int L, float invL) {
    const int q = (int)((float)j * invL);
    int k = j - q * L;
    k += k < 0 ? L : 0;
    k -= k >= L ? L : 0;
    return k;
}

// one mixed-radix Stockham stage of radix R (span L) over N points, by one
// wave: all of a lane's reads before its writes (a wave's LDS operations
// are processed in order, so no lane's write overtakes another's read);
// stage twiddles from the workgroup's LDS copy of T
template <int R, int NMAX>
__device__ __forceinline__ void wmr_stage(double2 *buf, int N, int L, const double2 *tw, int lane) {
    constexpr int QM = (NMAX / R + 63) / 64;
    const int nb = N / R, ts = N / (R * L);
    const float invL = 1.0f / (float)L;
    double2 x[QM][R];
#pragma unroll
    for (int q = 0; q < QM; ++q) {
        const int j = lane + 64 * q;
        if (j < nb) {
            const int k = mod_small(j, L, invL);
#pragma unroll
            for (int r = 0; r < R; ++r) x[q][r] = buf[j + r * nb];
#pragma unroll
            for (int r = 1; r < R; ++r) x[q][r] = cmul(x[q][r], tw[r * k * ts]);
            dft_small<R>(x[q], false);
        }
    }
    wfft::wave_sync();
#pragma unroll
    for (int q = 0; q < QM; ++q) {
        const int j = lane + 64 * q;
        if (j < nb) {
            const int k = mod_small(j, L, invL);
            const int o = (j - k) * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) buf[o + r * L] = x[q][r];
        }
    }
    wfft::wave_sync();
}

// radix 7 and the prime factors above it: the generic-radix stage (one
// output per lane per pass, R LDS loads and products each; no butterfly
// arrays, so no spill at the four-wave budget).  Inline: a call from this
// kernel (out-of-line stages, round 5) faulted on the device.
template <int NMAX>
__device__ __forceinline__ void wmr_stage_g(double2 *buf, int N, int L, int R, const double2 *tw, int lane) {
    double2 y[NMAX / 64];
    gr_stage_read4<NMAX / 64>(buf, N, L, R, tw, false, lane, 64, y);
    wfft::wave_sync();
    gr_stage_write<NMAX / 64>(buf, N, lane, 64, y);
    wfft::wave_sync();
}

// NMAX: the largest N of the instantiation (512: <= 128 VGPRs, four waves
// per SIMD; 1024: two), which sizes every stage's register footprint (a
// lane holds all of its butterflies between the stage's reads and writes)
// (the LDS of a workgroup -- four row buffers and the twiddles -- admits
// three of them per CU at NMAX 512 and two at 1024, so the register budget
// is three / two waves per SIMD)
#ifndef PPF_WM_PRE
#define PPF_WM_PRE 1
#endif
// ODD: odd nbin (<= 1023), the row as NF = nbin complex points with zero
// imaginary parts (rfft_len), X_k = Z_k for k <= nbin / 2: no pair post-pass.
template <int DT, int NMAX, bool ODD>
__global__ __launch_bounds__(64 * kWmW) __attribute__((amdgpu_waves_per_eu(NMAX <= 512 ? 3 : 2)))
void k_xspec_wm(XspecArgs a) {
    const int N = a.nbin >> 1, NH = N + 1;
    const int NF = ODD ? a.nbin : N;           // complex points per row
    // even: [0, N] Z then X, [N + 1] 1/errs_FT^2; odd: Z in [0, NF), X in
    // [0, N] and 1/errs_FT^2 in [N + 1] after the post-pass (N + 1 < NF)
    const int SL = ODD ? NF : N + 2, IE = N + 1;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *buf = lds + wave * SL;
    double2 *twl = lds + kWmW * SL;            // T[0, NF): the stage twiddles
    int s, cb;
    block_map(a.xcd_swizzle, a.nblk, s, cb, a.nsub);
    if (a.needx && !a.needx[s]) return;
    for (int i = threadIdx.x; i < NF; i += 64 * kWmW) twl[i] = a.T[i];
    __syncthreads();
    const int cbase = cb * a.cb, cend = min(a.nchan, cbase + a.cb);
    const int nround = (a.cb + kWmW - 1) / kWmW;
    const int mi = a.model_index ? a.model_index[s] : 0;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double sqrtN = sqrt((double)a.nbin / 2.0);
    double2 *Xs = a.X + (int64_t)(a.xslot ? a.xslot[s] : s) * NH * a.nchan;
    int kw = NH;
    if (a.KC) {
        const int nn = (cbase & ~63) + lane;
        kw = (int)wave_max(nn < a.nchan ? (double)a.KC[(int64_t)mi * a.nchan + nn] : 1.0);
    }
    const int mlane = (cbase + lane < cend && (!mask || mask[cbase + lane])) ? 1 : 0;
    auto usable = [&](int n) {
        return n < cend && __builtin_amdgcn_readlane(mlane, n - cbase) != 0;
    };
    const int nl = cbase + lane;
    const double ch_mpow = nl < cend ? a.Mpow[(int64_t)mi * a.nchan + nl] : 0.0;
    const double ch_err = (a.errs && nl < cend) ? a.errs[(int64_t)s * a.nchan + nl] : 0.0;
    const bool two0 = !ODD && (__builtin_ctz((unsigned)N) & 1) != 0;
#if PPF_WM_PRE
    // the wave's next row in registers while this one is transformed
    // (unconditional loads of a valid row: the prefetch stays in VGPRs)
    using ET = typename std::conditional<DT == 0, float, double>::type;
    using LT = typename std::conditional<ODD, ET, typename std::conditional<DT == 0, float2, double2>::type>::type;
    constexpr int PJ = NMAX / 64;
    LT pre[PJ];
    auto fetch = [&](int m) {
        const LT *src = reinterpret_cast<const LT *>(a.data) + ((int64_t)s * a.nchan + m) * (int64_t)NF;
#pragma unroll
        for (int i = 0; i < PJ; ++i) {
            const int t = lane + 64 * i;
            pre[i] = ld_stream(src + (t < NF ? t : NF - 1));
        }
    };
    fetch(min(cbase + wave, cend - 1));
#endif
    for (int r = 0, n = cbase + wave; r < nround; ++r, n += kWmW) {
        const bool live = usable(n);
        if (n < cend && !live && lane < 4) a.chan[((int64_t)s * a.nchan + n) * 4 + lane] = 0.0;
#if PPF_WM_PRE
        if (live) {
#pragma unroll
            for (int i = 0; i < PJ; ++i) {
                const int t = lane + 64 * i;
                if constexpr (ODD) {
                    if (t < NF) buf[t] = cmk((double)pre[i], 0.0);
                } else {
                    if (t < N) buf[t] = cmk((double)pre[i].x, (double)pre[i].y);
                }
            }
        }
        fetch(min(n + kWmW, cend - 1));
#endif
        if (live) {
            const int64_t crow = (int64_t)s * a.nchan + n;
#if !PPF_WM_PRE
            static_assert(!ODD, "odd nbin needs PPF_WM_PRE");
            if (DT == 0) {
                const float2 *src = reinterpret_cast<const float2 *>(a.data) + crow * (int64_t)N;
                for (int j = lane; j < N; j += 64) {
                    const float2 v = src[j];
                    buf[j] = cmk((double)v.x, (double)v.y);
                }
            } else {
                const double2 *src = reinterpret_cast<const double2 *>(a.data) + crow * (int64_t)N;
                for (int j = lane; j < N; j += 64) buf[j] = src[j];
            }
#endif
            wfft::wave_sync();
            // the stages in fft_radices' order (one 2 when the power of two
            // is odd, 4s, then the odd primes ascending), wave-uniform
            int L = 1, rem = NF;
            bool two = two0;
            while (rem > 1) {
                int R;
                if (two) { R = 2; two = false; }
                else if ((rem & 3) == 0) R = 4;
                else { R = 3; while (rem % R) R += 2; }
                switch (R) {
                    case 2: wmr_stage<2, NMAX>(buf, NF, L, twl, lane); break;
                    case 3: wmr_stage<3, NMAX>(buf, NF, L, twl, lane); break;
                    case 4: wmr_stage<4, NMAX>(buf, NF, L, twl, lane); break;
                    case 5: wmr_stage<5, NMAX>(buf, NF, L, twl, lane); break;
                    default: wmr_stage_g<NMAX>(buf, NF, L, R, twl, lane); break;
                }
                L *= R;
                rem /= R;
            }
            // real post-pass on the pairs (k, N - k), k <= N/2, in place:
            // X_k into slot k, X_{N-k} into slot N - k (k = 0: X_N into
            // slot N); unscaled, the write-out applies 1/errs_FT^2
            const double2 *Mrow = a.Mft + ((int64_t)mi * a.nchan + n) * NH;
            double pn = 0.0, pd = 0.0;
            // odd nbin: X_k = Z_k (k <= N), each lane its own slots
            for (int k = lane; ODD && k <= N; k += 64) {
                const double2 dk = buf[k];
                const double p0 = cabs2(dk);
                if (k >= a.kc) pn += p0;
                if (k >= 1) pd += p0;
                if (k < kw) buf[k] = k == 0 ? cmk(0.0, 0.0) : cmulc(dk, Mrow[k]);
            }
            for (int k = lane; !ODD && k <= N / 2; k += 64) {
                const int kn = N - k;
                const double2 dk = rfft_bin(buf, N, a.T2, k);
                const double2 dn = rfft_bin(buf, N, a.T2, kn);
                const double p0 = cabs2(dk), p1 = cabs2(dn);
                if (k >= a.kc) pn += p0;
                if (k >= 1) pd += p0;
                if (kn != k) {
                    if (kn >= a.kc) pn += p1;
                    pd += p1;
                }
                // (every read of this pair is done: rfft_bin read slots k
                // and N - k only, and no other lane touches them)
                if (k < kw) buf[k] = k == 0 ? cmk(0.0, 0.0) : cmulc(dk, Mrow[k]);
                if (kn < kw) buf[kn] = cmulc(dn, Mrow[kn]);
            }
            pn = wave_sum(pn);
            pd = wave_sum(pd);
            const int rr = n - cbase;
            double errs_FT;
            if (a.errs) errs_FT = readlane_d(ch_err, rr) * sqrtN;
            else errs_FT = sqrt(pn / (double)(NH - a.kc) / (double)a.nbin) * sqrtN;
            const double inv_e2 = 1.0 / (errs_FT * errs_FT);
            const double mpow = readlane_d(ch_mpow, rr);
            if (lane == 0) {
                reinterpret_cast<double *>(buf + IE)[0] = inv_e2;
                double *chan = a.chan + crow * 4;
                chan[0] = errs_FT;
                chan[1] = inv_e2;
                chan[2] = pd * inv_e2;          // Sd_n
                chan[3] = mpow * inv_e2;        // S_n at tau = 0
            }
        }
        __syncthreads();
        // write-out: thread t -> channel c = t % 4 of the round, harmonics
        // k = t / 4 + 64 j
        {
            const int c = threadIdx.x % kWmW, nc = cbase + r * kWmW + c;
            if (nc < cend) {
                const bool ok = !mask || mask[nc];
                const double2 *b = lds + c * SL;
                const double ie2 = ok ? reinterpret_cast<const double *>(b + IE)[0] : 0.0;
                for (int k = threadIdx.x / kWmW; k < kw; k += 64)
                    st_stream(Xs + (int64_t)k * a.nchan + nc, ok ? cscale(b[k], ie2) : cmk(0.0, 0.0));
            }
        }
        __syncthreads();
    }
}

// ===========================================================================
// k_xspec_wo: the spectrum pass for odd nbin < 1024 with TWO real rows per
// complex transform: row A as the real part, row B as the imaginary part,
// Z = FFT_NF(a + i b) (NF = nbin points, the stages of k_xspec_wm), then
// X_A(k) = (Z_k + conj Z_{NF-k}) / 2 and X_B(k) = (Z_k - conj Z_{NF-k}) / 2i
// for k <= N = nbin / 2: half the transform work per row of the one-row
// path (k_xspec_wm<ODD>, PPF_XSPEC_WO=0).  A round is 8 rows, two per wave
// (rows w and w + 4 of the round).  Each pair (k, NF - k) is read and
// written back by one lane in its own two slots: the unscaled X of row A at
// slot k, of row B at slot NF - k (k = 1 .. N); the k = 0 positions (X_0 = 0:
// F0_fact), slot 0 and slot NF, carry the rows' 1/errs_FT^2 for the
// write-out, which stores 8 channels (128 B) per harmonic.
// ===========================================================================
template <int DT, int NMAX>
__global__ __launch_bounds__(64 * kWmW) __attribute__((amdgpu_waves_per_eu(NMAX <= 512 ? 3 : 2)))
void k_xspec_wo(XspecArgs a) {
    const int N = a.nbin >> 1, NH = N + 1, NF = a.nbin;
    const int SL = NF + 1;                     // = 2 NH
    constexpr int RW = 2 * kWmW;               // rows per round
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *buf = lds + wave * SL;
    double2 *twl = lds + kWmW * SL;            // T[0, NF): the stage twiddles
    int s, cb;
    block_map(a.xcd_swizzle, a.nblk, s, cb, a.nsub);
    if (a.needx && !a.needx[s]) return;
    for (int i = threadIdx.x; i < NF; i += 64 * kWmW) twl[i] = a.T[i];
    __syncthreads();
    const int cbase = cb * a.cb, cend = min(a.nchan, cbase + a.cb);
    const int nround = (a.cb + RW - 1) / RW;
    const int mi = a.model_index ? a.model_index[s] : 0;
    const uint8_t *mask = a.mask ? a.mask + (int64_t)s * a.nchan : nullptr;
    const double sqrtN = sqrt((double)a.nbin / 2.0);
    double2 *Xs = a.X + (int64_t)(a.xslot ? a.xslot[s] : s) * NH * a.nchan;
    int kw = NH;
    if (a.KC) {
        const int nn = (cbase & ~63) + lane;
        kw = (int)wave_max(nn < a.nchan ? (double)a.KC[(int64_t)mi * a.nchan + nn] : 1.0);
    }
    const int mlane = (cbase + lane < cend && (!mask || mask[cbase + lane])) ? 1 : 0;
    auto usable = [&](int n) {
        return n < cend && __builtin_amdgcn_readlane(mlane, n - cbase) != 0;
    };
    const int nl = cbase + lane;
    const double ch_mpow = nl < cend ? a.Mpow[(int64_t)mi * a.nchan + nl] : 0.0;
    const double ch_err = (a.errs && nl < cend) ? a.errs[(int64_t)s * a.nchan + nl] : 0.0;
    // the wave's next two rows in registers while these are transformed
    using ET = typename std::conditional<DT == 0, float, double>::type;
    constexpr int PJ = NMAX / 64;
    ET pa[PJ], pb[PJ];
    auto fetch = [&](ET (&p)[PJ], int m) {
        const ET *src = reinterpret_cast<const ET *>(a.data) + ((int64_t)s * a.nchan + m) * (int64_t)NF;
#pragma unroll
        for (int i = 0; i < PJ; ++i) {
            const int t = lane + 64 * i;
            p[i] = ld_stream(src + (t < NF ? t : NF - 1));
        }
    };
    fetch(pa, min(cbase + wave, cend - 1));
    fetch(pb, min(cbase + wave + kWmW, cend - 1));
    for (int r = 0, nA = cbase + wave; r < nround; ++r, nA += RW) {
        const int nB = nA + kWmW;
        const bool liveA = usable(nA), liveB = usable(nB), live = liveA || liveB;
        if (nA < cend && !liveA && lane < 4) a.chan[((int64_t)s * a.nchan + nA) * 4 + lane] = 0.0;
        if (nB < cend && !liveB && lane < 4) a.chan[((int64_t)s * a.nchan + nB) * 4 + lane] = 0.0;
        if (live) {
#pragma unroll
            for (int i = 0; i < PJ; ++i) {
                const int t = lane + 64 * i;
                if (t < NF) buf[t] = cmk(liveA ? (double)pa[i] : 0.0, liveB ? (double)pb[i] : 0.0);
            }
        }
        fetch(pa, min(nA + RW, cend - 1));
        fetch(pb, min(nB + RW, cend - 1));
        if (live) {
            wfft::wave_sync();
            int L = 1, rem = NF;
            while (rem > 1) {
                int R = 3;
                while (rem % R) R += 2;
                switch (R) {
                    case 3: wmr_stage<3, NMAX>(buf, NF, L, twl, lane); break;
                    case 5: wmr_stage<5, NMAX>(buf, NF, L, twl, lane); break;
                    default: wmr_stage_g<NMAX>(buf, NF, L, R, twl, lane); break;
                }
                L *= R;
                rem /= R;
            }
            // the pairs (Z_k, Z_{NF-k}), k <= N: each lane reads and
            // rewrites only its own pairs' two slots
            const double2 *MA = a.Mft + ((int64_t)mi * a.nchan + min(nA, cend - 1)) * NH;
            const double2 *MB = a.Mft + ((int64_t)mi * a.nchan + min(nB, cend - 1)) * NH;
            double pnA = 0.0, pdA = 0.0, pnB = 0.0, pdB = 0.0;
            for (int k = lane; k <= N; k += 64) {
                const int kn = k == 0 ? 0 : NF - k;
                const double2 zk = buf[k], c = cconj(buf[kn]);
                const double2 xa = cscale(cadd(zk, c), 0.5);
                const double2 d = csub(zk, c);
                const double2 xb = cmk(0.5 * d.y, -0.5 * d.x);       // d / 2i
                const double qa = cabs2(xa), qb = cabs2(xb);
                if (k >= a.kc) { pnA += qa; pnB += qb; }
                if (k >= 1) { pdA += qa; pdB += qb; }
                if (k >= 1 && k < kw) {
                    buf[k] = cmulc(xa, MA[k]);
                    buf[kn] = cmulc(xb, MB[k]);
                }
            }
            pnA = wave_sum(pnA);
            pdA = wave_sum(pdA);
            pnB = wave_sum(pnB);
            pdB = wave_sum(pdB);
            const int rA = nA - cbase, rB = min(nB - cbase, 63);
            double eA, eB;
            if (a.errs) {
                eA = readlane_d(ch_err, rA) * sqrtN;
                eB = readlane_d(ch_err, rB) * sqrtN;
            } else {
                eA = sqrt(pnA / (double)(NH - a.kc) / (double)a.nbin) * sqrtN;
                eB = sqrt(pnB / (double)(NH - a.kc) / (double)a.nbin) * sqrtN;
            }
            const double ieA = 1.0 / (eA * eA), ieB = 1.0 / (eB * eB);
            const double mpA = readlane_d(ch_mpow, rA), mpB = readlane_d(ch_mpow, rB);
            if (lane == 0) {
                buf[0] = cmk(ieA, 0.0);
                buf[NF] = cmk(ieB, 0.0);
                if (liveA) {
                    double *chan = a.chan + ((int64_t)s * a.nchan + nA) * 4;
                    chan[0] = eA;
                    chan[1] = ieA;
                    chan[2] = pdA * ieA;          // Sd_n
                    chan[3] = mpA * ieA;          // S_n at tau = 0
                }
                if (liveB) {
                    double *chan = a.chan + ((int64_t)s * a.nchan + nB) * 4;
                    chan[0] = eB;
                    chan[1] = ieB;
                    chan[2] = pdB * ieB;
                    chan[3] = mpB * ieB;
                }
            }
        }
        __syncthreads();
        // write-out: thread t -> channel c = t % 8 of the round, harmonics
        // k = t / 8 + 32 j (X_0 = 0; slot 0 holds the row's 1/errs_FT^2)
        {
            const int c = threadIdx.x % RW, nc = cbase + r * RW + c;
            if (nc < cend) {
                const bool ok = !mask || mask[nc];
                // row A: X_k at slot k; row B: at slot NF - k (k = 0: 1/errs_FT^2)
                const double2 *b = lds + (c % kWmW) * SL;
                const int o0 = c < kWmW ? 0 : NF, st = c < kWmW ? 1 : -1;
                const double ie2 = ok ? b[o0].x : 0.0;
                for (int k = threadIdx.x / RW; k < kw; k += 64 * kWmW / RW)
                    st_stream(Xs + (int64_t)k * a.nchan + nc, (ok && k) ? cscale(b[o0 + st * k], ie2) : cmk(0.0, 0.0));
            }
        }
        __syncthreads();
    }
}

// nbin / 2 <= 1024 not a power of two; odd nbin < 1024 (NF = nbin points)
bool xspec_wm_supported(int nbin) {
    if (nbin & 1) return nbin >= 33 && nbin < kWmMaxN;
    const int N = nbin / 2;
    return !is_pow2(N) && N <= kWmMaxN && fft_len_supported(N);
}

#define PPF_WM_LAUNCH(NM, ODD)                                                           \
    do {                                                                                 \
        if (a.dtype == 0) hipLaunchKernelGGL((k_xspec_wm<0, NM, ODD>), g, b, lds, st, a); \
        else hipLaunchKernelGGL((k_xspec_wm<1, NM, ODD>), g, b, lds, st, a);              \
    } while (0)

// odd nbin: two rows per transform (k_xspec_wo) unless PPF_XSPEC_WO=0
// (environment, read once: the one-row k_xspec_wm<ODD>)
static bool use_xspec_wo() {
    static const bool on = [] {
        const char *e = getenv("PPF_XSPEC_WO");
        return e ? atoi(e) != 0 : true;
    }();
    return on;
}

hipError_t launch_xspec_wm(const XspecArgs &a, hipStream_t st) {
    const bool odd = a.nbin & 1;
    const int NF = rfft_len(a.nbin);
    if (odd && use_xspec_wo()) {
        const size_t lds = ((size_t)kWmW * (NF + 1) + NF) * sizeof(double2);
        dim3 g((unsigned)((int64_t)a.nsub * a.nblk)), b(64 * kWmW);
        if (NF <= 512) {
            if (a.dtype == 0) hipLaunchKernelGGL((k_xspec_wo<0, 512>), g, b, lds, st, a);
            else hipLaunchKernelGGL((k_xspec_wo<1, 512>), g, b, lds, st, a);
        } else {
            if (a.dtype == 0) hipLaunchKernelGGL((k_xspec_wo<0, 1024>), g, b, lds, st, a);
            else hipLaunchKernelGGL((k_xspec_wo<1, 1024>), g, b, lds, st, a);
        }
        return hipGetLastError();
    }
    const size_t lds = ((size_t)kWmW * (odd ? NF : NF + 2) + NF) * sizeof(double2);
    dim3 g((unsigned)((int64_t)a.nsub * a.nblk)), b(64 * kWmW);
    if (NF <= 512) {
        if (odd) PPF_WM_LAUNCH(512, true);
        else PPF_WM_LAUNCH(512, false);
    } else {
        if (odd) PPF_WM_LAUNCH(1024, true);
        else PPF_WM_LAUNCH(1024, false);
    }
    return hipGetLastError();
}

// k_xspec_w2 at 1024 points unless PPF_XSPEC2=0 (environment, read once)
static bool use_xspec2() {
    static const bool on = [] {
        const char *e = getenv("PPF_XSPEC2");
        return e ? atoi(e) != 0 : (PPF_XSPEC2 != 0);
    }();
    return on;
}

// ===========================================================================
// launchers
// ===========================================================================
template <int L2, int DT>
static void launch_w(const XspecArgs &a, hipStream_t st) {
    if constexpr (L2 == 10) {
        if (use_xspec2()) {
            const size_t lds = (size_t)kX2W * kX2SL * sizeof(double2);
            dim3 g((unsigned)((int64_t)a.nsub * a.nblk)), b(64 * kX2W);
            if (a.gflag)
                hipLaunchKernelGGL((k_xspec_w2<DT, true>), g, b, lds + (size_t)guess_slots(10) * sizeof(double2),
                                   st, a);
            else hipLaunchKernelGGL((k_xspec_w2<DT, false>), g, b, lds, st, a);
            return;
        }
    }
    const size_t lds = ((size_t)xsw<L2>() * xspec_slw<L2>() + (PPF_TW_LDS ? tw_slots<L2>() : 0)) *
                       sizeof(double2);
    dim3 g((unsigned)((int64_t)a.nsub * a.nblk)), b(64 * xsw<L2>());
    if (a.gflag && xspec_guess_fused(L2))
        hipLaunchKernelGGL((k_xspec_w<L2, DT, xspec_guess_fused(L2)>), g, b,
                           lds + (size_t)guess_slots(L2) * sizeof(double2), st, a);
    else hipLaunchKernelGGL((k_xspec_w<L2, DT, false>), g, b, lds, st, a);
}

bool xspec_wave_supported(int log2N, int cb) {
    return log2N >= 7 && log2N <= 10 && cb % xsw<7>() == 0 && cb % xsw<10>() == 0 && cb % kXW == 0;
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

// ===========================================================================
// k_noise_w: get_noise_PS per row (pplib.py:2312-2332) with one row per wave:
// the register radix FFT of k_xspec_w (next row in flight during the
// transform), the real post-pass, and the mean power of harmonics >= kc.
// Rows are dealt to the waves round-robin (4 waves per workgroup, as many
// workgroups as keep every CU's LDS busy); the block kernel k_noise (one
// 256-thread workgroup per row, a barrier per FFT stage) remains for the
// other lengths.
// ===========================================================================
constexpr int kNoiseW = 4;
template <int LOG2N, int DT>
__global__ __launch_bounds__(64 * kNoiseW) void k_noise_w(NoiseArgs a, int64_t nrows) {
    using P = wfft::Plan<LOG2N>;
    constexpr int N = P::N, R = P::R, NP = N / 128;
    constexpr int SL = wfft::buf_slots<LOG2N>();
    using RowT = typename std::conditional<DT == 0, vf2, vd2>::type;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *buf = lds + wave * SL;
    double2 *tw = lds + kNoiseW * SL;
    for (int i = threadIdx.x; i < tw_slots<LOG2N>(); i += 64 * kNoiseW) tw[i] = a.T[i];
    __syncthreads();
    const double2 w_seed = a.T2[lane], w_step = a.T2[64];
    const RowT *rows = reinterpret_cast<const RowT *>(a.in);
    const int64_t nw = (int64_t)gridDim.x * kNoiseW;
    int64_t row = (int64_t)blockIdx.x * kNoiseW + wave;
    RowT zr[R];
    auto fetch = [&](int64_t rr) {
        const RowT *src = rows + rr * N;
#pragma unroll
        for (int q = 0; q < R; ++q) zr[q] = src[lane + 64 * q];
    };
    if (row < nrows) fetch(row);
    for (; row < nrows; row += nw) {
        double2 x[R];
#pragma unroll
        for (int q = 0; q < R; ++q) x[q] = cmk((double)zr[q].x, (double)zr[q].y);
        if (row + nw < nrows) fetch(row + nw);
        wfft::fft_row<LOG2N>(x, buf, tw, lane);
        double pn = 0.0;
        double2 w = w_seed;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int klo = lane + 64 * i, khi = N - klo;
            double2 Dlo, Dhi;
            rfft_pair<LOG2N>(buf, klo, w, Dlo, Dhi);
            w = cmul(w, w_step);
            if (klo >= a.kc) pn += cabs2(Dlo);
            if (khi >= a.kc) pn += cabs2(Dhi);
        }
        if (lane == 0 && N / 2 >= a.kc) pn += cabs2(buf[wfft::pad<LOG2N>(N / 2)]);
        pn = wave_sum(pn);
        if (lane == 0) a.out[row] = sqrt(pn / (double)a.nbin / (double)(N + 1 - a.kc));
    }
}

// k_noise_h: k_noise_w on the half-buffer FFT (wfft::fft_row_h) without the
// next-row prefetch: 8.7 KB of LDS and fewer VGPRs per wave at 1024 points,
// so more waves per SIMD; bit-identical results (round-4 prototype of the
// wave-FFT restructure; PPF_NOISE_HALF=1 selects it).
#ifndef PPF_NOISE_HALF
#define PPF_NOISE_HALF 0
#endif
#ifndef PPF_NOISE_HALF_WPE
#define PPF_NOISE_HALF_WPE 3
#endif
template <int LOG2N, int DT>
__global__ __launch_bounds__(64 * kNoiseW) __attribute__((amdgpu_waves_per_eu(PPF_NOISE_HALF_WPE)))
void k_noise_h(NoiseArgs a, int64_t nrows) {
    using P = wfft::Plan<LOG2N>;
    constexpr int N = P::N, R = P::R, NP = N / 128;
    constexpr int SL = wfft::buf_slots<LOG2N>();
    using RowT = typename std::conditional<DT == 0, vf2, vd2>::type;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *tw = lds;
    double *hb = reinterpret_cast<double *>(lds + tw_slots<LOG2N>()) + wave * SL;
    for (int i = threadIdx.x; i < tw_slots<LOG2N>(); i += 64 * kNoiseW) tw[i] = a.T[i];
    __syncthreads();
    const double2 w_seed = a.T2[lane], w_step = a.T2[64];
    const RowT *rows = reinterpret_cast<const RowT *>(a.in);
    const int64_t nw = (int64_t)gridDim.x * kNoiseW;
    // the first PF of the next row's R loads per lane are in flight during
    // this row's transform (PPF_NOISE_HALF_PF; 0: none)
#ifndef PPF_NOISE_HALF_PF
#define PPF_NOISE_HALF_PF 0
#endif
    constexpr int PF = PPF_NOISE_HALF_PF < R ? PPF_NOISE_HALF_PF : R;
    RowT zp[PF > 0 ? PF : 1];
    int64_t row = (int64_t)blockIdx.x * kNoiseW + wave;
    if (PF > 0 && row < nrows) {
#pragma unroll
        for (int q = 0; q < PF; ++q) zp[q] = rows[row * N + lane + 64 * q];
    }
    for (; row < nrows; row += nw) {
        double2 x[R];
        const RowT *src = rows + row * N;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const RowT z = q < PF ? zp[q % (PF > 0 ? PF : 1)] : src[lane + 64 * q];
            x[q] = cmk((double)z.x, (double)z.y);
        }
        if (PF > 0 && row + nw < nrows) {
#pragma unroll
            for (int q = 0; q < PF; ++q) zp[q] = rows[(row + nw) * N + lane + 64 * q];
        }
        typename wfft::HBlk<LOG2N, P::NST - 1>::T vl;
        wfft::fft_row_h<LOG2N>(x, hb, tw, lane, vl);
        // the (k, N - k) pairs: real parts, then imaginary parts
        double zr[2 * NP + 1], zi[2 * NP + 1];
        wfft::hwrite_last<LOG2N, 0>(hb, lane, vl);
        wfft::wave_sync();
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int k = lane + 64 * i;
            zr[2 * i] = hb[wfft::pad<LOG2N>(k)];
            zr[2 * i + 1] = hb[k == 0 ? 0 : wfft::pad<LOG2N>(N - k)];
        }
        zr[2 * NP] = hb[wfft::pad<LOG2N>(N / 2)];
        wfft::wave_sync();
        wfft::hwrite_last<LOG2N, 1>(hb, lane, vl);
        wfft::wave_sync();
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int k = lane + 64 * i;
            zi[2 * i] = hb[wfft::pad<LOG2N>(k)];
            zi[2 * i + 1] = hb[k == 0 ? 0 : wfft::pad<LOG2N>(N - k)];
        }
        zi[2 * NP] = hb[wfft::pad<LOG2N>(N / 2)];
        wfft::wave_sync();
        double pn = 0.0;
        double2 w = w_seed;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int klo = lane + 64 * i, khi = N - klo;
            // rfft_pair on register copies of the two bins
            const double2 zk = cmk(zr[2 * i], zi[2 * i]), zn = cmk(zr[2 * i + 1], zi[2 * i + 1]);
            const double2 e = cmk(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y));
            const double2 o = cmk(0.5 * (zk.x - zn.x), 0.5 * (zk.y + zn.y));
            const double2 wo = cmul(w, o);
            const double2 Dlo = cmk(e.x + wo.y, e.y - wo.x);
            const double2 Dhi = cmk(e.x - wo.y, -(e.y + wo.x));
            w = cmul(w, w_step);
            if (klo >= a.kc) pn += cabs2(Dlo);
            if (khi >= a.kc) pn += cabs2(Dhi);
        }
        if (lane == 0 && N / 2 >= a.kc) pn += cabs2(cmk(zr[2 * NP], zi[2 * NP]));
        pn = wave_sum(pn);
        if (lane == 0) a.out[row] = sqrt(pn / (double)a.nbin / (double)(N + 1 - a.kc));
    }
}

template <int LOG2N, int DT>
static void launch_nh(const NoiseArgs &a, int64_t nrows, hipStream_t st) {
    const size_t lds = (size_t)tw_slots<LOG2N>() * sizeof(double2) +
                       (size_t)kNoiseW * wfft::buf_slots<LOG2N>() * sizeof(double);
    const int64_t want = (nrows + kNoiseW - 1) / kNoiseW;
    const unsigned grid = (unsigned)std::min<int64_t>(want, 256 * 24);
    hipLaunchKernelGGL((k_noise_h<LOG2N, DT>), dim3(grid), dim3(64 * kNoiseW), lds, st, a, nrows);
}

template <int LOG2N, int DT>
static void launch_nw(const NoiseArgs &a, int64_t nrows, hipStream_t st) {
    if (PPF_NOISE_HALF && LOG2N == 10) {
        launch_nh<LOG2N, DT>(a, nrows, st);
        return;
    }
    const size_t lds = ((size_t)kNoiseW * wfft::buf_slots<LOG2N>() + tw_slots<LOG2N>()) * sizeof(double2);
    // two to four workgroups per CU by LDS; a few rows per wave
    const int64_t want = (nrows + kNoiseW - 1) / kNoiseW;
    const unsigned grid = (unsigned)std::min<int64_t>(want, 256 * 16);
    hipLaunchKernelGGL((k_noise_w<LOG2N, DT>), dim3(grid), dim3(64 * kNoiseW), lds, st, a, nrows);
}

bool noise_wave_supported(int log2N) { return log2N >= 7 && log2N <= 10; }

hipError_t launch_noise_wave(const NoiseArgs &a, int64_t nrows, hipStream_t st) {
    switch (a.log2N * 2 + a.dtype) {
        case 14: launch_nw<7, 0>(a, nrows, st); break;
        case 15: launch_nw<7, 1>(a, nrows, st); break;
        case 16: launch_nw<8, 0>(a, nrows, st); break;
        case 17: launch_nw<8, 1>(a, nrows, st); break;
        case 18: launch_nw<9, 0>(a, nrows, st); break;
        case 19: launch_nw<9, 1>(a, nrows, st); break;
        case 20: launch_nw<10, 0>(a, nrows, st); break;
        case 21: launch_nw<10, 1>(a, nrows, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ===========================================================================
// k_align_part_w: ppalign accumulation (ppalign.py:236-247) with one row per
// wave.  Block = (channel n, group g of sub-ints) of kXW waves; wave w takes
// the group's sub-ints s0 + w, s0 + w + kXW, ... in order: register radix
// FFT of the row (next row in flight), real post-pass, times
// w exp(2 pi i k phase) (phasors by recurrence from exp(2 pi i lane phase),
// step exp(2 pi i 64 phase)), summed in registers.  The waves' sums are then
// added in wave order through LDS (fixed order: bitwise reproducible) and
// written as the group partial that k_align_fin reduces and inverts.
// ===========================================================================
template <int LOG2N, int DT>
__global__ __launch_bounds__(64 * kXW) void k_align_part_w(AlignArgs a) {
    using P = wfft::Plan<LOG2N>;
    constexpr int N = P::N, R = P::R, NP = N / 128;
    constexpr int SL = xspec_slw<LOG2N>();
    constexpr int SMID = SL - 2, SW = SL - 1;         // harmonic N/2, weight sum
    using RowT = typename std::conditional<DT == 0, vf2, vd2>::type;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *buf = lds + wave * SL;
    const int n = blockIdx.x % a.nchan, g = blockIdx.x / a.nchan;
    const int per = (a.nsub + a.ngroup - 1) / a.ngroup;
    const int s0 = g * per, s1 = min(a.nsub, s0 + per);
    const double2 w_seed = a.T2[lane], w_step = a.T2[64];
    const RowT *rows = reinterpret_cast<const RowT *>(a.in);
#if PPF_TW_LDS
    double2 *twl = lds + kXW * SL;
    for (int i = threadIdx.x; i < tw_slots<LOG2N>(); i += 64 * kXW) twl[i] = a.T[i];
    __syncthreads();
    const double2 *tw = twl;
#else
    const double2 *tw = a.T;
#endif
    double2 Alo[NP], Ahi[NP], Am = cmk(0.0, 0.0);
#pragma unroll
    for (int i = 0; i < NP; ++i) Alo[i] = Ahi[i] = cmk(0.0, 0.0);
    double wtot = 0.0;
    RowT zr[R];
    auto next_live = [&](int s) {      // rows with w == 0 are skipped (uniform per wave)
        while (s < s1 && a.weights[(int64_t)s * a.nchan + n] == 0.0) s += kXW;
        return s;
    };
    auto fetch = [&](int s) {
        const RowT *src = rows + ((int64_t)s * a.nchan + n) * N;
#pragma unroll
        for (int q = 0; q < R; ++q) zr[q] = ld_stream(src + lane + 64 * q);
    };
    int s = next_live(s0 + wave);
    if (s < s1) fetch(s);
    while (s < s1) {
        const int64_t row = (int64_t)s * a.nchan + n;
        const double w = a.weights[row], ph = a.phases[row];
        wtot += w;
        double2 x[R];
#pragma unroll
        for (int q = 0; q < R; ++q) x[q] = cmk((double)zr[q].x, (double)zr[q].y);
        const int sn = next_live(s + kXW);
        if (sn < s1) fetch(sn);                        // next row in flight during this FFT
        wfft::fft_row<LOG2N>(x, buf, tw, lane);
        const double2 Es = cexp2pi(64.0 * ph);
        double2 E = cexp2pi((double)lane * ph);                        // k = lane + 64 i
        double2 Eh = cmul(cexp2pi((double)N * ph), cconj(E));           // k = N - lane - 64 i
        double2 wt = w_seed;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int klo = lane + 64 * i;
            double2 Dlo, Dhi;
            rfft_pair<LOG2N>(buf, klo, wt, Dlo, Dhi);
            wt = cmul(wt, w_step);
            Alo[i] = cadd(Alo[i], cscale(cmul(Dlo, E), w));
            Ahi[i] = cadd(Ahi[i], cscale(cmul(Dhi, Eh), w));
            E = cmul(E, Es);
            Eh = cmul(Eh, cconj(Es));
        }
        if (lane == 0) {
            const double2 zm = buf[wfft::pad<LOG2N>(N / 2)];
            Am = cadd(Am, cscale(cmul(cmk(zm.x, -zm.y), cexp2pi((double)(N / 2) * ph)), w));
        }
        s = sn;
    }
    // this wave's sums into its buffer: k -> pad(k), N - k -> pad(N - k)
    // (k = 0: N -> pad(N / 2)), N / 2 -> SMID, weight sum -> SW
    wfft::wave_sync();
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int klo = lane + 64 * i;
        buf[wfft::pad<LOG2N>(klo)] = Alo[i];
        buf[klo == 0 ? wfft::pad<LOG2N>(N / 2) : wfft::pad<LOG2N>(N - klo)] = Ahi[i];
    }
    if (lane == 0) {
        buf[SMID] = Am;
        buf[SW] = cmk(wtot, 0.0);
    }
    __syncthreads();
    double2 *Pp = a.part + ((int64_t)g * a.nchan + n) * (N + 1);
    for (int k = threadIdx.x; k <= N; k += 64 * kXW) {
        const int slot = k == N ? wfft::pad<LOG2N>(N / 2) : (k == N / 2 ? SMID : wfft::pad<LOG2N>(k));
        double2 acc = lds[slot];
#pragma unroll
        for (int w2 = 1; w2 < kXW; ++w2) acc = cadd(acc, lds[w2 * SL + slot]);
        Pp[k] = acc;
    }
    if (threadIdx.x == 0) {
        double wsum = lds[SW].x;
        for (int w2 = 1; w2 < kXW; ++w2) wsum += lds[w2 * SL + SW].x;
        a.wpart[(int64_t)g * a.nchan + n] = wsum;
    }
}

template <int L2, int DT>
static void launch_align_w_t(const AlignArgs &a, hipStream_t st) {
    const size_t lds = ((size_t)kXW * xspec_slw<L2>() + (PPF_TW_LDS ? tw_slots<L2>() : 0)) * sizeof(double2);
    hipLaunchKernelGGL((k_align_part_w<L2, DT>), dim3((unsigned)((int64_t)a.ngroup * a.nchan)),
                       dim3(64 * kXW), lds, st, a);
}

bool align_wave_supported(int log2N) { return log2N >= 7 && log2N <= 10; }

hipError_t launch_align_part_w(const AlignArgs &a, hipStream_t st) {
    switch (a.log2N * 2 + a.dtype) {
        case 14: launch_align_w_t<7, 0>(a, st); break;
        case 15: launch_align_w_t<7, 1>(a, st); break;
        case 16: launch_align_w_t<8, 0>(a, st); break;
        case 17: launch_align_w_t<8, 1>(a, st); break;
        case 18: launch_align_w_t<9, 0>(a, st); break;
        case 19: launch_align_w_t<9, 1>(a, st); break;
        case 20: launch_align_w_t<10, 0>(a, st); break;
        case 21: launch_align_w_t<10, 1>(a, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_btab(int N, double *Bt, hipStream_t st) {
    hipLaunchKernelGGL(k_btab, dim3((unsigned)((N / 2 * 16 + 255) / 256)), dim3(256), 0, st, N, Bt);
    return hipGetLastError();
}

template <int L2, int DT>
static void launch_xg(const XmomArgs &a, bool full, hipStream_t st) {
    const size_t lds = xmom_g_lds<L2>();
    static_assert(xmom_g_lds<10>() <= 163840, "k_xmom_g LDS");
    dim3 g((unsigned)((int64_t)((a.nsub + 7) / 8) * a.nblk)), b(512);
    if (a.nmodel == 1) {
        if (full) hipLaunchKernelGGL((k_xmom_g<L2, DT, true, true>), g, b, lds, st, a);
        else hipLaunchKernelGGL((k_xmom_g<L2, DT, true, false>), g, b, lds, st, a);
    } else {
        if (full) hipLaunchKernelGGL((k_xmom_g<L2, DT, false, true>), g, b, lds, st, a);
        else hipLaunchKernelGGL((k_xmom_g<L2, DT, false, false>), g, b, lds, st, a);
    }
}

hipError_t launch_xmom(const XmomArgs &a, bool full, hipStream_t st) {
    switch (a.log2N * 2 + a.dtype) {
        case 14: launch_xg<7, 0>(a, full, st); break;
        case 15: launch_xg<7, 1>(a, full, st); break;
        case 16: launch_xg<8, 0>(a, full, st); break;
        case 17: launch_xg<8, 1>(a, full, st); break;
        case 18: launch_xg<9, 0>(a, full, st); break;
        case 19: launch_xg<9, 1>(a, full, st); break;
        case 20: launch_xg<10, 0>(a, full, st); break;
        case 21: launch_xg<10, 1>(a, full, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_model_pow(const double2 *Mft, int nchan, int nharm, int nmodel, double *out,
                            hipStream_t st) {
    const int nrows = nchan * nmodel;
    hipLaunchKernelGGL(k_model_pow, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, st, Mft, nrows,
                       nharm, out);
    return hipGetLastError();
}

// |M_nk|^2 in harmonic-major layout for the scattering pass: 64 x 4 tiles
// through LDS (reads along k, writes along n)
__global__ __launch_bounds__(256) void k_model_pow_t(const double2 *Mft, int nchan, int nharm,
                                                     double *MP) {
    __shared__ double t[64][65];
    const int m = blockIdx.z;
    const int k0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
    const double2 *M = Mft + (int64_t)m * nchan * nharm;
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int nl = i >> 6, kl = i & 63, n = n0 + nl, k = k0 + kl;
        t[nl][kl] = (n < nchan && k < nharm && k > 0) ? cabs2(M[(int64_t)n * nharm + k]) : 0.0;
    }
    __syncthreads();
    double *out = MP + (int64_t)m * nharm * nchan;
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int kl = i >> 6, nl = i & 63, n = n0 + nl, k = k0 + kl;
        if (n < nchan && k < nharm) out[(int64_t)k * nchan + n] = t[nl][kl];
    }
}

hipError_t launch_model_pow_t(const double2 *Mft, int nchan, int nharm, int nmodel, double *MP,
                              hipStream_t st) {
    dim3 g((unsigned)((nharm + 63) / 64), (unsigned)((nchan + 63) / 64), (unsigned)nmodel);
    hipLaunchKernelGGL(k_model_pow_t, g, dim3(256), 0, st, Mft, nchan, nharm, MP);
    return hipGetLastError();
}

// Harmonic cutoff per (model, channel): KC = 1 + the last k with
// |M_k|^2 > rel * max_k |M_k|^2 (>= 1).  Every term of the pass sums beyond
// it carries |M_k| < 1e-14 max |M| (rel = kCutRel = 1e-28) -- the level of
// a float64 template's own FFT rounding floor; summed over the dropped
// harmonics these terms change C, C', C'' and S by < 1e-12 relative -- so
// k_pass stops there (the example template at 512 x 2048: median 226 of
// 1025 harmonics; at 16384 x 1024 over 400-800 MHz the narrow component
// reaches Nyquist and nothing is cut).
// rel < 0 (ppf_fit_desc.options PPF_OPT_NO_HCUT): KC = nharm.
// workgroup = 64 channels (lanes) x 16 waves, each wave a 1/16 share of the
// harmonics (loads coalesced across the channels), reduced through LDS
constexpr int kCutWaves = 16;
__global__ __launch_bounds__(64 * kCutWaves) void k_model_cut(const double *MP, int nchan, int nharm,
                                                             int nmodel, double rel, int32_t *KC) {
    __shared__ double smx[kCutWaves][64];
    __shared__ int skc[kCutWaves][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int cblk = (nchan + 63) / 64;
    const int m = blockIdx.x / cblk, n = (blockIdx.x % cblk) * 64 + lane;
    const bool on = n < nchan;
    const double *p = MP + (int64_t)m * nharm * nchan + (on ? n : 0);
    double mx = 0.0;
    if (rel >= 0.0 && on)
        for (int k = w; k < nharm; k += kCutWaves) mx = fmax(mx, p[(int64_t)k * nchan]);
    smx[w][lane] = mx;
    __syncthreads();
    mx = 0.0;
    for (int q = 0; q < kCutWaves; ++q) mx = fmax(mx, smx[q][lane]);
    const double thr = rel * mx;
    // last harmonic k >= 1 above the threshold (KC = k + 1; 1 when none)
    int kc = 1;
    if (rel >= 0.0 && on)
        for (int k = w; k < nharm; k += kCutWaves)
            if (k >= 1 && p[(int64_t)k * nchan] > thr) kc = k + 1;
    skc[w][lane] = kc;
    __syncthreads();
    if (w == 0 && on) {
        for (int q = 1; q < kCutWaves; ++q) kc = max(kc, skc[q][lane]);
        KC[(int64_t)m * nchan + n] = rel >= 0.0 ? kc : nharm;
    }
}

hipError_t launch_model_cut(const double *MP, int nchan, int nharm, int nmodel, bool off,
                            int32_t *KC, hipStream_t st) {
    const int cblk = (nchan + 63) / 64;
    hipLaunchKernelGGL(k_model_cut, dim3((unsigned)(nmodel * cblk)), dim3(64 * kCutWaves), 0, st, MP,
                       nchan, nharm, nmodel, off ? -1.0 : kCutRel, KC);
    return hipGetLastError();
}

hipError_t launch_model_sum(const double2 *Mft, int nchan, int nharm, int nmodel, double2 *out,
                            hipStream_t st) {
    dim3 g((unsigned)((nharm + 15) / 16), (unsigned)nmodel);
    hipLaunchKernelGGL(k_model_sum, g, dim3(256), 0, st, Mft, nchan, nharm, nmodel, out);
    return hipGetLastError();
}

}  // namespace ppf

#ifdef PPF_XM_PROF
extern "C" int ppf_debug_xprof(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ppf::g_xprof), sizeof(unsigned long long) * 8) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(ppf::g_xprof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
