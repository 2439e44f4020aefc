// ppf_wfft.hpp -- wave-private register/LDS FFT for gfx950 (wave64).
//
// One wave transforms one row of N = 2^LOG2N complex points (128 <= N <= 1024)
// with no workgroup barrier: each lane holds R = N/64 points in registers,
// every Stockham stage is a radix-R (last stage: the remaining radix) DFT
// done entirely in registers, and the data is exchanged between stages
// through the wave's own LDS buffer.  The buffer is padded by one slot per
// 2^S (pad(idx) = idx + (idx >> S), S = max(3, log2 R)), so the stride-R
// stores of the first stage are conflict-free and every access is a
// lane-dependent base plus a compile-time offset (folded into the ds_*
// immediate: no per-element address registers held across the row loop).
// Stage twiddles: one read of w = T[k N/(radix L)] (global table, L1/L2
// resident) per butterfly, the other powers by recurrence.
//
// Plan for N = 1024: radix 16 (L=1) -> radix 16 (L=16) -> radix 4 (L=256).
#pragma once
#include "ppf_device.hpp"

namespace ppf {
namespace wfft {

// exp(-2 pi i j / 16), j < 16 (exact decimal expansions)
__device__ constexpr double kC16[16] = {
    1.0, 0.92387953251128675613, 0.70710678118654752440, 0.38268343236508977173,
    0.0, -0.38268343236508977173, -0.70710678118654752440, -0.92387953251128675613,
    -1.0, -0.92387953251128675613, -0.70710678118654752440, -0.38268343236508977173,
    0.0, 0.38268343236508977173, 0.70710678118654752440, 0.92387953251128675613};
__device__ constexpr double kS16[16] = {
    0.0, -0.38268343236508977173, -0.70710678118654752440, -0.92387953251128675613,
    -1.0, -0.92387953251128675613, -0.70710678118654752440, -0.38268343236508977173,
    0.0, 0.38268343236508977173, 0.70710678118654752440, 0.92387953251128675613,
    1.0, 0.92387953251128675613, 0.70710678118654752440, 0.38268343236508977173};

// multiply by exp(-2 pi i e / 16) (compile-time e), special-casing the
// trivial and 45-degree factors
template <int E>
__device__ __forceinline__ double2 mul_w16(double2 a) {
    constexpr int e = E & 15;
    if constexpr (e == 0) return a;
    else if constexpr (e == 4) return cmk(a.y, -a.x);            // -i
    else if constexpr (e == 8) return cmk(-a.x, -a.y);           // -1
    else if constexpr (e == 12) return cmk(-a.y, a.x);           // +i
    else if constexpr (e == 2) {
        constexpr double h = 0.70710678118654752440;
        return cmk((a.x + a.y) * h, (a.y - a.x) * h);
    } else if constexpr (e == 6) {
        constexpr double h = 0.70710678118654752440;
        return cmk((a.y - a.x) * h, -(a.x + a.y) * h);
    } else if constexpr (e == 10) {
        constexpr double h = 0.70710678118654752440;
        return cmk(-(a.x + a.y) * h, (a.x - a.y) * h);
    } else if constexpr (e == 14) {
        constexpr double h = 0.70710678118654752440;
        return cmk((a.x - a.y) * h, (a.x + a.y) * h);
    } else {
        return cmul(a, cmk(kC16[e], kS16[e]));
    }
}

template <int R>
__device__ constexpr int log2c() { return R <= 1 ? 0 : 1 + log2c<R / 2>(); }

template <int I, int BITS>
__device__ constexpr int bitrev() {
    int r = 0;
    for (int b = 0; b < BITS; ++b) r |= ((I >> b) & 1) << (BITS - 1 - b);
    return r;
}

// in-register forward DFT of R = 2, 4, 8 or 16 points, natural order in/out
template <int R, int LEN, int I, int J>
__device__ __forceinline__ void dft_bfly(double2 (&y)[R]) {
    if constexpr (J < LEN / 2) {
        constexpr int a = I + J, b = I + J + LEN / 2;
        const double2 v = mul_w16<J * (16 / LEN)>(y[b]);
        const double2 u = y[a];
        y[a] = cadd(u, v);
        y[b] = csub(u, v);
        dft_bfly<R, LEN, I, J + 1>(y);
    }
}
template <int R, int LEN, int I>
__device__ __forceinline__ void dft_group(double2 (&y)[R]) {
    if constexpr (I < R) {
        dft_bfly<R, LEN, I, 0>(y);
        dft_group<R, LEN, I + LEN>(y);
    }
}
template <int R, int LEN>
__device__ __forceinline__ void dft_levels(double2 (&y)[R]) {
    if constexpr (LEN <= R) {
        dft_group<R, LEN, 0>(y);
        dft_levels<R, LEN * 2>(y);
    }
}
template <int R, int I>
__device__ __forceinline__ void dft_perm(const double2 *x, double2 (&y)[R]) {
    if constexpr (I < R) {
        y[I] = x[bitrev<I, log2c<R>()>()];
        dft_perm<R, I + 1>(x, y);
    }
}
template <int R>
__device__ __forceinline__ void dft(double2 *x) {   // x[0..R) in place
    double2 y[R];
    dft_perm<R, 0>(x, y);
    dft_levels<R, 2>(y);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = y[i];
}

// compile-time plan: lane-local radix R = N/64 while it fits, then the rest
template <int LOG2N>
struct Plan {
    static constexpr int N = 1 << LOG2N;
    static constexpr int R = N / 64;                  // points per lane
    static constexpr int LR = LOG2N - 6;
    static constexpr int NFULL = LOG2N / LR;          // full radix-R stages
    static constexpr int LAST = 1 << (LOG2N - NFULL * LR);   // 1: none
    static constexpr int NST = NFULL + (LAST > 1 ? 1 : 0);
    static constexpr int S = LR > 3 ? LR : 3;          // swizzle shift
    static constexpr int radix(int s) { return s < NFULL ? R : LAST; }
    static constexpr int L(int s) { return s == 0 ? 1 : L(s - 1) * radix(s - 1); }
    static constexpr int L2 = NST > 1 ? R : N;         // L of stage 1
    // twiddle-table offset of stage s >= 1: L(s) - L(1)
    static constexpr int toff(int s) { return L(s) - L2; }
};

// Element idx -> LDS slot.  Default: the padding above.  PPF_LDS_XOR=1: slot
// = idx ^ ((idx >> SH) & MK), a permutation inside aligned blocks, no padding.
// Priced with MI355X_MICROARCH.md's LDS lane groups (tools/lds_conflicts.py),
// the XOR map cuts the extra bank-conflict cycles of a 1024-point row from
// 2.25 to 0.75 per ds_*_b128 (the padding moves lanes 16-31 of a
// ds_read_b128 group one slot onto lanes 0-15's banks) and makes the
// eight-channel write-out of k_xspec_w conflict-free.  Measured on MI355X
// (89 GPU tests green with it): C3 unchanged, k_xmom_g 3% slower (31.8 vs
// 30.8 ms; the kernels are f64-issue bound, not LDS bound), C5 7% slower (k_xspec_w<9> needs 136
// VGPRs instead of 124: three waves per SIMD instead of four).  Kept off.
#ifndef PPF_LDS_XOR
#define PPF_LDS_XOR 0
#endif
template <int LOG2N>
__host__ __device__ constexpr bool use_xor() { return PPF_LDS_XOR != 0; }
template <int LOG2N>
struct Swz {
    static constexpr int SH = LOG2N == 7 ? 2 : (LOG2N == 10 ? 4 : 3);
    static constexpr int MK = LOG2N == 7 ? 3 : 7;
    // offsets that are multiples of FREE commute with the map
    static constexpr int FREE = use_xor<LOG2N>() ? (MK + 1) << SH : 1 << Plan<LOG2N>::S;
};
template <int LOG2N>
__device__ __forceinline__ constexpr int pad(int idx) {
    if constexpr (use_xor<LOG2N>()) return idx ^ ((idx >> Swz<LOG2N>::SH) & Swz<LOG2N>::MK);
    else return idx + (idx >> Plan<LOG2N>::S);
}
// pad(a + C) given pad(a), for a compile-time C that is a multiple of FREE
template <int LOG2N, int C>
__device__ __forceinline__ int pad_add(int pa) {
    static_assert(C % Swz<LOG2N>::FREE == 0, "offset must commute with the slot map");
    if constexpr (use_xor<LOG2N>()) return pa + C;
    else return pa + C + (C >> Plan<LOG2N>::S);
}
// LDS slots of one wave buffer
template <int LOG2N>
__host__ __device__ constexpr int buf_slots() {
    if constexpr (use_xor<LOG2N>()) return Plan<LOG2N>::N;
    else return Plan<LOG2N>::N + (Plan<LOG2N>::N >> Plan<LOG2N>::S);
}
// slot of element lane + C, C a compile-time multiple of 64: one of two
// lane bases (lb[0] = pad(lane), lb[1] = pad(lane + 64) - 64) plus a constant
template <int LOG2N, int C>
__device__ __forceinline__ int lane_slot(const int (&lb)[2]) {
    constexpr int F = Swz<LOG2N>::FREE;
    if constexpr (F <= 64) return pad_add<LOG2N, C>(lb[0]);
    else return pad_add<LOG2N, C - C % F>(lb[(C % F) / 64]) + C % F;
}

__device__ __forceinline__ void wave_sync() { wave_lds_sync(); }

// One Stockham stage ST >= 1: read from buf, twiddle, DFT, write to buf.
// Reads j + q NB (j = lane + 64 b): pad(lane) + const.  Writes o + q L with
// o = (j - k) rad + k: pad(o) + const when 2^S divides L, else computed.
template <int LOG2N, int ST, int B, int Q>
__device__ __forceinline__ void stage_read_q(double2 *buf, const int (&lb)[2], double2 (&v)[Plan<LOG2N>::N / Plan<LOG2N>::radix(ST) / 64][Plan<LOG2N>::radix(ST)]) {
    using P = Plan<LOG2N>;
    constexpr int rad = P::radix(ST), NB = P::N / rad;
    if constexpr (Q < rad) {
        v[B][Q] = buf[lane_slot<LOG2N, 64 * B + Q * NB>(lb)];
        stage_read_q<LOG2N, ST, B, Q + 1>(buf, lb, v);
    }
}
template <int LOG2N, int ST, int B>
__device__ __forceinline__ void stage_read(double2 *buf, const int (&lb)[2], double2 (&v)[Plan<LOG2N>::N / Plan<LOG2N>::radix(ST) / 64][Plan<LOG2N>::radix(ST)]) {
    using P = Plan<LOG2N>;
    constexpr int rad = P::radix(ST), NB = P::N / rad, BPL = NB / 64;
    if constexpr (B < BPL) {
        stage_read_q<LOG2N, ST, B, 0>(buf, lb, v);
        stage_read<LOG2N, ST, B + 1>(buf, lb, v);
    }
}
template <int LOG2N, int ST>
__device__ __forceinline__ void stage(double2 *buf, const double2 *__restrict__ T, int lane) {
    using P = Plan<LOG2N>;
    constexpr int N = P::N, rad = P::radix(ST), L = P::L(ST);
    constexpr int NB = N / rad, BPL = NB / 64, TS = N / (rad * L);
    const int lb[2] = {pad<LOG2N>(lane), pad<LOG2N>(lane + 64) - 64};
    double2 v[BPL][rad];
    stage_read<LOG2N, ST, 0>(buf, lb, v);
#pragma unroll
    for (int b = 0; b < BPL; ++b) {
        const int j = lane + 64 * b, k = j & (L - 1);
        // twiddles w^q, w = exp(-2 pi i k / (rad L)) = T[k N / (rad L)], by
        // recurrence from one table read (no rad-1 twiddles live at once;
        // every power read from a table instead, k_xmom_g at 1024 points:
        // 34.6 vs 30.8 ms)
        const double2 w1 = T[k * TS];
        double2 wq = w1;
        v[b][1] = cmul(v[b][1], w1);
#pragma unroll
        for (int q = 2; q < rad; ++q) {
            wq = cmul(wq, w1);
            v[b][q] = cmul(v[b][q], wq);
        }
        dft<rad>(v[b]);
    }
    wave_sync();
#pragma unroll
    for (int b = 0; b < BPL; ++b) {
        const int j = lane + 64 * b, k = j & (L - 1);
        const int o = (j - k) * rad + k;
        if constexpr (L % Swz<LOG2N>::FREE == 0) {
            const int ob = pad<LOG2N>(o);
#pragma unroll
            for (int q = 0; q < rad; ++q) buf[ob + q * L + (use_xor<LOG2N>() ? 0 : (q * L) >> P::S)] = v[b][q];
        } else {
#pragma unroll
            for (int q = 0; q < rad; ++q) buf[pad<LOG2N>(o + q * L)] = v[b][q];
        }
    }
    wave_sync();
}
template <int LOG2N, int ST>
__device__ __forceinline__ void stages_from(double2 *buf, const double2 *__restrict__ T, int lane) {
    if constexpr (ST < Plan<LOG2N>::NST) {
        stage<LOG2N, ST>(buf, T, lane);
        stages_from<LOG2N, ST + 1>(buf, T, lane);
    }
}

// Full forward FFT of the row whose stage-0 inputs x[q] = z[lane + 64 q]
// (q < R) are in registers; result in natural order in buf (padded).
template <int LOG2N>
__device__ __forceinline__ void fft_row(double2 (&x)[Plan<LOG2N>::R], double2 *buf,
                                        const double2 *__restrict__ T, int lane) {
    using P = Plan<LOG2N>;
    constexpr int R = P::R;
    dft<R>(x);
    wave_sync();
    // stage 0 output: o = lane R + q (L = 1, k = 0).  Padding: pad(lane R +
    // q) = pad(lane R) + q (q < R <= 2^S).  XOR map: the lane's R outputs are
    // permuted inside their block, slot = lane R + (q ^ f_lane) when R <=
    // 2^SH, else computed per element
    if constexpr (use_xor<LOG2N>()) {
#pragma unroll
        for (int q = 0; q < R; ++q) buf[pad<LOG2N>(lane * R + q)] = x[q];
    } else {
        const int ob = pad<LOG2N>(lane * R);
#pragma unroll
        for (int q = 0; q < R; ++q) buf[ob + q] = x[q];
    }
    wave_sync();
    stages_from<LOG2N, 1>(buf, T, lane);
}

// ---------------------------------------------------------------------------
// Half-buffer variant (round-4 prototype, k_noise_h): the same stages and
// arithmetic as fft_row, but each exchange goes through a buffer of doubles
// (the padded slot map of the complex buffer, 8 B per slot) in two sweeps,
// real parts then imaginary parts.  Half the LDS per wave (8.7 KB at 1024
// points instead of 17.4 KB), so the LDS no longer caps a CU at two waves
// per SIMD; the results are bit-identical to fft_row (only the exchange
// differs).  hb: the wave's buffer_slots<LOG2N>() doubles.
template <int LOG2N, int ST, int B, int Q, int PART>
__device__ __forceinline__ void hstage_read_q(const double *hb, const int (&lb)[2],
                                              double2 (&v)[Plan<LOG2N>::N / Plan<LOG2N>::radix(ST) / 64][Plan<LOG2N>::radix(ST)]) {
    using P = Plan<LOG2N>;
    constexpr int rad = P::radix(ST), NB = P::N / rad;
    if constexpr (Q < rad) {
        const double t = hb[lane_slot<LOG2N, 64 * B + Q * NB>(lb)];
        if constexpr (PART == 0) v[B][Q].x = t;
        else v[B][Q].y = t;
        hstage_read_q<LOG2N, ST, B, Q + 1, PART>(hb, lb, v);
    }
}
template <int LOG2N, int ST, int B, int PART>
__device__ __forceinline__ void hstage_read(const double *hb, const int (&lb)[2],
                                            double2 (&v)[Plan<LOG2N>::N / Plan<LOG2N>::radix(ST) / 64][Plan<LOG2N>::radix(ST)]) {
    using P = Plan<LOG2N>;
    constexpr int rad = P::radix(ST), NB = P::N / rad, BPL = NB / 64;
    if constexpr (B < BPL) {
        hstage_read_q<LOG2N, ST, B, 0, PART>(hb, lb, v);
        hstage_read<LOG2N, ST, B + 1, PART>(hb, lb, v);
    }
}
// write the stage outputs v (PART of each) to their slots
template <int LOG2N, int ST, int PART>
__device__ __forceinline__ void hstage_write(double *hb, int lane,
                                             const double2 (&v)[Plan<LOG2N>::N / Plan<LOG2N>::radix(ST) / 64][Plan<LOG2N>::radix(ST)]) {
    using P = Plan<LOG2N>;
    constexpr int N = P::N, rad = P::radix(ST), L = P::L(ST);
    constexpr int NB = N / rad, BPL = NB / 64;
#pragma unroll
    for (int b = 0; b < BPL; ++b) {
        const int j = lane + 64 * b, k = j & (L - 1);
        const int o = (j - k) * rad + k;
#pragma unroll
        for (int q = 0; q < rad; ++q) {
            const double t = PART == 0 ? v[b][q].x : v[b][q].y;
            if constexpr (L % Swz<LOG2N>::FREE == 0)
                hb[pad<LOG2N>(o) + q * L + (use_xor<LOG2N>() ? 0 : (q * L) >> P::S)] = t;
            else
                hb[pad<LOG2N>(o + q * L)] = t;
        }
    }
}
// stage ST >= 1 whose inputs are the previous stage's outputs vp (still in
// registers): exchange them through hb (two sweeps), twiddle, DFT; the
// outputs stay in v
template <int LOG2N, int ST, int PST>
__device__ __forceinline__ void hstage(double *hb, const double2 *__restrict__ T, int lane,
                                       const double2 (&vp)[Plan<LOG2N>::N / Plan<LOG2N>::radix(PST) / 64][Plan<LOG2N>::radix(PST)],
                                       double2 (&v)[Plan<LOG2N>::N / Plan<LOG2N>::radix(ST) / 64][Plan<LOG2N>::radix(ST)]) {
    using P = Plan<LOG2N>;
    constexpr int N = P::N, rad = P::radix(ST), L = P::L(ST);
    constexpr int NB = N / rad, BPL = NB / 64, TS = N / (rad * L);
    const int lb[2] = {pad<LOG2N>(lane), pad<LOG2N>(lane + 64) - 64};
    hstage_write<LOG2N, PST, 0>(hb, lane, vp);
    wave_sync();
    hstage_read<LOG2N, ST, 0, 0>(hb, lb, v);
    wave_sync();
    hstage_write<LOG2N, PST, 1>(hb, lane, vp);
    wave_sync();
    hstage_read<LOG2N, ST, 0, 1>(hb, lb, v);
    wave_sync();
#pragma unroll
    for (int b = 0; b < BPL; ++b) {
        const int j = lane + 64 * b, k = j & (L - 1);
        const double2 w1 = T[k * TS];
        double2 wq = w1;
        v[b][1] = cmul(v[b][1], w1);
#pragma unroll
        for (int q = 2; q < rad; ++q) {
            wq = cmul(wq, w1);
            v[b][q] = cmul(v[b][q], wq);
        }
        dft<rad>(v[b]);
    }
}
// the whole transform from registers x (stage-0 inputs, as fft_row) to the
// last stage's outputs in registers (vl: [N / radix(NST-1) / 64][radix]),
// written nowhere: the caller reads them out through hb (hwrite_last)
template <int LOG2N, int ST>
struct HBlk {
    using P = Plan<LOG2N>;
    using T = double2[P::N / P::radix(ST) / 64][P::radix(ST)];
};
template <int LOG2N, int ST>
__device__ __forceinline__ void hstages_from(double *hb, const double2 *__restrict__ T, int lane,
                                             const typename HBlk<LOG2N, ST - 1>::T &vp,
                                             typename HBlk<LOG2N, Plan<LOG2N>::NST - 1>::T &vl) {
    if constexpr (ST == Plan<LOG2N>::NST - 1) {
        hstage<LOG2N, ST, ST - 1>(hb, T, lane, vp, vl);
    } else {
        typename HBlk<LOG2N, ST>::T v;
        hstage<LOG2N, ST, ST - 1>(hb, T, lane, vp, v);
        hstages_from<LOG2N, ST + 1>(hb, T, lane, v, vl);
    }
}
template <int LOG2N>
__device__ __forceinline__ void fft_row_h(double2 (&x)[Plan<LOG2N>::R], double *hb,
                                          const double2 *__restrict__ T, int lane,
                                          typename HBlk<LOG2N, Plan<LOG2N>::NST - 1>::T &vl) {
    using P = Plan<LOG2N>;
    static_assert(P::NST >= 2, "half-buffer FFT: at least two stages");
    dft<P::R>(x);
    typename HBlk<LOG2N, 0>::T v0;
#pragma unroll
    for (int q = 0; q < P::R; ++q) v0[0][q] = x[q];
    hstages_from<LOG2N, 1>(hb, T, lane, v0, vl);
}
// the last stage's outputs, PART (0: re, 1: im), to their natural-order slots
template <int LOG2N, int PART>
__device__ __forceinline__ void hwrite_last(double *hb, int lane,
                                            const typename HBlk<LOG2N, Plan<LOG2N>::NST - 1>::T &vl) {
    hstage_write<LOG2N, Plan<LOG2N>::NST - 1, PART>(hb, lane, vl);
}

}  // namespace wfft
}  // namespace ppf
