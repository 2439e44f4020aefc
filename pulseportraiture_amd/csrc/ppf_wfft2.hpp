// ppf_wfft2.hpp -- 1024-point wave FFT with one LDS exchange (gfx950).
//
// One wave transforms one row of N = 1024 complex points (a 2048-bin real
// row packed z_j = x_2j + i x_2j+1), 16 points per lane, as the four-step
// split 1024 = 16 (registers) x 64 (lanes), 64 = 4 x 16:
//
//   in:  x[q] = z[l + 64 q]            (lane l, register q)
//   A  DFT16 over q -> k1, twiddle W1024^(l k1)                  (registers)
//   B  lane bits 4, 5 <-> register bits 2, 3: v_permlane16_swap /
//      v_permlane32_swap (VALU, no LDS), then DFT4 over them -> m1, and the
//      twiddle W64^(l_lo e(m1))                                  (registers)
//   C  one LDS exchange (16 ds_write_b128 + 16 ds_read_b128) that gives
//      every lane the 16 l_lo values of one kappa = k1 + 16 m1, then DFT16
//      over them -> m2                                           (registers)
//
// The wave-FFT of ppf_wfft.hpp exchanges three times (radix 16 x 16 x 4) and
// writes the row back in natural order for the real post-pass: four LDS
// round trips per row.  Here: one, and the output layout is chosen so that
// the real post-pass partner Z[N - k] of every element sits in the SAME
// register of the lane l ^ 32 (a v_permlane32_swap per dword, section D):
//
//   lanes l < 32:  kappa = l,                           x[m] = Z[kappa + 64 m]
//   lanes l >= 32: kappa = 96 - l (l = 32: kappa = 32),  x[m] = Z[kappa + 64 (15 - m)]
//
// The upper lanes' reversed order costs nothing: their DFT16 inputs are
// read in reversed order from the exchange buffer and pre-multiplied by
// W16^(-l_lo), which the writer folds into its W64 twiddle (e(m1) = m1 - 4
// for m1 >= 2, i.e. exactly the kappa >= 32 destinations).  Negation mod 64
// has two fixed points (kappa = 0 and 32: lanes 0 and 32), whose pairs lie
// inside their own registers; those two lanes take their post-pass operands
// from a 32-slot LDS side buffer (exec-masked stores and loads).
//
// Exchange buffer: slot(lambda, r') = 65 r' + lambda (complex), 16,640 B per
// wave; the writes of a ds_write_b128 lane group land on 8 distinct rows
// (bank offset 4 per row: conflict-free), the reads are lane-contiguous.
#pragma once
#include "ppf_wfft.hpp"

namespace ppf {
namespace wf2 {

// scheduling fences between the sections (keeps the compiler from hoisting
// a later section's twiddle arithmetic into an earlier one, which holds
// dozens of extra VGPRs)
#ifndef PPF_WF2_CUT
#define PPF_WF2_CUT 1
#endif
#if PPF_WF2_CUT
#define WF2_CUT() __builtin_amdgcn_sched_barrier(0)
#else
#define WF2_CUT()
#endif

constexpr int kN = 1024;
constexpr int kXS = 65;                 // exchange row stride (complex slots)
constexpr int kXSlots = 16 * kXS;       // 1040 complex slots per wave
constexpr int kSpSlots = 32;            // side buffer of lanes 0 and 32

// per-lane constants of the transform (computed once per wave)
struct Seeds {
    double2 w1;     // W1024^lane
    double2 v1;     // W64^(lane & 15)
};

__device__ __forceinline__ Seeds make_seeds(int lane) {
    Seeds s;
    double sn, cs;
    sincospi(-2.0 * (double)lane / 1024.0, &sn, &cs);
    s.w1 = cmk(cs, sn);
    sincospi(-2.0 * (double)(lane & 15) / 64.0, &sn, &cs);
    s.v1 = cmk(cs, sn);
    return s;
}

// v_permlane{16,32}_swap on the four dwords of a complex double
template <bool S32>
__device__ __forceinline__ void pswap1(double &a, double &b) {
    const unsigned alo = __double2loint(a), ahi = __double2hiint(a);
    const unsigned blo = __double2loint(b), bhi = __double2hiint(b);
    unsigned nalo, nahi, nblo, nbhi;
    if constexpr (S32) {
        const auto lo = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
        nalo = lo[0]; nblo = lo[1]; nahi = hi[0]; nbhi = hi[1];
    } else {
        const auto lo = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
        nalo = lo[0]; nblo = lo[1]; nahi = hi[0]; nbhi = hi[1];
    }
    a = __hiloint2double((int)nahi, (int)nalo);
    b = __hiloint2double((int)nbhi, (int)nblo);
}
template <bool S32>
__device__ __forceinline__ void pswap(double2 &a, double2 &b) {
    pswap1<S32>(a.x, b.x);
    pswap1<S32>(a.y, b.y);
}

// In-register 16-point DFT (natural order in and out), radix-2 DIT as
// wfft::dft<16> but with every twiddled butterfly fused into FMAs: a 45-degree
// twiddle as u +- h (b.x + b.y, b.y - b.x) (2 adds + 4 fma instead of 8 ops),
// a general one in Linzer-Feig form u +- c (b.x - t b.y, b.y + t b.x) with c =
// cos, t = tan of the angle (6 fma).  148 f64 operations instead of 168.
template <int E>
__device__ __forceinline__ void bfly16(double2 &u, double2 &v) {
    constexpr int e = E & 15;
    constexpr double h = 0.70710678118654752440;
    const double2 a = u, b = v;
    if constexpr (e == 0) {
        u = cmk(a.x + b.x, a.y + b.y);
        v = cmk(a.x - b.x, a.y - b.y);
    } else if constexpr (e == 4) {                       // b * -i
        u = cmk(a.x + b.y, a.y - b.x);
        v = cmk(a.x - b.y, a.y + b.x);
    } else if constexpr (e == 2 || e == 6) {
        // e = 2: b w = h (b.x + b.y, b.y - b.x); e = 6: h (b.y - b.x, -(b.x + b.y))
        const double s = b.x + b.y, d = b.y - b.x;
        const double px = e == 2 ? s : d, py = e == 2 ? d : -s;
        u = cmk(fma(h, px, a.x), fma(h, py, a.y));
        v = cmk(fma(-h, px, a.x), fma(-h, py, a.y));
    } else {
        // w = exp(-2 pi i e / 16) = c (1 + i t)
        constexpr double C[8] = {1.0, 0.92387953251128675613, 0.0, 0.38268343236508977173, 0.0,
                                 -0.38268343236508977173, 0.0, -0.92387953251128675613};
        constexpr double T[8] = {0.0, -0.41421356237309504880, 0.0, -2.41421356237309504880, 0.0,
                                 2.41421356237309504880, 0.0, 0.41421356237309504880};
        const double p = fma(-T[e], b.y, b.x), q = fma(T[e], b.x, b.y);
        u = cmk(fma(C[e], p, a.x), fma(C[e], q, a.y));
        v = cmk(fma(-C[e], p, a.x), fma(-C[e], q, a.y));
    }
}
template <int LEN, int I, int J>
__device__ __forceinline__ void dft16_bfly(double2 (&y)[16]) {
    if constexpr (J < LEN / 2) {
        bfly16<J * (16 / LEN)>(y[I + J], y[I + J + LEN / 2]);
        dft16_bfly<LEN, I, J + 1>(y);
    }
}
template <int LEN, int I>
__device__ __forceinline__ void dft16_group(double2 (&y)[16]) {
    if constexpr (I < 16) {
        dft16_bfly<LEN, I, 0>(y);
        dft16_group<LEN, I + LEN>(y);
    }
}
#ifndef PPF_WF2_FDFT
#define PPF_WF2_FDFT 1
#endif
__device__ __forceinline__ void dft16(double2 (&x)[16]) {
    if constexpr (PPF_WF2_FDFT == 0) {
        wfft::dft<16>(x);
    } else {
        double2 y[16];
        wfft::dft_perm<16, 0>(x, y);
        dft16_group<2, 0>(y);
        dft16_group<4, 0>(y);
        dft16_group<8, 0>(y);
        dft16_group<16, 0>(y);
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = y[i];
    }
}

// Sections A-C.  x: the row as above; xb: the wave's kXSlots exchange slots.
// Returns with x[m] in the output layout of the header.
// The seeds are made opaque per call: their powers are loop-invariant, and
// hoisted out of a row loop they would hold 64 VGPRs for the whole kernel.
__device__ __forceinline__ void opaque(double2 &v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y));
}
__device__ __forceinline__ void fft1024(double2 (&x)[16], double2 *xb, int lane, const Seeds &sd0) {
    Seeds sd = sd0;
    opaque(sd.w1);
    opaque(sd.v1);
    // A: DFT16 over q, twiddle W1024^(l k1)
    dft16(x);
    {
        double2 wq = sd.w1;
        x[1] = cmul(x[1], wq);
#pragma unroll
        for (int k = 2; k < 16; ++k) {
            wq = cmul(wq, sd.w1);
            x[k] = cmul(x[k], wq);
        }
    }
    WF2_CUT();
    // B: lane bit 5 <-> register bit 3, lane bit 4 <-> register bit 2
#pragma unroll
    for (int r = 0; r < 8; ++r) pswap<true>(x[r], x[r + 8]);
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if ((r & 4) == 0) pswap<false>(x[r], x[r + 4]);
    // registers now k1lo + 4 l_hi (l_hi = old lane >> 4); lane = l_lo + 16 k1hi.
    // DFT4 over l_hi -> m1, then W64^(l_lo e(m1)), e = 0, 1, -2, -1
    const double2 v2 = cmul(sd.v1, sd.v1);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        double2 t[4] = {x[a], x[a + 4], x[a + 8], x[a + 12]};
        wfft::dft<4>(t);
        x[a] = t[0];
        x[a + 4] = cmul(t[1], sd.v1);
        x[a + 8] = cmulc(t[2], v2);
        x[a + 12] = cmulc(t[3], sd.v1);
    }
    WF2_CUT();
    // C: exchange.  Element (lane: l_lo, k1hi; register a + 4 m1) has kappa
    // = a + 4 k1hi + 16 m1 and goes to reader lane lambda(kappa), position
    // r' = l_lo (m1 < 2) or -l_lo mod 16 (m1 >= 2).
    const int llo = lane & 15, k1hi = lane >> 4;
    const int lb0 = kXS * llo + 4 * k1hi;
    const int lb1 = kXS * ((16 - llo) & 15) - 4 * k1hi + 32;
    const int lb8 = lb1 + (k1hi == 0 ? 0 : 32);       // kappa = 32 -> lane 32
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        xb[lb0 + a] = x[a];                            // m1 = 0: lambda = kappa
        xb[lb0 + a + 16] = x[a + 4];                   // m1 = 1
        if (a == 0) xb[lb8] = x[8];                    // m1 = 2: lambda = 96 - kappa
        else xb[lb1 + 32 - a] = x[a + 8];
        xb[lb1 + 16 - a] = x[a + 12];                  // m1 = 3
    }
    wfft::wave_sync();
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = xb[lane + kXS * r];
    wfft::wave_sync();
    dft16(x);
}

// kappa held by a lane, and the harmonic of x[m] (the header's layout)
__device__ __forceinline__ int lane_kappa(int lane) {
    return lane < 32 ? lane : (lane == 32 ? 32 : 96 - lane);
}
__device__ __forceinline__ int out_index(int lane, int m) {
    const int kap = lane_kappa(lane);
    return lane < 32 ? kap + 64 * m : kap + 64 * (15 - m);
}

// D: the real post-pass operands.  After pairs(): for slot i < 8 every lane
// holds A[i] = Z[kA + 64 i] and B[i] = Z[N - kA - 64 i], kA = pair_k0(lane)
// (lane 0: slot 0 is the pair (0, N) -> Z0 twice).  Lane 0 also returns
// Z[N/2] in zm.  sp: the wave's kSpSlots side slots.
__device__ __forceinline__ int pair_k0(int lane) {
    return lane == 32 ? 32 : (lane & 31) + (lane >= 32 ? 512 : 0);
}
__device__ __forceinline__ void pairs(double2 (&x)[16], double2 *sp, int lane, double2 &zm) {
    const bool special = (lane & 31) == 0;
    if (special) {
        const int b = (lane >> 5) * 16;
#pragma unroll
        for (int m = 0; m < 16; ++m) sp[b + m] = x[m];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) pswap<true>(x[i], x[i + 8]);
    wfft::wave_sync();
    if (special) {
        // lane 0: pairs (64 i, N - 64 i) of its own registers; lane 32:
        // (32 + 64 i, N - 32 - 64 i), its registers reversed
        const bool l0 = lane == 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            x[i] = sp[l0 ? i : 31 - i];
            x[i + 8] = sp[l0 ? ((16 - i) & 15) : 16 + i];
        }
        if (l0) zm = sp[8];
    }
    wfft::wave_sync();
}

}  // namespace wf2
}  // namespace ppf
