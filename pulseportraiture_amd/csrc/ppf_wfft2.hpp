// ppf_wfft2.hpp -- two-wave (128-lane) register/LDS FFT of a 1024-point row
// for gfx950.
//
// ppf_wfft.hpp gives a whole row to one wave: 16 points per lane and a 16 KB
// LDS buffer per wave, so at most eight or nine waves per CU fit in LDS (two
// per SIMD).  Here two waves share one row: each of the 128 lanes holds 8
// points, the Stockham stages are radix 8, 8, 8, 2 (L = 1, 8, 64, 512), and
// the exchanges go through the pair's LDS buffer with workgroup barriers
// between stages (all waves of the workgroup take every barrier).  With eight
// rows per workgroup that is sixteen waves per CU, four per SIMD.
// Slots are padded by one per 8 elements (pad(idx) = idx + (idx >> 3)): the
// stride-8 stores of the first stage then land on eight different 16-B bank
// groups.
#pragma once
#include "ppf_wfft.hpp"

namespace ppf {
namespace wfft2 {

constexpr int N = 1024, P = 128, R0 = 8;        // points, lanes per row, points per lane
constexpr int NST = 4;
__host__ __device__ constexpr int radix(int s) { return s < 3 ? 8 : 2; }
__host__ __device__ constexpr int Ls(int s) { return s == 0 ? 1 : Ls(s - 1) * radix(s - 1); }

__device__ __forceinline__ constexpr int pad(int idx) { return idx + (idx >> 3); }
__host__ __device__ constexpr int buf_slots() { return N + (N >> 3); }

// one Stockham stage ST >= 1 (reads, barrier, writes, barrier); lane L in
// [0, 128).  Every wave takes both barriers; live = false skips the work.
template <int ST>
__device__ __forceinline__ void stage(double2 *buf, const double2 *__restrict__ T, int L, bool live) {
    constexpr int rad = radix(ST), Lst = Ls(ST), NB = N / rad, BPL = NB / P, TS = N / (rad * Lst);
    double2 v[BPL][rad];
    if (live) {
        const int lb = pad(L);
#pragma unroll
        for (int b = 0; b < BPL; ++b)
#pragma unroll
            for (int q = 0; q < rad; ++q) {
                const int c = P * b + q * NB;           // multiple of 8: pad(L + c) = pad(L) + c + c/8
                v[b][q] = buf[lb + c + (c >> 3)];
            }
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            const int j = L + P * b, k = j & (Lst - 1);
            const double2 w1 = T[k * TS];
            double2 wq = w1;
            v[b][1] = cmul(v[b][1], w1);
#pragma unroll
            for (int q = 2; q < rad; ++q) {
                wq = cmul(wq, w1);
                v[b][q] = cmul(v[b][q], wq);
            }
            wfft::dft<rad>(v[b]);
        }
    }
    __syncthreads();
    if (live) {
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            const int j = L + P * b, k = j & (Lst - 1);
            const int o = (j - k) * rad + k;
            if constexpr ((Lst & 7) == 0) {
                const int ob = pad(o);
#pragma unroll
                for (int q = 0; q < rad; ++q) buf[ob + q * Lst + ((q * Lst) >> 3)] = v[b][q];
            } else {
#pragma unroll
                for (int q = 0; q < rad; ++q) buf[pad(o + q * Lst)] = v[b][q];
            }
        }
    }
    __syncthreads();
}

// Full forward FFT of the row whose stage-0 inputs x[q] = z[L + 128 q] are in
// registers (live = false: this pair has no row this round and only takes
// the barriers); result in natural order in buf (padded).  Starts with a
// barrier (the buffer's previous readers are done) and ends after one.
__device__ __forceinline__ void fft_row(double2 (&x)[R0], double2 *buf, const double2 *__restrict__ T,
                                        int L, bool live) {
    if (live) wfft::dft<R0>(x);
    __syncthreads();
    if (live) {
        const int ob = pad(L * R0);                    // pad(8L + q) = pad(8L) + q
#pragma unroll
        for (int q = 0; q < R0; ++q) buf[ob + q] = x[q];
    }
    __syncthreads();
    stage<1>(buf, T, L, live);
    stage<2>(buf, T, L, live);
    stage<3>(buf, T, L, live);
}

}  // namespace wfft2
}  // namespace ppf
