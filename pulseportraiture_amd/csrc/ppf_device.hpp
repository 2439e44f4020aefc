// ppf_device.hpp -- device building blocks of the gfx950 wideband FFTFIT engine.
//
// Complex fp64 helpers, wave64/workgroup reductions, an LDS-resident Stockham
// radix-4/2 FFT shared by every FFT-using kernel, the real<->half-length
// complex FFT packing, the scipy trust-ncg replica and the exact trust-region
// subproblem (Jacobi eigendecomposition and the secular equation) of the
// Newton solver, and a
// companion-matrix polynomial root finder (np.roots replacement for the
// zero-covariance GM cases).  Everything is fp64; the one dense contraction
// on the path (the Taylor moments of k_xmom_g, ppf_xspec.hip) is f64 MFMA.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ppf {

constexpr double kPi = 3.14159265358979323846;
constexpr double kTwoPi = 6.28318530717958647692;
constexpr double kDconst = 1.0 / 0.000241;   // pplib.py:64-67 (Dconst_trad)
constexpr double kLn10 = 2.30258509299404568402;
constexpr int kBlock = 256;                  // threads per workgroup (4 waves)
constexpr int kWaves = kBlock / 64;
constexpr int kMaxBfly = 4;                  // radix-4 butterflies / thread / pass

// ---------------------------------------------------------------------------
// complex fp64
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ double2 cmk(double r, double i) {
    double2 z; z.x = r; z.y = i; return z;
}
// Streaming accesses (round 6): data rows are read once and the cross
// spectrum X is written once per pass, so they are issued nontemporal and
// do not evict what IS re-read from the XCD's L2 (model rows, |M|^2, twiddle
// and moment tables).  C2: k_xspec_w2 24.09 vs 24.83 ms per 10k, 302.4k vs
// 294.3k fits/s; C3 / C5 +1-2 % (profiles/r06/ab_nt_status.txt).
#ifndef PPF_NT
#define PPF_NT 1
#endif
template <typename T>
__device__ __forceinline__ T ld_stream(const T *p) {
#if PPF_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
__device__ __forceinline__ float2 ld_stream(const float2 *p) {
    typedef float v2 __attribute__((ext_vector_type(2)));
    const v2 v = ld_stream(reinterpret_cast<const v2 *>(p));
    return float2(v.x, v.y);
}
__device__ __forceinline__ double2 ld_stream(const double2 *p) {
    typedef double v2 __attribute__((ext_vector_type(2)));
    const v2 v = ld_stream(reinterpret_cast<const v2 *>(p));
    return cmk(v.x, v.y);
}
__device__ __forceinline__ void st_stream(double2 *p, double2 v) {
#if PPF_NT
    typedef double v2 __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(v2{v.x, v.y}, reinterpret_cast<v2 *>(p));
#else
    *p = v;
#endif
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return cmk(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return cmk(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cscale(double2 a, double s) { return cmk(a.x * s, a.y * s); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return cmk(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// a * conj(b)
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {
    return cmk(fma(a.x, b.x, a.y * b.y), fma(a.y, b.x, -a.x * b.y));
}
__device__ __forceinline__ double2 cconj(double2 a) { return cmk(a.x, -a.y); }
__device__ __forceinline__ double cabs2(double2 a) { return fma(a.x, a.x, a.y * a.y); }

// exp(2 pi i t) with exact argument reduction of t to [-1/2, 1/2].
__device__ __forceinline__ double2 cexp2pi(double t) {
    double r = t - rint(t);
    double s, c;
    sincospi(2.0 * r, &s, &c);
    return cmk(c, s);
}

// ---------------------------------------------------------------------------
// reductions (fixed order -> bitwise reproducible)
// ---------------------------------------------------------------------------
// DPP move of a double (two 32-bit halves); lanes outside row_mask keep 0
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane63_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// Wave reductions on the DPP network (no LDS round trips): quad xor 1, xor
// 2, half-row mirror, row mirror (every lane of a row then holds the row
// total, bit-identically), then row_bcast15 / row_bcast31 fold rows 0+1 and
// 2+3 and the pairs into lane 63, read back as a wave-uniform value.  Fixed
// order: ((r3 + r2) + (r1 + r0)).  Needs all 64 lanes active.
template <typename Op>
__device__ __forceinline__ double wave_reduce(double v, Op op) {
    v = op(v, dpp_d<0xB1, 0xf>(v));     // quad_perm [1,0,3,2]
    v = op(v, dpp_d<0x4E, 0xf>(v));     // quad_perm [2,3,0,1]
    v = op(v, dpp_d<0x141, 0xf>(v));    // row_half_mirror
    v = op(v, dpp_d<0x140, 0xf>(v));    // row_mirror
    {
        const double t = dpp_d<0x142, 0xa>(v);   // row_bcast:15 -> rows 1, 3
        const int r = (threadIdx.x >> 4) & 3;
        if (r & 1) v = op(v, t);
    }
    {
        const double t = dpp_d<0x143, 0xc>(v);   // row_bcast:31 -> rows 2, 3
        if ((threadIdx.x & 63) >= 32) v = op(v, t);
    }
    return readlane63_d(v);
}

// the scattering kernel 1 / (1 + i b) of pplib.scattering_portrait_FT:
// NumPy's complex reciprocal (loops CDOUBLE_reciprocal) of 1 + i b
__device__ __forceinline__ double2 scat_recip(double b) {
#pragma clang fp contract(off)
    if (fabs(b) <= 1.0) {
        const double r = b / 1.0, d = 1.0 + b * r;
        return cmk(1.0 / d, -r / d);
    }
    const double r = 1.0 / b, d = 1.0 * r + b;
    return cmk(r / d, -1.0 / d);
}

#ifdef PPF_SHFL_REDUCE
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    return v;
}
#else
__device__ __forceinline__ double wave_sum(double v) {
    return wave_reduce(v, [](double x, double y) { return x + y; });
}

__device__ __forceinline__ double wave_max(double v) {
    return wave_reduce(v, [](double x, double y) { return fmax(x, y); });
}
#endif

// wave-uniform copies of a double held by the first / a given lane
__device__ __forceinline__ double readfirst_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)b);
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// wave-scope ordering of LDS traffic (no hardware barrier: a wave's LDS
// operations are processed in issue order; this keeps the compiler from
// moving them across the exchange point)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sum K values per thread over the whole block; result valid in every thread.
// scratch must hold kWaves*K doubles.  Contains two __syncthreads().
// Max of K values per thread over the block (same contract as block_sum).
template <int K, int NW = kWaves>
__device__ __forceinline__ void block_max(double (&v)[K], double *scratch) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < K; ++i) v[i] = wave_max(v[i]);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < K; ++i) scratch[wave * K + i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double s = scratch[i];
        for (int w = 1; w < NW; ++w) s = fmax(s, scratch[w * K + i]);
        v[i] = s;
    }
    __syncthreads();
}

template <int K, int NW = kWaves>
__device__ __forceinline__ void block_sum(double (&v)[K], double *scratch) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < K; ++i) v[i] = wave_sum(v[i]);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < K; ++i) scratch[wave * K + i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double s = 0.0;
        for (int w = 0; w < NW; ++w) s += scratch[w * K + i];
        v[i] = s;
    }
    __syncthreads();
}

// block_sum / block_max for a TB-thread block: one wave (TB = 64) reduces
// with DPP alone (no LDS round trip, no barrier); otherwise the block forms
template <int K, int TB>
__device__ __forceinline__ void blk_sum(double (&v)[K], double *scratch) {
    if constexpr (TB == 64) {
#pragma unroll
        for (int i = 0; i < K; ++i) v[i] = wave_sum(v[i]);
    } else {
        block_sum<K, TB / 64>(v, scratch);
    }
}
template <int K, int TB>
__device__ __forceinline__ void blk_max(double (&v)[K], double *scratch) {
    if constexpr (TB == 64) {
#pragma unroll
        for (int i = 0; i < K; ++i) v[i] = wave_max(v[i]);
    } else {
        block_max<K, TB / 64>(v, scratch);
    }
}

// ---------------------------------------------------------------------------
// LDS FFT (Stockham autosort, radix-4 with one leading radix-2 pass when
// log2 N is odd).  In place in buf[0..N); every thread of the block must call
// it (it synchronises).  T[t] = exp(-2 pi i t / N), t < N (global, cached).
// inverse: exp(+...) kernel, no 1/N scaling.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double2 twid(const double2 *__restrict__ T, int idx, bool inverse) {
    double2 w = T[idx];
    return inverse ? cconj(w) : w;
}

__device__ void lds_fft(double2 *buf, int log2N, const double2 *__restrict__ T, bool inverse) {
    const int N = 1 << log2N;
    const int tid = threadIdx.x;
    int L = 1;
    if (log2N & 1) {  // radix-2, L = 1: no twiddles
        const int nb = N >> 1;
        double2 a[2 * kMaxBfly], b[2 * kMaxBfly];
#pragma unroll
        for (int q = 0; q < 2 * kMaxBfly; ++q) {
            int j = tid + q * kBlock;
            if (j < nb) { a[q] = buf[j]; b[q] = buf[j + nb]; }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 2 * kMaxBfly; ++q) {
            int j = tid + q * kBlock;
            if (j < nb) {
                buf[2 * j] = cadd(a[q], b[q]);
                buf[2 * j + 1] = csub(a[q], b[q]);
            }
        }
        __syncthreads();
        L = 2;
    }
    const int nb = N >> 2;
    while (L < N) {
        const int tstride = N / (4 * L);
        double2 x[kMaxBfly][4];
#pragma unroll
        for (int q = 0; q < kMaxBfly; ++q) {
            int j = tid + q * kBlock;
            if (j < nb) {
                int k = j & (L - 1);
#pragma unroll
                for (int r = 0; r < 4; ++r) x[q][r] = buf[j + r * nb];
                if (k) {
                    x[q][1] = cmul(x[q][1], twid(T, k * tstride, inverse));
                    x[q][2] = cmul(x[q][2], twid(T, 2 * k * tstride, inverse));
                    x[q][3] = cmul(x[q][3], twid(T, 3 * k * tstride, inverse));
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kMaxBfly; ++q) {
            int j = tid + q * kBlock;
            if (j < nb) {
                int k = j & (L - 1);
                double2 s02 = cadd(x[q][0], x[q][2]), d02 = csub(x[q][0], x[q][2]);
                double2 s13 = cadd(x[q][1], x[q][3]), d13 = csub(x[q][1], x[q][3]);
                // forward: y1 = d02 - i d13, y3 = d02 + i d13
                double2 id13 = inverse ? cmk(-d13.y, d13.x) : cmk(d13.y, -d13.x);
                int o = (j - k) * 4 + k;
                buf[o] = cadd(s02, s13);
                buf[o + L] = cadd(d02, id13);
                buf[o + 2 * L] = csub(s02, s13);
                buf[o + 3 * L] = csub(d02, id13);
            }
        }
        __syncthreads();
        L <<= 2;
    }
}

// ---------------------------------------------------------------------------
// Mixed-radix LDS FFT for any N <= 4096 (nbin = 2N not a power
// of two: 1000, 1536, 600, ...; numpy's pocketfft takes any length,
// pptoaslib.py:1022-1025, pplib.py:2455).  Stockham autosort as lds_fft:
// stage with radix R and span L reads x_q = buf[j + q N/R] (j < N/R,
// k = j mod L), twiddles x_q by T[q k N/(R L)], takes the R-point DFT and
// writes buf[(j - k) R + k + q L].  Radices: 4s (one 2 first when the
// power of two is odd), then 3s, 5s, 7s, then larger prime factors on the
// generic-radix stage (mr_stage_g).  Power-of-two N goes to lds_fft
// (bitwise unchanged).
// ---------------------------------------------------------------------------
constexpr int kMaxFftN = 4096;

// Stage radices of N in order: 4s (one 2 first when the power of two is
// odd), 3s, 5s, 7s, then any larger prime factors (the generic-radix stage
// below).  Returns their count, 0 for N < 2.
__host__ __device__ inline int fft_radices(int N, int *r) {
    if (N < 2) return 0;
    int n = N, p2 = 0, c = 0;
    while ((n & 1) == 0) { n >>= 1; ++p2; }
    if (p2 & 1) r[c++] = 2;
    for (int i = 0; i < p2 / 2; ++i) r[c++] = 4;
    for (int f = 3; f * f <= n; f += 2)
        while (n % f == 0) { n /= f; r[c++] = f; }
    if (n > 1) r[c++] = n;
    return c;
}
// N = 2^a 3^b 5^c 7^d: every stage has a hard-coded butterfly
__host__ __device__ inline bool fft_len_smooth(int N) {
    if (N < 2) return false;
    int n = N;
    const int f[4] = {2, 3, 5, 7};
    for (int p : f)
        while (n % p == 0) n /= p;
    return n == 1;
}
__host__ __device__ inline bool fft_len_supported(int N) { return N >= 2 && N <= kMaxFftN; }
__host__ __device__ inline bool is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }
// Complex FFT length of a real row of nbin samples: even nbin packs
// z_j = x_2j + i x_2j+1 into nbin / 2 points (rfft_bin / irfft_prebin); odd
// nbin transforms the row itself, nbin points with zero imaginary parts
// (X_k = Z_k for k <= nbin / 2, the inverse from the Hermitian-filled buffer)
__host__ __device__ inline int rfft_len(int nbin) { return (nbin & 1) ? nbin : nbin >> 1; }

// cos / sin (2 pi m / R), m < R, for the odd radices (exact decimal expansions)
__device__ constexpr double kCos3[3] = {1.0, -0.5, -0.5};
__device__ constexpr double kSin3[3] = {0.0, 0.86602540378443864676, -0.86602540378443864676};
__device__ constexpr double kCos5[5] = {1.0, 0.30901699437494742410, -0.80901699437494742410,
                                        -0.80901699437494742410, 0.30901699437494742410};
__device__ constexpr double kSin5[5] = {0.0, 0.95105651629515357212, 0.58778525229247312917,
                                        -0.58778525229247312917, -0.95105651629515357212};
__device__ constexpr double kCos7[7] = {1.0, 0.62348980185873353053, -0.22252093395631440429,
                                        -0.90096886790241912624, -0.90096886790241912624,
                                        -0.22252093395631440429, 0.62348980185873353053};
__device__ constexpr double kSin7[7] = {0.0, 0.78183148246802980871, 0.97492791218182360702,
                                        0.43388373911755812048, -0.43388373911755812048,
                                        -0.97492791218182360702, -0.78183148246802980871};

// R-point DFT in place (natural order), forward exp(-2 pi i m q / R)
template <int R>
__device__ __forceinline__ void dft_small(double2 (&x)[R], bool inv) {
    if constexpr (R == 2) {
        const double2 a = x[0], b = x[1];
        x[0] = cadd(a, b);
        x[1] = csub(a, b);
    } else if constexpr (R == 4) {
        const double2 s02 = cadd(x[0], x[2]), d02 = csub(x[0], x[2]);
        const double2 s13 = cadd(x[1], x[3]), d13 = csub(x[1], x[3]);
        const double2 id13 = inv ? cmk(-d13.y, d13.x) : cmk(d13.y, -d13.x);
        x[0] = cadd(s02, s13);
        x[1] = cadd(d02, id13);
        x[2] = csub(s02, s13);
        x[3] = csub(d02, id13);
    } else {
        // odd R over the pairs a_j = x_j + x_{R-j}, b_j = x_j - x_{R-j}
        // (j = 1 .. H): c_m = x_0 + sum_j cos(2 pi j m / R) a_j,
        // d_m = sum_j sin(2 pi j m / R) b_j, and y_m = c_m -+ i d_m,
        // y_{R-m} = c_m +- i d_m (forward / inverse): H^2 real-by-complex
        // products per part instead of (R-1)^2 complex ones
        constexpr int H = (R - 1) / 2;
        const double *C = R == 3 ? kCos3 : (R == 5 ? kCos5 : kCos7);
        const double *S = R == 3 ? kSin3 : (R == 5 ? kSin5 : kSin7);
        double2 pa[H], pb[H];
        double2 y0 = x[0];
#pragma unroll
        for (int j = 1; j <= H; ++j) {
            pa[j - 1] = cadd(x[j], x[R - j]);
            pb[j - 1] = csub(x[j], x[R - j]);
            y0 = cadd(y0, pa[j - 1]);
        }
        double2 y[R];
        y[0] = y0;
#pragma unroll
        for (int m = 1; m <= H; ++m) {
            double2 c = x[0], d = cmk(0.0, 0.0);
#pragma unroll
            for (int j = 1; j <= H; ++j) {
                const int e = (j * m) % R;
                c = cmk(fma(C[e], pa[j - 1].x, c.x), fma(C[e], pa[j - 1].y, c.y));
                d = cmk(fma(S[e], pb[j - 1].x, d.x), fma(S[e], pb[j - 1].y, d.y));
            }
            // -i d (forward) / +i d (inverse)
            const double2 id = inv ? cmk(-d.y, d.x) : cmk(d.y, -d.x);
            y[m] = cadd(c, id);
            y[R - m] = csub(c, id);
        }
#pragma unroll
        for (int m = 0; m < R; ++m) x[m] = y[m];
    }
}

template <int R>
__device__ void mr_stage(double2 *buf, int N, int L, const double2 *__restrict__ T, bool inv) {
    constexpr int QM = (kMaxFftN / R + kBlock - 1) / kBlock;   // butterflies / thread
    const int nb = N / R, ts = N / (R * L);
    double2 x[QM][R];
#pragma unroll
    for (int q = 0; q < QM; ++q) {
        const int j = threadIdx.x + q * kBlock;
        if (j < nb) {
            const int k = j % L;
#pragma unroll
            for (int r = 0; r < R; ++r) x[q][r] = buf[j + r * nb];
            if (k) {
#pragma unroll
                for (int r = 1; r < R; ++r) x[q][r] = cmul(x[q][r], twid(T, r * k * ts, inv));
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < QM; ++q) {
        const int j = threadIdx.x + q * kBlock;
        if (j < nb) {
            const int k = j % L;
            dft_small<R>(x[q], inv);
            const int o = (j - k) * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) buf[o + r * L] = x[q][r];
        }
    }
    __syncthreads();
}

// Generic-radix stage for a prime factor R > 7 of N (1002 = 2 * 3 * 167,
// 1022 = 2 * 7 * 73 bins ...), the same Stockham step with the stage twiddle
// and the R-point DFT folded into one table index: the output at
// o = (j - k) R + k + m L is sum_q buf[j + q N/R] T[q (k N/(R L) + m N/R) mod N].
// One output per thread per pass (NT threads starting at t0), O(N R) work;
// all of a thread's reads are done before the caller's barrier, its writes
// after it.
template <int QO>
__device__ __forceinline__ void gr_stage_read(const double2 *buf, int N, int L, int R,
                                              const double2 *__restrict__ T, bool inv, int t0, int NT,
                                              double2 (&y)[QO]) {
    const int nb = N / R, ts = N / (R * L), RL = R * L;
#pragma unroll
    for (int i = 0; i < QO; ++i) {
        const int o = t0 + i * NT;
        if (o < N) {
            const int blk = o / RL, rem = o - blk * RL, m = rem / L, k = rem - m * L;
            const int j = blk * L + k;
            int e = k * ts + m * nb;
            e = e >= N ? e - N : e;
            double2 acc = buf[j];
            for (int q = 1, idx = e; q < R; ++q) {
                const double2 w = twid(T, idx, inv);
                acc = cadd(acc, cmul(buf[j + q * nb], w));
                idx += e;
                idx = idx >= N ? idx - N : idx;
            }
            y[i] = acc;
        }
    }
}
// gr_stage_read with the outputs formed G = 4 at a time and the q loop
// outside, so a lane has four independent LDS read chains in flight instead
// of one dependent chain per output (the same arithmetic per output, so the
// same bits); an output past N is computed on a clamped index and dropped.
// The wave-per-row kernels take it (k_xspec_wm / k_xspec_wo: nbin 1022 and
// 1023 +3-4 %); in the block-FFT kernels its registers cost more than it
// gains (k_guess at nbin 1000 / 1536: 152 -> 185 / 248 -> 278 ms per 72
// calls, profiles/r05/ab_r5g_status.txt), so they keep the loop above.
template <int QO>
__device__ __forceinline__ void gr_stage_read4(const double2 *buf, int N, int L, int R,
                                              const double2 *__restrict__ T, bool inv, int t0, int NT,
                                              double2 (&y)[QO]) {
    const int nb = N / R, ts = N / (R * L), RL = R * L;
    constexpr int G = QO >= 4 ? 4 : QO;
    static_assert(QO % G == 0, "QO must be a multiple of the group size");
#pragma unroll
    for (int i0 = 0; i0 < QO; i0 += G) {
        if (t0 + i0 * NT >= N) break;            // no output of this thread from here on
        int j[G], e[G], idx[G];
        double2 acc[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            int o = t0 + (i0 + g) * NT;
            o = o < N ? o : N - 1;
            const int blk = o / RL, rem = o - blk * RL, m = rem / L, k = rem - m * L;
            j[g] = blk * L + k;
            const int ee = k * ts + m * nb;
            e[g] = ee >= N ? ee - N : ee;
            idx[g] = e[g];
            acc[g] = buf[j[g]];
        }
        for (int q = 1; q < R; ++q) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const double2 w = twid(T, idx[g], inv);
                acc[g] = cadd(acc[g], cmul(buf[j[g] + q * nb], w));
                idx[g] += e[g];
                idx[g] = idx[g] >= N ? idx[g] - N : idx[g];
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) y[i0 + g] = acc[g];
    }
}
template <int QO>
__device__ __forceinline__ void gr_stage_write(double2 *buf, int N, int t0, int NT, const double2 (&y)[QO]) {
#pragma unroll
    for (int i = 0; i < QO; ++i) {
        const int o = t0 + i * NT;
        if (o < N) buf[o] = y[i];
    }
}
__device__ __noinline__ void mr_stage_g(double2 *buf, int N, int L, int R, const double2 *__restrict__ T,
                                        bool inv) {
    constexpr int QO = kMaxFftN / kBlock;
    double2 y[QO];
    gr_stage_read<QO>(buf, N, L, R, T, inv, threadIdx.x, kBlock, y);
    __syncthreads();
    gr_stage_write<QO>(buf, N, threadIdx.x, kBlock, y);
    __syncthreads();
}

// Any supported N (fft_len_supported); every thread of the block calls it.
__device__ void lds_fft(double2 *buf, int log2N, const double2 *__restrict__ T, bool inverse);
__device__ __forceinline__ void lds_fft_mixed(double2 *buf, int N, const double2 *__restrict__ T,
                                           bool inverse) {
    int r[32];
    const int ns = fft_radices(N, r);
    int L = 1;
    for (int s = 0; s < ns; ++s) {
        switch (r[s]) {
            case 2: mr_stage<2>(buf, N, L, T, inverse); break;
            case 3: mr_stage<3>(buf, N, L, T, inverse); break;
            case 4: mr_stage<4>(buf, N, L, T, inverse); break;
            case 5: mr_stage<5>(buf, N, L, T, inverse); break;
            case 7: mr_stage<7>(buf, N, L, T, inverse); break;
            default: mr_stage_g(buf, N, L, r[s], T, inverse); break;
        }
        L *= r[s];
    }
}
// MX = false: N is a power of two (the caller's launcher checked) and the
// kernel carries none of the mixed-radix code, whose registers would
// otherwise set its VGPR budget: with the stages inlined a block-FFT kernel
// needs ~190 VGPRs (two waves per SIMD), with them behind a call 248 VGPRs +
// 32 AGPRs and scratch (one wave), against ~100 without (round 4: k_guess at
// C4 0.60 vs 0.30 ms per launch).  Launchers instantiate MX = true only for
// nbin / 2 not a power of two.
template <bool MX = true>
__device__ __forceinline__ void lds_fft_n(double2 *buf, int N, const double2 *__restrict__ T,
                                          bool inverse) {
    if (!MX || is_pow2(N)) lds_fft(buf, __builtin_ctz((unsigned)N), T, inverse);
    else if constexpr (MX) lds_fft_mixed(buf, N, T, inverse);
}

// Compile-time-size variant of lds_fft (exact register footprint, unrolled
// passes); T may live in LDS or global memory.
template <int LOG2N, bool INV>
__device__ __forceinline__ void lds_fft_t(double2 *buf, const double2 *T) {
    constexpr int N = 1 << LOG2N;
    const int tid = threadIdx.x;
    int L = 1;
    if constexpr ((LOG2N & 1) != 0) {
        constexpr int nb = N / 2;
        constexpr int Q = (nb + kBlock - 1) / kBlock;
        double2 a[Q], b[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int j = tid + q * kBlock;
            if (j < nb) { a[q] = buf[j]; b[q] = buf[j + nb]; }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int j = tid + q * kBlock;
            if (j < nb) { buf[2 * j] = cadd(a[q], b[q]); buf[2 * j + 1] = csub(a[q], b[q]); }
        }
        __syncthreads();
        L = 2;
    }
    constexpr int nb = N / 4;
    constexpr int Q = (nb + kBlock - 1) / kBlock;
#pragma unroll
    for (int pass = 0; pass < LOG2N / 2; ++pass) {
        const int tstride = N / (4 * L);
        double2 x[Q][4];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int j = tid + q * kBlock;
            if (j < nb) {
                const int k = j & (L - 1);
#pragma unroll
                for (int r = 0; r < 4; ++r) x[q][r] = buf[j + r * nb];
                if (k) {
                    x[q][1] = cmul(x[q][1], twid(T, k * tstride, INV));
                    x[q][2] = cmul(x[q][2], twid(T, 2 * k * tstride, INV));
                    x[q][3] = cmul(x[q][3], twid(T, 3 * k * tstride, INV));
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int j = tid + q * kBlock;
            if (j < nb) {
                const int k = j & (L - 1);
                const double2 s02 = cadd(x[q][0], x[q][2]), d02 = csub(x[q][0], x[q][2]);
                const double2 s13 = cadd(x[q][1], x[q][3]), d13 = csub(x[q][1], x[q][3]);
                const double2 id13 = INV ? cmk(-d13.y, d13.x) : cmk(d13.y, -d13.x);
                const int o = (j - k) * 4 + k;
                buf[o] = cadd(s02, s13);
                buf[o + L] = cadd(d02, id13);
                buf[o + 2 * L] = csub(s02, s13);
                buf[o + 3 * L] = csub(d02, id13);
            }
        }
        __syncthreads();
        L <<= 2;
    }
}

// Real FFT post-pass: X_k (k = 0..N) from Z = FFT_N(x_even + i x_odd).
// T2[k] = exp(-i pi k / N), k < N.
__device__ __forceinline__ double2 rfft_bin(const double2 *buf, int N, const double2 *__restrict__ T2, int k) {
    // k in [0, N]: Z_{k mod N} and Z_{(N - k) mod N} (any N)
    double2 zk = buf[k == N ? 0 : k];
    double2 zc = cconj(buf[k == 0 ? 0 : N - k]);
    double2 e = cscale(cadd(zk, zc), 0.5);
    double2 o = cscale(csub(zk, zc), 0.5);       // (Z_k - conj Z_{N-k}) / 2
    double2 w = (k < N) ? T2[k] : cmk(-1.0, 0.0);
    // X_k = e - i w o
    double2 wo = cmul(w, o);
    return cmk(e.x + wo.y, e.y - wo.x);
}

// Inverse real FFT pre-pass: Z_k (k < N) from X_0..X_N (imaginary parts of
// X_0 and X_N ignored, as numpy.fft.irfft does).  Xk, XNk = X_k, X_{N-k}.
__device__ __forceinline__ double2 irfft_prebin(double2 Xk, double2 XNk, double2 w /*T2[k]*/) {
    double2 xc = cconj(XNk);
    double2 e = cscale(cadd(Xk, xc), 0.5);
    double2 d = cscale(csub(Xk, xc), 0.5);
    double2 o = cmul(cconj(w), d);               // exp(+i pi k/N) (X_k - conj X_{N-k}) / 2
    return cmk(e.x - o.y, e.y + o.x);            // E + i O
}

// ---------------------------------------------------------------------------
// scipy trust-ncg replica (scipy/optimize/_trustregion.py:_minimize_trust_region
// with _trustregion_ncg.py:CGSteihaugSubproblem), on the fitted subspace.
// ---------------------------------------------------------------------------
struct TRModel {
    double f;
    double g[5];
    double H[5][5];
};

// The subspace dimension N (number of fitted parameters) is a template
// argument: every loop unrolls and the vectors stay in registers (a runtime
// bound made them scratch arrays, one memory round trip per element access
// on the solver's serial path).
template <int N>
__device__ __forceinline__ double dotn(const double *a, const double *b) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i) s += a[i] * b[i];
    return s;
}
template <int N>
__device__ __forceinline__ void hessp(const TRModel &m, const double *p, double *out) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) s += m.H[i][j] * p[j];
        out[i] = s;
    }
}
template <int N>
__device__ __forceinline__ double model_value(const TRModel &m, const double *p) {
    double Hp[5];
    hessp<N>(m, p, Hp);
    return m.f + dotn<N>(m.g, p) + 0.5 * dotn<N>(p, Hp);
}
// || z + t d || == R  ->  (ta, tb) sorted
template <int N>
__device__ __forceinline__ void boundary_t(const double *z, const double *d, double R, double &ta,
                                           double &tb) {
    double a = dotn<N>(d, d), b = 2.0 * dotn<N>(z, d), c = dotn<N>(z, z) - R * R;
    double sq = sqrt(b * b - 4.0 * a * c);
    double aux = b + copysign(sq, b);
    double t1 = -aux / (2.0 * a), t2 = -2.0 * c / aux;
    ta = fmin(t1, t2);
    tb = fmax(t1, t2);
}
// Returns hits_boundary; p (length N) is the step.
template <int N>
__device__ bool cg_steihaug(const TRModel &m, double jac_mag, double R, double *p) {
    double tol = fmin(0.5, sqrt(jac_mag)) * jac_mag;
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = 0.0;
    if (jac_mag < tol) return false;
    double z[5], r[5], d[5], Bd[5];
#pragma unroll
    for (int i = 0; i < N; ++i) { z[i] = 0.0; r[i] = m.g[i]; d[i] = -m.g[i]; }
#pragma unroll 1
    for (int it = 0; it < 64; ++it) {
        hessp<N>(m, d, Bd);
        double dBd = dotn<N>(d, Bd);
        if (dBd <= 0.0) {
            double ta, tb;
            boundary_t<N>(z, d, R, ta, tb);
            double pa[5], pb[5];
#pragma unroll
            for (int i = 0; i < N; ++i) { pa[i] = z[i] + ta * d[i]; pb[i] = z[i] + tb * d[i]; }
            bool usea = model_value<N>(m, pa) < model_value<N>(m, pb);
#pragma unroll
            for (int i = 0; i < N; ++i) p[i] = usea ? pa[i] : pb[i];
            return true;
        }
        double rr = dotn<N>(r, r);
        double alpha = rr / dBd;
        double zn[5];
#pragma unroll
        for (int i = 0; i < N; ++i) zn[i] = z[i] + alpha * d[i];
        if (sqrt(dotn<N>(zn, zn)) >= R) {
            double ta, tb;
            boundary_t<N>(z, d, R, ta, tb);
#pragma unroll
            for (int i = 0; i < N; ++i) p[i] = z[i] + tb * d[i];
            return true;
        }
        double rn[5];
#pragma unroll
        for (int i = 0; i < N; ++i) rn[i] = r[i] + alpha * Bd[i];
        double rnn = dotn<N>(rn, rn);
        if (sqrt(rnn) < tol) {
#pragma unroll
            for (int i = 0; i < N; ++i) p[i] = zn[i];
            return false;
        }
        double beta = rnn / rr;
#pragma unroll
        for (int i = 0; i < N; ++i) { d[i] = -rn[i] + beta * d[i]; z[i] = zn[i]; r[i] = rn[i]; }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = z[i];
    return false;
}

// ---------------------------------------------------------------------------
// Exact trust-region subproblem for the Newton solver of the scattering fits
// (PPF_TR_NEWTON): min_p g.p + p.H p / 2 subject to |p| <= R, H symmetric
// N x N (N <= 5), by the eigendecomposition of H (cyclic Jacobi) and Newton
// iterations on the secular equation 1/|p(l)| = 1/R, p(l) = -(H + l I)^-1 g
// (More & Sorensen 1983; Nocedal & Wright, Numerical Optimization, alg. 4.3,
// with the "hard case" of a g orthogonal to the lowest eigenvector).
// Returns hits_boundary; p (length N) is the step.  __host__ as well so the
// CPU tests check it against a NumPy restatement (ppf_tr_subproblem_host).
// ---------------------------------------------------------------------------
template <int N>
__host__ __device__ inline void sym_eig_jacobi(double (&A)[5][5], double (&V)[5][5]) {
    #pragma unroll
    for (int i = 0; i < N; ++i)
        #pragma unroll
        for (int j = 0; j < N; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 40; ++sweep) {
        double off = 0.0, dia = 0.0;
        #pragma unroll
        for (int p = 0; p < N; ++p) {
            dia += A[p][p] * A[p][p];
            #pragma unroll
            for (int q = p + 1; q < N; ++q) off += A[p][q] * A[p][q];
        }
        if (!(off > 1e-34 * dia)) break;
        #pragma unroll
        for (int p = 0; p < N; ++p) {
            #pragma unroll
            for (int q = p + 1; q < N; ++q) {
                const double apq = A[p][q];
                if (apq == 0.0) continue;
                const double th = (A[q][q] - A[p][p]) / (2.0 * apq);
                const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                #pragma unroll
                for (int k = 0; k < N; ++k) {          // A J
                    const double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
                #pragma unroll
                for (int k = 0; k < N; ++k) {          // J^T (A J)
                    const double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
                A[p][q] = A[q][p] = 0.0;
                #pragma unroll
                for (int k = 0; k < N; ++k) {          // V J
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
        }
    }
}

template <int N>
__host__ __device__ inline bool tr_exact(const double (&H)[5][5], const double *g, double R, double *p) {
    double A[5][5], V[5][5], lam[5], gp[5], q[5];
    #pragma unroll
    for (int i = 0; i < N; ++i)
        #pragma unroll
        for (int j = 0; j < N; ++j) A[i][j] = H[i][j];
    sym_eig_jacobi<N>(A, V);
    int imin = 0;
    double gn2 = 0.0;
    #pragma unroll
    for (int i = 0; i < N; ++i) {
        lam[i] = A[i][i];
        if (lam[i] < lam[imin]) imin = i;
        double s = 0.0;
        #pragma unroll
        for (int k = 0; k < N; ++k) s += V[k][i] * g[k];
        gp[i] = s;
        gn2 += s * s;
    }
    const double lmin = lam[imin];
    bool hb = true;
    if (lmin > 0.0) {
        double n2 = 0.0;
        #pragma unroll
        for (int i = 0; i < N; ++i) { q[i] = gp[i] / lam[i]; n2 += q[i] * q[i]; }
        if (n2 <= R * R) hb = false;      // interior Newton step
    }
    if (hb) {
        const double lo = lmin > 0.0 ? 0.0 : -lmin;
        // hard case: g (almost) orthogonal to the lowest eigenvector and the
        // step at l = lo inside the region -> add that eigenvector
        if (lmin <= 0.0 && fabs(gp[imin]) <= 1e-10 * sqrt(gn2)) {
            double n2 = 0.0;
            #pragma unroll
            for (int i = 0; i < N; ++i) {
                const double d = lam[i] + lo;
                q[i] = (i == imin || d <= 0.0) ? 0.0 : gp[i] / d;
                n2 += q[i] * q[i];
            }
            if (n2 < R * R) {
                q[imin] = -sqrt(R * R - n2);      // p = -V q below
                #pragma unroll
                for (int k = 0; k < N; ++k) {
                    double s = 0.0;
                    #pragma unroll
                    for (int i = 0; i < N; ++i) s += V[k][i] * q[i];
                    p[k] = -s;
                }
                return true;
            }
        }
        // iterate on the shift e = l - lo >= 0 with d_i = (lam_i + lo) + e
        // (exactly e for the lowest eigenvalue when lo = -lam_min: no
        // cancellation when lo is large).  Start where |p| >= R (|p| >=
        // |gp_min| / e and |p| >= |g| / (e + lo + lam_max)): Newton on
        // 1/|p| - 1/R from there increases e monotonically to the root
        double sh[5], lmax = lam[0];
        #pragma unroll
        for (int i = 0; i < N; ++i) { sh[i] = (i == imin && lo > 0.0) ? 0.0 : lam[i] + lo; lmax = fmax(lmax, lam[i]); }
        double e = fmax(fabs(gp[imin]) / R, sqrt(gn2) / R - lmax - lo);
        if (!(e > 0.0)) e = 1e-300;
        for (int it = 0; it < 100; ++it) {
            double n2 = 0.0, w = 0.0;
            #pragma unroll
            for (int i = 0; i < N; ++i) {
                const double d = sh[i] + e;
                q[i] = gp[i] / d;
                n2 += q[i] * q[i];
                w += q[i] * q[i] / d;
            }
            const double nq = sqrt(n2);
            if (fabs(nq - R) <= 1e-13 * R || !(w > 0.0)) break;
            double en = e + (n2 / w) * (nq - R) / R;
            if (!(en > 0.0)) en = 0.5 * e;
            if (en == e) break;
            e = en;
        }
        double n2 = 0.0;
        #pragma unroll
        for (int i = 0; i < N; ++i) { q[i] = gp[i] / (sh[i] + e); n2 += q[i] * q[i]; }
        if (n2 > R * R) {                 // round onto the sphere
            const double sc = R / sqrt(n2);
            #pragma unroll
            for (int i = 0; i < N; ++i) q[i] *= sc;
        }
    }
    #pragma unroll
    for (int k = 0; k < N; ++k) {
        double s = 0.0;
        #pragma unroll
        for (int i = 0; i < N; ++i) s += V[k][i] * q[i];
        p[k] = -s;
    }
    return hb;
}

// ---------------------------------------------------------------------------
// small dense inverse (Gauss-Jordan, partial pivoting); returns false if
// singular.  n <= 5.
// ---------------------------------------------------------------------------
__host__ __device__ inline bool invert_small(double (*A)[5], double (*Ainv)[5], int n) {
    double M[5][10];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 2 * n; ++j) M[i][j] = (j < n) ? A[i][j] : (j - n == i ? 1.0 : 0.0);
    for (int c = 0; c < n; ++c) {
        int piv = c;
        double best = fabs(M[c][c]);
        for (int r = c + 1; r < n; ++r)
            if (fabs(M[r][c]) > best) { best = fabs(M[r][c]); piv = r; }
        if (best == 0.0 || !(best == best)) return false;
        if (piv != c)
            for (int j = 0; j < 2 * n; ++j) { double t = M[c][j]; M[c][j] = M[piv][j]; M[piv][j] = t; }
        double inv = 1.0 / M[c][c];
        for (int j = 0; j < 2 * n; ++j) M[c][j] *= inv;
        for (int r = 0; r < n; ++r) {
            if (r == c) continue;
            double f = M[r][c];
            if (f != 0.0)
                for (int j = 0; j < 2 * n; ++j) M[r][j] -= f * M[c][j];
        }
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) Ainv[i][j] = M[i][j + n];
    return true;
}

// ---------------------------------------------------------------------------
// Polynomial roots as np.roots: eigenvalues of the companion matrix
// (balanced, then Francis double-shift QR on the Hessenberg form).  Only the
// real roots (exact zero imaginary part, as LAPACK reports them) are returned.
// coeffs[0..deg] highest power first.  Returns the number of real roots.
// ---------------------------------------------------------------------------
#define PPF_SIGN(a, b) ((b) >= 0.0 ? fabs(a) : -fabs(a))

__host__ __device__ inline void balance_small(double (*a)[8], int n) {
    const double radix = 2.0, sqrdx = radix * radix;
    int last = 0;
    while (last == 0) {
        last = 1;
        for (int i = 0; i < n; ++i) {
            double r = 0.0, c = 0.0;
            for (int j = 0; j < n; ++j)
                if (j != i) { c += fabs(a[j][i]); r += fabs(a[i][j]); }
            if (c != 0.0 && r != 0.0) {
                double g = r / radix, f = 1.0, s = c + r;
                while (c < g) { f *= radix; c *= sqrdx; }
                g = r * radix;
                while (c > g) { f /= radix; c /= sqrdx; }
                if ((c + r) / f < 0.95 * s) {
                    last = 0;
                    g = 1.0 / f;
                    for (int j = 0; j < n; ++j) a[i][j] *= g;
                    for (int j = 0; j < n; ++j) a[j][i] *= f;
                }
            }
        }
    }
}

// a: upper Hessenberg n x n (n <= 8), destroyed.  wr/wi eigenvalues.
// Returns false on non-convergence.
__host__ __device__ inline bool hqr_small(double (*a)[8], int n, double *wr, double *wi) {
    int nn, m, l, k, j, its, i, mmin;
    double z = 0, y, x, w, v, u, t, s, r = 0, q = 0, p = 0, anorm = 0.0;
    for (i = 0; i < n; ++i)
        for (j = (i - 1 > 0 ? i - 1 : 0); j < n; ++j) anorm += fabs(a[i][j]);
    nn = n - 1;
    t = 0.0;
    while (nn >= 0) {
        its = 0;
        do {
            for (l = nn; l >= 1; --l) {
                s = fabs(a[l - 1][l - 1]) + fabs(a[l][l]);
                if (s == 0.0) s = anorm;
                if (fabs(a[l][l - 1]) + s == s) { a[l][l - 1] = 0.0; break; }
            }
            x = a[nn][nn];
            if (l == nn) {
                wr[nn] = x + t;
                wi[nn--] = 0.0;
            } else {
                y = a[nn - 1][nn - 1];
                w = a[nn][nn - 1] * a[nn - 1][nn];
                if (l == nn - 1) {
                    p = 0.5 * (y - x);
                    q = p * p + w;
                    z = sqrt(fabs(q));
                    x += t;
                    if (q >= 0.0) {
                        z = p + PPF_SIGN(z, p);
                        wr[nn - 1] = wr[nn] = x + z;
                        if (z != 0.0) wr[nn] = x - w / z;
                        wi[nn - 1] = wi[nn] = 0.0;
                    } else {
                        wr[nn - 1] = wr[nn] = x + p;
                        wi[nn - 1] = -(wi[nn] = z);
                    }
                    nn -= 2;
                } else {
                    if (its == 60) return false;
                    if (its == 10 || its == 20) {
                        t += x;
                        for (i = 0; i <= nn; ++i) a[i][i] -= x;
                        s = fabs(a[nn][nn - 1]) + fabs(a[nn - 1][nn - 2]);
                        y = x = 0.75 * s;
                        w = -0.4375 * s * s;
                    }
                    ++its;
                    for (m = nn - 2; m >= l; --m) {
                        z = a[m][m];
                        r = x - z;
                        s = y - z;
                        p = (r * s - w) / a[m + 1][m] + a[m][m + 1];
                        q = a[m + 1][m + 1] - z - r - s;
                        r = a[m + 2][m + 1];
                        s = fabs(p) + fabs(q) + fabs(r);
                        p /= s; q /= s; r /= s;
                        if (m == l) break;
                        u = fabs(a[m][m - 1]) * (fabs(q) + fabs(r));
                        v = fabs(p) * (fabs(a[m - 1][m - 1]) + fabs(z) + fabs(a[m + 1][m + 1]));
                        if (u + v == v) break;
                    }
                    for (i = m + 2; i <= nn; ++i) {
                        a[i][i - 2] = 0.0;
                        if (i != m + 2) a[i][i - 3] = 0.0;
                    }
                    for (k = m; k <= nn - 1; ++k) {
                        if (k != m) {
                            p = a[k][k - 1];
                            q = a[k + 1][k - 1];
                            r = 0.0;
                            if (k != nn - 1) r = a[k + 2][k - 1];
                            if ((x = fabs(p) + fabs(q) + fabs(r)) != 0.0) { p /= x; q /= x; r /= x; }
                        }
                        if ((s = PPF_SIGN(sqrt(p * p + q * q + r * r), p)) != 0.0) {
                            if (k == m) {
                                if (l != m) a[k][k - 1] = -a[k][k - 1];
                            } else {
                                a[k][k - 1] = -s * x;
                            }
                            p += s;
                            x = p / s; y = q / s; z = r / s; q /= p; r /= p;
                            for (j = k; j <= nn; ++j) {
                                p = a[k][j] + q * a[k + 1][j];
                                if (k != nn - 1) { p += r * a[k + 2][j]; a[k + 2][j] -= p * z; }
                                a[k + 1][j] -= p * y;
                                a[k][j] -= p * x;
                            }
                            mmin = nn < k + 3 ? nn : k + 3;
                            for (i = l; i <= mmin; ++i) {
                                p = x * a[i][k] + y * a[i][k + 1];
                                if (k != nn - 1) { p += z * a[i][k + 2]; a[i][k + 2] -= p * r; }
                                a[i][k + 1] -= p * q;
                                a[i][k] -= p;
                            }
                        }
                    }
                }
            }
        } while (l < nn - 1);
    }
    return true;
}

// Real roots of sum_i c[i] x^(deg-i).  out receives them; returns count, or
// -1 if the QR iteration failed.
__host__ __device__ inline int poly_real_roots(const double *c, int deg, double *out) {
    int lead = 0;
    while (lead <= deg && c[lead] == 0.0) ++lead;
    if (lead > deg) return 0;
    int trail = 0;
    while (deg - trail > lead && c[deg - trail] == 0.0) ++trail;
    int n = deg - lead - trail;  // companion size
    int cnt = 0;
    for (int i = 0; i < trail; ++i) out[cnt++] = 0.0;
    if (n <= 0) return cnt;
    double a[8][8];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) a[i][j] = 0.0;
    for (int j = 0; j < n; ++j) a[0][j] = -c[lead + 1 + j] / c[lead];
    for (int i = 1; i < n; ++i) a[i][i - 1] = 1.0;
    balance_small(a, n);
    double wr[8], wi[8];
    if (!hqr_small(a, n, wr, wi)) return -1;
    for (int i = 0; i < n; ++i)
        if (wi[i] == 0.0) out[cnt++] = wr[i];
    return cnt;
}

}  // namespace ppf
