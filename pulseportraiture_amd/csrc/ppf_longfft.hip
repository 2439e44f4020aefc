// Long 1-D transforms on the device (round 6): get_noise_PS of rows longer
// than the LDS FFTs take -- pplib.get_noise_PS(chans=False) ravels a whole
// portrait (pplib.py:2334-2338: nchan * nbin samples, 2^20 at 512 x 2048),
// and rows of any length with chans=True (pplib.py:2312-2332).  Until round
// 5 these went to the FFT library through torch.fft.
//
//   * transform length n: nbin / 2 complex points for an even row (two real
//     samples packed per point, split after the transform), the row itself
//     as n complex points for an odd one (ppf::rfft_len's convention);
//   * n a power of two (>= 64): one four-step transform of M = n = M1 M2
//     points, M1, M2 <= 4096, each step a batch of block LDS FFTs (lds_fft):
//       P1  for each n2 < M2: FFT over n1 of x[M2 n1 + n2], times
//           exp(-2 pi i n2 k1 / M), stored at [k1][n2]
//       P2  for each k1 < M1: FFT over n2 of row k1, stored at [k1][k2]
//     so X[k1 + M1 k2] ends at k1 M2 + k2 (the power sums read it there);
//   * any other n: Bluestein's chirp z-transform, X_k = w_k sum_j (x_j w_j)
//     conj(w_{k-j}), w_j = exp(-i pi j^2 / n), as a circular convolution of
//     length M = pow2 >= 2n - 1 (>= 64): P1 P2 of the chirped row and of the
//     chirp, the product, and the inverse four-step (I1 = P2's batches
//     inverse with the twiddle after, I2 = P1's inverse) back to natural
//     order.  j^2 is reduced mod 2n in integers before the sincospi, so the
//     chirp is exact to an ulp for every n <= 2^23;
//   * k_lf_pow: |F_k|^2 / nbin for k >= kc = int((1 - 1/frac) nharm) in
//     fixed-order block partials, k_lf_fin: sqrt of their mean.
// Every kernel here streams; none is on the fit's hot path.
#include <hip/hip_runtime.h>

#include "ppf_device.hpp"
#include "ppf_internal.hpp"

namespace ppf {

namespace {

// exp(i pi e / d), e reduced into [0, 2d)
__device__ __forceinline__ double2 phasor_pi(int64_t e, int64_t d, double sign) {
    double s, c;
    sincospi(sign * (double)e / (double)d, &s, &c);
    return cmk(c, s);
}

// w_j = exp(-i pi j^2 / n)
__device__ __forceinline__ double2 chirp(int64_t j, int64_t n) {
    const int64_t e = (j % (2 * n)) * (j % (2 * n)) % (2 * n);
    return phasor_pi(e, n, -1.0);
}

}  // namespace

// real rows [nrows][nbin] -> complex sequences [nrows][M] (packed / as is,
// chirped and zero-padded for Bluestein)
__global__ __launch_bounds__(kBlock) void k_lf_load(LongNoiseArgs a, double2 *A) {
    const int64_t r = blockIdx.y;
    const char *base = reinterpret_cast<const char *>(a.in);
    const size_t esz = a.in_dtype == PPF_F32 ? 4 : 8;
    const char *row = base + (size_t)(a.row0 + r) * (size_t)a.nbin * esz;
    auto x = [&](int64_t t) -> double {
        return a.in_dtype == PPF_F32 ? (double)ld_stream(reinterpret_cast<const float *>(row) + t)
                                     : ld_stream(reinterpret_cast<const double *>(row) + t);
    };
    double2 *out = A + r * a.M;
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < a.M; j += (int64_t)gridDim.x * kBlock) {
        double2 z = cmk(0.0, 0.0);
        if (j < a.n) {
            z = a.packed ? cmk(x(2 * j), x(2 * j + 1)) : cmk(x(j), 0.0);
            if (a.bluestein) z = cmul(z, chirp(j, a.n));
        }
        out[j] = z;
    }
}

// the convolution kernel b_j = conj(w_|j|) on the circle of M points
__global__ __launch_bounds__(kBlock) void k_lf_chirp(LongNoiseArgs a, double2 *B) {
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < a.M; j += (int64_t)gridDim.x * kBlock) {
        double2 b = cmk(0.0, 0.0);
        if (j < a.n) b = cconj(chirp(j, a.n));
        else if (j > a.M - a.n) b = cconj(chirp(a.M - j, a.n));
        B[j] = b;
    }
}

// one four-step pass: grid (nbatch, nrows), a block LDS FFT per batch
__global__ __launch_bounds__(kBlock) void k_lf_pass(LongPassArgs p) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int64_t b = blockIdx.x, r = blockIdx.y;
    const double2 *src = p.in + r * p.row_elems + b * p.in_bstride;
    for (int j = threadIdx.x; j < p.len; j += kBlock) lds[j] = src[(int64_t)j * p.in_stride];
    __syncthreads();
    lds_fft(lds, p.log2len, p.T, p.inverse != 0);
    __syncthreads();
    double2 *dst = p.out + r * p.row_elems + b * p.out_bstride;
    for (int k = threadIdx.x; k < p.len; k += kBlock) {
        double2 v = lds[k];
        // exp(-+ 2 pi i b k / M) = exp(-+ i pi (2 b k mod 2M) / M)
        if (p.twiddle) v = cmul(v, phasor_pi((2 * b * k) % (2 * p.M), p.M, p.inverse ? 1.0 : -1.0));
        dst[(int64_t)k * p.out_stride] = v;
    }
}

// Bluestein: A[r] *= FFT(b) / M (both in the four-step's [k1][k2] order)
__global__ __launch_bounds__(kBlock) void k_lf_mul(LongNoiseArgs a, double2 *A, const double2 *Bf) {
    const int64_t r = blockIdx.y;
    const double s = 1.0 / (double)a.M;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < a.M; i += (int64_t)gridDim.x * kBlock)
        A[r * a.M + i] = cscale(cmul(A[r * a.M + i], Bf[i]), s);
}

// block partials of sum_{k >= kc} |F_k|^2 / nbin, F the real row's rFFT
__global__ __launch_bounds__(kBlock) void k_lf_pow(LongNoiseArgs a, const double2 *A, double *part) {
    __shared__ double red[kWaves];
    const int64_t r = blockIdx.y;
    const double2 *Z = A + r * a.M;
    // the complex transform's bin k (k = n wraps to 0)
    auto zk = [&](int64_t k) -> double2 {
        if (k >= a.n) k -= a.n;
        if (a.bluestein) return cmul(Z[k], chirp(k, a.n));
        return Z[(k & (a.M1 - 1)) * a.M2 + (k >> a.log2M1)];   // X[k1 + M1 k2] at k1 M2 + k2
    };
    double acc[1] = {0.0};
    for (int64_t k = a.kc + (int64_t)blockIdx.x * kBlock + threadIdx.x; k < a.nharm;
         k += (int64_t)gridDim.x * kBlock) {
        double2 F;
        if (a.packed) {
            // F_k = (Z_k + conj Z_{n-k}) / 2 - i e^{-2 pi i k / nbin} (Z_k - conj Z_{n-k}) / 2
            const double2 z1 = zk(k), z2 = cconj(zk(a.n - k));
            const double2 e = cscale(cadd(z1, z2), 0.5), o = cscale(csub(z1, z2), 0.5);
            const double2 w = phasor_pi(2 * k, a.nbin, -1.0);
            const double2 wo = cmul(w, o);
            F = cmk(e.x + wo.y, e.y - wo.x);
        } else {
            F = zk(k);
        }
        acc[0] += (F.x * F.x + F.y * F.y) / (double)a.nbin;
    }
    block_sum<1>(acc, red);
    if (threadIdx.x == 0) part[r * gridDim.x + blockIdx.x] = acc[0];
}

__global__ __launch_bounds__(kBlock) void k_lf_fin(LongNoiseArgs a, const double *part, int nblk, double *out) {
    __shared__ double red[kWaves];
    const int64_t r = blockIdx.x;
    double acc[1] = {0.0};
    for (int i = threadIdx.x; i < nblk; i += kBlock) acc[0] += part[r * nblk + i];
    block_sum<1>(acc, red);
    if (threadIdx.x == 0) out[a.row0 + r] = sqrt(acc[0] / (double)(a.nharm - a.kc));
}

int lf_pow_blocks(const LongNoiseArgs &a) {
    const int64_t span = a.nharm - a.kc;
    const int64_t b = (span + kBlock - 1) / kBlock;
    return (int)(b < 1 ? 1 : (b > 256 ? 256 : b));
}

static unsigned stride_blocks(int64_t n) {
    const int64_t b = (n + kBlock - 1) / kBlock;
    return (unsigned)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

// the four-step of the rows [0, nrows) of X (in place through Y)
static hipError_t four_step(const LongNoiseArgs &a, int64_t nrows, double2 *X, double2 *Y, bool inverse,
                            const double2 *T1, const double2 *T2, hipStream_t st) {
    LongPassArgs c{};     // P1 / I2: columns (length M1, batch n2 = 0..M2)
    c.nbatch = a.M2; c.len = (int)a.M1; c.log2len = a.log2M1;
    c.in_stride = a.M2; c.in_bstride = 1; c.out_stride = a.M2; c.out_bstride = 1;
    c.row_elems = a.M; c.M = a.M; c.T = T1; c.inverse = inverse ? 1 : 0;
    LongPassArgs w{};     // P2 / I1: rows (length M2, batch k1 = 0..M1)
    w.nbatch = a.M1; w.len = (int)a.M2; w.log2len = (int)(a.log2M - a.log2M1);
    w.in_stride = 1; w.in_bstride = a.M2; w.out_stride = 1; w.out_bstride = a.M2;
    w.row_elems = a.M; w.M = a.M; w.T = T2; w.inverse = inverse ? 1 : 0;
    if (!inverse) {
        c.twiddle = 1; c.in = X; c.out = Y;
        w.twiddle = 0; w.in = Y; w.out = X;
    } else {
        w.twiddle = 1; w.in = X; w.out = Y;
        c.twiddle = 0; c.in = Y; c.out = X;
    }
    const LongPassArgs first = inverse ? w : c, second = inverse ? c : w;
    for (const LongPassArgs &p : {first, second}) {
        hipLaunchKernelGGL(k_lf_pass, dim3((unsigned)p.nbatch, (unsigned)nrows), dim3(kBlock),
                           sizeof(double2) * (size_t)p.len, st, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_chirp_ft(const LongNoiseArgs &a, double2 *Bf, double2 *Bs, const double2 *T1,
                           const double2 *T2, hipStream_t st) {
    hipLaunchKernelGGL(k_lf_chirp, dim3(stride_blocks(a.M)), dim3(kBlock), 0, st, a, Bf);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return four_step(a, 1, Bf, Bs, false, T1, T2, st);
}

hipError_t launch_noise_long(const LongNoiseArgs &a, int64_t nrows, double2 *A, double2 *Y,
                             const double2 *Bf, double *part, double *out, const double2 *T1,
                             const double2 *T2, hipStream_t st) {
    hipError_t e;
    hipLaunchKernelGGL(k_lf_load, dim3(stride_blocks(a.M), (unsigned)nrows), dim3(kBlock), 0, st, a, A);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = four_step(a, nrows, A, Y, false, T1, T2, st)) != hipSuccess) return e;
    if (a.bluestein) {
        hipLaunchKernelGGL(k_lf_mul, dim3(stride_blocks(a.M), (unsigned)nrows), dim3(kBlock), 0, st, a, A, Bf);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = four_step(a, nrows, A, Y, true, T1, T2, st)) != hipSuccess) return e;
    }
    const int nb = lf_pow_blocks(a);
    hipLaunchKernelGGL(k_lf_pow, dim3((unsigned)nb, (unsigned)nrows), dim3(kBlock), 0, st, a, A, part);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_lf_fin, dim3((unsigned)nrows), dim3(kBlock), 0, st, a, part, nb, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Rotation of rows of any length (ppf_rotate_long, round 6): rotate_data's
// irfft(rfft(x) e^{2 pi i k phi}) (pplib.py:2427-2515) where the block
// kernels' LDS transforms do not reach.  Both transforms are Bluestein's
// (natural order in and out, any length): the forward one on the packed /
// odd row as in ppf_noise_long, the inverse as conj(DFT(conj Y)) of the
// spectrum repacked for a real output -- even output length L = 2 No:
// Y_j = E_j + i O_j, E_j = (R_j + conj R_{No-j}) / 2, O_j = e^{2 pi i j / L}
// (R_j - conj R_{No-j}) / 2, so IDFT_No(Y)_j = x_2j + i x_2j+1; odd L = nbin:
// the Hermitian fill R_j, conj R_{L-j}.  R = X e^{2 pi i k phi} with the
// imaginary parts irfft ignores (R_0, and R_No at even L) dropped.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_lr_mid(LongRotArgs r, const double2 *Yf, double2 *A2) {
    const int64_t row = blockIdx.y;
    const LongNoiseArgs &f = r.f, &b = r.b;
    const double2 *Z = Yf + row * f.M;
    const double phi = r.phases ? r.phases[f.row0 + row] : 0.0;
    const double tn = r.taus ? r.taus[f.row0 + row] : 0.0;
    auto zk = [&](int64_t k) -> double2 {
        if (k >= f.n) k -= f.n;
        return cmul(Z[k], chirp(k, f.n));
    };
    // the rotated spectrum R_k, 0 <= k <= nbin / 2
    auto Rk = [&](int64_t k) -> double2 {
        double2 X;
        if (f.packed) {
            const double2 z1 = zk(k), z2 = cconj(zk(f.n - k));
            const double2 e = cscale(cadd(z1, z2), 0.5), o = cscale(csub(z1, z2), 0.5);
            const double2 wo = cmul(phasor_pi(2 * k, f.nbin, -1.0), o);
            X = cmk(e.x + wo.y, e.y - wo.x);
        } else {
            X = zk(k);
        }
        double2 R = r.phases ? cmul(X, cexp2pi((double)k * phi)) : X;
        if (tn != 0.0) R = cmul(R, scat_recip((2.0 * kPi * (double)k) * tn));
        if (k == 0 || (r.out_even && k == b.n)) R.y = 0.0;
        return R;
    };
    double2 *out = A2 + row * b.M;
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < b.M; j += (int64_t)gridDim.x * kBlock) {
        double2 y = cmk(0.0, 0.0);
        if (j < b.n) {
            double2 Y;
            if (r.out_even) {
                const double2 r1 = Rk(j), r2 = cconj(Rk(b.n - j));
                const double2 E = cscale(cadd(r1, r2), 0.5);
                const double2 O = cmul(phasor_pi(2 * j, 2 * b.n, 1.0), cscale(csub(r1, r2), 0.5));
                Y = cmk(E.x - O.y, E.y + O.x);            // E + i O
            } else {
                const int64_t N = b.n / 2;                  // odd L = b.n: k <= N stored
                Y = j <= N ? Rk(j) : cconj(Rk(b.n - j));
            }
            // inverse DFT as conj(DFT(conj Y)): Bluestein input conj(Y) w_j
            y = cmul(cconj(Y), chirp(j, b.n));
        }
        out[j] = y;
    }
}

__global__ __launch_bounds__(kBlock) void k_lr_out(LongRotArgs r, const double2 *Yb) {
    const int64_t row = blockIdx.y;
    const LongNoiseArgs &b = r.b;
    const double2 *Y = Yb + row * b.M;
    double *out = r.out + (r.b.row0 + row) * r.nout;
    const double s = 1.0 / (double)b.n;
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < b.n; j += (int64_t)gridDim.x * kBlock) {
        // IDFT(Y)_j = conj(w_j y_j) / n
        const double2 v = cscale(cconj(cmul(Y[j], chirp(j, b.n))), s);
        if (r.out_even) {
            out[2 * j] = v.x;
            out[2 * j + 1] = v.y;
        } else {
            out[j] = v.x;
        }
    }
}

// rFFT bins X_k, k < nbin / 2 + 1, of rows transformed by the forward
// Bluestein plan f (natural-order y in Yf) -> out[row0 + row][k] (the fit's
// long-row spectra: model rows for Mft, data rows for k_xspec_spec)
__global__ __launch_bounds__(kBlock) void k_lr_spec(LongNoiseArgs f, const double2 *Yf, double2 *out) {
    const int64_t row = blockIdx.y;
    const double2 *Z = Yf + row * f.M;
    const int64_t nharm = f.nbin / 2 + 1;
    auto zk = [&](int64_t k) -> double2 {
        if (k >= f.n) k -= f.n;
        return cmul(Z[k], chirp(k, f.n));
    };
    double2 *o = out + (f.row0 + row) * nharm;
    for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < nharm; k += (int64_t)gridDim.x * kBlock) {
        if (f.packed) {
            const double2 z1 = zk(k), z2 = cconj(zk(f.n - k));
            const double2 e = cscale(cadd(z1, z2), 0.5), q = cscale(csub(z1, z2), 0.5);
            const double2 wo = cmul(phasor_pi(2 * k, f.nbin, -1.0), q);
            o[k] = cmk(e.x + wo.y, e.y - wo.x);
        } else {
            o[k] = zk(k);
        }
    }
}

hipError_t launch_rfft_long(const LongNoiseArgs &f, int64_t nrows, double2 *A, double2 *Y, const double2 *Bf,
                            double2 *out, const double2 *T1, const double2 *T2, hipStream_t st) {
    hipError_t e;
    hipLaunchKernelGGL(k_lf_load, dim3(stride_blocks(f.M), (unsigned)nrows), dim3(kBlock), 0, st, f, A);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = four_step(f, nrows, A, Y, false, T1, T2, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_lf_mul, dim3(stride_blocks(f.M), (unsigned)nrows), dim3(kBlock), 0, st, f, A, Bf);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = four_step(f, nrows, A, Y, true, T1, T2, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_lr_spec, dim3(stride_blocks(f.nbin / 2 + 1), (unsigned)nrows), dim3(kBlock), 0, st, f,
                       A, out);
    return hipGetLastError();
}

hipError_t launch_rotate_long(const LongRotArgs &r, int64_t nrows, double2 *A, double2 *Y, const double2 *Bff,
                              const double2 *Bfb, const double2 *T1f, const double2 *T2f, const double2 *T1b,
                              const double2 *T2b, hipStream_t st) {
    hipError_t e;
    const LongNoiseArgs &f = r.f, &b = r.b;
    // forward: chirped row -> DFT_n in natural order (in A)
    hipLaunchKernelGGL(k_lf_load, dim3(stride_blocks(f.M), (unsigned)nrows), dim3(kBlock), 0, st, f, A);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = four_step(f, nrows, A, Y, false, T1f, T2f, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_lf_mul, dim3(stride_blocks(f.M), (unsigned)nrows), dim3(kBlock), 0, st, f, A, Bff);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = four_step(f, nrows, A, Y, true, T1f, T2f, st)) != hipSuccess) return e;
    // rotate, repack, chirp for the inverse (into Y, row stride b.M)
    hipLaunchKernelGGL(k_lr_mid, dim3(stride_blocks(b.M), (unsigned)nrows), dim3(kBlock), 0, st, r, A, Y);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = four_step(b, nrows, Y, A, false, T1b, T2b, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_lf_mul, dim3(stride_blocks(b.M), (unsigned)nrows), dim3(kBlock), 0, st, b, Y, Bfb);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = four_step(b, nrows, Y, A, true, T1b, T2b, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_lr_out, dim3(stride_blocks(b.n), (unsigned)nrows), dim3(kBlock), 0, st, r, Y);
    return hipGetLastError();
}

}  // namespace ppf
