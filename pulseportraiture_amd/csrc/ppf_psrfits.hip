// ppf_psrfits.hip -- device side of the PSRCHIVE-free PSRFITS fast path
// (pulseportraiture_amd/psrfits.py): the raw DATA bytes of
// a fold-mode SUBINT table arrive as they sit in the file and are turned
// into the float32 total-intensity rows load_data would hand get_TOAs
// (pplib.py:2749-2915 with pscrunch=True, rm_baseline=True), plus the
// per-profile baseline statistics and S/N.
//
//   k_unpack      WG = (sub-int, block of kUnpackChans channels), thread =
//                 bin pairs: big-endian int16 / uint8 / float32 samples (or
//                 native float32 rows: load_data's statistics pass after
//                 dedispersion / tscrunch, DAT_SCL = 1, DAT_OFFS = 0) ->
//                 DATA * DAT_SCL + DAT_OFFS in float32 arithmetic (two
//                 roundings, no fma: PSRCHIVE's loader) -> total intensity
//                 (npol 1: itself; AA+BB / AABBCRCI: AA + BB; IQUV: I) ->
//                 rows [nsub][nchan][nbin]; the weighted channel sum of the
//                 block (fixed channel order) -> partials [nsub][nblk][nbin]
//   k_base_window WG per sub-int: total profile = sum of the partials in
//                 block order; PSRCHIVE's BaselineWindow: the circular window
//                 of W = rint(0.15 nbin) bins with the smallest sum (first
//                 minimum) -> window start, total profile out
//   k_row_stats   wave per row: off-pulse mean over the window (subtracted
//                 from the row in place when rm_baseline), off-pulse sigma,
//                 S/N = sum over the on-pulse bins / (sigma sqrt(n_on))
// All of it is HBM-streaming integer/byte work (no MFMA): a few bytes per
// sample against the 2 B per sample that crossed PCIe.
#include "ppf_device.hpp"
#include "ppf_internal.hpp"

namespace ppf {

constexpr int kUnpackChans = 16;

__device__ __forceinline__ float sample_f32(const uint8_t *p, int elem, int64_t i) {
    if (elem == 0) {
        const uint16_t u = reinterpret_cast<const uint16_t *>(p)[i];
        return (float)(int16_t)__builtin_bswap16(u);
    }
    if (elem == 1) return (float)p[i];
    if (elem == 3) return reinterpret_cast<const float *>(p)[i];   // native rows
    const uint32_t u = __builtin_bswap32(reinterpret_cast<const uint32_t *>(p)[i]);
    return __uint_as_float(u);
}

__global__ __launch_bounds__(256) void k_unpack(UnpackArgs a) {
    // DATA * DAT_SCL + DAT_OFFS rounds twice, as PSRCHIVE's (and NumPy's)
    // float32 arithmetic does: the product is pinned in a register before
    // the add, so the compiler cannot fuse them (-ffp-contract=fast)
    const int nblk = (a.nchan + kUnpackChans - 1) / kUnpackChans;
    const int s = blockIdx.x / nblk, blk = blockIdx.x % nblk;
    const uint8_t *raw = a.raw + (int64_t)s * a.sub_stride;
    const float *scl = a.scl + (int64_t)s * a.npol * a.nchan;
    const float *off = a.offs + (int64_t)s * a.npol * a.nchan;
    const int n0 = blk * kUnpackChans, n1 = min(a.nchan, n0 + kUnpackChans);
    const int npol_used = a.pol_mode == 1 ? 2 : 1;
    for (int b = threadIdx.x; b < a.nbin; b += blockDim.x) {
        double part = 0.0;
        for (int n = n0; n < n1; ++n) {
            float v = 0.0f;
            for (int p = 0; p < npol_used; ++p) {
                const int64_t i = ((int64_t)p * a.nchan + n) * a.nbin + b;
                float prod = sample_f32(raw, a.elem, i) * scl[p * a.nchan + n];
                asm volatile("" : "+v"(prod));      // rounded product: no fma
                const float x = prod + off[p * a.nchan + n];
                v = p == 0 ? x : v + x;
            }
            a.out[((int64_t)s * a.nchan + n) * a.nbin + b] = v;
            const double w = a.wts ? (double)a.wts[(int64_t)s * a.nchan + n] : 1.0;
            if (w != 0.0) part += w * (double)v;
        }
        a.part[((int64_t)s * nblk + blk) * a.nbin + b] = part;
    }
}

__global__ __launch_bounds__(256) void k_base_window(UnpackArgs a) {
    extern __shared__ double tot[];
    const int s = blockIdx.x;
    const int nblk = (a.nchan + kUnpackChans - 1) / kUnpackChans;
    for (int b = threadIdx.x; b < a.nbin; b += blockDim.x) {
        double t = 0.0;
        for (int k = 0; k < nblk; ++k) t += a.part[((int64_t)s * nblk + k) * a.nbin + b];
        tot[b] = t;
        a.total[(int64_t)s * a.nbin + b] = t;
    }
    __syncthreads();
    // window sums by thread: each thread scans its share of start bins with
    // a direct sum for its first start and a sliding update after that;
    // the per-thread minima are then reduced in start order (first minimum)
    const int W = a.win;
    const int per = (a.nbin + blockDim.x - 1) / blockDim.x;
    const int b0 = threadIdx.x * per, b1 = min(a.nbin, b0 + per);
    double best = INFINITY;
    int bi = a.nbin;
    if (b0 < b1) {
        double w = 0.0;
        for (int j = 0; j < W; ++j) w += tot[(b0 + j) % a.nbin];
        for (int b = b0; b < b1; ++b) {
            if (b > b0) w += tot[(b - 1 + W) % a.nbin] - tot[b - 1];
            if (w < best) { best = w; bi = b; }
        }
    }
    __shared__ double rb[256];
    __shared__ int ri[256];
    rb[threadIdx.x] = best;
    ri[threadIdx.x] = bi;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = rb[0];
        int mi = ri[0];
        for (int t = 1; t < (int)blockDim.x; ++t)
            if (rb[t] < m) { m = rb[t]; mi = ri[t]; }
        a.wstart[s] = mi < a.nbin ? mi : 0;
    }
}

__global__ __launch_bounds__(256) void k_row_stats(UnpackArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= (int64_t)a.nsub * a.nchan) return;
    const int s = (int)(row / a.nchan);
    float *x = a.out + row * a.nbin;
    const int w0 = a.wstart[s], W = a.win;
    double sm = 0.0;
    for (int j = lane; j < W; j += 64) sm += (double)x[(w0 + j) % a.nbin];
    const double mean = wave_sum(sm) / (double)W;
    double sq = 0.0;
    for (int j = lane; j < W; j += 64) {
        const double d = (double)x[(w0 + j) % a.nbin] - mean;
        sq += d * d;
    }
    const double var = wave_sum(sq) / (double)W;
    double on = 0.0;
    for (int b = lane; b < a.nbin; b += 64) {
        const int rel = (b - w0 + a.nbin) % a.nbin;
        const double v = (double)x[b] - mean;
        if (rel >= W) on += v;
        if (a.rm_baseline) x[b] = (float)v;
    }
    on = wave_sum(on);
    const int non = a.nbin - W;
    if (lane == 0) {
        double *o = a.stats + row * 3;
        o[0] = mean;
        o[1] = sqrt(var);
        o[2] = (var > 0.0 && non > 0) ? on / (sqrt(var) * sqrt((double)non)) : 0.0;
    }
}

hipError_t launch_unpack(const UnpackArgs &a, hipStream_t st) {
    const int nblk = (a.nchan + kUnpackChans - 1) / kUnpackChans;
    hipLaunchKernelGGL(k_unpack, dim3((unsigned)((int64_t)a.nsub * nblk)), dim3(256), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_base_window, dim3((unsigned)a.nsub), dim3(256), (size_t)a.nbin * sizeof(double),
                       st, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int64_t rows = (int64_t)a.nsub * a.nchan;
    hipLaunchKernelGGL(k_row_stats, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, a);
    return hipGetLastError();
}

// Device-side copy out of page-locked host memory (zero-copy reads over
// PCIe by the CUs): the fit inputs' staging buffer reaches HBM without a
// copy-engine transfer, so it never queues behind an archive upload.
__global__ __launch_bounds__(256) void k_copy_host(const uint4 *__restrict__ src,
                                                   uint4 *__restrict__ dst, int64_t n16) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        dst[i] = src[i];
}

__global__ __launch_bounds__(64) void k_copy_host_tail(const uint8_t *__restrict__ src,
                                                       uint8_t *__restrict__ dst, int64_t n) {
    const int64_t i = threadIdx.x;
    if (i < n) dst[i] = src[i];
}

hipError_t launch_copy_host(const void *src_dev, void *dst, int64_t nbytes, hipStream_t st) {
    const int64_t n16 = nbytes / 16, tail = nbytes - n16 * 16;
    if (n16 > 0) {
        const int64_t want = (n16 + 255) / 256;
        const unsigned grid = (unsigned)(want < 1024 ? want : 1024);
        hipLaunchKernelGGL(k_copy_host, dim3(grid), dim3(256), 0, st, (const uint4 *)src_dev,
                           (uint4 *)dst, n16);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (tail > 0) {
        hipLaunchKernelGGL(k_copy_host_tail, dim3(1), dim3(64), 0, st,
                           (const uint8_t *)src_dev + n16 * 16, (uint8_t *)dst + n16 * 16, tail);
        return hipGetLastError();
    }
    return hipSuccess;
}

size_t unpack_partials(int nsub, int nchan, int nbin) {
    return (size_t)nsub * ((nchan + kUnpackChans - 1) / kUnpackChans) * nbin;
}

}  // namespace ppf
