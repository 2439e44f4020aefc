// Host file I/O of the PSRFITS fast path: the DATA column read straight into
// the page-locked upload buffer by native threads (include/ppfit.h,
// ppf_read_rows).  The Python loader issued one positioned read per row from
// a thread pool; every row re-took the interpreter lock, so under the GetTOAs
// pipeline (fit worker, bookkeeping and loader threads all in Python) the
// 134 MB read of a 64 x 512 x 2048 archive stretched from 2.0 to 3-4 ms.
#include <unistd.h>
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstring>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/ppfit.h"

extern "C" int ppf_read_rows(int32_t fd, int64_t offset, int64_t row_stride, int64_t nbytes,
                             int64_t nrows, void *dst, int64_t dst_stride, int32_t nthreads) {
    if (fd < 0 || offset < 0 || nbytes < 0 || nrows < 0 || (nrows > 0 && nbytes > 0 && !dst) ||
        row_stride < nbytes || dst_stride < nbytes || nthreads < 1 || nthreads > 64)
        return PPF_EINVAL;
    if (nrows == 0 || nbytes == 0) return PPF_OK;
    const int64_t piece = 4ll << 20;
    const int64_t per_row = (nbytes + piece - 1) / piece;
    const int64_t npieces = per_row * nrows;
    std::atomic<int64_t> next{0};
    std::atomic<int> failed{0};
    auto work = [&]() {
        for (;;) {
            const int64_t i = next.fetch_add(1, std::memory_order_relaxed);
            if (i >= npieces || failed.load(std::memory_order_relaxed)) return;
            const int64_t r = i / per_row, p = i % per_row;
            const int64_t b0 = p * piece, b1 = std::min(nbytes, b0 + piece);
            char *out = (char *)dst + r * dst_stride;
            int64_t done = b0;
            while (done < b1) {
                const ssize_t k = pread(fd, out + done, (size_t)(b1 - done),
                                        (off_t)(offset + r * row_stride + done));
                if (k < 0 && errno == EINTR) continue;
                if (k <= 0) {
                    failed.store(1);
                    return;
                }
                done += k;
            }
        }
    };
    const int nt = (int)std::min<int64_t>(nthreads, npieces);
    std::vector<std::thread> pool;
    // no exception may cross the C ABI: a thread that cannot be started
    // (thread limit, memory) leaves its pieces to the threads that did
    // start (they all take pieces from the shared counter), the calling
    // thread included
    try {
        pool.reserve(nt > 0 ? nt - 1 : 0);
        for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    } catch (const std::exception &) {
    }
    work();
    for (auto &th : pool) th.join();
    return failed.load() ? PPF_EIO : PPF_OK;
}

// Parallel host memcpy (the pageable -> page-locked staging copy of
// GetTOAs' in-memory archives, pptoas._Stager): nbytes from src to dst in
// 4-MiB pieces taken in turn by nthreads threads (1..64), outside the
// interpreter lock.  Host memory only; no device, no context.
extern "C" int ppf_host_copy(void *dst, const void *src, int64_t nbytes, int32_t nthreads) {
    if (nbytes < 0 || (nbytes > 0 && (!dst || !src)) || nthreads < 1 || nthreads > 64)
        return PPF_EINVAL;
    if (nbytes == 0) return PPF_OK;
    const int64_t piece = 4ll << 20;
    const int64_t npieces = (nbytes + piece - 1) / piece;
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        for (;;) {
            const int64_t i = next.fetch_add(1, std::memory_order_relaxed);
            if (i >= npieces) return;
            const int64_t b0 = i * piece, b1 = std::min(nbytes, b0 + piece);
            std::memcpy((char *)dst + b0, (const char *)src + b0, (size_t)(b1 - b0));
        }
    };
    const int nt = (int)std::min<int64_t>(nthreads, npieces);
    std::vector<std::thread> pool;
    try {
        pool.reserve(nt > 0 ? nt - 1 : 0);
        for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    } catch (const std::exception &) {
    }
    work();
    for (auto &th : pool) th.join();
    return PPF_OK;
}
