#!/bin/bash
# Host sanitizer run: the CPU tests that
# call into libppfit's host code -- the C-ABI exports and struct layouts,
# workspace sizing and descriptor validation, the host root finder and
# trust-region subproblem, the native PSRFITS reader (ppf_read_rows: up to 64
# pread threads writing into caller buffers) -- against the library built
# with AddressSanitizer + UndefinedBehaviorSanitizer on its host code
# (`make asan`).  Python itself is not instrumented, so clang's ASan runtime
# is preloaded; leak checking is off (the interpreter and the HIP runtime
# keep allocations to exit).  usage: tools/asan_tests.sh [LOG]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
make -s asan || exit 1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
LOG=${1:-profiles/r05/asan_cpu_tests.log}
mkdir -p "$(dirname "$LOG")"
{
  echo "# $(date -u +%FT%TZ) libppfit host code under ASan+UBSan ($RT)"
  LD_PRELOAD="$RT" PPFIT_LIB="$PWD/pulseportraiture_amd/lib/asan/libppfit.so" \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:print_summary=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    python -m pytest -q -m "not gpu" -p no:cacheprovider tests/test_abi.py tests/test_psrfits.py 2>&1
} | tee "$LOG"
rc=$?
# the sanitizer is live: a deliberate overflow (ppf_read_rows told to write
# 2 rows into a 1-row numpy buffer) must be caught and reported
{
  echo "# expected-failure check: ppf_read_rows overflowing its destination"
  out=$(ASAN_OPTIONS=detect_leaks=0 LD_PRELOAD="$RT" \
        PPFIT_LIB="$PWD/pulseportraiture_amd/lib/asan/libppfit.so" python - 2>&1 <<'PY'
import ctypes, os, tempfile
import numpy as np
from pulseportraiture_amd import _lib
lib = _lib.load()
assert "asan" in lib._name
fd, fn = tempfile.mkstemp()
os.write(fd, b"x" * 8192)
dst = np.zeros(4096, dtype=np.uint8)
lib.ppf_read_rows(fd, 0, 4096, 4096, 2, dst.ctypes.data, 4096, 1)
PY
)
  echo "$out" | grep -m1 -E "ERROR: AddressSanitizer: [a-z-]+" || { echo "NOT CAUGHT"; exit 1; }
} | tee -a "$LOG"
exit $((rc || $?))
