# Build libppfit.so (HIP, gfx950) in-tree.  `make -j8`; `make clean`.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := pulseportraiture_amd/csrc
OUT := pulseportraiture_amd/lib/libppfit.so
SRCS := $(CSRC)/ppf_kernels.hip $(CSRC)/ppf_longfft.hip $(CSRC)/ppf_xspec.hip $(CSRC)/ppf_solve.hip $(CSRC)/ppf_psrfits.hip $(CSRC)/ppf_api.cpp $(CSRC)/ppf_io.cpp
HDRS := $(CSRC)/ppf_device.hpp $(CSRC)/ppf_state.hpp $(CSRC)/ppf_wfft.hpp $(CSRC)/ppf_wfft2.hpp $(CSRC)/ppf_internal.hpp include/ppfit.h
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-pass-failed \
            -ffp-contract=fast -munsafe-fp-atomics

OBJS := $(CSRC)/ppf_kernels.o $(CSRC)/ppf_longfft.o $(CSRC)/ppf_xspec.o $(CSRC)/ppf_solve.o $(CSRC)/ppf_psrfits.o $(CSRC)/ppf_api.o $(CSRC)/ppf_io.o

all: $(OUT)

$(CSRC)/ppf_kernels.o: $(CSRC)/ppf_kernels.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/ppf_longfft.o: $(CSRC)/ppf_longfft.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/ppf_xspec.o: $(CSRC)/ppf_xspec.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/ppf_solve.o: $(CSRC)/ppf_solve.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/ppf_psrfits.o: $(CSRC)/ppf_psrfits.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/ppf_api.o: $(CSRC)/ppf_api.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

# host-only: the native DATA reader (no device code)
$(CSRC)/ppf_io.o: $(CSRC)/ppf_io.cpp include/ppfit.h
	$(HIPCC) -O2 -std=c++17 -fPIC -Wall -pthread -c $< -o $@

$(OUT): $(OBJS)
	@mkdir -p $(dir $(OUT))
	$(HIPCC) --offload-arch=$(ARCH) -shared -pthread -o $@ $(OBJS)

clean:
	rm -f $(OBJS) $(OUT)

.PHONY: all clean

# Host sanitizer build: the same library with its HOST code
# under AddressSanitizer + UndefinedBehaviorSanitizer (device code is not
# instrumented: GPU sanitizers are unavailable on the pool).  Run the CPU
# tests against it with tools/asan_tests.sh (LD_PRELOADs clang's runtime).
ASAN_DIR := pulseportraiture_amd/lib/asan
ASAN_OUT := $(ASAN_DIR)/libppfit.so
ASAN_HOST := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
             -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=undefined
ASAN_OBJS := $(patsubst $(CSRC)/%.o,$(ASAN_DIR)/%.o,$(OBJS))

asan: $(ASAN_OUT)

$(ASAN_DIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(HIPFLAGS) -O1 $(ASAN_HOST) -c $< -o $@

$(ASAN_DIR)/ppf_api.o: $(CSRC)/ppf_api.cpp $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(HIPFLAGS) -O1 $(ASAN_HOST) -x hip -c $< -o $@

$(ASAN_DIR)/ppf_io.o: $(CSRC)/ppf_io.cpp include/ppfit.h
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) -O1 -g -std=c++17 -fPIC -Wall -pthread -fsanitize=address,undefined \
	    -fno-omit-frame-pointer -fno-sanitize-recover=undefined -c $< -o $@

$(ASAN_OUT): $(ASAN_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -pthread -shared-libasan \
	    -fsanitize=address,undefined -o $@ $(ASAN_OBJS)

.PHONY: asan
