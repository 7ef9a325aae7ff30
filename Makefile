# Builds liborbgpu.so (HIP kernels + C ABI, gfx950) and the CPU oracle (test infrastructure).
#   make            -> orb-slam3_byzyh_amd/lib/liborbgpu.so + oracle/_build/liborb_oracle.so
# -ffp-contract=off everywhere: float results must match the reference's rounding exactly.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := orb-slam3_byzyh_amd
SRC := $(PKG)/csrc
LIBDIR := $(PKG)/lib
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -I$(SRC) \
            -Wall -Wno-unused-function -Wno-sign-compare -Wno-unused-value -Wno-unused-result -Wno-pass-failed
HIP_SRCS := $(wildcard $(SRC)/*.hip)
HIP_OBJS := $(patsubst $(SRC)/%.hip,build/obj/%.o,$(HIP_SRCS))
DEPS := $(wildcard $(SRC)/*.h) $(wildcard $(SRC)/*.inc) include/orbgpu.h

all: $(LIBDIR)/liborbgpu.so oracle shims

build/obj/%.o: $(SRC)/%.hip $(DEPS)
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/liborbgpu.so: $(HIP_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIP_OBJS)

oracle:
	$(MAKE) -C oracle

oracle/_build/liborb_oracle.so: $(wildcard oracle/*.cpp) $(wildcard oracle/*.h)
	$(MAKE) -C oracle

# The C++ drop-in headers linked to the real library, each checked against the oracle on the GPU
# (tests/test_shims_gpu.py).  Test programs, built here so that the GPU box runs them without a build.
SHIM_BINS := build/tests/local_ba_shim_gpu build/tests/matcher_shim_gpu build/tests/cv_shim_gpu
SHIM_FLAGS := -O2 -std=c++17 -ffp-contract=off -pthread -Wall -Werror -Iinclude -Itests/native/mock_cv
SHIM_LIBS := -L$(LIBDIR) -lorbgpu -Loracle/_build -lorb_oracle \
             -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,'$$ORIGIN/../../oracle/_build'
shims: $(SHIM_BINS)

build/tests/%_gpu: tests/native/%_gpu.cpp $(wildcard include/*.h*) $(LIBDIR)/liborbgpu.so oracle/_build/liborb_oracle.so
	@mkdir -p build/tests
	g++ $(SHIM_FLAGS) $< -o $@ $(SHIM_LIBS)

clean:
	rm -rf build $(LIBDIR) oracle/_build
.PHONY: all oracle shims clean
