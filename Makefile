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

all: $(LIBDIR)/liborbgpu.so oracle

build/obj/%.o: $(SRC)/%.hip $(DEPS)
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/liborbgpu.so: $(HIP_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIP_OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIBDIR) oracle/_build
.PHONY: all oracle clean
