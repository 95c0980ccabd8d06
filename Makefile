# Build everything in-tree (the .so files travel to the GPU box with the snapshot).
#   make            libsdr_amd.so (HIP, gfx950) + oracle/liboracle.so (+ oracle/_ref when the
#                   reference tree is present in this container)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := real-time-sdr_amd
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
            -mllvm -pragma-unroll-threshold=1000000 \
            -Wall -Iinclude
LIB      := $(PKG)/libsdr_amd.so
SRCS     := $(PKG)/csrc/sdr_kernels.hip $(PKG)/csrc/sdr_taps.cpp
HDRS     := include/sdr_amd.h

.PHONY: all lib oracle clean
all: lib oracle

lib: $(LIB)

$(LIB): $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(LIB)
	$(MAKE) -C oracle clean
