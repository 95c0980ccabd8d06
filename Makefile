# Build everything in-tree (the .so files travel to the GPU box with the snapshot).
#   make            libsdr_amd.so (HIP kernels + C ABI, gfx950), libsdr_host.so (the reference's
#                   C++ stage/primitive API over the C ABI), bin/sdr_project (the receiver CLI),
#                   bin/sdr_multi (the multi-channel receiver),
#                   oracle/liboracle.so (+ oracle/_ref when the reference tree is present here)
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ROCM     ?= /opt/rocm
ARCH     ?= gfx950
PKG      := real-time-sdr_amd
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
            -mllvm -pragma-unroll-threshold=1000000 \
            -Wall -Iinclude
LIB      := $(PKG)/libsdr_amd.so
SRCS     := $(PKG)/csrc/sdr_kernels.hip $(PKG)/csrc/sdr_frontend.hip $(PKG)/csrc/sdr_pll.hip $(PKG)/csrc/sdr_taps.cpp
OBJS     := $(patsubst $(PKG)/csrc/%,build/%.o,$(SRCS))
HDRS     := include/sdr_amd.h $(PKG)/csrc/pll_math.h $(PKG)/csrc/sdr_internal.h

# host C++ (no device code): compiled by the system g++ against the HIP runtime headers
HOSTFLAGS := -O2 -std=c++17 -fPIC -Wall -Wextra -pthread -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include \
             -Iinclude -Iinclude/dropin -I$(PKG)/host
HOSTLIB   := $(PKG)/libsdr_host.so
HOSTSRCS  := $(PKG)/host/dropin_primitives.cpp $(PKG)/host/dropin_stages.cpp $(PKG)/host/rds_frame.cpp \
             $(PKG)/host/sdr_multi_engine.cpp
HOSTHDRS  := $(wildcard include/dropin/*.h) $(PKG)/host/hip_util.h include/sdr_amd.h include/sdr_multi.h
CLI       := $(PKG)/bin/sdr_project
MULTI     := $(PKG)/bin/sdr_multi

.PHONY: all lib host oracle clean
all: lib host oracle

lib: $(LIB)
host: $(HOSTLIB) $(CLI) $(MULTI)

# one object per translation unit (compiled in parallel), linked into the shared library
# the stage kernels keep their f32 multiply-adds scalar (packed f32 runs at half rate): no SLP;
# the lane-pair PLL step is faster scalar too (packed-f32 results cost a wait state on gfx950,
# profiles/r03/ab_pll_split3.txt)
build/sdr_kernels.hip.o: HIPFLAGS += -fno-slp-vectorize
build/sdr_pll.hip.o: HIPFLAGS += -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-ilp
# (the lane-pair PLL step scheduled for ILP: 212.4 -> 210.4 shader cycles per step, profiles/r04/ab_sched.txt)

build/%.o: $(PKG)/csrc/% $(HDRS) Makefile
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -fPIC -shared -Wl,-soname,libsdr_amd.so -o $@ $(OBJS)

$(HOSTLIB): $(HOSTSRCS) $(HOSTHDRS) $(LIB)
	$(CXX) $(HOSTFLAGS) -shared -o $@ $(HOSTSRCS) -L$(PKG) -lsdr_amd -L$(ROCM)/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(ROCM)/lib

$(CLI): $(PKG)/host/sdr_project.cpp $(HOSTLIB)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -o $@ $< -L$(PKG) -lsdr_host -Wl,-rpath,'$$ORIGIN/..'

$(MULTI): $(PKG)/host/sdr_multi.cpp include/sdr_multi.h $(HOSTLIB)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -o $@ $< -L$(PKG) -lsdr_host -lsdr_amd -L$(ROCM)/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/..' -Wl,-rpath,$(ROCM)/lib

oracle: host
	$(MAKE) -C oracle

clean:
	rm -f $(LIB) $(HOSTLIB) $(CLI) $(MULTI)
	rm -rf build
	$(MAKE) -C oracle clean
