# Build a variant of libsdr_amd.so with extra -D flags into build/variants/<name>.so, for A/B timing
# through SDR_AMD_LIB=<path> (tools/gpu/*.sh). Usage: bash tools/build_variant.sh <name> -DFOO=1 ...
set -e
name=$1; shift
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -mllvm -pragma-unroll-threshold=1000000 -Iinclude "$@" -shared -Wl,-soname,libsdr_amd.so \
  -o build/variants/$name.so real-time-sdr_amd/csrc/sdr_kernels.hip real-time-sdr_amd/csrc/sdr_frontend.hip \
  real-time-sdr_amd/csrc/sdr_pll.hip real-time-sdr_amd/csrc/sdr_taps.cpp
echo build/variants/$name.so
