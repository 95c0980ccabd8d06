# Build a variant of libsdr_amd.so with extra flags into build/variants/<name>.so, for A/B timing
# through SDR_AMD_LIB=<path> (tools/gpu/*.sh); per-file flags as in the Makefile.
#   bash tools/build_variant.sh <name> -DFOO=1 ...
#   PLLFLAGS="-mllvm ..." bash tools/build_variant.sh <name>    (flags for sdr_pll.hip only;
#   FEFLAGS for sdr_frontend.hip, KFLAGS for sdr_kernels.hip)
set -e
name=$1; shift
d=build/variants/$name.obj
mkdir -p $d
common="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -mllvm -pragma-unroll-threshold=1000000 -Iinclude"
pids=""
for f in sdr_kernels.hip sdr_frontend.hip sdr_pll.hip sdr_taps.cpp; do
  extra=""
  case $f in
    sdr_kernels.hip) extra="-fno-slp-vectorize ${KFLAGS:-}";;
    sdr_frontend.hip) extra="${FEFLAGS:-}";;
    sdr_pll.hip) extra="-fno-slp-vectorize ${PLLFLAGS--mllvm -amdgpu-sched-strategy=max-ilp}";;
  esac
  /opt/rocm/bin/hipcc $common $extra "$@" -c -o $d/$f.o ${SRC:-real-time-sdr_amd/csrc}/$f & pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -Wl,-soname,libsdr_amd.so -o build/variants/$name.so $d/*.o
rm -rf $d
echo build/variants/$name.so
