#!/bin/bash
# tools/build_variants.sh N... — builds librt_hip.so variants with
# __launch_bounds__(256, N) (N waves per SIMD) into variants/wN/ for A/B runs
# (select one with RTNW_LIB=variants/wN/librt_hip.so).
set -e
cd "$(dirname "$0")/../peter-shirley-ray-tracing-the-next-week_amd"
make -s librt_hip.so
for n in "$@"; do
  mkdir -p ../variants/w$n
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc -Icsrc/host --offload-arch=gfx950 \
      -munsafe-fp-atomics -DRT_WAVES_PER_SIMD=$n -c csrc/hip/rt_kernel.hip -o ../variants/w$n/rt_kernel.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../variants/w$n/librt_hip.so ../variants/w$n/rt_kernel.o \
      build/capi.o build/bvh.o build/flatten.o build/rtnw.o -Wl,-rpath,/opt/rocm/lib
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc -Icsrc/host --offload-arch=gfx950 \
      -DRT_WAVES_PER_SIMD=$n -c csrc/hip/rt_kernel.hip -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 \
      | grep -A8 "ILb0ELb0" | grep -E "VGPRs:|Scratch|Occupancy" | sed "s/^/w$n: /"
done
