#!/bin/bash
# tools/build_variants.sh NAME "DEFINES" ... — builds librt_hip.so variants of the
# megakernel with extra -D flags into variants/NAME/ for A/B runs
# (select one with RTNW_LIB=variants/NAME/librt_hip.so; tools/ab.py).
# RT_SRC=path builds from another kernel source (e.g. a previous revision).
set -e
cd "$(dirname "$0")/../peter-shirley-ray-tracing-the-next-week_amd"
make -s librt_hip.so
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p ../variants/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc -Icsrc/host --offload-arch=gfx950 \
      -Icsrc/hip -munsafe-fp-atomics $defs -c "${RT_SRC:-csrc/hip/rt_kernel.hip}" -o ../variants/$name/rt_kernel.o \
      -Rpass-analysis=kernel-resource-usage 2> ../variants/$name/resource.txt
  grep -A8 "ILb0ELb0" ../variants/$name/resource.txt | grep -E "VGPRs:|Scratch" | sed "s/.*remark: */$name: /"
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../variants/$name/librt_hip.so ../variants/$name/rt_kernel.o \
      build/capi.o build/bvh.o build/flatten.o build/rtnw.o build/png.o build/dist.o -lz -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
