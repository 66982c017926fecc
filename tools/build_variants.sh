#!/bin/bash
# tools/build_variants.sh NAME "DEFINES" ... — builds librt_hip.so variants of the
# megakernel with extra -D flags into variants/NAME/ for A/B runs, in parallel
# (select one with RTNW_LIB=variants/NAME/librt_hip.so; tools/ab.py).
# RT_SRC=path builds from another kernel source (e.g. a previous revision).
set -e
cd "$(dirname "$0")/../peter-shirley-ray-tracing-the-next-week_amd"
make -s librt_hip.so
build_one() {
  local name=$1 defs=$2
  mkdir -p ../variants/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc -Icsrc/host --offload-arch=gfx950 \
      -Icsrc/hip -munsafe-fp-atomics -cuid=rt_kernel $defs -c "${RT_SRC:-csrc/hip/rt_kernel.hip}" -o ../variants/$name/rt_kernel.o \
      -Rpass-analysis=kernel-resource-usage 2> ../variants/$name/resource.txt
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../variants/$name/librt_hip.so ../variants/$name/rt_kernel.o \
      build/capi.o build/bvh.o build/flatten.o build/rtnw.o build/png.o build/dist.o -lz -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
}
pids=()
names=()
while [ $# -ge 2 ]; do
  build_one "$1" "$2" &
  pids+=($!); names+=("$1")
  shift 2
done
rc=0
for i in "${!pids[@]}"; do
  wait "${pids[$i]}" || { echo "variant ${names[$i]} failed"; rc=1; }
  grep -A8 "ILb0ELb0ELi2ELi16ELi1E" ../variants/${names[$i]}/resource.txt | grep -E "VGPRs:|Scratch" | sed "s/.*remark: */${names[$i]}: /"
done
exit $rc
