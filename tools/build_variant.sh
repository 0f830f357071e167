#!/bin/bash
# Build an A/B variant of libfpm_hip.so with extra compiler flags into
# fpm-opencv_amd/lib_var/NAME/ (load it with FPM_HIP_LIB=<path>).
#   bash tools/build_variant.sh NAME "<extra hipcc flags>"
set -e
NAME=$1; shift
EXTRA="$*"
cd "$(dirname "$0")/../fpm-opencv_amd"
OUT=lib_var/$NAME
mkdir -p $OUT/obj
F="--offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -fPIC -Wall -Wno-unused-result -I../include $EXTRA"
pids=()
for s in $(cd csrc && ls *.hip | sed "s/\.hip$//"); do
  /opt/rocm/bin/hipcc $F -c csrc/$s.hip -o $OUT/obj/$s.o & pids+=($!)
done
/opt/rocm/bin/hipcc $F -x hip -c csrc/api.cpp -o $OUT/obj/api.o & pids+=($!)
for p in ${pids[@]}; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libfpm_hip.so $OUT/obj/*.o
rm -rf $OUT/obj
echo "built $OUT/libfpm_hip.so"
