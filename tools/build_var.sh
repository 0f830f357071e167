#!/bin/bash
# build a variant of libfpm_hip.so with extra compile flags into
# fpm-opencv_amd/lib_<name>/ (same-box A/B runs load it via FPM_HIP_LIB)
#   tools/build_var.sh <name> "<HIPFLAGS_EXTRA>" [git ref: build that commit's sources]
#   MAKEVARS="MMC_FILES='np1024 objcrop'" tools/build_var.sh ...: extra make variables
set -e
name=$1; flags=$2; ref=$3
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=/tmp/fpm_var_$name
rm -rf $tmp && mkdir -p $tmp
cp -r $root/include $tmp/ && mkdir -p $tmp/fpm-opencv_amd $tmp/tests
if [ -n "$ref" ]; then
  (cd $root && git archive $ref fpm-opencv_amd/csrc fpm-opencv_amd/Makefile include) | tar -x -C $tmp
else
  cp -r $root/fpm-opencv_amd/csrc $root/fpm-opencv_amd/Makefile $tmp/fpm-opencv_amd/
fi
eval make -s -C $tmp/fpm-opencv_amd -j8 lib/libfpm_hip.so HIPFLAGS_EXTRA=\"$flags\" ${MAKEVARS:-}
mkdir -p $root/fpm-opencv_amd/lib_$name
cp $tmp/fpm-opencv_amd/lib/libfpm_hip.so $root/fpm-opencv_amd/lib_$name/
echo "built fpm-opencv_amd/lib_$name/libfpm_hip.so ($flags)"
