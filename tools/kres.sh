#!/bin/bash
# per-kernel register use of the fused kernels (compiler resource remarks):
#   tools/kres.sh [csrc dir]   -> kernel  VGPRs  VGPR-spill  SGPR-spill  occupancy
src=${1:-fpm-opencv_amd/csrc}
for f in ${KRES_FILES:-fpm_fused fused_dist fused_s90 fused_mr fused_small np1024}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -fPIC -I${src}/../../include -I$(dirname $0)/../include \
    -c $src/$f.hip -o /tmp/kres_$f.o --offload-device-only -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/{n=$NF=="";split($0,a,"Function Name: ");split(a[2],b," ");k=b[1]}
       /VGPRs:/&&!/Spill/{split($0,a,"VGPRs: ");split(a[2],b," ");v=b[1]}
       /SGPRs Spill:/{split($0,a,"Spill: ");split(a[2],b," ");ss=b[1]}
       /VGPRs Spill:/{split($0,a,"Spill: ");split(a[2],b," ");vs=b[1]}
       /Occupancy/{split($0,a,"]: ");split(a[2],b," ");o=b[1]}
       /LDS Size/{printf "%-60s vgpr %4s vspill %3s sspill %4s occ %s\n", k, v, vs, ss, o}'
done
