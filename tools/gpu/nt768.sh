# 768-thread variant of k_fused_iteration (FPM_FUSED_NT=768): parity vs the
# 512-thread kernel, then the metric bench, for two builds (P / F parked, or
# held in registers with spills)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/nt768
mkdir -p $O
cat > $O/chk.py <<'PY'
import os, sys, numpy as np
import torch  # its HIP runtime first (tests/conftest.py)
import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack
Np, L, r, B = 256, 512, 33, 4
x0, y0, order = grid_geometry(Np, L, 5, 20)
stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=3)
prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=B, path=fpm_amd.PATH_FUSED)
outs = []
for nt in ("512", "768"):
    os.environ["FPM_FUSED_NT"] = nt
    with fpm_amd.Solver(prob) as s:
        s.upload(stack); s.init(); s.run(2); outs.append(s.download())
for k in ("objF", "objCrop", "pupil"):
    print(k, max(rel_l2(outs[1][k][b], outs[0][k][b]) for b in range(B)), np.array_equal(outs[1][k], outs[0][k]))
PY
for V in park768 nopark768; do
  export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so
  echo "== $V"
  PYTHONPATH=fpm-opencv_amd/python:oracle:tests:. timeout -k 10 120 python $O/chk.py 2>&1 | tail -4 || exit 1
done
for i in 1 2; do
  for V in default park768 nopark768; do
    if [ $V = default ]; then unset FPM_HIP_LIB; NT=512; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; NT=768; fi
    FPM_FUSED_NT=$NT timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/$V$i.json 2> $O/$V$i.err || { echo "$V rc=$?"; tail -3 $O/$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$V$i.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['config'].get('kernel'))"
  done
done
