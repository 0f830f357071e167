# tail pixels re-homed (in-tree) vs before (lib_var): bit-identical outputs, tests, metric A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tailre
mkdir -p $O
cat > $O/run.py <<'PY'
import sys, numpy as np
import torch
sys.path[:0] = ["fpm-opencv_amd/python", "oracle", "tests", "."]
import fpm_amd
from test_gpu_configs import _probe_geometry
p, x0, y0 = _probe_geometry("geometry_dogStomach_metric.json")
Np, L, r = p["np"], p["nlarge"], p["na_radius"]
order = np.arange(len(x0))
B = 260  # > CUs / 2: one workgroup per patch
rng = np.random.default_rng(7)
stack = rng.integers(0, 30000, (len(x0), B, Np, Np)).astype(np.uint16)
prob = fpm_amd.Problem(Np, L, order, x0, y0, r, p["delta1"], p["delta2"], n_patch=B, path=fpm_amd.PATH_FUSED)
with fpm_amd.Solver(prob) as s:
    print("wg", s.info().wg_per_patch, s.info().fused_kernel)
    s.upload(stack); s.init(); s.run(2)
    out = s.download(support=False)
np.savez(sys.argv[1], objCrop=out["objCrop"][::37], pupil=out["pupil"], objF=out["objF"][::37])
PY
timeout -k 10 300 python $O/run.py $O/new.npz && FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_var/libfpm_hip.so timeout -k 10 300 python $O/run.py $O/old.npz && python3 -c "
import numpy as np
a=np.load('$O/new.npz'); b=np.load('$O/old.npz')
for k in a.files: print(k, np.array_equal(a[k], b[k]))
assert all(np.array_equal(a[k], b[k]) for k in a.files)
" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_metric.py tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
TAG=tailre/ab bash tools/gpu/ab_lib.sh
