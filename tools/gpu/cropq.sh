# L = 768 objCrop column pass in quarter strips (FPM_CROP_Q=1) vs halves: parity, then metric A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cropq
mkdir -p $O
FPM_CROP_Q=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_metric.py -x -q -k "objcrop or metric or bench" --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
AB_ENV=FPM_CROP_Q=1 TAG=cropq/ab bash tools/gpu/ab_env.sh
