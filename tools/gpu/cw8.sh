# Np 1024 column pass 8 columns per block (FPM_N1K_CW=8) vs 4: tests + config 5 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cw8
mkdir -p $O
FPM_N1K_CW=${CW:-16} timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_configs.py -k "np1024 or config5" -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -5 $O/t.log; exit 1; }
tail -2 $O/t.log
AB_STEPS="--steps 3 --warmup 1" AB_ENV=FPM_N1K_CW=${CW:-16} BENCH_ARGS="--config c5" TAG=cw8/ab bash tools/gpu/ab_env.sh
