# interleaved column halves (in-tree) vs HEAD's contiguous halves (lib_head):
# Np 256 parity tests, metric / 128-patch benches, phase stamps of both
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ipart2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_metric.py tests/test_gpu_configs.py -x -v -s --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
grep -E "passed|failed" $O/t.log | tail -1
VARS="head" TAG=ipart2/metric bash tools/gpu/ab_multi.sh || exit 1
VARS="head" ROUNDS=2 BENCH_ARGS="--patches 128" TAG=ipart2/pt128 bash tools/gpu/ab_multi.sh || exit 1
for V in default head; do
  if [ $V = head ]; then export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_head/libfpm_hip.so; else unset FPM_HIP_LIB; fi
  FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/st_$V.json 2> $O/st_$V.err || exit 1
  echo "== $V"; grep "fpm stamps" $O/st_$V.err
done
