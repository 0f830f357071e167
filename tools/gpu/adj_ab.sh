# interleaved halves: pass-B column blocks on adjacent columns (lib_adj) vs
# spread by 16 (in-tree) vs HEAD's contiguous halves (lib_head); stamps of each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/adj
mkdir -p $O
FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_adj/libfpm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_metric.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
VARS="adj head" TAG=adj/metric bash tools/gpu/ab_multi.sh || exit 1
for V in default adj head; do
  if [ $V = default ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
  FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/st_$V.json 2> $O/st_$V.err || exit 1
  echo "== $V"; grep "fpm stamps" $O/st_$V.err
done
