# Np 200 fused kernel: its parity tests, config 3 literal, config-3 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-mr}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_mr.py tests/test_gpu_configs.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert|rel" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { echo "BENCH c3 rc=$?"; tail $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
FPM_STAMPS=1 timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 0 --no-cpu-baseline > $O/stamps_c3.json 2> $O/stamps_c3.err || { echo "STAMPS rc=$?"; exit 1; }
grep stamps $O/stamps_c3.err | tail -1
