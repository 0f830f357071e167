# Np 1024 register kernels: their tests, config 5, config-5 bench on both implementations + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-n1k}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_np1024.py tests/test_gpu_configs.py -x -v -k "np1024 or config5 or fp16" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert|rel" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "BENCH c5 rc=$?"; tail $O/bench_c5.err; exit 1; }
FPM_NO_REG1024=1 timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5_lds.json 2> $O/bench_c5l.err || { echo "BENCH c5 lds rc=$?"; tail $O/bench_c5l.err; exit 1; }
for f in bench_c5 bench_c5_lds; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('led_ms_per_step'), d.get('objcrop_ms_per_step'))"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { echo "PROF c5 rc=$?"; exit 1; }
python3 tools/prof_summary.py $O/prof_c5 $O/kernel_stats_c5.csv fpm
rm -rf $O/prof_c5
head -12 $O/kernel_stats_c5.csv
