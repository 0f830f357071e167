set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $O/split_tests.log 2>&1 || { echo "SPLIT TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/split_tests.log | head -20; exit 1; }
tail -1 $O/split_tests.log
for T in 64 32; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --patches-total $T --no-cpu-baseline > $O/bench_pt$T.json 2> $O/bench_pt$T.err || { echo "BENCH pt$T rc=$?"; tail $O/bench_pt$T.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_pt$T.json')); print('patches-total $T', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['config']['workgroups_per_patch'])"
done
TAG=${TAG:-r03c}/flops bash tools/gpu/prof_flops.sh
TAG=${TAG:-r03c}/pmc_metric bash tools/gpu/prof_counters.sh && head -60 $O/pmc_metric/pmc_summary.txt
