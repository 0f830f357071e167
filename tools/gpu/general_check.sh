# all GPU tests + general-path configs (c3, c5 at 8 and 1 patches) + c5 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-gen}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for C in "c3 0" "c5 0" "c5 1"; do
  set -- $C
  timeout -k 10 400 python bench.py --config $1 --patches $2 --steps 2 --warmup 1 > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || { echo "$C FAILED rc=$?"; tail $O/bench_$1_$2.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$1_$2.json')); print('$C', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
done
timeout -k 10 400 python bench.py --path general --no-cpu-baseline --steps 2 --warmup 1 > $O/bench_metric_general.json 2> $O/bench_mg.err || { echo "metric general FAILED rc=$?"; tail $O/bench_mg.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/bench_metric_general.json')); print('metric general', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 1 --warmup 0 > $O/prof_c3.log 2>&1 || { echo "PROF rc=$?"; exit 1; }
python3 tools/prof_summary.py $O/prof_c3 $O/kernel_stats_c3.csv fpm
