# Round-6 evidence run: the whole GPU suite, counter passes of every workload
# kernel (the split / distributed instances included: plain co-resident
# launches exit cleanly under rocprofv3 since round 4), the bench lines of
# every workload reading those fresh counter files (--pmc), the kernel-trace
# stats of the headline command, and phase stamps of the shard workloads.
# tools/collect_profiles.py gpurun_out/<TAG> r06f copies the results to profiles/.
# A GPU call is limited to 20 minutes, so the run comes in parts:
#   PMC="metric pt128 pt64" (counter passes of these workloads only; SKIP_TESTS=1 skips the suite)
#   BENCH=1 SKIP_TESTS=1 SKIP_PMC=1 (bench lines reading the collected profiles/pmc_* files,
#   kernel trace, stamps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r06p}
O=gpurun_out/$T
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --durations 10 > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
  tail -1 $O/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
W_ALL="metric: c2:--config_c2 c3:--config_c3 c5:--config_c5 pt128:--patches-total_128 pt64:--patches-total_64 pt32:--patches-total_32 c2np256:--config_c2_--np_256"
if [ -z "$SKIP_PMC" ]; then
  for W in $W_ALL; do
    N=${W%%:*}; A=${W#*:}
    case " ${PMC:-metric c2 c3 c5 pt128 pt64 pt32 c2np256} " in *" $N "*) ;; *) continue;; esac
    TAG=$T/pmc_$N BENCH_ARGS="${A//_/ }" bash tools/gpu/prof_counters.sh || { echo "pmc $N failed"; exit 1; }
    echo "pmc $N done"
  done
fi
bl() {  # name, args
  timeout -k 10 400 python bench.py $2 > $O/bench_$1.json 2> $O/bench_$1.err || { echo "BENCH $1 rc=$?"; tail -3 $O/bench_$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'], r['kernel'], r['frac'], r['hbm']['frac'], r.get('traffic'))"
}
[ -z "$BENCH" ] && { echo "evidence part done"; exit 0; }
pm() { [ -f $O/pmc_$1/pmc.json ] && echo "--pmc $O/pmc_$1/pmc.json"; }
bl metric "--steps 20 --warmup 5 $(pm metric)" && \
bl c2 "--config c2 --steps 20 --warmup 3 --no-cpu-baseline $(pm c2)" && \
bl c3 "--config c3 --steps 20 --warmup 3 --no-cpu-baseline $(pm c3)" && \
bl c5 "--config c5 --steps 3 --warmup 1 --no-cpu-baseline $(pm c5)" && \
bl pt128 "--patches-total 128 --steps 20 --warmup 3 --no-cpu-baseline $(pm pt128)" && \
bl pt64 "--patches-total 64 --steps 20 --warmup 3 --no-cpu-baseline $(pm pt64)" && \
bl pt32 "--patches-total 32 --steps 20 --warmup 3 --no-cpu-baseline $(pm pt32)" && \
bl c2np256 "--config c2 --np 256 --steps 5 --warmup 1 --no-cpu-baseline $(pm c2np256)" && \
bl default_cmd "" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || { echo "kernel trace rc=$?"; tail -5 $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_metric.csv \;
find $O/kt -name "*kernel_trace.csv" -delete
for P in 128 64 32; do
  FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gather --patches-total $P > $O/st_pt$P.json 2> $O/st_pt$P.err || { echo "stamps pt$P rc=$?"; exit 1; }
  echo "== stamps pt$P"; grep "fpm stamps" $O/st_pt$P.err | tail -2
done
for C in metric c2 c3; do
  A=$([ $C = metric ] || echo "--config $C")
  FPM_STAMPS=1 timeout -k 10 120 python bench.py $A --steps 2 --warmup 1 --no-cpu-baseline --no-gather > $O/st_$C.json 2> $O/st_$C.err || { echo "stamps $C rc=$?"; exit 1; }
  echo "== stamps $C"; grep "fpm stamps" $O/st_$C.err | tail -2
done
echo "evidence done"
