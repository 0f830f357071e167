# round-3 evidence run: bench lines of every workload, the kernel-trace stats
# of the headline command, and counter passes per workload kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03p}
mkdir -p $O
bl() {  # name, args
  timeout -k 10 400 python bench.py $2 > $O/bench_$1.json 2> $O/bench_$1.err || { echo "BENCH $1 rc=$?"; tail -3 $O/bench_$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'], r['kernel'], r['frac'], r['hbm']['frac'], d.get('setup'))"
}
bl metric "--steps 20 --warmup 5" && \
bl c2 "--config c2 --steps 20 --warmup 3 --no-cpu-baseline" && \
bl c3 "--config c3 --steps 20 --warmup 3 --no-cpu-baseline" && \
bl c5 "--config c5 --steps 3 --warmup 1 --no-cpu-baseline" && \
bl pt128 "--patches-total 128 --steps 20 --warmup 3 --no-cpu-baseline" && \
bl pt64 "--patches-total 64 --steps 20 --warmup 3 --no-cpu-baseline" && \
bl pt32 "--patches-total 32 --steps 20 --warmup 3 --no-cpu-baseline" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || { echo "kernel trace rc=$?"; tail -5 $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_metric.csv \;
find $O/kt -name "*kernel_trace.csv" -delete
head -8 $O/kernel_stats_metric.csv
# counter passes: the split / distributed (cooperative-launch) workloads end
# in a segfault of the profiled process at exit on this pool (DESIGN.md
# section 5), so by default only the one-workgroup-per-patch workloads
for W in "metric:" "c2:--config c2" "c3:--config c3" "c5:--config c5"; do
  N=${W%%:*}; A=${W#*:}
  TAG=${TAG:-r03p}/pmc_$N BENCH_ARGS="$A" bash tools/gpu/prof_counters.sh || { echo "pmc $N failed"; exit 1; }
  echo "pmc $N done"
done
