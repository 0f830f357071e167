# Kernel trace of the dataset_mono Np 256 / r 84 general path (c2np256) and
# of config 5: per-kernel durations per LED step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06t}
mkdir -p $O
for W in ${WL:-c2np256}; do
  case $W in
    c2np256) A="--config c2 --np 256 --steps 3 --warmup 1";;
    c5) A="--config c5 --steps 2 --warmup 1";;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_$W -o run -- python3 $GRAFT_REPO_ROOT/bench.py $A --no-cpu-baseline > $O/kt_$W.log 2>&1 || { echo "kernel trace $W rc=$?"; tail -5 $O/kt_$W.log; exit 1; }
  find $O/kt_$W -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$W.csv \;
  if [ -n "$KEEP_TRACE" ]; then find $O/kt_$W -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace_$W.csv \; ; fi
  find $O/kt_$W -name "*kernel_trace.csv" -delete
  echo "== $W"; cut -d, -f1-4 $O/kernel_stats_$W.csv | grep -v "at::" | head -14
done
