# Kernel-trace stats (rocprofv3 --kernel-trace --stats) of the bench command of
# each workload on the final tree: gpurun_out/<TAG>/kernel_stats_<w>.csv
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05t}
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
for W in ${LINES:-c2:--config_c2 c3:--config_c3 c5:--config_c5 pt32:--patches-total_32}; do
  N=${W%%:*}; A=${W#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_$N -o run -- python3 $GRAFT_REPO_ROOT/bench.py ${A//_/ } --steps 3 --warmup 1 --no-cpu-baseline --no-gather > $O/kt_$N.log 2>&1 || { echo "kernel trace $N rc=$?"; tail -5 $O/kt_$N.log; exit 1; }
  find $O/kt_$N -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$N.csv \;
  rm -rf $O/kt_$N
  echo "trace $N done"
done
