# kernel-trace stats for the general-path configs (c3 at 256 patches, c5 at 8 patches)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-pc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 1 --warmup 0 > $O/prof_c3.log 2>&1 || { echo "PROF c3 rc=$?"; exit 1; }
python3 tools/prof_summary.py $O/prof_c3 $O/kernel_stats_c3.csv fpm
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 1 --warmup 0 > $O/prof_c5.log 2>&1 || { echo "PROF c5 rc=$?"; exit 1; }
python3 tools/prof_summary.py $O/prof_c5 $O/kernel_stats_c5.csv fpm
