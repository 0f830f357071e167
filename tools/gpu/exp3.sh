# variant builds: fused parity tests + per-kernel rocprof stats for fpm kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for V in "$@"; do
  (cd fpm-opencv_amd && make clean > /dev/null && make HIPFLAGS_EXTRA="$V" > /dev/null 2>&1) || { echo "BUILD FAILED $V"; exit 1; }
  timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "fused or metric" > gpurun_out/e_t.log 2>&1 || { echo "TESTS FAILED [$V] rc=$?"; tail -15 gpurun_out/e_t.log; continue; }
  rm -rf gpurun_out/e_prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/e_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/e_prof.log 2>&1 || { echo "PROF rc=$?"; exit 1; }
  echo "VARIANT [$V] $(tail -1 gpurun_out/e_t.log)"
  python3 tools/prof_summary.py gpurun_out/e_prof /tmp/e.csv fpm:: | head -8
done
