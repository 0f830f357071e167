# config 5: hoisted-load row kernels at 4 waves (default) vs 3 waves (lib_var)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-c5ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_np1024.py -x -q --timeout 300 --timeout-method thread > $O/np1024_tests.log 2>&1 || { echo "NP1024 TESTS FAILED"; tail -20 $O/np1024_tests.log; exit 1; }
tail -1 $O/np1024_tests.log
for V in default var; do
  if [ $V = var ]; then export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_var/libfpm_hip.so; fi
  timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$V.json 2> $O/c5_$V.err || { echo "c5 $V rc=$?"; tail -3 $O/c5_$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$V.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
done
unset FPM_HIP_LIB
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/kt.log 2>&1 || { echo "kt rc=$?"; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c5.csv \;
rm -rf $O/kt
grep -E "k_rows1024|k_cols1024|k_tile|k_pupil" $O/kernel_stats_c5.csv | cut -d, -f1-4
