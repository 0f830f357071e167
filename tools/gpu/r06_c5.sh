# Config 5 A/B: the in-tree lib ("new") against lib_<name> variants, the
# np1024 / config 5 GPU tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06c5}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_np1024.py tests/test_gpu_configs.py::test_config5_fp16_storage_65_leds_2_iterations tests/test_gpu_configs.py::test_config5_fp16_storage_np1024_l4096 tests/test_gpu_groups.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert|rel L2" $O/tests.log | head -30; exit 1; }
grep -E "passed|failed|rel L2" $O/tests.log | tail -14
venv() { case $1 in new) echo "FPM_X=1";; dp32) echo "FPM_DP32=1";; *) echo "FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$1/libfpm_hip.so";; esac; }
for R in $(seq 1 ${ROUNDS:-2}); do
for V in ${VARS:-new base}; do
  env $(venv $V) timeout -k 10 300 python bench.py --config c5 --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > $O/c5_${V}$R.json 2> $O/c5_${V}$R.err || { echo "bench $V rc=$?"; tail -3 $O/c5_${V}$R.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_${V}$R.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
done
done
