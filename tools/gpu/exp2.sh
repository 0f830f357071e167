# build variants (hipcc defines), each: fused parity tests + bench + stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
for V in "$@"; do
  (cd fpm-opencv_amd && make clean > /dev/null && make HIPFLAGS_EXTRA="$V" > /dev/null 2>&1) || { echo "BUILD FAILED $V"; exit 1; }
  timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "fused or metric" > gpurun_out/e_t.log 2>&1 || { echo "TESTS FAILED [$V] rc=$?"; tail -15 gpurun_out/e_t.log; continue; }
  FPM_STAMPS=1 timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/e_b.json 2> gpurun_out/e_b.err || { echo "bench rc=$? [$V]"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/e_b.json')); print('VARIANT [$V]', 'led', d['led_ms_per_step'], 'crop', d['objcrop_ms_per_step'], 'tests:', open('gpurun_out/e_t.log').read().strip().splitlines()[-1])"
  grep "fpm stamps" gpurun_out/e_b.err | tail -1
done
