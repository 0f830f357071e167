# timing-only variants (no parity tests: for deliberately incomplete builds)
set -o pipefail
cd $GRAFT_REPO_ROOT
for V in "$@"; do
  (cd fpm-opencv_amd && make clean > /dev/null && make HIPFLAGS_EXTRA="$V" > /dev/null 2>&1) || { echo "BUILD FAILED $V"; exit 1; }
  FPM_STAMPS=1 timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/e_b.json 2> gpurun_out/e_b.err || { echo "bench rc=$? [$V]"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/e_b.json')); print('VARIANT [$V]', 'led', d['led_ms_per_step'], 'crop', d['objcrop_ms_per_step'])"
  grep "fpm stamps" gpurun_out/e_b.err | tail -1
done
