# objCrop timing experiments: for each EXP_LIST entry (hipcc defines, ','
# separated, '-' = none) rebuild the library on the box and print the bench's
# objCrop and fused-kernel time per step (results not checked: parity tests
# run separately on the default build)
set -o pipefail
cd $GRAFT_REPO_ROOT
for e in ${EXP_LIST:--}; do
  flags=""
  [ "$e" != "-" ] && flags=$(echo "$e" | tr ',' ' ')
  (cd fpm-opencv_amd && make clean > /dev/null && make HIPFLAGS_EXTRA="$flags" > /dev/null 2>&1) || { echo "BUILD FAILED $e"; exit 1; }
  timeout -k 10 240 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/cexp.json 2> gpurun_out/cexp.err || { echo "exp rc=$?"; tail -5 gpurun_out/cexp.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cexp.json')); print('EXP', '$e', 'crop', d['objcrop_ms_per_step'], 'led', d['led_ms_per_step'], 'value', d['value'])"
done
