# quick iteration: fused-path GPU tests, bench, phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/qt.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 gpurun_out/qt.log; exit 1; }
tail -1 gpurun_out/qt.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/qb.json 2> gpurun_out/qb.err || { echo "BENCH FAILED rc=$?"; tail gpurun_out/qb.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/qb.json')); print('value', d['value'], 'ms/step', d['ms_per_step'], 'led', d['led_ms_per_step'], 'crop', d['objcrop_ms_per_step'], 'frac', d['roofline']['frac'])"
FPM_STAMPS=1 timeout -k 10 240 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> gpurun_out/qs.err || { echo "stamps rc=$?"; exit 1; }
grep "fpm stamps" gpurun_out/qs.err | tail -1
