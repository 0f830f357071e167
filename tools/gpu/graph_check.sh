# general path with and without hipGraph replay: parity tests + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gt.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 gpurun_out/gt.log; exit 1; }
tail -1 gpurun_out/gt.log
timeout -k 10 300 python bench.py --path general --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g1.json 2> gpurun_out/g1.err || { echo "BENCH graph rc=$?"; tail gpurun_out/g1.err; exit 1; }
FPM_NO_GRAPH=1 timeout -k 10 300 python bench.py --path general --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g0.json 2> gpurun_out/g0.err || { echo "BENCH nograph rc=$?"; tail gpurun_out/g0.err; exit 1; }
python3 -c "
import json
for f in ('g1','g0'):
    d=json.load(open('gpurun_out/%s.json'%f)); print(f, 'value', d['value'], 'ms/step', d['ms_per_step'], 'led', d['led_ms_per_step'])"
