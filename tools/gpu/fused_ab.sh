# A/B of the fused kernel variants on one box: parity tests of the fused path
# (default variant), bench lines for 1024 and 512 threads, phase stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multirank.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench1024.json 2> $O/bench1024.err || { echo "BENCH1024 rc=$?"; tail $O/bench1024.err; exit 1; }
FPM_FUSED_NT=512 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench512.json 2> $O/bench512.err || { echo "BENCH512 rc=$?"; tail $O/bench512.err; exit 1; }
FPM_STAMPS=1 timeout -k 10 300 python bench.py --steps 2 --warmup 0 --no-cpu-baseline > $O/stamps1024.json 2> $O/stamps1024.err || { echo "STAMPS rc=$?"; tail $O/stamps1024.err; exit 1; }
FPM_FUSED_NT=512 FPM_STAMPS=1 timeout -k 10 300 python bench.py --steps 2 --warmup 0 --no-cpu-baseline > $O/stamps512.json 2> $O/stamps512.err || { echo "STAMPS512 rc=$?"; exit 1; }
python3 - <<'PY'
import json,os
O=os.environ.get("TAG","ab")
for v in ("1024","512"):
    d=json.load(open(f"gpurun_out/{O}/bench{v}.json"))
    print(v, d["value"], d["ms_per_step"], d["roofline"]["launch_ms"], d["objcrop_ms_per_step"])
PY
grep "stamps" $O/stamps1024.err | tail -1
grep "stamps" $O/stamps512.err | tail -1
