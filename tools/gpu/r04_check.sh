# Round 4 check: full GPU suite (one pytest process), the default bench line,
# phase stamps of the small-shard modes, and one rocprofv3 kernel-trace pass
# of a plain-launched split-mode instance (the cooperative launch of round 3
# ended every profiled run of these instances in a SIGSEGV at exit).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04a}
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --durations 15 > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH rc=$?"; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'], d['scaling'])"
run() {  # name, bench args
  FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gather $2 > $O/$1.json 2> $O/$1.err || { echo "$1 rc=$?"; tail -3 $O/$1.err; return 1; }
  echo "== $1: $(python3 -c "import json; d=json.load(open('$O/$1.json')); print(d['value'], d['led_ms_per_step'], d['config']['kernel'])")"
  grep "fpm stamps" $O/$1.err | tail -2
}
line() {  # name, bench args: a timed line without stamps
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-gather $2 > $O/$1.json 2> $O/$1.err || { echo "$1 rc=$?"; tail -3 $O/$1.err; return 1; }
  echo "== $1: $(python3 -c "import json; d=json.load(open('$O/$1.json')); print(d['value'], d['led_ms_per_step'], d['objcrop_ms_per_step'], d['config']['kernel'])")"
}
line pt128 "--patches-total 128" && line pt64 "--patches-total 64" && line pt32 "--patches-total 32" && \
run st_pt64 "--patches-total 64" && run st_pt32 "--patches-total 32" && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_fused" --output-format csv -d $O/kt128 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-gather --patches-total 128 > $O/kt128.log 2>&1; echo "kt128 rc=$?"; tail -3 $O/kt128.log
