# Round 4 check: full GPU suite (one pytest process), the default bench line,
# small-shard lines of the in-tree library against lib_v1 (round-3
# distributed kernel with round-4 polling), phase stamps, and one rocprofv3
# kernel-trace pass of a plain-launched split-mode instance (the cooperative
# launch of round 3 ended every profiled run of these in a SIGSEGV at exit).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04a}
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --durations 15 > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH rc=$?"; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'], d['scaling'])"
line() {  # name, lib variant (or default), env, bench args
  if [ $2 = default ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$2/libfpm_hip.so; fi
  env $3 timeout -k 10 120 python bench.py --no-cpu-baseline --no-gather $4 > $O/$1.json 2> $O/$1.err || { echo "$1 rc=$?"; tail -3 $O/$1.err; return 1; }
  echo "== $1: $(python3 -c "import json; d=json.load(open('$O/$1.json')); print(d['value'], d['led_ms_per_step'], d['objcrop_ms_per_step'], d['config']['kernel'])")"
}
stamps() {  # name, env, bench args
  unset FPM_HIP_LIB
  env $2 FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gather $3 > $O/$1.json 2> $O/$1.err || { echo "$1 rc=$?"; tail -3 $O/$1.err; return 1; }
  echo "== $1: $(python3 -c "import json; d=json.load(open('$O/$1.json')); print(d['value'], d['led_ms_per_step'], d['config']['kernel'])")"
  grep "fpm stamps" $O/$1.err | tail -2
}
for r in 1 2; do
  line pt64_v2_$r default "FPM_X=0" "--patches-total 64" && line pt64_v1_$r v1 "FPM_X=0" "--patches-total 64" && \
  line pt32_v2_$r default "FPM_X=0" "--patches-total 32" && line pt32_v1_$r v1 "FPM_X=0" "--patches-total 32" || exit 1
done
line pt128_split default "FPM_X=0" "--patches-total 128" && line pt128_d2 default "FPM_DIST=2" "--patches-total 128" && \
line pt128_d2v1 v1 "FPM_DIST=2" "--patches-total 128" && line pt64_split default "FPM_NO_DIST=1" "--patches-total 64" && \
stamps st_pt64 "FPM_X=0" "--patches-total 64" && stamps st_pt32 "FPM_X=0" "--patches-total 32" && stamps st_pt128d2 "FPM_DIST=2" "--patches-total 128" || exit 1
unset FPM_HIP_LIB
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_fused" --output-format csv -d $O/kt128 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-gather --patches-total 128 > $O/kt128.log 2>&1; echo "kt128 rc=$?"; tail -3 $O/kt128.log
