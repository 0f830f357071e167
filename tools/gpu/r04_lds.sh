# Round 4: LDS bank layouts of the Np 90 / Np 200 kernels.  Parity tests of
# both kernels, same-box alternating A/B of the bank-friendly layout against
# the dense one (FPM_S90_DENSE / FPM_MR_DENSE), one LDS counter pass each, then
# (PMC_SHARDS=1) the counter passes of the split / distributed instances.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04b}
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for c in c2 c3 c5; do
  K=$([ $c = c2 ] && echo FPM_S90_DENSE=1 || { [ $c = c3 ] && echo FPM_MR_DENSE=1 || echo FPM_T32=1; })
  for i in 1 2 3; do
    for V in fast dense; do
      E=$([ $V = dense ] && echo $K || echo FPM_AB_NONE=1)
      env $E timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/${c}_$V$i.json 2> $O/${c}_$V$i.err || { echo "$c $V rc=$?"; tail -3 $O/${c}_$V$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${c}_$V$i.json')); print('$c $V', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
    done
  done
  [ $c = c5 ] && continue
  for V in fast dense; do
    E=$([ $V = dense ] && echo $K || echo FPM_AB_NONE=1)
    env $E timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --kernel-include-regex "k_fused" --output-format csv -d $O/lds_${c}_$V -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 2 --warmup 0 --no-cpu-baseline > $O/lds_${c}_$V.log 2>&1 || { echo "pmc $c $V rc=$?"; tail -3 $O/lds_${c}_$V.log; exit 1; }
    python3 - <<PY
import csv, glob, collections
f = glob.glob("$O/lds_${c}_$V/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(float); n = collections.Counter()
for row in csv.DictReader(open(f[0])):
    if "k_fused" in row["Kernel_Name"]:
        acc[row["Counter_Name"]] += float(row["Counter_Value"])
print("$c $V", {k: v for k, v in acc.items()}, "bank-conflict share of LDS cycles %.3f" % (acc["SQ_LDS_BANK_CONFLICT"] / acc["SQ_LDS_IDX_ACTIVE"]))
PY
  done
done
if [ -n "$PMC_SHARDS" ]; then
  for P in 128 64 32; do
    TAG=$(basename $O)/pmc_pt$P BENCH_ARGS="--patches-total $P" bash tools/gpu/prof_counters.sh || exit 1
    echo "pmc pt$P done"
  done
fi
# distributed mode: this tree against lib_v1 (DIST_AB=1), alternating
if [ -n "$DIST_AB" ]; then
  for i in 1 2; do
    for V in cur v1; do
      for P in 256 64 32; do
        if [ $V = v1 ]; then export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_v1/libfpm_hip.so; else unset FPM_HIP_LIB; fi
        timeout -k 10 120 python bench.py --no-cpu-baseline --no-gather --patches-total $P > $O/pt${P}_$V$i.json 2> $O/pt${P}_$V$i.err || { echo "pt$P $V rc=$?"; tail -3 $O/pt${P}_$V$i.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/pt${P}_$V$i.json')); print('pt$P $V', d['value'], d['led_ms_per_step'], d['config']['kernel'])"
      done
    done
  done
  unset FPM_HIP_LIB
fi
# phase stamps of the distributed instances (cycles per LED)
for P in 64 32; do
  FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gather --patches-total $P > $O/st_pt$P.json 2> $O/st_pt$P.err || { echo "stamps pt$P rc=$?"; tail -3 $O/st_pt$P.err; exit 1; }
  echo "== st_pt$P"; grep "fpm stamps" $O/st_pt$P.err | tail -2
done
