# same-box A/B of an environment knob: AB_ENV (e.g. FPM_MR_XT100=1) vs none, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abenv}
mkdir -p $O
for i in 1 2 3; do
  for V in default knob; do
    if [ $V = knob ]; then E="$AB_ENV"; else E="FPM_AB_NONE=1"; fi
    env $E timeout -k 10 300 python bench.py ${AB_STEPS:---steps 20 --warmup 3} --no-cpu-baseline ${BENCH_ARGS:-} > $O/$V$i.json 2> $O/$V$i.err || { echo "$V rc=$?"; tail -3 $O/$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$V$i.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
  done
done
