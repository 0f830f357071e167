# same-box A/B of several library variants (fpm-opencv_amd/lib_<v>/) against
# the in-tree library, metric bench (or BENCH_ARGS), alternating, N rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abm}
mkdir -p $O
for i in $(seq 1 ${ROUNDS:-3}); do
  for V in default $VARS; do
    if [ $V = default ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
    timeout -k 10 300 python bench.py ${AB_STEPS:---steps 20 --warmup 3} --no-cpu-baseline ${BENCH_ARGS:-} > $O/$V$i.json 2> $O/$V$i.err || { echo "$V rc=$?"; tail -3 $O/$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$V$i.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
  done
done
