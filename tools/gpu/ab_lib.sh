# same-box A/B: the in-tree library vs fpm-opencv_amd/lib_var (metric bench, alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab}
mkdir -p $O
for i in 1 2 3; do
  for V in default var; do
    if [ $V = var ]; then export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_var/libfpm_hip.so; else unset FPM_HIP_LIB; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $O/$V$i.json 2> $O/$V$i.err || { echo "$V rc=$?"; tail -3 $O/$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$V$i.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
  done
done
