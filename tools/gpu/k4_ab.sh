# config 5: in-tree library (batched K4 tile loads) vs lib_var (previous K4), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/k4_ab
mkdir -p $O
for i in 1 2 3; do
  for V in default var; do
    if [ $V = var ]; then export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_var/libfpm_hip.so; else unset FPM_HIP_LIB; fi
    timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/$V$i.json 2> $O/$V$i.err || { echo "$V rc=$?"; tail -3 $O/$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$V$i.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
  done
done
unset FPM_HIP_LIB
cd /tmp && export TMPDIR=/tmp
for V in default var; do
  if [ $V = var ]; then export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_var/libfpm_hip.so; else unset FPM_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$V -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_$V.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  f=$(find $GRAFT_REPO_ROOT/$O/prof_$V -name "*kernel_stats.csv" | head -1); cp $f $GRAFT_REPO_ROOT/$O/kstats_$V.csv
  find $GRAFT_REPO_ROOT/$O/prof_$V -name "*.csv" ! -name "*kernel_stats.csv" -delete
  grep -E "k_tile_rows|rows1024|cols1024" $GRAFT_REPO_ROOT/$O/kstats_$V.csv | cut -d, -f1-4 | sed "s/^/$V /"
done
