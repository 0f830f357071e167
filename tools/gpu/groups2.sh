set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/groups2
mkdir -p $O
for i in 1 2; do
  for V in "FPM_PATCH_GROUPS=1_FPM_NO_GRAPH=1" "FPM_PATCH_GROUPS=2_FPM_NO_GRAPH=1" "FPM_PATCH_GROUPS=3_FPM_NO_GRAPH=1" "FPM_PATCH_GROUPS=4_FPM_NO_GRAPH=1" "FPM_PATCH_GROUPS=2"; do
    E=$(echo $V | tr '_' ' ' | sed 's/FPM PATCH GROUPS/FPM_PATCH_GROUPS/; s/FPM NO GRAPH/FPM_NO_GRAPH/')
    env $E timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/$V$i.json 2> $O/$V$i.err || { echo "$V rc=$?"; tail -3 $O/$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$V$i.json')); print('$E', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
  done
done
