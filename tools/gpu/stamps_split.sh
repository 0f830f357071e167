# phase stamps (FPM_STAMPS=1) of the Np 256 fused kernel per workgroups-per-patch
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-stamps}
mkdir -p $O
run() {  # name, env, bench args
  env $2 FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-gather $3 > $O/$1.json 2> $O/$1.err || { echo "$1 rc=$?"; tail -3 $O/$1.err; return 1; }
  echo "== $1: $(python3 -c "import json; d=json.load(open('$O/$1.json')); print(d['value'], d['led_ms_per_step'], d['config']['workgroups_per_patch'])")"
  grep "fpm stamps" $O/$1.err
}
run ks1_256 "FPM_X=0" "" && run ks2_128 "FPM_X=0" "--patches-total 128" && run ks4_64 "FPM_X=0" "--patches-total 64" && run ks2_64 "FPM_SPLIT=2" "--patches-total 64" && run ks4_32 "FPM_X=0" "--patches-total 32"
