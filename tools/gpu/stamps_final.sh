# phase stamps (FPM_STAMPS=1, cycles per LED step) of the metric config's
# one-workgroup kernel and of config 3 / config 2 on the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/stf
mkdir -p $O
for W in "metric:" "c3:--config c3" "c2:--config c2"; do
  N=${W%%:*}; A=${W#*:}
  FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline $A > $O/$N.json 2> $O/$N.err || exit 1
  echo "== $N"; grep "stamps" $O/$N.err
done
