# Patch groups vs hardware queues: the general path's groups run on their own
# streams; with GPU_MAX_HW_QUEUES=4 (the box default) more than ~3 streams
# share queues.  c2np256 and c5 at 2 / 3 / 4 groups, default and 8 queues.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06q}
mkdir -p $O
for W in ${WL:-c2np256 c5}; do
  case $W in c2np256) A="--config c2 --np 256 --steps 5";; c5) A="--config c5 --steps 2";; esac
  for V in ${VARS:-g2 g3 g4 q8g2 q8g3 q8g4}; do
    E="FPM_PATCH_GROUPS=${V: -1}"
    case $V in q8*) E="$E GPU_MAX_HW_QUEUES=8";; esac
    env $E timeout -k 10 300 python bench.py $A --warmup 1 --no-cpu-baseline > $O/${W}_$V.json 2> $O/${W}_$V.err || { echo "bench $W $V rc=$?"; tail -3 $O/${W}_$V.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${W}_$V.json')); print('$W $V', d['value'], d['led_ms_per_step'])"
  done
done
