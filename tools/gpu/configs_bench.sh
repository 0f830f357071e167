# bench lines of the non-headline BASELINE configs on one box:
# c2 (dataset_mono, Np 90, 64 patches), c3 (dogStomach literal, Np 200 fused), c4 shard (128 of 1024
# patches), c5 (Np 1024 fp16, general path)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cfg}
mkdir -p $O
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail $O/c3.err; exit 1; }
FPM_STAMPS=1 timeout -k 10 300 python bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep stamps > $O/c3_stamps.txt || true
timeout -k 10 300 python bench.py --patches-total 128 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_shard128.json 2> $O/c4s.err || { echo "c4 shard rc=$?"; tail $O/c4s.err; exit 1; }
timeout -k 10 400 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { echo "c5 rc=$?"; tail $O/c5.err; exit 1; }
timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { echo "c2 rc=$?"; tail $O/c2.err; exit 1; }
for f in c2 c3 c4_shard128 c5; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('led_ms_per_step'), d.get('objcrop_ms_per_step'))"; done
cat $O/c3_stamps.txt
