# Strong-scaling pieces of bench.py on one box: the config-4 single-GPU shard
# (128 of 1024 patches) and a 2-rank gloo rehearsal of the N > 1 path
# (--patches-total, shard_range, gather + stitch) with both ranks on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-strong}
mkdir -p $O
timeout -k 10 300 python bench.py --patches-total 128 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_shard128.json 2> $O/c4s.err || { echo "c4 shard rc=$?"; tail $O/c4s.err; exit 1; }
cat $O/c4_shard128.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --backend gloo --patches-total 64 --steps 2 --warmup 1 --no-cpu-baseline > $O/gloo2.json 2> $O/gloo2.err || { echo "gloo2 rc=$?"; tail -20 $O/gloo2.err; exit 1; }
cat $O/gloo2.json
