# device-upload layout copy variants (FPM_LAYOUT_VAR 0 / 1 non-temporal / 2 128-column strips)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/layout_ab
mkdir -p $O
for V in 0 1 2; do
  FPM_LAYOUT_VAR=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_torch_interop.py -x -q --timeout 300 --timeout-method thread > $O/t$V.log 2>&1 || { echo "TESTS FAILED var $V"; tail -20 $O/t$V.log; exit 1; }
done
for i in 1 2 3; do
  for V in 0 1 2; do
    FPM_LAYOUT_VAR=$V timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/b$V$i.json 2> $O/b$V$i.err || { echo "bench rc=$?"; tail -3 $O/b$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b$V$i.json')); print('var $V', d['value'], d['setup']['upload_and_permute_ms'], d['setup']['init_ms'])"
  done
done
