# L = 600 objCrop column-pass shapes (config 3): parity then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c600
mkdir -p $O
for V in 1 2 4; do
  FPM_CROP600_VAR=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_mr.py "tests/test_gpu_configs.py::test_config3_dogstomach_literal_256_patches" -x -q --timeout 300 --timeout-method thread > $O/t$V.log 2>&1 || { echo "TESTS FAILED $V"; tail -5 $O/t$V.log; exit 1; }
  tail -1 $O/t$V.log
done
for i in 1 2; do
  for V in 0 1 2 3 4; do
    FPM_CROP600_VAR=$V timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/b$V$i.json 2> $O/b$V$i.err || { echo "bench rc=$?"; tail -3 $O/b$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b$V$i.json')); print('var $V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
  done
done
