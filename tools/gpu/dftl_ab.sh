# packed dft256_full (in-tree) vs scalar (lib_dftls): objCrop and Np 1024
# tests, then metric (objCrop ms per step) and config 5 benches, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/dftl
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_np1024.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_groups.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  for V in default dftls; do
    if [ $V = default ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/m_$V$i.json 2> $O/m_$V$i.err || exit 1
    python3 -c "import json; d=json.load(open('$O/m_$V$i.json')); print('metric $V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
  done
done
for i in 1 2; do
  for V in default dftls; do
    if [ $V = default ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
    timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$V$i.json 2> $O/c5_$V$i.err || exit 1
    python3 -c "import json; d=json.load(open('$O/c5_$V$i.json')); print('c5 $V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
  done
done
