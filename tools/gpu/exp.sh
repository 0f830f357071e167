# timing-only experiment build (results not checked): EXP_FLAGS are extra hipcc defines
set -o pipefail
cd $GRAFT_REPO_ROOT/fpm-opencv_amd
make clean > /dev/null && make HIPFLAGS_EXTRA="$EXP_FLAGS" > /dev/null 2>&1 || { echo BUILD FAILED; exit 1; }
cd $GRAFT_REPO_ROOT
FPM_STAMPS=1 timeout -k 10 240 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/exp.json 2> gpurun_out/exp.err || { echo "exp rc=$?"; tail -5 gpurun_out/exp.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/exp.json')); print('EXP', '$EXP_FLAGS', 'led', d['led_ms_per_step'])"
grep "fpm stamps" gpurun_out/exp.err | tail -1
