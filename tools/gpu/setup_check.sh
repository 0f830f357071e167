set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-setup}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_torch_interop.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for W in "metric:" "c3:--config c3"; do N=${W%%:*}; A=${W#*:}
timeout -k 10 300 python bench.py $A --steps 5 --warmup 1 --no-cpu-baseline > $O/b_$N.json 2> $O/b_$N.err || { echo "bench rc=$?"; tail -3 $O/b_$N.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_$N.json')); print('$N', d['value'], d['setup']['upload_and_permute_ms'], d['setup']['init_ms'])"
done
