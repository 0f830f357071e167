cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -k "fused or metric" > gpurun_out/t4.log 2>&1
grep -E "PASS|FAIL|assert .* <|passed|failed" gpurun_out/t4.log | head -40
