# Full GPU check of the tree in one box call:
#   GPU parity tests, smoke, kernel-trace stats of the bench command, the PMC
#   passes (HBM bytes + SQ counters, one counter group per pass, kernel-trace
#   only alongside --pmc), then the default bench line reading the counter
#   profile of THIS tree (src_hash stamped by tools/pmc_to_json.py).
# usage (on the box): TAG=r02x bash tools/gpu/round_profile.sh
#   SKIP_TESTS=1 skips pytest/smoke; KRE = kernel regex for the PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-rp}
mkdir -p $O
export TMPDIR=/tmp
lscpu > $O/lscpu.txt 2>&1 || true
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED rc=$?"; tail $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "PROF rc=$?"; tail $O/prof.log; exit 1; }
python3 tools/prof_summary.py $O/prof $O/kernel_stats.csv
python3 tools/prof_summary.py $O/prof $O/kernel_stats_fpm.csv "fpm::" > /dev/null
rm -rf $O/prof   # full traces of the synthetic-input torch kernels exceed gpurun's 64 MiB copy-back
KRE=${KRE:-"k_fused|k_meas_layout|k_crop"}
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$KRE" --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_p$i.log 2>&1 || { echo "PMC pass $i rc=$?"; tail -5 $O/pmc_p$i.log; exit 1; }
  echo "pmc pass $i done"
done
# FP32 instruction mix (only when this rocprofv3 lists the counters)
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
if grep -q SQ_INSTS_VALU_FMA_F32 $O/counters_list.txt; then
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "$KRE" --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc/p9 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_p9.log 2>&1 || { echo "PMC pass 9 rc=$?"; tail -5 $O/pmc_p9.log; exit 1; }
  echo "pmc pass 9 done"
fi
python3 tools/pmc_to_json.py $O/pmc $O/pmc_latest.json > $O/pmc_summary.txt || { echo "pmc_to_json failed"; exit 1; }
cat $O/pmc_summary.txt
find $O/pmc -name '*kernel_trace.csv' -delete
timeout -k 10 600 python bench.py --pmc $O/pmc_latest.json > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED rc=$?"; tail $O/bench.err; exit 1; }
cat $O/bench.json
