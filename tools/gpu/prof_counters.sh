# HBM traffic passes (MI355X_MICROARCH.md "HBM [CDNA4]"): FETCH_SIZE and
# WRITE_SIZE in separate passes, --kernel-trace only alongside --pmc.
# k_meas_layout moves a known byte count (reported as a FETCH_SIZE check).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "k_fused|k_meas_layout|k_fft_batch|k_crop" --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_to_json.py $OUT gpurun_out/pmc_latest.json
