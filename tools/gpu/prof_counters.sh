# Counter passes for ONE bench workload (MI355X_MICROARCH.md "HBM [CDNA4]"):
# FETCH_SIZE and WRITE_SIZE in separate passes, the L2->fabric read requests
# by size, and three SQ passes; --kernel-trace only beside --pmc.  Reduced
# with tools/pmc_to_json.py to gpurun_out/<TAG>/pmc.json (stamped with the
# csrc hash).  usage: TAG=name BENCH_ARGS="--config c2" bash tools/gpu/prof_counters.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-pmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
RX="k_fused|k_meas|k_crop|k_fft|k_colpass|k_gather|k_rowfft|k_rows1024|k_cols1024|k_rows256|k_cols256|k_tile|k_pupil|k_row_max"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM" \
         "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-gather ${BENCH_ARGS:-} > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
# the profiled run is one iteration (--steps 1 --warmup 0): recorded in the
# file, bench.py divides a kernel's dispatches by it
PMC_BENCH_ITERS=1 python3 tools/pmc_to_json.py $OUT $OUT/pmc.json > $OUT/pmc_summary.txt
rm -rf $OUT/p[0-9]*/   # raw rocprofv3 output: too large to copy back; pmc.json keeps the per-kernel means
