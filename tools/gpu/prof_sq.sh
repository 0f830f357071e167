# SQ counter passes on the fused kernel (one counter group per pass, --kernel-trace only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/sq
mkdir -p $OUT
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM" \
         "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "k_fused" --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/p$i.log; }
done
FPM_STAMPS=1 timeout -k 10 240 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/stamps.json 2> $OUT/stamps.err || echo "stamps rc=$?"
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/sq/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        print(r["Counter_Name"], r["Counter_Value"])
PY
grep "fpm stamps" $OUT/stamps.err | tail -2
