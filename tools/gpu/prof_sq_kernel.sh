# SQ counter passes on one kernel of a bench.py run (one counter group per pass,
# --kernel-trace only).  KRE = kernel-name regex, ARGS = bench.py arguments.
#   TAG=sqc3 KRE=k_colpass ARGS="--config c3 --steps 1 --warmup 0" bash tools/gpu/prof_sq_kernel.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-sqk}
mkdir -p $OUT
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAVES" \
         "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$KRE" --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); disp = collections.defaultdict(set)
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
for k in sorted(tot):
    n = max(len(disp[k]), 1)
    print(f"{k:28s} per-dispatch {tot[k] / n:16.1f}  ({n} dispatches)")
PY
