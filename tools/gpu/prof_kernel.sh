# SQ/TCP counter passes on one kernel (regex $1), bench as the workload
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RX="$1"
OUT=$GRAFT_REPO_ROOT/gpurun_out/pk
rm -rf $OUT; mkdir -p $OUT
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $OUT/p$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(dict)
for f in sorted(glob.glob("gpurun_out/pk/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[(r["Dispatch_Id"], r["Kernel_Name"][:40])][r["Counter_Name"]] = float(r["Counter_Value"])
# collapse by kernel name + grid: print per-dispatch in order of first pass
seen = collections.defaultdict(list)
for (d, k), c in agg.items():
    seen[k].append(c)
for k, lst in seen.items():
    keys = sorted(set().union(*lst))
    print(k, "dispatch-samples", len(lst))
    for key in keys:
        vals = [c[key] for c in lst if key in c]
        print(f"   {key:28s} " + " ".join(f"{v:.4g}" for v in vals[:6]))
PY
