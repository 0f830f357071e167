# How SQ_INSTS_VALU_*_F32 count packed FP32 instructions (tools/gpu/micro/flop_count.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-flops}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $OUT/p1 -o run -- $GRAFT_REPO_ROOT/tools/gpu/micro/bin/flop_count > $OUT/flops.log 2>&1 || { echo "flops rc=$?"; tail $OUT/flops.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] = float(r["Counter_Value"])
for k, d in sorted(acc.items()):
    print(k, {c: int(v) for c, v in sorted(d.items())})
PY
grep expected $OUT/flops.log; rm -rf $OUT/p1/
