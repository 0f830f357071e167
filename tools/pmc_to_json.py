"""Reduce rocprofv3 --pmc passes to per-launch counters per kernel
(bench.py's roofline.traffic and roofline.counters).

usage: python tools/pmc_to_json.py <pmc dir with p*/**/*counter_collection.csv> <out.json>

Every counter is averaged over the dispatches of one kernel (one value per
launch).  The output is stamped with tools/srchash.py's hash of the csrc tree
it was measured on; bench.py ignores a file whose hash differs.

Units and corrections (MI355X_MICROARCH.md, HBM [CDNA4] and PMC notes):
  * FETCH_SIZE / WRITE_SIZE are KiB.  On gfx950 FETCH_SIZE = TCC_EA0_RDREQ x
    64 B while the L2 issues 128-B requests, so it reports half the bytes.
    When the request-size pass (TCC_EA0_RDREQ_32B/_64B/_128B) is present the
    read bytes are 32 n32 + 64 n64 + 128 n128 -- calibrated on
    k_meas_layout_copy, which reads exactly n_img Np^2 2 bytes (75008 images:
    9.830e9 B predicted, 128 x 7.681e7 = 9.832e9 B counted); otherwise FETCH is
    doubled.
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs: kernel cycles = value / 8.
  * SQ_INSTS_VALU counts wave instructions; a wave64 FP32 VALU instruction
    occupies its SIMD for 2 cycles, so VALU issue fraction =
    2 * SQ_INSTS_VALU / (1024 SIMDs * kernel cycles).
  * SQ_WAVE_CYCLES, SQ_ACTIVE_INST_*, SQ_WAIT_* count quad-cycles; ratios
    between them are unit-free.
  * FP32 flops counted = 64 lanes * (2 FMA + ADD + MUL + TRANS) wave
    instructions of the SQ_INSTS_VALU_*_F32 counters (when collected).  These
    count a PACKED instruction once, like its scalar form
    (tools/gpu/micro/flop_count.hip: 2^26 v_pk_fma_f32 -> 2^26 FMA_F32 on
    MI355X, profiles/r03_flop_count.txt), so for the packed-FP32 fused
    kernels fp32_flops is half of the flops executed by the packed part:
    fp32_flops_packed_upper (2x) bounds the executed flops from above.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from srchash import src_hash  # noqa: E402

N_SIMD = 1024


def short(name):
    """Kernel key: the Np 256 fused kernels keep their template instance
    (k_fused_iteration<NT,KS>, k_fused_dist<KS>: workgroups per patch) so a
    profile of a split-mode instance is never read as the one-workgroup
    kernel's."""
    import re
    m = re.search(r"k_fused_iteration<(\d+),\s*(\d+)>", name)
    if m:
        return f"k_fused_iteration<{m.group(1)},{m.group(2)}>"
    m = re.search(r"k_fused_dist<(\d+)>", name)
    if m:
        return f"k_fused_dist<{m.group(1)}>"
    for k in ("k_fused_mr", "k_fused_small", "k_fused_s90", "k_meas_layout", "k_meas_transpose_tiles", "k_meas_transpose",
              "k_fft_batch<true>", "k_fft_batch<false>", "k_crop_rows600", "k_crop_cols600", "k_crop_rows",
              "k_crop_cols", "k_colpass_wave", "k_colpass_tiled", "k_gather_rowifft_tiled",
              "k_rowfft_update_tiled", "k_rows1024_inv", "k_rows1024_fwd", "k_cols1024", "k_rows256_inv",
              "k_rows256_fwd", "k_cols256", "k_tile_rows",
              "k_tile_max_all", "k_row_max_all", "k_pupil_commit"):
        if k in name:
            return k
    return name.split("(")[0][:60]


def derive(c):
    d = {}
    cyc = c.get("GRBM_GUI_ACTIVE")
    if cyc:
        cyc /= 8.0
        d["kernel_cycles"] = cyc
        if "SQ_INSTS_VALU" in c:
            d["valu_issue_frac"] = 2.0 * c["SQ_INSTS_VALU"] / (N_SIMD * cyc)
        f32 = [c.get(k) for k in ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
                                  "SQ_INSTS_VALU_TRANS_F32")]
        if all(v is not None for v in f32):
            fl = 64.0 * (2 * f32[0] + f32[1] + f32[2] + f32[3])
            d["fp32_flops"] = fl
            d["fp32_flops_packed_upper"] = 2.0 * fl
            d["fp32_flops_per_cycle_frac"] = fl / (N_SIMD * 64.0 * cyc)
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY",
                  "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in c:
                d[k.lower().replace("sq_", "") + "_per_wave_cycle"] = c[k] / wc
    if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c:
        d["lds_bank_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    return d


def main():
    src, out = sys.argv[1], sys.argv[2]
    acc = defaultdict(lambda: defaultdict(list))
    perm = []  # (work-items, FETCH bytes) per k_meas_layout dispatch
    if src.endswith(".json"):  # re-reduce an earlier output (its raw means and stamp)
        with open(src) as fh:
            prev = json.load(fh)
        raw, stamp = prev["raw_per_launch"], prev["src_hash"]
        disp = prev.get("dispatches", {})
        iters = prev.get("bench_iterations", 1)
    else:
        iters = 1
        for f in sorted(glob.glob(os.path.join(src, "*", "**", "*counter_collection.csv"), recursive=True)):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = short(r["Kernel_Name"])
                    v = float(r["Counter_Value"])
                    acc[k][r["Counter_Name"]].append(v)
                    if k == "k_meas_layout" and r["Counter_Name"] == "FETCH_SIZE" and "Grid_Size" in r:
                        perm.append((int(r["Grid_Size"]), v * 1024.0))
        raw = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
        # dispatches of each kernel in the profiled run (one row per dispatch
        # in the FETCH_SIZE pass): the general path's per-LED kernels run once
        # per patch group, so bench.py turns per-dispatch bytes into bytes per
        # LED step of the whole context with them
        disp = {k: len(d["FETCH_SIZE"]) for k, d in acc.items() if "FETCH_SIZE" in d}
        stamp = src_hash()
    res = {"src_hash": stamp, "raw_per_launch": raw, "per_launch_hbm_bytes": {}, "read_scale": {},
           "derived": {}, "dispatches": disp,
           # iterations of the profiled bench run (tools/gpu/prof_counters.sh: 1)
           "bench_iterations": int(os.environ.get("PMC_BENCH_ITERS", iters))}
    if perm and "k_meas_layout" in raw and "TCC_EA0_RDREQ_128B" in raw["k_meas_layout"]:
        # k_meas_layout_copy<256,16,64>: 4 blocks of 256 threads per Np 256 image (128 KiB read)
        known = sum(g // 1024 * 256 * 256 * 2.0 for g, _ in perm) / len(perm)
        r = raw["k_meas_layout"]
        res["layout_known_read_bytes"] = known
        res["layout_counted_read_bytes"] = 128.0 * r["TCC_EA0_RDREQ_128B"] + 64.0 * r["TCC_EA0_RDREQ_64B"]
    for k, d in raw.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            if all(c in d for c in ("TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_128B")):
                rd = 32.0 * d["TCC_EA0_RDREQ_32B"] + 64.0 * d["TCC_EA0_RDREQ_64B"] + 128.0 * d["TCC_EA0_RDREQ_128B"]
                res["read_scale"][k] = rd / (d["FETCH_SIZE"] * 1024.0) if d["FETCH_SIZE"] else None
            else:
                rd = d["FETCH_SIZE"] * 1024.0 * 2.0
                res["read_scale"][k] = 2.0
            res["per_launch_hbm_bytes"][k] = rd + d["WRITE_SIZE"] * 1024.0
        dv = derive(d)
        if dv:
            res["derived"][k] = dv
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({"src_hash": res["src_hash"], "per_launch_hbm_bytes": res["per_launch_hbm_bytes"],
                      "derived": res["derived"]}, indent=1))


if __name__ == "__main__":
    main()
