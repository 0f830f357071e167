"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes to per-launch HBM
bytes per kernel (bench.py's roofline.traffic).

usage: python tools/pmc_to_json.py <pmc dir with p*/run_counter_collection.csv> <out.json>

Units and corrections (MI355X_MICROARCH.md, HBM [CDNA4]): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of 16-B/lane
coalesced reads and other widths are uncalibrated.  k_permute_meas reads and
writes exactly n_img * Np^2 * 2 bytes with 2-B/lane row reads -- the access
width of the fused kernel's measurement stream -- so its FETCH ratio is used
as the read calibration for k_fused_iteration; k_fft_batch (8-B/lane) uses the
guide's x2.  Raw values are kept next to the corrected ones.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    for k in ("k_fused_iteration", "k_permute_meas", "k_fft_batch<true>", "k_fft_batch<false>", "k_crop_rows",
              "k_crop_cols"):
        if k in name:
            return k
    return name[:60]


def main():
    src, out = sys.argv[1], sys.argv[2]
    acc = defaultdict(lambda: defaultdict(list))
    perm = []  # (work-items, FETCH bytes) per k_permute_meas dispatch
    for f in glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]) * 1024.0)
                if k == "k_permute_meas" and r["Counter_Name"] == "FETCH_SIZE":
                    perm.append((int(r["Grid_Size"]), float(r["Counter_Value"]) * 1024.0))
    raw = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
    res = {"raw_bytes_per_launch": raw, "per_launch_hbm_bytes": {}, "read_scale": {}}
    # calibration from the permutation kernel: known bytes read per launch
    # = grid_blocks(y) * Np^2 * 2 ; its grid is (Np/64 * 256 threads) x n_img
    cal = None
    if perm:
        # grid (Np/64, n_img) x 256 threads: work-items = 4 * 256 * n_img at Np 256
        np_ = 256
        known = sum(g // (np_ // 64 * 256) * np_ * np_ * 2.0 for g, _ in perm)
        cal = known / sum(v for _, v in perm)
        res["permute_known_read_bytes"] = known
    for k, d in raw.items():
        if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            continue
        scale = cal if (k == "k_fused_iteration" and cal) else 2.0
        res["read_scale"][k] = scale
        res["per_launch_hbm_bytes"][k] = d["FETCH_SIZE"] * scale + d["WRITE_SIZE"]
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
