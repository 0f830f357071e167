"""Copy a GPU evidence run (tools/gpu/r03_prof.sh output under gpurun_out/<tag>)
into profiles/: bench lines as profiles/<round>_bench_<workload>.json, the
kernel-trace stats as profiles/<round>_kernel_stats_metric.csv, and each
workload's counter reduction as profiles/pmc_<config>_<kernel>.json (the file
bench.py's default_pmc reads; bench.py reports its traffic only while its
csrc hash matches the tree).

usage: python tools/collect_profiles.py gpurun_out/<tag> <round>
"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIG = {"metric": "metric", "c2": "c2", "c3": "c3", "c5": "c5", "pt128": "metric", "pt64": "metric",
          "pt32": "metric", "c2np256": "c2", "default_cmd": None}  # None: a bench line without counters


def led_kernel(pmc):
    """The workload's LED-update kernel key in a counter file (bench.py
    kernel_name): the fused kernel profiled, or the general path's LED step."""
    keys = json.load(open(pmc))["per_launch_hbm_bytes"].keys()
    fused = [k for k in keys if k.startswith("k_fused")]
    return fused[0] if len(fused) == 1 else "general_led_step"


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    for w, cfg in CONFIG.items():
        b = os.path.join(src, f"bench_{w}.json")
        pmc = os.path.join(src, f"pmc_{w}", "pmc.json")
        if os.path.exists(b):
            shutil.copy(b, os.path.join(prof, f"{rnd}_bench_{w}.json"))
        if cfg and os.path.exists(pmc):
            # the counter run of an evidence part may come without its bench
            # line (tools/gpu/r04_prof.sh runs in parts): key from the file
            kern = json.load(open(b))["config"]["kernel"] if os.path.exists(b) else led_kernel(pmc)
            k = kern.replace("<", "_").replace(">", "").replace(",", "_")
            shutil.copy(pmc, os.path.join(prof, f"pmc_{cfg}_{k}.json"))
            s = os.path.join(src, f"pmc_{w}", "pmc_summary.txt")
            if os.path.exists(s):
                shutil.copy(s, os.path.join(prof, f"{rnd}_pmc_summary_{w}.txt"))
    ks = os.path.join(src, "kernel_stats_metric.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(prof, f"{rnd}_kernel_stats_metric.csv"))


if __name__ == "__main__":
    main()
