"""Summarise a same-box A/B run (tools/gpu/ab_multi.sh output directories).

usage: python tools/ab_summary.py gpurun_out/<tag>/<workload> [...]
prints one line per bench json: workload, variant+round, LED-updates/s,
ms per step, LED-update kernel ms per launch, then the per-variant medians.
"""
import json
import os
import re
import statistics
import sys

for d in sys.argv[1:]:
    per = {}
    for f in sorted(os.listdir(d)):
        if not f.endswith(".json"):
            continue
        j = json.load(open(os.path.join(d, f)))
        v = re.sub(r"\d+$", "", f[:-5])
        per.setdefault(v, []).append(j["led_ms_per_step"])
        print(os.path.basename(d), f[:-5], j["value"], j["ms_per_step"], j["led_ms_per_step"])
    for v, xs in per.items():
        print(os.path.basename(d), v, "median led ms", statistics.median(xs))
