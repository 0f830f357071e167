#!/usr/bin/env python3
"""Benchmark: LED-updates/s of the MI355X FPM solver (BASELINE.json metric).

Workload (SURVEY.md 8(d) metric config): dataset_dogStomach optics
(6.5 um pixel, mag 8.1485, objNA 0.1, lambda 0.6292), all 293 LEDs of its
holeCoordinates array (maxIlluminationNA raised to 0.6), cropSizeX Np = 256
-> resImprovementFactor 3, L = 768, naRadius 33, delta1 = 10, delta2 = 3,
and north_star's fixed field of 256 independent patches: at N GPUs it is
statically sharded over the ranks (fpm_amd.parallel.shard_range: 256 / 128 /
64 / 32 patches per rank at N = 1 / 2 / 4 / 8; strong scaling), synthetic
seeded forward-model stacks resident in HBM.  `--weak` gives every rank its
own --patches (BASELINE config 4: `--patches-total 1024`, 128 per rank at 8).

One step = one runFPM iteration (fpmMain.cpp:345-482) over every patch:
293 sequential LED updates per patch plus the per-iteration objCrop IDFT.
value = field patches x LEDs x steps / (max over ranks of the timed wall
time).  Launch: `python bench.py` (1 GPU) or torch.distributed.run with
--nproc-per-node N (one rank per GPU, RCCL).  After the timed region, ranks
> 0 send their objCrop tiles to rank 0 with one RCCL gather (the stitched-field
exchange of SURVEY.md 8(e)); its time is reported separately, not in value.
`--backend gloo` rehearses the N > 1 path (barrier, max-over-ranks timing,
gather) with several ranks sharing one GPU; bench numbers use nccl (RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fpm-opencv_amd", "python"), os.path.join(ROOT, "tests")]

METRIC = "LED-updates/sec (patch·LED/s), 256² patch × 293 LEDs; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
F32_PEAK_TFLOPS = 157.3    # FP32 vector == FP32 MFMA dense peak (MI355X_MICROARCH.md)
F32_FLOPS_PER_CYCLE = 1024 * 64  # 256 CUs x 4 SIMDs x 64 f32 flops per cycle: the peak at any clock

DOG_KEYS = {"cropSizeX": 256, "pixelSize": 6.5, "objectiveMag": 8.1485, "objectiveNA": 0.1,
            "maxIlluminationNA": 0.6, "lambda": 0.6292, "delta1": 10, "delta2": 3,
            "arrayRotation": 0, "flipDatasetX": False, "flipDatasetY": False}


def metric_geometry(np_=256, max_na=0.6):
    from fpm_amd import host
    keys = dict(DOG_KEYS, cropSizeX=np_, maxIlluminationNA=max_na)
    ds = host.Dataset(json_text=host.dataset_json(keys, host.dogstomach_led_table(), trailing_comma=True))
    ds.set_present(range(1, 294))
    n = ds.geometry()
    cfg = ds.config()
    x0, y0 = ds.crops()
    return dict(np_=cfg.np, L=cfg.nlarge, r=cfg.na_radius, d1=cfg.delta1, d2=cfg.delta2, n_led=n,
                order_leds=ds.order(), x0=x0, y0=y0)


WORKLOADS = {
    "metric": "dataset_dogStomach optics, 293 LEDs (maxIlluminationNA 0.6), Np=256, L=768, naRadius 33, "
              "one runFPM iteration per step",
    "c3": "dataset_dogStomach.json literal (Np=200, maxIlluminationNA 0.4: 157 LEDs, L=600, naRadius 26), "
          "one runFPM iteration per step",
    "c5": "config 5: Np=1024, L=4096 spectrum in fp16, naRadius 333, 512-LED synthetic grid, "
          "one runFPM iteration per step",
    "c2": "config 2: dataset_mono.json with the dome fallback (Np=90, L=360, naRadius 30, 193 LEDs), "
          "64 patches, one runFPM iteration per step",
    "c2np256": "config 2 geometry at Np=256: dataset_mono.json with the dome fallback, cropSizeX 256 (L=1024, "
               "naRadius 84, 193 LEDs; general path on the Np 256 register kernels), 64 patches, one runFPM "
               "iteration per step",
}


def config_geometry(name, np_=256):
    """Geometry of the workload `name` (BASELINE.json configs):
      metric  configs[1]-style headline: dogStomach optics, Np 256, 293 LEDs
      c3      configs[2] literal dataset_dogStomach.json: Np 200, maxNA 0.4 ->
              L 600, naRadius 26, 157 LEDs (general path, mixed radix)
      c2      configs[1]: dataset_mono.json + dome fallback (the config-1
              geometry: Np 90, L 360, r 30, 193 LEDs), 64 patches (general path)
      c5      configs[4]: Np 1024, L 4096, naRadius 333 (mono optics at
              Np 1024), 512 LEDs of a synthetic square grid
              (23 x 23 at a 128-px k-space pitch, the 512 nearest the centre),
              fp16 spectrum storage
    Only `metric` is the headline bench line; the others are measured for
    DESIGN.md."""
    if name == "metric":
        return metric_geometry(np_)
    if name == "c3":
        return metric_geometry(200, max_na=0.4)
    if name == "c2":
        import numpy as np
        g = config1_geometry(np_)
        g["order_leds"] = np.arange(g["n_led"])
        return g
    if name == "c5":
        import numpy as np
        from tools.synth import grid_geometry
        Np, L = 1024, 4096
        x0, y0, order = grid_geometry(Np, L, 23, 128)
        keep = np.array(order[:512])
        return dict(np_=Np, L=L, r=333, d1=5, d2=10, n_led=512, order_leds=keep,
                    x0=np.asarray(x0)[keep], y0=np.asarray(y0)[keep])
    raise ValueError(name)


def algorithmic_flops_per_update(np_, nb, support_px):
    """Flops of the support-pruned update per LED-update (DESIGN.md 'Roofline'):
    5 N log2 N per executed 1-D DFT (nb row IDFTs, Np column IDFT+DFT pairs, nb
    row DFTs), 12 flops/px amplitude replacement, 60 flops per support pixel for
    the object + pupil updates."""
    import math
    lg = math.log2(np_)
    return 5.0 * np_ * lg * (2 * nb + 2 * np_) + 12.0 * np_ * np_ + 60.0 * support_px


def dense_flops_per_update(np_):
    """SURVEY.md 8(d) 'Algorithmic flops': two dense 2-D FFTs of Np^2 points
    (5 N log2 N each) + ~70 Np^2 element-wise flops per LED-update."""
    import math
    return 2 * 5.0 * np_ * np_ * math.log2(np_ * np_) + 70.0 * np_ * np_


def dense_bytes_per_update(np_):
    """SURVEY.md 8(d) dense definition: read I (2) + read/write O ROI (8+8) +
    read/write P (8+8) per ROI pixel = 34 Np^2.  Reported as a labelled
    dense-equivalent figure only: the fused kernel keeps T in LDS and P in
    registers, so these bytes never move."""
    return 34.0 * np_ * np_


def min_bytes_per_update(np_, support_px, meas_bytes=2):
    """Minimum HBM bytes one LED-update must move on the support-pruned path
    (the headline roofline): read the measurement I (meas_bytes per pixel,
    uint16 in the C-ABI layout) + read and write the spectrum O on the pupil
    support (8 + 8 bytes per support pixel).  The pupil, tile maxima and
    max|P| stay on chip for the whole launch (their per-launch bytes are
    below 0.1 %)."""
    return float(meas_bytes) * np_ * np_ + 16.0 * support_px


def load_pmc(path, kernel, n_led=None):
    """(per-launch HBM bytes, derived counter view, note) for `kernel` from a
    tools/pmc_to_json.py file -- only when its src_hash matches the current
    csrc tree, so a profile of older kernels is never reported as traffic."""
    from tools.srchash import src_hash
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception as e:  # noqa: BLE001
        return None, None, f"no counter profile ({type(e).__name__})"
    if d.get("src_hash") != src_hash():
        return None, None, f"counter profile {os.path.basename(path)} is for csrc {d.get('src_hash')}, " \
                           f"tree is {src_hash()}: not reported"
    pl = d.get("per_launch_hbm_bytes", {})
    if kernel == "general_led_step":
        # one LED step of the general path = its per-LED launches (the Np 1024
        # / Np 256 register kernels or the LDS kernels, then the tile maxima).
        # Each kernel runs once per patch group and LED (the commit of the
        # register paths once per group and iteration): the counter file's
        # per-dispatch bytes times its dispatches over the profiled run's LED
        # steps (tools/gpu/prof_counters.sh: one iteration of n_led LEDs)
        ks = [k for k in ("k_rows1024_inv", "k_cols1024", "k_rows1024_fwd", "k_rows256_inv", "k_cols256",
                          "k_rows256_fwd", "k_gather_rowifft_tiled",
                          "k_colpass_wave", "k_colpass_tiled", "k_rowfft_update_tiled", "k_tile_rows",
                          "k_pupil_commit") if k in pl]
        disp = d.get("dispatches", {})
        steps = n_led * d.get("bench_iterations", 1) if n_led else 0
        if ks and steps and all(k in disp for k in ks):
            tot = sum(pl[k] * disp[k] for k in ks) / steps
            how = f"sum of per-dispatch bytes x dispatches / {steps} LED steps of {', '.join(ks)}"
        else:
            tot = sum(pl[k] for k in ks) if ks else None
            how = f"sum of per-dispatch bytes of {', '.join(ks)} (one patch group's LED step)"
        return (tot, {k: d.get("derived", {}).get(k) for k in ks},
                f"{os.path.basename(path)} (csrc {d['src_hash']}; {how})")
    return (pl.get(kernel), d.get("derived", {}).get(kernel),
            f"{os.path.basename(path)} (csrc {d['src_hash']})")


def kernel_name(info):
    """Name of the LED-update kernel the context launches (rocprof / pmc key):
    the template instance (threads and workgroups per patch, fpm_info) for
    the Np 256 kernels."""
    import fpm_amd
    if info.fused_kernel == fpm_amd.KERNEL_FUSED_NP256:
        return f"k_fused_iteration<{info.threads_per_wg or 512},{info.wg_per_patch}>"
    if info.fused_kernel == fpm_amd.KERNEL_FUSED_NP256_DIST:
        return f"k_fused_dist<{info.wg_per_patch}>"
    return fpm_amd.KERNEL_NAMES[info.fused_kernel]


def default_pmc(args, info):
    """Counter profile of this workload's kernel (tools/gpu/prof_counters.sh
    writes one per workload: profiles/pmc_<config>_<kernel>.json)."""
    k = kernel_name(info).replace("<", "_").replace(">", "").replace(",", "_")
    return os.path.join(ROOT, "profiles", f"pmc_{args.config}_{k}.json")


def fp32_roof_updates_per_s(np_, nb, support_px):
    """LED-updates/s at the FP32 peak: the ceiling of a compute-bound kernel
    on the algorithmic flop model (7.61 MFLOP at the metric)."""
    return F32_PEAK_TFLOPS * 1e12 / algorithmic_flops_per_update(np_, nb, support_px)


def roofline_line(geo, info, per_launch_ms, per_launch_updates, pmc_path, clock=None):
    """roofline object of the bench line for the context's LED-update kernel.

    The fused kernels keep T in LDS and P in registers: they move the
    measurement plus the spectrum on the support (1.02x that by counters at
    the metric), so the HBM roof is far away and what binds is FP32 VALU issue
    (SQ counters in `counters`).  `bound` is therefore "valu": `achieved` is
    the algorithmic flop rate (support-pruned transform model) against the
    157.3 TFLOP/s FP32 peak.  The HBM view (minimum bytes, SURVEY.md 8(d)'s
    support-restricted 2 Np^2 + 32 |S| and dense 34 Np^2 figures) sits in
    `hbm`; `ceiling` states what the north-star '>= 70 % of HBM' target maps
    to on this kernel (the FP32 roof reached first)."""
    np_, S = geo["np_"], info.support_px
    t = per_launch_ms * 1e-3
    kname = kernel_name(info)
    traffic, counters, pmc_note = load_pmc(pmc_path, kname, geo.get("n_led"))
    flops = algorithmic_flops_per_update(np_, info.box, S) * per_launch_updates
    achieved_tf = flops / t / 1e12
    min_bytes = min_bytes_per_update(np_, S) * per_launch_updates
    sup_bytes = (2.0 * np_ * np_ + 32.0 * S) * per_launch_updates
    dense_bytes = dense_bytes_per_update(np_) * per_launch_updates
    roof_u = fp32_roof_updates_per_s(np_, info.box, S)
    # the counters' FP32 view: SQ_INSTS_VALU_*_F32 count a packed
    # instruction once, so the counted flops are a lower bound of the executed
    # ones and twice them an upper bound; the 5 N log2 N model (frac above)
    # exceeds even that upper bound (radix-16 transforms need fewer operations)
    cyc = clock["kernel_cycles_per_launch"] if clock and clock.get("kernel_cycles_per_launch") else None
    fl_cnt = counters.get("fp32_flops") if counters else None
    counted = None
    if fl_cnt:
        counted = dict(
            fp32_frac_counted=round(fl_cnt / t / 1e12 / F32_PEAK_TFLOPS, 4),
            fp32_frac_counted_packed_upper=round(2 * fl_cnt / t / 1e12 / F32_PEAK_TFLOPS, 4),
            counted_flops_per_launch=fl_cnt, model_over_packed_upper=round(flops / (2 * fl_cnt), 3),
            note="SQ_INSTS_VALU_*_F32 count a v_pk_* instruction once: counted flops bound the executed ones "
                 "from below, 2x counted from above; fractions of the 157.3 TF peak at the measured launch time")
        if cyc:
            counted["fp32_frac_counted_per_cycle"] = round(fl_cnt / (cyc * F32_FLOPS_PER_CYCLE), 4)
    hbm = dict(achieved=round(min_bytes / t / 1e9, 1), peak=HBM_PEAK_GBS, unit="GB/s",
               frac=round(min_bytes / t / 1e9 / HBM_PEAK_GBS, 4),
               bytes_model=f"2*Np^2 (uint16 I) + 16*|S| (O read+write on the {S}-px support) per LED-update "
                           f"x {per_launch_updates} LED-updates per launch",
               algorithmic_bytes_per_launch=min_bytes,
               support_restricted_frac=round(sup_bytes / t / 1e9 / HBM_PEAK_GBS, 4),
               support_restricted_note="SURVEY.md 8(d): 2*Np^2 + 32*|S| B per LED-update",
               dense_equivalent_frac=round(dense_bytes / t / 1e9 / HBM_PEAK_GBS, 4),
               dense_note="SURVEY.md 8(d) dense 34*Np^2 definition; bytes this design never moves",
               measured_GBs=(round(traffic / t / 1e9, 1) if traffic else None),
               traffic_over_algorithmic=(round(traffic / min_bytes, 3) if traffic else None))
    return dict(bound="valu", achieved=round(achieved_tf, 2), peak=F32_PEAK_TFLOPS, unit="TFLOP/s",
                frac=round(achieved_tf / F32_PEAK_TFLOPS, 4),
                fp32_frac_counted=counted["fp32_frac_counted"] if counted else None,
                frac_per_cycle=(round(flops / (cyc * F32_FLOPS_PER_CYCLE), 4) if cyc else None),
                frac_per_cycle_note="model flops / (in-kernel cycles per launch x 65536 f32 flops per cycle): "
                                    "the fraction independent of the box's clock",
                fp32_counted=counted, traffic=traffic,
                kernel=kname, launch_ms=round(per_launch_ms, 4),
                flops_model=f"5 N log2 N per executed pruned 1-D DFT (nb={info.box} row IDFTs + Np column "
                            f"IDFT/DFT pairs + nb row DFTs) + 12 flop/px amplitude + 60 flop per support px, "
                            f"x {per_launch_updates} LED-updates per launch",
                algorithmic_flops_per_launch=flops,
                hbm=hbm,
                ceiling=dict(fp32_roof_led_updates_per_s=round(roof_u, 1),
                             hbm_frac_at_fp32_roof=round(roof_u * min_bytes_per_update(np_, S) / 1e9 / HBM_PEAK_GBS, 4),
                             note="north_star asks >= 70 % of the HBM roof; on the minimum bytes that needs "
                                  "more flops than the FP32 peak, so the FP32 roof is the reachable ceiling"),
                traffic_source=pmc_note, counters=counters)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """Cores this job may use on the host: the CPU affinity mask, capped by a
    cgroup CPU quota when one is set (a GPU box shares its host between
    jobs; nproc reports the whole machine).  Returns (cores, description)."""
    n_aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    cores = min(n_aff, quota) if quota else n_aff
    return cores, f"nproc {os.cpu_count()}, affinity {n_aff}, cgroup quota {quota or 'none'}"


def config1_geometry(np_=90):
    """BASELINE configs[0]: dataset_mono.json with the 508-LED dome fallback
    (geometry and order from the reference's own jsoncpp probe,
    tests/golden/geometry_mono_dome.json): Np 90, L 360, r 30, 193 LEDs;
    np_=256: the same dataset at cropSizeX 256 (geometry_mono_dome_np256.json:
    L 1024, r 84, 193 LEDs)."""
    import numpy as np
    fx = {90: "geometry_mono_dome.json", 256: "geometry_mono_dome_np256.json"}[np_]
    with open(os.path.join(ROOT, "tests", "golden", fx)) as f:
        p = json.load(f)["probe"]
    leds = {l["led"]: l for l in p["leds"]}
    order = p["sorted_indices"]
    return dict(np_=p["np"], L=p["nlarge"], r=p["na_radius"], d1=p["delta1"], d2=p["delta2"], n_led=len(order),
                x0=np.array([leds[n]["crop_x0"] for n in order], np.int32),
                y0=np.array([leds[n]["crop_y0"] for n in order], np.int32))


def cpu_baseline(geo, stack_host, threads, cores_note):
    """C++ fp64 reference-faithful restatement (oracle/liboracle.so, 'port'),
    one patch per thread, all LEDs, one iteration; wall-clock.  SURVEY.md 8(d)
    asks for the rate on all host cores (one patch per thread, patches are
    independent), on one core, and for config 1 (dataset_mono, Np 90, 1
    patch, 5 iterations) on one core: all three are measured, `value` is the
    first."""
    import numpy as np
    import oracle_lib
    from tools.synth import make_stack
    order = np.arange(geo["n_led"], dtype=np.int32)

    def timed(stk, g, nthr, iters=1):
        o = np.arange(g["n_led"], dtype=np.int32)
        t0 = time.perf_counter()
        oracle_lib.run_fpm_batch(stk, o, g["x0"], g["y0"], g["np_"], g["L"], g["r"],
                                 g["d1"], g["d2"], iters, nthr, outputs=False)
        return time.perf_counter() - t0

    dt = timed(stack_host, geo, threads)
    dt1 = timed(np.ascontiguousarray(stack_host[:, :1]), geo, 1)
    c1 = config1_geometry()
    s1 = make_stack(c1["np_"], c1["L"], c1["r"], c1["x0"], c1["y0"], n_patch=1, seed=20261015)
    dtc1 = timed(s1, c1, 1, iters=5)
    B = stack_host.shape[1]
    del order
    return dict(value=round(B * geo["n_led"] / dt, 1), unit="LED-updates/s", cores=threads, kind="port",
                single_core_value=round(geo["n_led"] / dt1, 1), cpu_model=cpu_model(), host_cores=cores_note,
                config1_single_core=dict(value=round(5 * c1["n_led"] / dtc1, 1), unit="LED-updates/s",
                                         seconds=round(dtc1, 2),
                                         sample="BASELINE configs[0]: dataset_mono + dome fallback, Np 90, L 360, "
                                                f"{c1['n_led']} LEDs, 1 patch, 5 iterations, 1 thread"),
                sample=f"{B} patches x {geo['n_led']} LEDs x 1 iteration, Np={geo['np_']} L={geo['L']}, "
                       f"complex128, one patch per thread on {threads} threads, {dt:.1f} s wall; "
                       f"single core: 1 patch x {geo['n_led']} LEDs, {dt1:.1f} s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)  # ~0.2 s of GPU time at the metric config
    ap.add_argument("--warmup", type=int, default=5)  # the first launches after setup run slower (clock ramp)
    ap.add_argument("--patches", type=int, default=0,
                    help="--weak: patches per GPU (0: 256, 8 for --config c5, 64 for c2)")
    ap.add_argument("--patches-total", type=int, default=0,
                    help="strong scaling: one field of T patches sharded over the ranks (parallel.shard_range), "
                         "gathered and stitched on rank 0 after the timed region (0: north_star's 256-patch field "
                         "for --config metric, weak scaling for the other configs)")
    ap.add_argument("--weak", action="store_true", help="weak scaling: every rank owns --patches patches")
    ap.add_argument("--np", type=int, default=0,
                    help="patch size: 256 for --config metric (other Np: dogStomach optics at that size), "
                         "90 for c2 (256: the same dataset at cropSizeX 256, naRadius 84, general path)")
    ap.add_argument("--config", default="metric", choices=["metric", "c2", "c3", "c5"],
                    help="workload (config_geometry); only 'metric' is the headline line")
    ap.add_argument("--fp16", action="store_true", help="fp16 spectrum storage (default for --config c5)")
    ap.add_argument("--path", default="auto", choices=["auto", "general", "fused"])
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this job may use (host_cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--pmc", default="", help="counter profile (tools/pmc_to_json.py); default: the workload's "
                                              "profiles/pmc_<config>_<kernel>.json")
    ap.add_argument("--pcie", action="store_true",
                    help="also time the host->device stack upload (fpm_upload_stack from host memory); "
                         "reported beside the line as upload, never in value")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path with several ranks on one GPU (CPU collectives)")
    ap.add_argument("--data", default="model", choices=["model", "random"],
                    help="random: uniform uint16 stack (profiling runs only; not a bench number)")
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # `bench.py --gpus N` without a launcher: start one rank per GPU under
        # torch.distributed.run as a CHILD process (nothing here has touched
        # the GPU yet) and exit with its status -- never a 1-GPU number
        # labelled as N
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        raise SystemExit(subprocess.call(cmd))
    if world_env is not None and int(world_env) != args.gpus and "--gpus" in " ".join(sys.argv):
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world_env}: launch one rank per GPU")

    import numpy as np
    import torch
    import torch.distributed as dist
    import fpm_amd
    from tools.synth_torch import make_stack

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and world > 1 and local >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {ndev} GPUs (use --backend gloo to rehearse)")
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    cdev = torch.device("cuda", local) if args.backend == "nccl" else torch.device("cpu")
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    if not args.np:
        args.np = 90 if args.config == "c2" else 256
    geo = config_geometry(args.config, args.np)
    fp16 = args.fp16 or args.config == "c5"
    if args.patches_total <= 0 and not args.weak and args.config == "metric":
        args.patches_total = 256  # north_star: a 256-patch x 293-LED stack at 1/2/4/8 GPUs
    strong = args.patches_total > 0 and not args.weak
    if strong:
        # strong scaling: one fixed field of T patches, contiguous shards
        # (parallel.shard_range); data seeded per global patch
        from fpm_amd import parallel
        lo, hi = parallel.shard_range(args.patches_total, world, rank)
        B, seed, poff = hi - lo, 20261015, lo
        if B < 1:
            raise SystemExit(f"rank {rank}: empty shard of {args.patches_total} patches over {world} ranks")
    else:
        B = args.patches if args.patches > 0 else {"c5": 8, "c2": 64}.get(args.config, 256)
        seed, poff = 20261015 + 1000 * rank, 0
    if args.data == "random":
        g = torch.Generator(device="cuda")
        g.manual_seed(rank)
        stack = torch.randint(0, 40000, (geo["n_led"], B, geo["np_"], geo["np_"]), generator=g, device="cuda",
                              dtype=torch.int32).to(torch.int16)
    else:
        stack = make_stack(geo["np_"], geo["L"], geo["r"], geo["x0"], geo["y0"], B,
                           seed=seed, device="cuda", patch_offset=poff)
    torch.cuda.synchronize()
    path = {"auto": fpm_amd.PATH_AUTO, "general": fpm_amd.PATH_GENERAL, "fused": fpm_amd.PATH_FUSED}[args.path]
    prob = fpm_amd.Problem(geo["np_"], geo["L"], np.arange(geo["n_led"]), geo["x0"], geo["y0"], geo["r"],
                           geo["d1"], geo["d2"], n_patch=B, path=path,
                           flags=fpm_amd.FLAG_SPEC_FP16 if fp16 else 0)
    solver = fpm_amd.Solver(prob, device=local)
    # one-time setup, reported beside the line (never in value): the device
    # stack copy incl. the fused path's measurement permutation, and fpm_init
    torch.cuda.synchronize()
    s0 = time.perf_counter()
    solver.upload_device(stack.data_ptr())
    solver.synchronize()
    s1 = time.perf_counter()
    solver.init()
    solver.synchronize()
    setup = dict(upload_and_permute_ms=round((s1 - s0) * 1e3, 2),
                 init_ms=round((time.perf_counter() - s1) * 1e3, 2),
                 note="once per reconstruction, excluded from value")
    info = solver.info()

    for _ in range(args.warmup):
        solver.run(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    led_ms = 0.0
    launches = 0
    crop_ms = 0.0
    clk_cyc = clk_ms = 0.0
    clk_n = 0
    for _ in range(args.steps):
        solver.run(1)
        t = solver.timing()
        led_ms += t.led_ms
        launches += t.led_launches
        crop_ms += t.objcrop_ms
        k = solver.clock()  # block 0's s_memtime / s_memrealtime over the launch (fused path)
        clk_cyc += k.cycles_per_launch * k.launches
        clk_ms += k.ms_per_launch * k.launches
        clk_n += k.launches
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    updates = (args.patches_total if strong else B * world) * geo["n_led"] * args.steps
    value = updates / elapsed
    per_launch_ms = led_ms / max(launches, 1)
    fused = info.path == fpm_amd.PATH_FUSED
    per_launch_updates = B * geo["n_led"] if fused else B
    clock = None
    if clk_n:
        clock = dict(clock_mhz=round(clk_cyc / (clk_ms * 1e-3) / 1e6, 1),
                     kernel_cycles_per_launch=round(clk_cyc / clk_n, 0),
                     probe_ms_per_launch=round(clk_ms / clk_n, 4), launches=clk_n,
                     note="block 0 of each LED-update launch: s_memtime (shader cycles) and s_memrealtime "
                          "(100 MHz) at entry and after its last LED; a slow box reads as a lower clock at the "
                          "same cycles (fpm_get_clock)")
    roofline = roofline_line(geo, info, per_launch_ms, per_launch_updates, args.pmc or default_pmc(args, info), clock)

    gather = None
    if world > 1 and not args.no_gather:
        # the final exchange of SURVEY.md 8(e): every rank's objCrop tiles to
        # rank 0 in one gather (RCCL over xGMI), then -- for a fixed field --
        # the stitched high-resolution field on rank 0's GPU; timed beside
        # the line, never inside value
        from fpm_amd import parallel
        L = geo["L"]
        mine = torch.empty((B, L, L, 2), dtype=torch.float32, device="cuda")
        solver.download_objcrop_device(mine.data_ptr())
        torch.cuda.synchronize()
        mine = mine.to(cdev)
        if world > 1:
            dist.barrier()
        g0 = time.perf_counter()
        tiles = parallel.gather_tiles(mine, dist, dst=0) if world > 1 else mine
        torch.cuda.synchronize()
        gms = (time.perf_counter() - g0) * 1e3
        gather = dict(ms=round(gms, 2), GB_to_rank0=round(mine.numel() * 4 * (world - 1) / 1e9, 3))
        if strong and rank == 0:
            grid = parallel.field_grid(args.patches_total)
            s0 = time.perf_counter()
            field = parallel.stitch(tiles, grid)
            torch.cuda.synchronize()
            gather.update(stitch_ms=round((time.perf_counter() - s0) * 1e3, 2),
                          field=f"{grid[0]}x{grid[1]} patches -> {field.shape[0]}x{field.shape[1]} complex64")
            del field
        del tiles

    upload = None
    if args.pcie and rank == 0:
        # the same stack from pinned host memory through the C ABI's host entry
        # point (PCIe + the fused-layout permutation), once per reconstruction
        host_stack = stack.cpu().pin_memory()
        torch.cuda.synchronize()
        u0 = time.perf_counter()
        import ctypes
        rc = fpm_amd._lib.fpm_upload_stack(solver._h, ctypes.cast(host_stack.data_ptr(),
                                                                   ctypes.POINTER(ctypes.c_uint16)))
        torch.cuda.synchronize()
        us = time.perf_counter() - u0
        if rc != 0:
            raise RuntimeError(fpm_amd._lib.fpm_last_error().decode())
        gb = host_stack.numel() * 2 / 1e9
        iters_equiv = us / (elapsed / args.steps)
        upload = dict(s=round(us, 3), GB=round(gb, 2), GBps=round(gb / us, 1),
                      iterations_equivalent=round(iters_equiv, 1),
                      led_updates_per_s_incl_upload_1_iteration=round(B * geo["n_led"] / (us + elapsed / args.steps), 1))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "metric":
        cores, note = host_cores()
        threads = args.cpu_threads or min(cores, B)
        host_stack = stack[:, :threads].contiguous().cpu().numpy().view(np.uint16)
        cpu = cpu_baseline(geo, host_stack, threads, note)

    step_ms = elapsed / args.steps * 1e3
    setup_ms = setup["upload_and_permute_ms"] + setup["init_ms"]
    per_rank = B * geo["n_led"]
    setup["led_updates_per_s_incl_setup"] = {
        f"{k}_iteration{'s' if k > 1 else ''}": round(k * per_rank / ((setup_ms + k * step_ms) * 1e-3), 1)
        for k in (1, 5)}
    setup["note"] = ("once per reconstruction (device-resident stack copied + permuted, fpm_init), excluded from "
                     "value; led_updates_per_s_incl_setup = one reconstruction of k iterations on this rank "
                     "including it")
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "LED-updates/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
            # the no-flag default changed in round 4 (weak, 256 patches per rank in rounds 1-3 -> strong,
            # one 256-patch field): multi-GPU lines of r01-r03 and r04+ are not comparable
            "scaling_note": "default since round 4: strong scaling of north_star's 256-patch field; "
                            "rounds 1-3 defaulted to weak scaling (256 patches per rank); --weak reproduces that",
            "dtype": "f32 (fp16 spectrum storage)" if fp16 else "f32",
            "data": ("synthetic: seeded FPM forward model (HR object, defocus pupil, Poisson noise), uint16"
                     if args.data == "model" else "random uint16 (profiling only)"),
            "config": {"workload": (WORKLOADS["c2np256"] if args.config == "c2" and args.np == 256 else
                                    WORKLOADS[args.config] if args.config != "metric" or args.np == 256 else
                                    f"dogStomach optics, Np={geo['np_']}, one runFPM iteration per step"),
                       "patches_per_gpu": B, "leds": int(geo["n_led"]), "np": int(geo["np_"]),
                       "patches_total": int(args.patches_total if strong else B * world),
                       "scaling_mode": (f"strong: one {args.patches_total}-patch field sharded over {world} rank(s)"
                                        if strong else f"weak: {B} patches per rank"),
                       "nlarge": int(geo["L"]), "na_radius": int(geo["r"]),
                       "path": "fused" if info.path == fpm_amd.PATH_FUSED else "general",
                       "kernel": kernel_name(info), "workgroups_per_patch": int(info.wg_per_patch),
                       "parallelism": f"patch-sharded x{world}"},
            "roofline": roofline,
            "clock_mhz": clock["clock_mhz"] if clock else None,
            "kernel_cycles_per_launch": clock["kernel_cycles_per_launch"] if clock else None,
            "clock": clock,
            "cpu_baseline": cpu,
            "setup": setup,
            "led_ms_per_step": round(led_ms / args.steps, 3),
            "objcrop_ms_per_step": round(crop_ms / args.steps, 3),
        }
        if gather:
            out["gather"] = gather
        if upload:
            out["upload"] = upload
        print(json.dumps(out), flush=True)
    solver.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
