"""A small synthetic dataset directory in the reference's on-disk format
(dataset JSON + iLED_<n>.tif 16-bit frames), shared by the loader and CLI
tests.  Frames are random uint16 with a per-frame background level, so the
background windows, the bgThresh clamp and the darkfield divide all act.
"""
from __future__ import annotations

import json
import os

import numpy as np

from fpm_amd import host

KEYS = {
    "filePrefix": "iLED_", "fileExtension": ".tif", "cropSizeX": 32, "pixelSize": 6.5,
    "objectiveMag": 8.1485, "objectiveNA": 0.1, "maxIlluminationNA": 0.2, "lambda": 0.6292,
    "cropX": 20, "cropY": 12, "bk1cropX": 1, "bk1cropY": 62, "bk2cropX": 70, "bk2cropY": 62,
    "bgThresh": 3000, "darkfieldExpMultiplier": 3, "delta1": 10, "delta2": 3,
    "arrayRotation": 0, "flipDatasetX": False, "flipDatasetY": False,
}
FRAME = (96, 104)        # height, width
N_FILES = 293            # LED numbers 1..N_FILES present on disk (all of dogStomach)


def make_dataset(root: str, seed: int = 7, keys: dict | None = None) -> dict:
    """Write dataset.json + frames under `root`; returns the keys and frames
    ({led number: uint16 [H][W]})."""
    os.makedirs(root, exist_ok=True)
    k = dict(KEYS, **(keys or {}))
    k["datasetRoot"] = root.rstrip("/") + "/"
    rng = np.random.default_rng(seed)
    frames = {}
    for led in range(1, N_FILES + 1):
        bg = int(rng.integers(200, 3000))          # some frames clamp at bgThresh
        f = bg + rng.integers(0, 3000, FRAME)
        f[10:60, 15:70] += rng.integers(0, 20000, (50, 55))   # object region over the crops
        f = np.clip(f, 0, 65535).astype(np.uint16)
        frames[led] = f
        host.write_tiff16(os.path.join(root, f"iLED_{led}.tif"), f)
    text = host.dataset_json(k, host.dogstomach_led_table())
    with open(os.path.join(root, "dataset.json"), "w") as fh:
        fh.write(text)
    return dict(keys=k, frames=frames, json=os.path.join(root, "dataset.json"))


def dump_keys(k: dict) -> str:
    return json.dumps(k, sort_keys=True)
