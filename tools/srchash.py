"""Hash of the device-code sources a counter profile was measured on.

bench.py only reports `roofline.traffic` (and the SQ counter view) from
profiles/pmc_latest.json when the file's `src_hash` equals the hash of the
current fpm-opencv_amd/csrc tree, so a stale profile is never attributed to
changed kernels.

usage: python tools/srchash.py      -> prints the hash
"""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fpm-opencv_amd", "csrc")


def src_hash(csrc: str = CSRC) -> str:
    h = hashlib.sha256()
    for name in sorted(os.listdir(csrc)):
        p = os.path.join(csrc, name)
        if not os.path.isfile(p) or not name.endswith((".hip", ".hpp", ".cpp", ".h")):
            continue
        h.update(name.encode())
        with open(p, "rb") as f:
            h.update(f.read())
    # the compile flags decide the machine code too (round 5: the scheduler
    # strategy); the HIPFLAGS line of the Makefile is part of the stamp
    mk = os.path.join(os.path.dirname(csrc), "Makefile")
    if os.path.isfile(mk):
        with open(mk, "rb") as f:
            for line in f.read().split(b"\n"):
                if b"HIPFLAGS" in line or b"amdgpu-" in line or b"MMC_FILES" in line:
                    h.update(line)
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(src_hash())
