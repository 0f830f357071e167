"""Generate tests/golden/geometry_*.json from the reference's own jsoncpp.

Runs oracle/_ref/ref_probe (oracle/ref_probe.cpp linked with the reference's
vendored jsoncpp, compiled in place from /root/reference/include/jsoncpp.cpp by
oracle/Makefile) on the shipped dataset JSONs.  Each fixture stores:
  keys     the JSON scalar keys (data: optics, crop, regularisers)
  trailing_comma  whether holeCoordinates ended with ", ]" in the source file
  probe    the probe's output: derived optics, per-LED position / NA / used /
           k-offsets / crop starts, sortedIndicies
The coordinates inside `probe.leds` are what the reference's jsoncpp returned
(asFloat), so tests can rebuild an equivalent dataset JSON without
/root/reference.  Run here (needs /root/reference); commit the outputs.
"""
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_probe")

CASES = [
    # name, json file, n_present, maxNA override, cropSizeX override
    ("dogStomach_literal", "dataset_dogStomach.json", 293, None, None),
    ("dogStomach_metric", "dataset_dogStomach.json", 293, 0.6, 256),
    ("cellScope_literal", "dataset_cellScope.json", 508, None, None),
    ("mono_no_coordinates", "dataset_mono.json", 508, None, None),
    # SURVEY.md 8(c) fallback: dataset_mono.json optics with the 508-LED dome
    # table of include/domeHoleCoordinates.h inserted as holeCoordinates
    ("mono_dome", "dataset_mono.json+dome", 508, None, None),
    # the same at cropSizeX 256 (Np 256, L 1024, naRadius 84,
    # 193 LEDs; BASELINE.md 3 "dataset_mono geometry (Np = 90 / 256)")
    ("mono_dome_np256", "dataset_mono.json+dome", 508, 0.45, 256),
]
DOME_H = "include/domeHoleCoordinates.h"


def dome_table():
    """The 508 (x, y, z) triples of domeHoleCoordinates.h, read as numbers."""
    text = open(os.path.join(REF, DOME_H)).read()
    rows = re.findall(r"\{\s*(-?[0-9.eE+-]+)\s*,\s*(-?[0-9.eE+-]+)\s*,\s*(-?[0-9.eE+-]+)\s*\}", text)
    assert len(rows) == 508, len(rows)
    return [[float(a), float(b), float(c)] for a, b, c in rows]


def with_dome(text):
    rows = ",\n".join('   [{"x":%r},{"y":%r},{"z":%r}]' % tuple(r) for r in dome_table())
    body = text.rstrip().rstrip("}").rstrip().rstrip(",")
    return body + ',\n  "holeCoordinates":[\n' + rows + "\n]\n}\n"

SCALAR_KEYS = ["cropSizeX", "pixelSize", "objectiveMag", "objectiveNA", "maxIlluminationNA", "lambda",
               "arrayRotation", "bgThresh", "delta1", "delta2", "ledCount", "flipDatasetX", "flipDatasetY",
               "isColor", "cropX", "cropY", "bk1cropX", "bk1cropY", "bk2cropX", "bk2cropY", "centerLED",
               "filePrefix", "fileExtension", "darkfieldExpMultiplier"]


def scalar_keys(text):
    out = {}
    for k in SCALAR_KEYS:
        m = re.search(r'"%s"\s*:\s*("[^"]*"|true|false|-?[0-9.eE+-]+)' % re.escape(k), text)
        if m:
            out[k] = json.loads(m.group(1))
    return out


def main():
    if not os.path.exists(PROBE):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "ref"])
    for name, fn, n, maxna, np_ in CASES:
        if fn.endswith("+dome"):
            text = with_dome(open(os.path.join(REF, fn[:-5])).read())
            path = "/tmp/fpm_mono_dome.json"
            with open(path, "w") as f:
                f.write(text)
        else:
            path = os.path.join(REF, fn)
            text = open(path).read()
        args = [PROBE, path, str(n)]
        if maxna is not None or np_ is not None:
            args += [str(maxna if maxna is not None else 0.7604 if "maxIlluminationNA" not in text else
                         scalar_keys(text)["maxIlluminationNA"])]
        if np_ is not None:
            args += [str(np_)]
        probe = json.loads(subprocess.check_output(args).decode())
        fixture = dict(source=fn if not fn.endswith("+dome") else fn[:-5] + " + " + DOME_H, n_present=n, max_na_override=maxna, np_override=np_,
                       keys=scalar_keys(text),
                       trailing_comma=bool(re.search(r",\s*\]\s*\}\s*$", text)),
                       probe=probe)
        out = os.path.join(HERE, f"geometry_{name}.json")
        with open(out, "w") as f:
            json.dump(fixture, f, indent=0)
        print("wrote", out, "used", probe.get("led_used_count"))


if __name__ == "__main__":
    sys.exit(main())
