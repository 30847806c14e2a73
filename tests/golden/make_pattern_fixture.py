#!/usr/bin/env python3
"""Generates the known-answer fixtures read as DATA from the reference text (run in the build
container, where /root/reference exists):

* tests/golden/pattern_fixture.json: the rBRIEF sampling pattern `bit_pattern_31_`
  (skaegy/ORBSLAM_MapSave src/ORBextractor.cc:149-407), the 1024 integers in table order — the
  check of include/orbfe_pattern.inc (tests/test_oracle_cpu.py);
* tests/golden/constants_fixture.json: PATCH_SIZE / HALF_PATCH_SIZE / EDGE_THRESHOLD
  (src/ORBextractor.cc:71-73), ORBmatcher::TH_HIGH / TH_LOW / HISTO_LENGTH
  (src/ORBmatcher.cc:37-39) and the ORBextractor.* parameters of
  Examples/ORB_RGB640x480.yaml:35-48 — checked against the oracle, the HIP library and the
  bench's parameters by tests/test_constants.py.
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
SRC = REF + "/src/ORBextractor.cc"


def parse(text: str) -> list[int]:
    m = re.search(r"static\s+int\s+bit_pattern_31_\s*\[\s*256\s*\*\s*4\s*\]\s*=\s*\{(.*?)\};",
                  text, re.S)
    if not m:
        raise SystemExit("bit_pattern_31_ not found")
    body = re.sub(r"/\*.*?\*/", " ", m.group(1), flags=re.S)
    vals = [int(v) for v in re.findall(r"-?\d+", body)]
    if len(vals) != 1024:
        raise SystemExit(f"expected 1024 values, found {len(vals)}")
    return vals


def _line_of(text: str, pos: int) -> int:
    return text[:pos].count("\n") + 1


def parse_consts(path: str, names: list[str], pattern: str) -> dict:
    """`const int NAME = value;` declarations (pattern has one %s for the name)."""
    text = open(path).read()
    out = {}
    for n in names:
        m = re.search(pattern % re.escape(n) + r"\s*=\s*(-?\d+)\s*;", text)
        if not m:
            raise SystemExit(f"{n} not found in {path}")
        out[n] = {"value": int(m.group(1)),
                  "source": f"{os.path.relpath(path, REF)}:{_line_of(text, m.start())}"}
    return out


def parse_yaml(path: str) -> dict:
    """The ORBextractor.* keys of an OpenCV YAML settings file (Tracking.cc:200-204 reads them)."""
    text = open(path).read()
    out = {}
    for m in re.finditer(r"^ORBextractor\.(\w+):\s*([-0-9.]+)\s*$", text, re.M):
        v = m.group(2)
        out[m.group(1)] = {"value": float(v) if "." in v else int(v),
                           "source": f"{os.path.relpath(path, REF)}:{_line_of(text, m.start())}"}
    for k in ("nFeatures", "scaleFactor", "nLevels", "iniThFAST", "minThFAST"):
        if k not in out:
            raise SystemExit(f"ORBextractor.{k} not found in {path}")
    return out


def write_constants() -> None:
    ext = parse_consts(SRC, ["PATCH_SIZE", "HALF_PATCH_SIZE", "EDGE_THRESHOLD"],
                       r"const\s+int\s+%s")
    mat = parse_consts(REF + "/src/ORBmatcher.cc", ["TH_HIGH", "TH_LOW", "HISTO_LENGTH"],
                       r"const\s+int\s+ORBmatcher::%s")
    yaml = parse_yaml(REF + "/Examples/ORB_RGB640x480.yaml")
    out = {"constants": {**ext, **mat}, "yaml_ORB_RGB640x480": yaml}
    with open(os.path.join(ROOT, "tests", "golden", "constants_fixture.json"), "w") as f:
        json.dump(out, f, indent=1)
    print({k: v["value"] for k, v in out["constants"].items()},
          {k: v["value"] for k, v in yaml.items()})


def main() -> None:
    write_constants()
    with open(sys.argv[1] if len(sys.argv) > 1 else SRC) as f:
        text = f.read()
    start = text[:text.index("static int bit_pattern_31_")].count("\n") + 1
    vals = parse(text)
    out = {"source": f"src/ORBextractor.cc:{start}-{start + 258}", "table": "bit_pattern_31_",
           "count": len(vals), "values": vals}
    with open(os.path.join(ROOT, "tests", "golden", "pattern_fixture.json"), "w") as f:
        json.dump(out, f)
    print(out["source"], len(vals), sum(vals))


if __name__ == "__main__":
    main()
