#!/usr/bin/env python3
"""Generates tests/golden/pattern_fixture.json: the reference's rBRIEF sampling pattern
`bit_pattern_31_` (skaegy/ORBSLAM_MapSave src/ORBextractor.cc:149-407), read as DATA from the
reference text (run in the build container, where /root/reference exists).  The fixture holds
the 1024 integers in table order and is the known-answer check of include/orbfe_pattern.inc
(tests/test_oracle_cpu.py::test_pattern_matches_reference_fixture).
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = "/root/reference/src/ORBextractor.cc"


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


def main() -> None:
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
