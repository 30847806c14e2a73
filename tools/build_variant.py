#!/usr/bin/env python3
"""Builds an A/B variant of liborbfe.so: python tools/build_variant.py NAME [-DFLAG=V ...]
-> orbslam_mapsave_amd/lib/liborbfe_NAME.so (selected at run time with ORBFE_LIB=...)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(ROOT, "orbslam_mapsave_amd", "lib", f"liborbfe_{name}.so")
subprocess.run(["/opt/rocm/bin/hipcc", *g.HIPCC_FLAGS, *flags, "-o", out,
                os.path.join(g.CSRC, "orbfe_lib.hip")], check=True)
print(out)
