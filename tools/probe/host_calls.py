#!/usr/bin/env python3
"""Latency of the host-form matcher calls (one call per tracked frame in the reference), for
A/B runs of two library builds: ORBFE_LIB selects the library (orbslam_mapsave_amd/native.py).

  python tools/probe/host_calls.py   (GPU box) -> one JSON line, ms per call
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def timed(fn, k, warm=5):
    for _ in range(warm):
        fn()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    return (time.perf_counter() - t0) / k * 1e3


def main():
    import scenarios as S
    from orbslam_mapsave_amd import native
    out = {"lib": os.environ.get("ORBFE_LIB", "in-tree")}
    c = S.sbp_keyframe_case(0)
    m = native.ORBmatcher(0.9, True, device=0)
    out["reloc_sbp"] = timed(lambda: m.SearchByProjectionKeyFrame(
        c["cur"], c["tcw_cur"], c["cam"], c["log_scale"], c["kf_angle"], c["kf_valid"], c["kf_bad"],
        c["found"], c["kf_xyz"], c["kf_desc"], c["kf_min"], c["kf_max"], 10, 100,
        frame_mp=c["frame_mp"], kf_ids=c["kf_ids"]), 200)
    c = S.sbp_last_case(0)
    args = (c["cur"], c["tcw_cur"], c["cam"], c["last_keys"], c["last_valid"], c["last_outlier"],
            c["last_xyz"], c["last_desc"], c["last_nobs"], c["tcw_last"])
    out["sbp_last"] = timed(lambda: m.SearchByProjectionLast(*args, 15.0, True, last_ids=c["last_ids"]), 200)
    f1, f2, prev = S.sfi_case(0)
    out["sfi"] = timed(lambda: m.SearchForInitialization(f1, f2, prev, 100), 100)
    m.close()
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
