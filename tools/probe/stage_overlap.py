#!/usr/bin/env python3
"""How well two stages of the extraction overlap when their kernels share the chip (the
co-scheduling question of DESIGN.md §5h): two extractor handles, each on its own stream with
its own 256-frame batch (c3 shape: 640x480 @1000, x86 reading), extract once; then each stage
pair (X on handle A, Y on handle B) is relaunched R times on both streams at once
(orbfe_debug_replay) and the wall time is compared with X alone and Y alone.

  python tools/probe/stage_overlap.py [W H NF B R]   (GPU box) -> JSON on stdout
overlap = (t_X + t_Y - t_XY) / min(t_X, t_Y): 1 = the shorter one hides entirely, 0 = serial.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    from orbslam_mapsave_amd import native
    from orbslam_mapsave_amd.synth import synthetic_batch
    W, H, NF, B, R = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (640, 480, 1000, 256, 20)))
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    hs = []
    for k in range(2):
        fr = torch.from_numpy(synthetic_batch(B, W, H, first_seed=1000 + 100 * k, distinct=32)).to(dev)
        e = native.ORBextractor(NF, 1.2, 8, 20, 7, device=0, max_width=W, max_height=H, max_batch=B)
        e.set_stream(streams[k].cuda_stream)
        cap = e.capacity(W, H)
        bufs = (fr, torch.empty((B, cap * 28), dtype=torch.uint8, device=dev),
                torch.empty((B, cap, 32), dtype=torch.uint8, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev))
        e.extract_batch_device(fr.data_ptr(), B, W, H, W, W * H, bufs[1].data_ptr(), cap,
                               bufs[2].data_ptr(), bufs[3].data_ptr())
        hs.append((e, bufs))
    torch.cuda.synchronize()

    def wall(jobs):
        """jobs: [(handle index, stages)]; each replayed R times on its stream, all at once."""
        for k, st in jobs:  # warm
            hs[k][0].replay(st, 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k, st in jobs:
            hs[k][0].replay(st, R)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / R * 1e3

    stages = [("resize",), ("fast",), ("octree",), ("describe",)]
    alone = {s[0]: wall([(0, s)]) for s in stages}
    pairs = {}
    for a, b in [("fast", "describe"), ("fast", "fast"), ("describe", "describe"), ("resize", "fast"),
                 ("resize", "describe"), ("octree", "describe"), ("octree", "fast"), ("resize", "resize")]:
        t = wall([(0, (a,)), (1, (b,))])
        ta, tb = alone[a], alone[b]
        pairs[f"{a}+{b}"] = {"ms": round(t, 4), "serial_ms": round(ta + tb, 4),
                             "overlap": round((ta + tb - t) / min(ta, tb), 3)}
    print(json.dumps({"shape": [W, H, NF, B], "reps": R,
                      "alone_ms": {k: round(v, 4) for k, v in alone.items()}, "pairs": pairs}, indent=1))


if __name__ == "__main__":
    main()
