"""Micro-benchmark of orbfe_bf_match_batch_device alone (config-3 shape by default):
    python tools/bf_bench.py [lib.so] [--nr 2007] [--nq 1007] [--batch 256]
prints the mean kernel time (HIP events of the matcher's profiler) per launch."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("lib", nargs="?")
ap.add_argument("--nr", type=int, nargs="+", default=[2007])
ap.add_argument("--nq", type=int, default=1007)
ap.add_argument("--cap", type=int, default=1280)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
torch.zeros(1, device="cuda")
from orbslam_mapsave_amd import native  # noqa: E402
if args.lib:
    native.LIB_PATH = os.path.abspath(args.lib)
from orbslam_mapsave_amd.native import ORBmatcher  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
B, cap = args.batch, args.cap
q = torch.randint(0, 256, (B, cap, 32), dtype=torch.uint8, device="cuda", generator=g)
nq = torch.full((B,), args.nq, dtype=torch.int32, device="cuda")
out = torch.empty((B, cap, 3), dtype=torch.int32, device="cuda")
mt = ORBmatcher(0.9, True, device=0)
mt.set_stream(torch.cuda.current_stream().cuda_stream)
for nr in args.nr:
    r = torch.randint(0, 256, (nr, 32), dtype=torch.uint8, device="cuda", generator=g)
    dnr = torch.full((B,), nr, dtype=torch.int32, device="cuda")
    run = lambda: mt.bf_match_batch_device(q.data_ptr(), cap * 32, nq.data_ptr(), cap, r.data_ptr(), 0,
                                           dnr.data_ptr(), B, out.data_ptr())
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    mt.profile(True)
    mt.profile_read()
    for _ in range(args.iters):
        run()
    ms, n = mt.profile_read()
    mt.profile(False)
    pairs = B * args.nq * nr
    print(f"{os.path.basename(native.LIB_PATH)} nr={nr} {ms / n * 1e3:.1f} us/launch "
          f"{pairs / (ms / n * 1e-3) / 1e12:.2f} Tpairs/s")
