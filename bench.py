#!/usr/bin/env python3
"""Benchmark of the MI355X ORB front-end (the hot path of skaegy/ORBSLAM_MapSave).

Default workload (BASELINE.json configs[2], the config its metric "frames/sec ORB
extract+match, 640x480 @1000 kp" is quoted on): every step, every rank extracts a batch of B
synthetic 640x480 frames (ORBextractor(1000, 1.2, 8, 32, 7), ORB_RGB640x480.yaml with
nFeatures=1000) and brute-force Hamming-matches each frame's descriptors against a 2000-kp
reference frame (best / second / index per query).  Frames are independent, so N ranks shard
them with no data-path collective ("scaling": "weak").  Inputs are resident in HBM before the
timed region; outputs stay on the device.

``--config c4`` runs BASELINE configs[3] instead: 1920x1080 @2000 kp, a global batch of 256
frames sharded round-robin over the ranks, an RCCL all-gather of the descriptor slabs and a
frame f vs frame f-1 match.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 through torch.distributed.run
(one process per GPU, RCCL).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ARITH = {"scalar": 0, "x86": 1}  # orbfe_set_arithmetic: ORBFE_ARITH_SCALAR / ORBFE_ARITH_X86_SIMD
METRIC = "frames/sec ORB extract+match, 640×480 @1000 kp, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md "HBM3E peak BW 8.0 TB/s spec"
# VALU issue peak: 256 CUs x 4 SIMD-32 units, a wave64 VALU instruction holds its SIMD for 2
# cycles (MI355X_MICROARCH.md "Each CU has 4 SIMD-32 units ... over 2 cycles"), 2.4 GHz peak
# engine clock: 1.2288 T wave-instructions / s
VALU_PEAK_INSTS = 256 * 4 * 2.4e9 / 2
# dense FP4 matrix-core peak (MI355X_MICROARCH.md: ~10 PF dense; AMD's 20 PF includes sparsity)
FP4_PEAK_TFLOPS = 10000.0
# bf_expand: the batch-shared reference set expanded to FP4 fragments once per match call (its
# own profiler stage, so bf_match's per-launch figures are the match kernel's alone)
STAGES = ("mask", "resize", "fast", "octree", "blur", "describe", "bf_match", "bf_expand")
# ORBextractor.{scaleFactor,nLevels,iniThFAST,minThFAST} of Examples/ORB_RGB640x480.yaml:38-48
# (its nFeatures, 2000, is config 4's; configs 2/3/5 extract the metric's 1000).  Pinned against
# the reference text by tests/test_constants.py (tests/golden/constants_fixture.json).
ORB_SCALE, ORB_LEVELS, ORB_INI_TH, ORB_MIN_TH = 1.2, 8, 32, 7
ORB_YAML_NFEATURES = 2000
ORB = (ORB_SCALE, ORB_LEVELS, ORB_INI_TH, ORB_MIN_TH)


def level_sizes(w, h, nlevels=8, scale=1.2):
    s = np.float32(1.0)
    out = []
    for l in range(nlevels):
        inv = np.float32(1.0) / s
        out.append((int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))))
        s = np.float32(np.float64(s) * np.float64(np.float32(scale)))
    return out


def algorithmic_bytes(stage: str, w: int, h: int, nkp: float, nref: float = 0.0) -> float:
    """Per-frame algorithmic bytes of one stage (DESIGN.md "Roofline")."""
    P = [a * b for a, b in level_sizes(w, h)]
    if stage == "resize":   # cascaded: read level l-1, write level l
        return float(sum(P[:-1]) + sum(P[1:]))
    if stage == "fast":     # every level read once
        return float(sum(P))
    if stage == "blur":     # read + write every level
        return float(2 * sum(P))
    if stage == "describe":  # 31x31 angle patch + 512 samples per keypoint, kp + desc out
        return float(nkp * (961 + 512 + 28 + 32))
    if stage == "octree":   # the level's FAST candidates (4 B) read, keypoints (4 B) written
        return float(nkp * 8)
    if stage == "bf_match":  # query + reference descriptors read, 12 B result per query
        return float(32 * (nkp + nref) + 12 * nkp)
    return 0.0


def committed_pmc(config: str, arith: str, frames: int) -> tuple[dict, str | None]:
    """Per-kernel VALU wave-instructions per launch (SQ_INSTS_VALU) from the rocprofv3 --pmc
    pass of this command committed as profiles/valu_<config>.json (tools/summarize_profile.py):
    PMC counters cannot be read inside this process.  Empty when absent or for another batch."""
    path = os.path.join(ROOT, "profiles", f"valu_{config}.json")
    if not os.path.exists(path):
        return {}, None
    with open(path) as fh:
        j = json.load(fh)
    if j.get("frames_per_launch") != frames:
        return {}, None
    suf = "" if arith == "scalar" else f"@{arith}"
    out = {k[:-len(suf)] if suf else k: v for k, v in j.items()
           if isinstance(v, dict) and (k.endswith(suf) if suf else "@" not in k)}
    return out, f"profiles/valu_{config}.json ({j.get('source', 'rocprofv3 --pmc SQ_INSTS_VALU')})"


# bench stage -> the kernels that implement it (the stage's launches in a step)
STAGE_KERNELS = {"resize": ("pyramid_kernel", "resize2_kernel", "resize_kernel", "resize_tail_kernel"),
                 "fast": ("fast_kernel", "fast_strip_kernel"), "octree": ("octree_kernel",),
                 "describe": ("describe_kernel",), "bf_match": ("bf_match_fp4e_kernel", "bf_match_fp4_kernel",
                                                             "bf_match_kernel")}


def host_cpu() -> dict:
    """Host core count and CPU model ("report the core count and model")."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        nproc = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    # the GPU box gives one GPU's job a share of the host (OMP_NUM_THREADS is set to it)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(nproc, share) if share > 0 else nproc
    return {"model": model, "nproc": nproc, "threads": max(1, threads)}


def cpu_baseline(frames: np.ndarray, ref_desc: np.ndarray | None, budget_s: float,
                 nfeatures: int = 1000, what: str = "", match: bool = True,
                 arith: str = "scalar") -> dict:
    """The CPU oracle (a port of the reference CPU path, oracle/orb_oracle.cpp, -O3) on the
    bench's own frames, BASELINE.md §2: (i) one thread, frames in sequence, after 50 warm-up
    frames, until >= 1000 frames or `budget_s`; (ii) all cores of this job's host share, one
    extractor state per thread (ctypes releases the GIL), for ~budget_s / 3.  Each frame is
    extract(nfeatures) + brute-force match against `ref_desc` (or against the previous frame's
    descriptors when ref_desc is None: config 4's f vs f-1); extract only with match=False
    (config 2).  arith "x86" switches the oracle to the x86 build's reading (H4/H5/H6)."""
    import concurrent.futures as cf
    import oracle  # test infrastructure: the cpu_baseline leg is allowed to load it
    oracle.set_variant(0 if arith == "scalar" else
                       oracle.VAR_H4_FMA | oracle.VAR_H5_SSE2 | oracle.VAR_H6_SIMD)
    p = oracle.params(nfeatures, *ORB)
    host = host_cpu()

    def one(i, prev):
        kps, desc = oracle.extract(p, frames[i % len(frames)])
        if match:
            oracle.bf_match(desc, ref_desc if ref_desc is not None else prev)
        return desc

    prev = oracle.extract(p, frames[-1])[1]
    for i in range(min(50, len(frames) * 2)):  # warm-up
        prev = one(i, prev)
    times = []
    t0 = time.perf_counter()
    while len(times) < 1000 and (time.perf_counter() - t0 < budget_s or len(times) < 5):
        a = time.perf_counter()
        prev = one(len(times), prev)
        times.append(time.perf_counter() - a)
    el1 = time.perf_counter() - t0
    T = host["threads"]
    budget_all = max(budget_s / 3, 2.0)
    stop = time.perf_counter() + budget_all

    def worker(k):
        n, pv = 0, oracle.extract(p, frames[k % len(frames)])[1]
        while time.perf_counter() < stop or n < 2:
            pv = one(k + n * T, pv)
            n += 1
        return n

    ta = time.perf_counter()
    with cf.ThreadPoolExecutor(T) as pool:
        done_all = sum(pool.map(worker, range(T)))
    el_all = time.perf_counter() - ta
    ms = np.array(times) * 1e3
    return {"value": round(len(times) / el1, 3), "unit": "frames/s", "cores": 1, "kind": "port",
            "threads": 1, "median_ms": round(float(np.median(ms)), 3),
            "mean_ms": round(float(ms.mean()), 3),
            "all_core": {"value": round(done_all / el_all, 3), "unit": "frames/s", "threads": T,
                         "frames": done_all, "seconds": round(el_all, 2)},
            "host": host,
            "sample": f"{len(times)} of the bench's frames {what} after 50 warm-up frames, 1 "
                      f"thread, {el1:.1f} s (oracle/orb_oracle.cpp -O3 -march=x86-64-v3); "
                      f"all-core: {done_all} frames on {T} threads in {el_all:.1f} s"}


C2_METRIC = ("frames/sec ORB extract (8-level pyramid + FAST-9 + oct-tree + rBRIEF), 640×480 "
             "@1000 kp, 1 MI355X")
C4_METRIC = ("frames/sec ORB extract+match, 1920×1080 @2000 kp, batch 256 sharded over 1/2/4/8 "
             "MI355X with an RCCL descriptor all-gather; % HBM roofline")
C5_METRIC = ("frames/sec tracking-loop SearchByProjection (isInFrustum + SearchByProjection) vs "
             "50k-MapPoint local map, 640×480, 1 MI355X")


def run_c5(args) -> None:
    """BASELINE configs[4]: Tracking::SearchLocalPoints against a 50k-point local map, one
    frame per step, frame and map resident in HBM (orbfe_search_local_points_device).  N ranks
    run independent replicas (one tracking thread per GPU); value = frames/s over all ranks."""
    import torch
    import torch.distributed as dist
    from orbslam_mapsave_amd.abi import Camera, MapPoints
    from orbslam_mapsave_amd.native import ORBextractor, ORBmatcher
    from orbslam_mapsave_amd.synth import synthetic_frame, synthetic_local_map

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    W, H, M = 640, 480, 50_000
    img = synthetic_frame(2024 + rank, W, H)
    ex = ORBextractor(1000, *ORB, device=local, max_width=W, max_height=H)
    keys, desc = ex(img)
    scale = ex.GetScaleFactors()
    ex.close()
    lm = synthetic_local_map(keys, desc, M, seed=rank)
    cam = Camera(500.0, 500.0, 320.0, 240.0, 40.0, 40.0 / 500.0)
    log_scale = float(np.log(np.float32(1.2)).astype(np.float32))
    T = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in lm.items()}
    d_keys = torch.from_numpy(keys.view(np.uint8).copy()).to(dev)
    d_desc = torch.from_numpy(np.ascontiguousarray(desc)).to(dev)
    d_inv = torch.zeros(M, dtype=torch.uint8, device=dev)
    # the frame's MapPoint slots and their Observations() side by side, so the per-step reset
    # (the call writes them) is one copy
    slots = torch.stack([T["frame_mp"], T["frame_mp_obs"]]).contiguous()
    T["frame_mp"], T["frame_mp_obs"] = slots[0], slots[1]
    slots0 = slots.clone()
    mt = ORBmatcher(0.8, False, device=local)
    # one stream of its own for the call and the slot reset in front of it (ordered with each
    # other; the legacy default stream's implicit ordering is not needed)
    cs = torch.cuda.Stream(dev)
    mt.set_stream(cs.cuda_stream)
    torch.cuda.synchronize(dev)
    out = {}

    def step():
        with torch.cuda.stream(cs):
            slots.copy_(slots0)
        out["r"] = mt.search_local_points_device(
            len(keys), d_keys.data_ptr(), d_desc.data_ptr(), None, W, H, scale, lm["tcw"], cam,
            log_scale, 0.5, M, T["xyz"].data_ptr(), T["normal"].data_ptr(),
            T["min_dist"].data_ptr(), T["max_dist"].data_ptr(), T["desc"].data_ptr(),
            T["nobs"].data_ptr(), T["bad"].data_ptr(), T["skip"].data_ptr(), T["ids"].data_ptr(),
            0.8, 1.0, T["frame_mp"].data_ptr(), T["frame_mp_obs"].data_ptr(), d_inv.data_ptr())

    # A14 alone ("time A17+A14 together and A14 alone"): the same
    # frame and map with isInFrustum's outputs already in HBM (computed once, untimed) —
    # SearchByProjection(F, vpLocalMapPoints, th) by itself
    sf_np = np.asarray(scale, np.float32)
    inv, px, py, pxr, pl, vc = mt.is_in_frustum(lm["xyz"], lm["normal"], lm["min_dist"],
                                                lm["max_dist"], lm["tcw"], cam,
                                                (0.0, float(W), 0.0, float(H)), log_scale, 0.5)
    inv[(lm["skip"] > 0) | (lm["bad"] > 0)] = 0
    A = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
         for k, v in dict(inv=inv, px=px, py=py, pxr=pxr, pl=pl, vc=vc).items()}

    def step_a14():
        with torch.cuda.stream(cs):
            slots.copy_(slots0)
        out["a14"] = mt.search_by_projection_local_device(
            len(keys), d_keys.data_ptr(), d_desc.data_ptr(), None, W, H, sf_np, M,
            A["inv"].data_ptr(), T["bad"].data_ptr(), A["px"].data_ptr(), A["py"].data_ptr(),
            A["pxr"].data_ptr(), A["pl"].data_ptr(), A["vc"].data_ptr(), T["desc"].data_ptr(),
            T["nobs"].data_ptr(), T["ids"].data_ptr(), 0.8, 1.0, T["frame_mp"].data_ptr(),
            T["frame_mp_obs"].data_ptr())

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def timed(fn):
        for _ in range(max(args.warmup, 1)):
            fn()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    dt_a14 = timed(step_a14)
    fmp_a14 = slots.clone()
    dt = timed(step)
    same_a14 = bool(torch.equal(fmp_a14, slots))  # both legs reach the same assignment
    if rank == 0:
        K = args.steps
        value = world * K / dt
        ms = dt / K * 1e3
        # algorithmic bytes per frame: map point reads (xyz 12, normal 12, min/max 8, descriptor
        # 32, Observations 4, bad 1, skip 1, id 4) + frame keypoints/descriptors (60 B each) +
        # the in-view byte written per point
        nbytes = M * (12 + 12 + 8 + 32 + 4 + 1 + 1 + 4 + 1) + len(keys) * 60
        achieved = nbytes / (ms / 1e3) / 1e9
        cpu = None
        if world == 1 and args.cpu_budget > 0:
            import oracle  # test infrastructure: the cpu_baseline leg is allowed to load it
            from orbslam_mapsave_amd.abi import Frame
            fr = Frame(keys, desc, W, H, scale)
            done, c0, t_sbp = 0, time.perf_counter(), 0.0
            while True:
                inv, px, py, pxr, pl, vc = oracle.is_in_frustum(
                    lm["xyz"], lm["normal"], lm["min_dist"], lm["max_dist"], lm["tcw"], cam,
                    (0.0, float(W), 0.0, float(H)), log_scale, 0.5)
                inv[(lm["skip"] > 0) | (lm["bad"] > 0)] = 0
                mps = MapPoints(px, py, pl, vc, lm["desc"], lm["nobs"], track_in_view=inv,
                                is_bad=lm["bad"], proj_xr=pxr)
                s0 = time.perf_counter()
                oracle.search_by_projection_local(fr, mps, 1.0, 0.8, lm["frame_mp"],
                                                  lm["frame_mp_obs"], lm["ids"])
                t_sbp += time.perf_counter() - s0
                done += 1
                el = time.perf_counter() - c0
                if el >= min(args.cpu_budget, 10.0) and done >= 3:
                    break
            cpu = {"value": round(done / el, 3), "unit": "frames/s", "cores": 1, "kind": "port",
                   "a14_alone_value": round(done / t_sbp, 3),
                   "sample": f"{done} calls of the same frame + 50k-point local map, isInFrustum "
                             f"+ SearchByProjection, 1 thread, oracle/orb_oracle.cpp -O3, "
                             f"{el:.1f} s"}
        nm, nto = out["r"]
        a14 = {"calls_per_s": round(world * K / dt_a14, 2),
               "ms_per_call": round(dt_a14 / K * 1e3, 4), "nmatches": out["a14"],
               "same_assignment_as_fused": same_a14,
               "note": "orbfe_search_by_projection_local_device: isInFrustum outputs resident in "
                       "HBM (computed once, untimed); grid + one kernel for the candidates "
                       "(fixed per-point slots) and the greedy initialisation + blind greedy "
                       "rounds + accept, one synchronisation (CSR path on overflow)"}
        line = {
            "metric": C5_METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: seeded textured 640x480 frame (GPU-extracted, 1000 kp) + 50k "
                    "world-space map points (synth.synthetic_local_map), resident in HBM",
            "config": {"workload": "configs[4]: Tracking::SearchLocalPoints (isInFrustum + "
                                   "SearchByProjection th=1, nnratio 0.8) vs 50k-MapPoint local map",
                       "arith": args.arith,
                       "map_points": M, "keypoints": int(len(keys)), "nToMatch": nto,
                       "nmatches": nm, "greedy_rounds": mt.last_rounds(),
                       "parallelism": f"replicas x{world}"},
            "roofline": {"bound": "hbm", "kernel": "search_local_points (frustum + candidates + "
                         "greedy rounds, whole call)", "achieved": round(achieved, 3),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
                         "bytes_per_launch": nbytes, "avg_launch_ms": round(ms, 4)},
            "cpu_baseline": cpu,
            "a14_alone": a14,
        }
        if cpu:
            line["gpu_over_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    mt.close()
    if world > 1:
        dist.destroy_process_group()


def e2e_bytes(w: int, h: int, nf: int, nq: int = 0, nr: int = 0) -> int:
    """SURVEY.md §8(d) end-to-end algorithmic bytes per frame: input + cascaded resize (read +
    write) + FAST read + blur read/write + N (31x31 patch + 512 samples + keypoint + descriptor),
    plus 32 (Q + R) + 12 Q for a brute-force match (6,261,674 B at 640x480 @1000; +108,000)."""
    P = [a * b for a, b in level_sizes(w, h)]
    b = w * h + sum(P[:-1]) + sum(P[1:]) + sum(P) + 2 * sum(P) + nf * (961 + 512) + nf * (28 + 32)
    if nq:
        b += 32 * (nq + nr) + 12 * nq
    return int(b)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); when WORLD_SIZE is unset and N > 1, "
                         "bench.py starts the N rank processes itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank launch: gloo backend, no GPU, the "
                         "config-4 exchange step on small random descriptor slabs")
    ap.add_argument("--arith", default="x86", choices=["scalar", "x86"],
                    help="arithmetic reading of the extractor (orbfe_set_arithmetic): the SSE2 "
                         "resize / blur bodies + FMA rotation of the reference's x86-64 build "
                         "(the default, as the library's), or OpenCV's portable scalar paths "
                         "(DESIGN.md §2)")
    # 100 timed steps: the two sub-batch streams' fill and drain at the ends of the timed region
    # (one stream's last kernels alone on the chip) weigh 1/K of it — c3 1.385 ms per step at
    # K = 20, 1.374 at K = 100 (profiles/r05/steps_k/)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--soak-s", type=float, default=8.0,
                    help="untimed wall-clock seconds of steps after the warmup (c2/c3/c4), so "
                         "that an external GPU-utilisation sampler sees the load; 0 = off")
    ap.add_argument("--batch", type=int, default=512,
                    help="frames per rank per step (c3; 512: +4 %% frames/s over 256, level at 1024)")
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--per-rank", type=int, default=0,
                    help="c4: frames per rank (default 256 / world; 32 rehearses the 8-GPU "
                         "per-rank shape on one GPU)")
    ap.add_argument("--distinct", type=int, default=32, help="distinct synthetic seeds (cycled)")
    ap.add_argument("--streams", type=int, default=0,
                    help="sub-batches per rank in the timed steps, each on its own HIP stream and "
                         "extractor handle (their latency-bound kernels overlap; c4: sub-batch "
                         "A's all-gather runs while B is extracted); 0 = 2.  The probe and "
                         "roofline legs always run the whole batch on one stream")
    ap.add_argument("--probe-steps", type=int, default=2,
                    help="steps after the warmup with events on every kernel, for the per-stage "
                         "table and the choice of the dominant kernel")
    ap.add_argument("--chunks", type=int, default=1,
                    help="extraction calls per stream per step (each a sub-batch / chunks)")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="1 (c3): each sub-batch extracted in two calls (orbfe_set_stage_mask: "
                         "pyramid + FAST + oct-tree, then describe + its match), and stream k's "
                         "first call waits for stream k-1's first, so one sub-batch's describe "
                         "runs beside the next one's FAST (DESIGN.md §5h)")
    ap.add_argument("--skew", type=int, default=0,
                    help="1: stream k starts k/streams of a step late (its first chunk waits "
                         "for stream 0's chunk k*chunks/streams - 1), so the streams run "
                         "different stages at the same time")
    ap.add_argument("--profile", type=int, default=1,
                    help="0: no per-kernel HIP events in the timed region (no roofline)")
    ap.add_argument("--cpu-budget", type=float, default=15.0,
                    help="seconds of CPU-baseline work on rank 0 (0 disables)")
    return ap.parse_args()


def run_extract(args, dev, rank, world, local, W, H, NF, NREF, B, mode, steps, warmup):
    """One extraction benchmark: every step, every rank extracts B frames (device-resident) and,
    by `mode`, matches nothing ("none", config 2), each frame against a 2000-kp reference
    ("ref", config 3), or each frame against its global predecessor after the descriptor
    all-gather ("pred", config 4).  Returns the measurement (rank 0) or None."""
    import torch
    import torch.distributed as dist
    from orbslam_mapsave_amd.native import ORBextractor, ORBmatcher
    from orbslam_mapsave_amd.shard import PredecessorMatch
    from orbslam_mapsave_amd.synth import synthetic_batch, synthetic_frame

    frames_np = synthetic_batch(B, W, H, first_seed=1000 * rank, distinct=args.distinct)
    frames = torch.from_numpy(frames_np).to(dev)
    S = max(1, min(args.streams or 2, B))
    while B % S:
        S -= 1
    C = B // S  # frames per sub-batch
    streams = [torch.cuda.Stream(dev) for _ in range(S)]

    # handle 0 also serves the single-stream legs (probe and roofline steps: the whole batch in
    # one call), so it is planned for B frames; the other sub-batch handles for C
    exs = []
    for k in range(S):
        e = ORBextractor(NF, *ORB, device=local, max_width=W, max_height=H,
                         max_batch=B if k == 0 else C)
        e.set_arithmetic(ARITH[args.arith])
        e.set_stream(streams[k].cuda_stream)
        exs.append(e)
    mt = ORBmatcher(0.9, True, device=local)
    cap = exs[0].capacity(W, H)
    d_kps = torch.empty((B, cap * 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(B, dtype=torch.int32, device=dev)
    d_out = torch.empty((B, cap, 3), dtype=torch.int32, device=dev)

    ref_desc_np = None
    if mode == "ref":  # reference frame (config 3): the 2x-feature extractor, once on the GPU
        ref_np = synthetic_frame(999_999, W, H)
        ex_ref = ORBextractor(NREF, *ORB, device=local, max_width=W, max_height=H)
        ex_ref.set_arithmetic(ARITH[args.arith])
        ref_kps, ref_desc_np = ex_ref(ref_np)
        ex_ref.close()
        ref_desc = torch.from_numpy(np.ascontiguousarray(ref_desc_np)).to(dev)
        d_nr = torch.full((B,), len(ref_desc_np), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)

    if mode == "pred":
        # the match's own stream (not the legacy default stream, whose implicit ordering the
        # step does not need: every dependency is an explicit wait below)
        main_stream = torch.cuda.Stream(dev)

        def bf(q, qn, r, rn, out):
            mt.set_stream(main_stream.cuda_stream)
            mt.bf_match_batch_device(q.data_ptr(), cap * 32, qn.data_ptr(), cap, r.data_ptr(),
                                     cap * 32, rn.data_ptr(), q.shape[0], out.data_ptr())

        # one exchange part per sub-batch stream: part k's all-gather is queued behind stream
        # k's extraction, so it runs while the later sub-batches are still being extracted
        pm = PredecessorMatch(rank, world, B, cap, dev, bf, parts=S)

    J = max(1, min(args.chunks, C))
    while C % J:
        J -= 1
    CJ = C // J  # frames per extraction call

    def extract_chunk(k, j=None):
        f0, n = (k * C, C) if j is None else (k * C + j * CJ, CJ)
        exs[k].extract_batch_device(frames[f0].data_ptr(), n, W, H, W, W * H,
                                    d_kps[f0].data_ptr(), cap, d_desc[f0].data_ptr(),
                                    d_n[f0:].data_ptr())

    skew_next = [False]

    def step_single():
        """The whole batch in one extraction call (+ one match launch) on stream 0: the probe
        and roofline legs, where a kernel's launch has the chip to itself."""
        exs[0].extract_batch_device(frames[0].data_ptr(), B, W, H, W, W * H, d_kps[0].data_ptr(),
                                    cap, d_desc[0].data_ptr(), d_n.data_ptr())
        mt.set_stream(streams[0].cuda_stream)
        if mode == "ref":
            mt.bf_match_batch_device(d_desc[0].data_ptr(), cap * 32, d_n.data_ptr(), cap,
                                     ref_desc.data_ptr(), 0, d_nr.data_ptr(), B,
                                     d_out[0].data_ptr())
        elif mode == "pred":  # the local predecessor stands in for the gathered one (leg only)
            mt.bf_match_batch_device(d_desc[0].data_ptr(), cap * 32, d_n.data_ptr(), cap,
                                     d_desc[0].data_ptr(), cap * 32, d_n.data_ptr(), B,
                                     d_out[0].data_ptr())

    G1, G2 = ("resize", "fast", "octree"), ("describe",)
    pipe_ev = [torch.cuda.Event() for _ in range(S)]

    def step_pipeline():
        """--pipeline 1: per sub-batch, stages up to the oct-tree, then describe + the match,
        with stream k's first part queued behind stream k-1's first part."""
        for k in range(S):
            f0 = k * C
            if k:
                streams[k].wait_event(pipe_ev[k - 1])
            exs[k].set_stages(G1)
            extract_chunk(k)
            pipe_ev[k].record(streams[k])
            exs[k].set_stages(G2)
            extract_chunk(k)
            exs[k].set_stages(None)
            if mode == "ref":
                mt.set_stream(streams[k].cuda_stream)
                mt.bf_match_batch_device(d_desc[f0].data_ptr(), cap * 32, d_n[f0:].data_ptr(), cap,
                                         ref_desc.data_ptr(), 0, d_nr[f0:].data_ptr(), C,
                                         d_out[f0].data_ptr())

    def step():
        if S == 1 and mode != "pred":
            return step_single()
        if args.pipeline and mode != "pred" and J == 1:
            return step_pipeline()
        if mode != "pred":  # sub-batch k: extract (+ match) on stream k, no cross-stream deps
            ev = {}
            for j in range(J):
                for k in range(S):
                    if skew_next[0] and j == 0 and k > 0:
                        src = max(0, k * J // S - 1)
                        if src in ev:
                            streams[k].wait_event(ev[src])
                    f0 = k * C + j * CJ
                    extract_chunk(k, j)
                    if mode == "ref":
                        mt.set_stream(streams[k].cuda_stream)
                        mt.bf_match_batch_device(d_desc[f0].data_ptr(), cap * 32,
                                                 d_n[f0:].data_ptr(), cap, ref_desc.data_ptr(), 0,
                                                 d_nr[f0:].data_ptr(), CJ, d_out[f0].data_ptr())
                    if skew_next[0] and k == 0:
                        ev[j] = torch.cuda.Event()
                        ev[j].record(streams[0])
            skew_next[0] = False
        else:  # sub-batch k: extract on stream k, then its all-gather behind it (RCCL's
            # stream waits for stream k only); the match runs on the main stream once every
            # part has arrived
            for k in range(S):
                extract_chunk(k)
                with torch.cuda.stream(streams[k]):
                    pm.gather_part(k, d_desc, d_n)
            for k in range(S):
                main_stream.wait_stream(streams[k])
            with torch.cuda.stream(main_stream):
                pm.finish(d_desc, d_n, d_out)
            for k in range(S):
                streams[k].wait_stream(main_stream)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def read_stages():
        acc = {st: (0.0, 0) for st in STAGES}
        for e in exs:
            for st, (ms, n) in e.profile_read().items():
                acc[st] = (acc[st][0] + ms, acc[st][1] + n)
        acc.update(mt.profile_read_stages())
        return acc

    def agreed(flag: bool) -> bool:
        """True once every rank reports flag (a MIN over ranks: collective counts pair up)."""
        if world == 1:
            return flag
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    for _ in range(warmup):
        step()
    barrier()
    # Soak (untimed, >= --soak-s seconds of wall clock of the same steps): the timed region of a
    # default run is tens of milliseconds, too short for an external utilisation sampler (rocm-smi
    # every few seconds) to see the GPU busy; the soak gives it a window of sustained load before
    # the measurement and settles the clocks.  Steady-state step time from 10 steps after the
    # warmup (the warmup's first calls include plan, workspace and graph setup); the soak then
    # runs in chunks of ~0.5 s and stops when every rank has passed --soak-s (collective counts
    # stay paired).
    soak = {"seconds": 0.0, "steps": 0}
    if args.soak_s > 0:
        ta = time.perf_counter()
        for _ in range(10):
            step()
        barrier()
        tw = (time.perf_counter() - ta) / 10
        chunk = max(1, min(int(0.5 / max(tw, 1e-5)), 20000))
        if world > 1:
            c = torch.tensor([chunk], dtype=torch.int64, device=dev)
            dist.all_reduce(c, op=dist.ReduceOp.MIN)
            chunk = int(c.item())
        ts = time.perf_counter()
        while True:
            for _ in range(chunk):
                step()
            barrier()
            soak["steps"] += chunk
            if agreed(time.perf_counter() - ts >= args.soak_s):
                break
        soak["seconds"] = round(time.perf_counter() - ts, 2)
        soak["steady_ms_per_step"] = round(tw * 1e3, 4)
    # Probe steps (untimed, single-stream): events on every kernel give the per-stage table and
    # pick the dominant kernel.
    probe_steps = max(args.probe_steps, 1) if args.profile else 0
    for e in exs:
        e.profile(bool(probe_steps))
        e.profile_read()
    mt.profile(bool(probe_steps))
    mt.profile_read()
    for _ in range(probe_steps):
        step_single()
    barrier()
    probe = read_stages()
    dom = max(STAGES, key=lambda st: probe[st][0]) if probe_steps else None
    for e in exs:
        e.profile(False)
    mt.profile(False)
    # Timed steps: the workload as it runs best (S sub-batch streams), no instrumentation.
    skew_next[0] = bool(args.skew) and S > 1 and J >= S
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    # Roofline leg (untimed for `value`): the same number of steps single-stream with HIP events
    # on the dominant kernel's launches alone, so each event pair times that kernel with the chip
    # to itself (with S streams a launch shares the chip with the other sub-batch's kernels).
    if dom is not None:
        exs[0].profile(dom != "bf_match", stages=(dom,))
        exs[0].profile_read()
        mt.profile(dom == "bf_match")
        mt.profile_read()
        for _ in range(steps):
            step_single()
        barrier()
    stages = read_stages()
    for e in exs:
        e.profile(False)
    mt.profile(False)
    nkp = float(d_n.float().mean().item())
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    for e in exs:
        e.close()
    mt.close()
    if rank != 0:
        return None
    K = steps
    per_step = {s_: probe[s_][0] / max(probe_steps, 1) for s_ in STAGES}
    dom_ms, dom_launches = stages[dom] if dom else (0.0, 0)
    nref = float(len(ref_desc_np)) if mode == "ref" else nkp
    bytes_per_step = algorithmic_bytes(dom, W, H, nkp, nref) * B if dom else 0.0
    achieved = bytes_per_step / (dom_ms / K / 1e3) / 1e9 if dom_ms > 0 else 0.0
    # HBM traffic of the dominant kernel per launch: PMC counters cannot be read inside this
    # process, so it comes from the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the same
    # command committed under profiles/ (traffic_source names the file and round)
    traffic, tsrc = None, None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tpath) and dom:
        with open(tpath) as fh:
            tj = json.load(fh)
        key = dom if args.arith == "scalar" else f"{dom}@{args.arith}"
        if isinstance(tj.get(key), (int, float)) and tj.get("frames_per_launch") == B:
            traffic = tj[key]
            tsrc = f"profiles/traffic_{args.config}.json ({tj.get('source', 'rocprofv3 --pmc')})"
    roof = {"bound": "hbm", "kernel": f"{dom}_kernel" if dom else None,
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "traffic_source": tsrc,
            "bytes_per_launch": round(bytes_per_step * K / max(dom_launches, 1)),
            "avg_launch_ms": round(dom_ms / max(dom_launches, 1), 4), "launches": dom_launches,
            "leg": (f"{K} single-stream steps of {B} frames after the timed region, HIP events on "
                    f"the {dom} launches only (the timed steps run {S} sub-batch streams, "
                    "uninstrumented)")}
    # the binding resources: VALU issue (SQ_INSTS_VALU of the committed PMC pass over the
    # launch's event time) for the dominant kernel and each stage, and the matrix cores for the
    # brute force (algorithmic FP4 flops: 2 x 256 per (query, reference) pair)
    pmc, pmc_src = committed_pmc(args.config, args.arith, B)

    def valu_of(stage, ms, launches):
        ks = [k for k in STAGE_KERNELS.get(stage, ()) if k in pmc]
        if not ks or ms <= 0 or launches <= 0:
            return None
        # a stage of several kernels (the 1080p pyramid): their launch-weighted mean
        nd = sum(pmc[k]["dispatches"] for k in ks)
        per = sum(pmc[k]["valu_per_launch"] * pmc[k]["dispatches"] for k in ks) / max(nd, 1)
        rate = per * launches / (ms / 1e3)
        return {"kernel": "+".join(ks), "insts_per_launch": round(per),
                "achieved": round(rate / 1e12, 4), "peak": round(VALU_PEAK_INSTS / 1e12, 4),
                "unit": "T wave-instructions/s", "frac": round(rate / VALU_PEAK_INSTS, 4)}
    if dom:
        v = valu_of(dom, dom_ms, dom_launches)
        if v:
            v["source"] = pmc_src
        roof["valu"] = v
    mfma = None
    if mode in ("ref", "pred") and per_step.get("bf_match", 0) > 0:
        pairs = nkp * (nref if mode == "ref" else nkp) * B  # (query, reference) pairs per step
        flops = 2.0 * 256 * pairs
        tfl = flops / (per_step["bf_match"] / 1e3) / 1e12
        mfma = {"kernel": "bf_match_fp4e_kernel" if mode == "ref" else "bf_match_fp4_kernel",
                "flops_per_step": round(flops), "ms_per_step": round(per_step["bf_match"], 4),
                "achieved": round(tfl, 1), "peak": FP4_PEAK_TFLOPS, "unit": "TFLOP/s (FP4, dense)",
                "frac": round(tfl / FP4_PEAK_TFLOPS, 4),
                "note": "algorithmic flops (2 x 256 per query x reference pair) over the probe "
                        "steps' event time; the padded tiles the kernel computes are not counted"}
    value = world * B * K / dt
    nq = NF if mode != "none" else 0
    e2e = e2e_bytes(W, H, NF, nq, NREF if mode == "ref" else (NF if mode == "pred" else 0))
    # every stage against the same HBM peak, from the probe steps' per-launch events (the
    # roofline object above is the dominant kernel's, timed live in the timed region)
    stage_roof = {}
    for s_ in STAGES:
        ms = per_step[s_]
        ab = algorithmic_bytes(s_, W, H, nkp, nref) * B
        if ms > 0 and ab > 0:
            gbs = ab / (ms / 1e3) / 1e9
            ent = stage_roof[f"{s_}_kernel" if s_ != "resize" else "pyramid_kernel"] = {
                "ms_per_step": round(ms, 4), "bytes_per_step": round(ab),
                "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
            v = valu_of(s_, probe[s_][0], probe[s_][1])
            if v:
                ent["valu_frac"] = v["frac"]
    if mfma:
        roof["mfma"] = mfma
    return {"value": value, "dt": dt, "K": K, "B": B, "S": S, "J": J, "nkp": nkp, "soak": soak,
            "roofline": roof, "per_step": per_step, "probe_steps": probe_steps,
            "stage_roofline": stage_roof,
            "ref_kp": len(ref_desc_np) if ref_desc_np is not None else None,
            "frames_np": frames_np, "ref_desc_np": ref_desc_np,
            "end_to_end": {"bytes_per_frame": e2e, "achieved": round(e2e * value / 1e9, 2),
                           "unit": "GB/s", "frac": round(e2e * value / 1e9 / HBM_PEAK_GBS, 5),
                           "model": "SURVEY.md §8(d) algorithmic bytes per frame x frames/s"}}


def launch_ranks(args) -> int:
    """`--gpus N` without a launcher: start N rank processes (this script again, with RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1) and return the worst exit
    code.  Runs before anything touches the GPU: the parent imports no torch, so every rank
    owns its device from the start."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                                      env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0:
                rc = rc or code
                for q in pending:  # one rank failed: the others would wait forever
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 1


def _cpu_bf(desc, counts, prev, prev_n, out) -> None:
    """Dry-run stand-in for the GPU matcher (first-wins best / second per query over a popcount
    table); only `--dry-run` uses it."""
    table = np.array([bin(i).count("1") for i in range(256)], np.int32)
    out.fill_(-1)
    for j in range(desc.shape[0]):
        q = desc[j, :int(counts[j])].numpy()
        r = prev[j, :int(prev_n[j])].numpy()
        if len(q) == 0 or len(r) == 0:
            continue
        d = table[q[:, None, :] ^ r[None, :, :]].sum(-1)
        bi = d.argmin(1)
        bd = d[np.arange(len(q)), bi]
        d[np.arange(len(q)), bi] = 257
        res = np.stack([bi, bd, d.min(1)], 1).astype(np.int32)
        out[j, :len(q)] = torch_from_numpy(res)


def torch_from_numpy(a):
    import torch
    return torch.from_numpy(a)


def run_dry(args) -> None:
    """`--dry-run`: the multi-rank plumbing on CPU (gloo) — rendezvous, world-size check, the
    config-4 exchange (shard.PredecessorMatch in `parts` sub-batches), barrier-bracketed timing
    and the max over ranks — at configs[3]'s shape: a global batch of 256 frames dealt
    round-robin (32 per rank at 8 ranks; --per-rank overrides), slabs of capacity(1920, 1080)
    rows (orbfe_keypoint_capacity_params, host arithmetic), random descriptors with up to 96
    keypoints per frame so the CPU stand-in matcher stays cheap.  Not a GPU measurement."""
    import torch
    import torch.distributed as dist
    from orbslam_mapsave_amd.native import keypoint_capacity
    from orbslam_mapsave_amd.shard import PredecessorMatch, global_frame

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
    if rank == 0 and world != args.gpus:
        print(f"bench.py: {world} ranks running but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(3)
    B = args.per_rank if args.per_rank > 0 else max(2, 256 // world)
    cap = keypoint_capacity(ORB_YAML_NFEATURES, *ORB, 1920, 1080)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8)
    cnt = torch.zeros(B, dtype=torch.int32)
    for j in range(B):
        rng = np.random.default_rng(global_frame(rank, world, j))
        n = int(rng.integers(48, 97))
        desc[j, :n] = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8))
        cnt[j] = n
    out = torch.zeros((B, cap, 3), dtype=torch.int32)
    parts = 2
    pm = PredecessorMatch(rank, world, B, cap, "cpu", _cpu_bf, parts=parts)

    def step():
        for p in range(parts):
            pm.gather_part(p, desc, cnt)
        pm.finish(desc, cnt, out)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # a checksum over every global frame's matches, identical for every world size
    chk = torch.tensor([sum(int(global_frame(rank, world, j) + 1) * int(out[j].long().sum())
                            for j in range(B))], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(chk)
    if rank == 0:
        K = args.steps
        print(json.dumps({
            "metric": C4_METRIC + " [dry run: CPU gloo plumbing rehearsal]",
            "match_checksum": int(chk.item()),
            "value": round(world * B * K / dt, 2), "unit": "frames/s", "n_gpus": world,
            "steps": K, "warmup": args.warmup, "ms_per_step": round(dt / K * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": f"synthetic random descriptor slabs ({B} frames x {cap} x 32 B per rank, "
                    "48-96 keypoints each)",
            "dry_run": True,
            "config": {"workload": "config-4 exchange step on CPU: gloo all-gather in 2 "
                                   "sub-batches + frame f vs f-1 brute force",
                       "frames_per_rank_per_step": B, "global_batch": B * world,
                       "parallelism": f"frame-sharded x{world} + gloo all-gather"}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def main() -> None:
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.dry_run:
        return run_dry(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if int(os.environ.get("RANK", "0")) == 0 and world != args.gpus:
        print(f"bench.py: {world} ranks running but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(3)
    if args.config == "c5":
        return run_c5(args)

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    sweep = None
    if args.config == "c2":
        W, H, NF, NREF = 640, 480, 1000, 0
        metric = C2_METRIC
        workload = ("configs[1]: 640x480 extract only (8-level pyramid, FAST-9, oct-tree, "
                    "rBRIEF, 1000 kp), batch sweep B in {1, 64, 256}, >= 1000 frames after 50 "
                    "warm-up frames per B; value at B = 256")
        sweep = {}
        for Bc in (1, 64, 256):
            r = run_extract(args, dev, rank, world, local, W, H, NF, NREF, Bc, "none",
                            max(args.steps, -(-1000 // Bc)), max(args.warmup, -(-50 // Bc)))
            if rank == 0:
                sweep[str(Bc)] = {"frames_per_s": round(r["value"], 1),
                                  "ms_per_call": round(r["dt"] / r["K"] * 1e3, 4),
                                  "frames": Bc * r["K"] * world,
                                  "dominant": r["roofline"]["kernel"],
                                  "dominant_frac": r["roofline"]["frac"],
                                  "stage_ms_per_call": {k: round(v, 4) for k, v in r["per_step"].items()}}
        B = 256
        parallelism = f"frame-sharded x{world}, no data-path collective"
    elif args.config == "c3":
        W, H, NF, NREF = 640, 480, 1000, 2000
        B = args.batch
        metric = METRIC
        workload = ("configs[2]: 640x480 extract (8-level pyramid, FAST-9, oct-tree, rBRIEF, "
                    "1000 kp) + brute-force Hamming match vs a 2000-kp reference frame")
        r = run_extract(args, dev, rank, world, local, W, H, NF, NREF, B, "ref", args.steps,
                        args.warmup)
        parallelism = f"frame-sharded x{world}, no data-path collective"
    else:
        W, H, NF, NREF = 1920, 1080, ORB_YAML_NFEATURES, ORB_YAML_NFEATURES
        B = args.per_rank if args.per_rank > 0 else max(1, 256 // world)
        metric = C4_METRIC
        workload = (f"configs[3]: 1920x1080 @2000 kp, global batch {B * world} sharded "
                    "round-robin, RCCL all-gather of descriptor slabs, frame f vs f-1 match")
        r = run_extract(args, dev, rank, world, local, W, H, NF, NREF, B, "pred", args.steps,
                        args.warmup)
        parallelism = f"frame-sharded x{world} + RCCL all-gather"

    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_budget > 0:
            if args.config == "c4":
                cpu = cpu_baseline(r["frames_np"][:min(args.distinct, 8)], None, args.cpu_budget,
                                   NF, "(1920x1080, extract 2000 kp + BF match vs frame f-1)",
                                   arith=args.arith)
            elif args.config == "c3":
                cpu = cpu_baseline(r["frames_np"][:args.distinct], r["ref_desc_np"],
                                   args.cpu_budget, NF,
                                   "(640x480, extract 1000 kp + BF match vs the 2000-kp reference)",
                                   arith=args.arith)
            else:
                cpu = cpu_baseline(r["frames_np"][:args.distinct], None, args.cpu_budget, NF,
                                   "(640x480, extract 1000 kp, no match)", match=False,
                                   arith=args.arith)
        K, S, J = r["K"], r["S"], r["J"]
        line = {
            "metric": metric, "value": round(r["value"], 2), "unit": "frames/s", "n_gpus": world,
            "steps": K, "warmup": args.warmup, "ms_per_step": round(r["dt"] / K * 1e3, 3),
            "higher_is_better": True, "scaling": "weak" if args.config != "c4" else "strong",
            "vs_baseline": None, "dtype": "u8",
            "data": f"synthetic: seeded textured {W}x{H} u8 frames ({args.distinct} distinct "
                    f"seeds per rank, cycled), resident in HBM",
            "config": {"workload": workload, "arith": args.arith,
                       "frames_per_rank_per_step": B,
                       "streams_per_rank": S, "chunks_per_stream": J,
                       "stream_skew": bool(args.skew) and S > 1 and J >= S,
                       "stage_pipeline": bool(args.pipeline) and S > 1 and args.config == "c3",
                       "global_batch": B * world, "nfeatures": NF, "reference_kp": r["ref_kp"],
                       "mean_kp_per_frame": round(r["nkp"], 1), "parallelism": parallelism},
            "roofline": r["roofline"],
            "end_to_end": r["end_to_end"],
            "cpu_baseline": cpu,
            "stage_ms_per_step": {k: round(v, 4) for k, v in r["per_step"].items()},
            "stage_roofline": r.get("stage_roofline"),
            "stage_note": (f"summed kernel durations per step over {r['probe_steps']} untimed "
                           "single-stream probe steps (events on every launch, the whole batch "
                           "in one call); the timed steps are uninstrumented" +
                           (f" and overlap {S} sub-batch streams, so ms_per_step is below the "
                            "sum" if S > 1 else "")),
            "soak": r["soak"],
        }
        if sweep is not None:
            line["batch_sweep"] = sweep
        if cpu:
            line["gpu_over_cpu"] = round(r["value"] / cpu["value"], 1)
            line["gpu_over_cpu_all_core"] = round(r["value"] / cpu["all_core"]["value"], 1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
