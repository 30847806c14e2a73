#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY — residuals of the oracle's pinned semantic choices (SURVEY §8a
H2/H4/H5/H6) against the other readings a real x86 build of the reference would take.

The reference cannot be built here (OpenCV 3.3.1 absent), so parity stays "unpinned"; what CAN
be measured is how often each build-dependent choice changes the output.  For every variant
the oracle (oracle/orb_oracle.cpp) is switched to the alternative reading (oracle.variant) and
its extraction is compared with the pinned oracle — the one the GPU is bit-exact against — on:

* frames: the bench's 32 synthetic 640x480 frames (seeds 0-31; seeds 0-4 are tests/golden's)
  at 1000 features, and seed 0 at 1920x1080 / 2000 features;
* keypoints: symmetric difference of the (x, y, octave) sets, and order differences when the
  sets agree;
* descriptors: over keypoints present in both, keypoints with any differing byte, differing
  bytes and bits;
* pixels: pyramid pixels (H5) and blurred-level pixels (H6) that differ.

Variants (orb_oracle.h): H2 oct-tree phase-2 ties by real glibc heap address (the reference's
allocation sequence replayed on this glibc), H4 glibc cosf/sinf, H4 FMA contraction (GCC -O3
-march=x86-64-v3 -ffp-contract=fast on the reference's expression), H5 OpenCV's SSE2
VResizeLinearVec_32s8u body, H6 OpenCV's SSE2 SymmColumnVec_32s8u (float) body, and all of
them together ("as_built_x86").

Usage (repo root): python -m oracle.residuals  -> tests/golden/residuals.json
"""
from __future__ import annotations

import json
import os
import platform
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from orbslam_mapsave_amd.synth import synthetic_frame  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "residuals.json")
VARIANTS = {
    "H2_heap_address": oracle.VAR_H2_ADDR,
    "H4_glibc_cosf": oracle.VAR_H4_COSF,
    "H4_fma_contraction": oracle.VAR_H4_FMA,
    "H4_cosf_and_fma": oracle.VAR_H4_COSF | oracle.VAR_H4_FMA,
    "H5_sse2_resize": oracle.VAR_H5_SSE2,
    "H6_simd_blur": oracle.VAR_H6_SIMD,
    "as_built_x86": 31,
}


def _key_ids(kps: np.ndarray) -> np.ndarray:
    rec = np.zeros(len(kps), [("x", "<f4"), ("y", "<f4"), ("o", "<i4")])
    rec["x"], rec["y"], rec["o"] = kps["x"], kps["y"], kps["octave"]
    return rec.view(np.void(12)).ravel() if len(kps) else np.zeros(0, np.void(12))


def compare(ck, cd, vk, vd) -> dict:
    """Counts of what a variant's extraction (vk, vd) changes vs the pinned one (ck, cd)."""
    a, b = _key_ids(ck), _key_ids(vk)
    sa, sb = set(a.tolist()), set(b.tolist())
    only_c, only_v = len(sa - sb), len(sb - sa)
    order = 0
    if not only_c and not only_v and len(a) == len(b):
        order = int((a != b).sum())
    pos_v = {k: i for i, k in enumerate(b.tolist())}
    kp_desc = bytes_ = bits = angle = 0
    for i, k in enumerate(a.tolist()):
        j = pos_v.get(k)
        if j is None:
            continue
        if ck["angle"][i] != vk["angle"][j]:
            angle += 1
        x = np.bitwise_xor(cd[i], vd[j])
        if x.any():
            kp_desc += 1
            bytes_ += int(np.count_nonzero(x))
            bits += int(np.unpackbits(x).sum())
    return dict(keypoints=len(ck), only_pinned=only_c, only_variant=only_v, order_diff=order,
                common=len(sa & sb), angle_diff=angle, desc_kp_diff=kp_desc,
                desc_byte_diff=bytes_, desc_bit_diff=bits)


def pixel_diffs(p, img, flags) -> dict:
    """Pyramid pixels (H5) and blurred-level pixels (H6) a variant changes."""
    out = {}
    base = oracle.pyramid(p, img)
    if flags & oracle.VAR_H5_SSE2:
        with oracle.variant(oracle.VAR_H5_SSE2):
            var = oracle.pyramid(p, img)
        out["pyramid_px_diff"] = [int((x != y).sum()) for x, y in zip(base, var)]
        out["pyramid_px"] = [int(x.size) for x in base]
    if flags & oracle.VAR_H6_SIMD:
        blur0 = [oracle.gaussian_blur(l) for l in base]
        with oracle.variant(oracle.VAR_H6_SIMD):
            blur1 = [oracle.gaussian_blur(l) for l in base]
        out["blur_px_diff"] = [int((x != y).sum()) for x, y in zip(blur0, blur1)]
        out["blur_px"] = [int(x.size) for x in base]
    return out


def frame_set(quick: bool = False):
    """(name, params, images): the bench's frames (and golden seeds) + one 1080p frame."""
    p1 = oracle.params(1000, 1.2, 8, 32, 7)
    seeds = [0] if quick else list(range(32))
    sets = [("640x480@1000", p1, [(s, synthetic_frame(s, 640, 480)) for s in seeds])]
    if not quick:
        sets.append(("1920x1080@2000", oracle.params(2000, 1.2, 8, 32, 7),
                     [(0, synthetic_frame(0, 1920, 1080))]))
    return sets


def measure(quick: bool = False, variants=None) -> dict:
    """Every variant against the portable scalar reading (variant 0)."""
    with oracle.variant(oracle.VAR_SCALAR):
        return _measure(quick, variants)


def _measure(quick: bool = False, variants=None) -> dict:
    variants = variants or VARIANTS
    res = {"variants": {}, "frames": {}}
    for name, p, frames in frame_set(quick):
        res["frames"][name] = [s for s, _ in frames]
        canon = [oracle.extract(p, img) for _, img in frames]
        for vname, flags in variants.items():
            # every frame through the variant first, so the H2 replay's heap history is the
            # extractor's own (frame after frame, as in Tracking), then the comparisons
            with oracle.variant(flags):
                var = [oracle.extract(p, img) for _, img in frames]
            per = []
            for (seed, img), (ck, cd), (vk, vd) in zip(frames, canon, var):
                c = compare(ck, cd, vk, vd)
                c["seed"] = seed
                c.update(pixel_diffs(p, img, flags & (oracle.VAR_H5_SSE2 | oracle.VAR_H6_SIMD)))
                per.append(c)
            tot = {k: int(sum(c[k] for c in per)) for k in
                   ("keypoints", "only_pinned", "only_variant", "order_diff", "common",
                    "angle_diff", "desc_kp_diff", "desc_byte_diff", "desc_bit_diff")}
            tot["frames"] = len(per)
            tot["frames_with_kp_set_diff"] = sum(1 for c in per if c["only_pinned"] or c["only_variant"])
            tot["frames_with_any_diff"] = sum(
                1 for c in per if c["only_pinned"] or c["only_variant"] or c["order_diff"]
                or c["desc_kp_diff"] or c["angle_diff"])
            for key in ("pyramid_px_diff", "blur_px_diff"):
                if key in per[0]:
                    tot[key] = int(sum(sum(c[key]) for c in per))
                    tot[key.replace("_diff", "")] = int(sum(sum(c[key.replace("_diff", "")]) for c in per))
            res["variants"].setdefault(vname, {})[name] = {"total": tot, "per_frame": per}
    return res


def host_info() -> dict:
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu": model, "glibc": " ".join(platform.libc_ver()), "machine": platform.machine()}


def h2_repeats(n: int = 4) -> list[int]:
    """H2 depends on the heap history: the 32-frame pass repeated in one process (the heap
    state each pass starts from is what the previous pass left), keypoints changed per pass."""
    with oracle.variant(oracle.VAR_SCALAR):
        return _h2_repeats(n)


def _h2_repeats(n: int) -> list[int]:
    p = oracle.params(1000, 1.2, 8, 32, 7)
    frames = [synthetic_frame(s, 640, 480) for s in range(32)]
    canon = [oracle.extract(p, img) for img in frames]
    out = []
    for _ in range(n):
        with oracle.variant(oracle.VAR_H2_ADDR):
            var = [oracle.extract(p, img) for img in frames]
        out.append(int(sum(compare(ck, cd, vk, vd)["only_pinned"]
                           for (ck, cd), (vk, vd) in zip(canon, var))))
    return out


def main() -> None:
    res = measure()
    res["h2_repeats_only_pinned"] = h2_repeats()
    res["host"] = host_info()
    res["note"] = ("counts vs the pinned oracle (variant 0); see oracle/residuals.py and "
                   "tests/golden/README.md")
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1)
    for vname, by in res["variants"].items():
        for fs, r in by.items():
            t = r["total"]
            print(f"{vname:20s} {fs:16s} frames {t['frames_with_any_diff']}/{t['frames']} "
                  f"kp-set {t['only_pinned']}/{t['keypoints']} order {t['order_diff']} "
                  f"desc-kp {t['desc_kp_diff']} bytes {t['desc_byte_diff']} "
                  f"px {t.get('pyramid_px_diff', '-')}/{t.get('blur_px_diff', '-')}")


if __name__ == "__main__":
    main()
