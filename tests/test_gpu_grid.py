"""A16 — the Frame grid, directly: Frame::AssignFeaturesToGrid / PosInGrid (Frame.cc:341-356,
500-510) and Frame::GetFeaturesInArea (Frame.cc:445-498) on the GPU (grid_lds_kernel for up to
8,192 keypoints, grid_kernel above; features_in_area and features_in_area_wave) against the
oracle's restatement (oracle/orb_oracle.cpp build_grid / features_in_area), candidate lists and
their ORDER compared exactly.

The cases pin what the matchers' first-wins ties depend on:
* insertion by roundf (half away from zero): keypoints whose (x - minX) * invW lands exactly on
  k + 0.5 (x = 10k + 5 at 640 / 64);
* keypoints outside the 64 x 48 grid (undistorted points can leave the image) are dropped;
* the level filter applies only if minLevel > 0 || maxLevel >= 0 (466, 479-486);
* floor / ceil cell bounds with radii that put the window edge exactly on a cell edge, and
  the strict |dx| < r, |dy| < r test;
* candidate order ix-major, then iy, then insertion (keypoint index) order.
"""
import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE, Frame

pytestmark = pytest.mark.gpu

SCALE = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
LEVELS = [(-1, -1), (0, 0), (1, 3), (0, -1), (2, -1), (-1, 2), (7, 7)]


def grid_frame(n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    k = np.zeros(n, KEYPOINT_DTYPE)
    k["x"] = rng.uniform(-8, 648, n).astype(np.float32)
    k["y"] = rng.uniform(-8, 488, n).astype(np.float32)
    # a fifth of the points on roundf's .5 boundaries (x = 10 i + 5, y = 10 j + 5)
    b = rng.random(n) < 0.2
    k["x"][b] = (10 * rng.integers(-1, 65, b.sum()) + 5).astype(np.float32)
    k["y"][b] = (10 * rng.integers(-1, 49, b.sum()) + 5).astype(np.float32)
    k["octave"] = rng.integers(0, 8, n)
    k["angle"] = rng.uniform(0, 360, n)
    k["size"] = 31.0
    k["class_id"] = -1
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    return Frame(k, desc, 640, 480, SCALE)


def queries(nq, seed):
    rng = np.random.Generator(np.random.PCG64(seed + 1000))
    x = rng.uniform(-30, 670, nq).astype(np.float32)
    y = rng.uniform(-30, 510, nq).astype(np.float32)
    r = rng.choice([1.0, 2.5, 4.0, 7.5, 15.0, 40.0, 100.0], nq).astype(np.float32)
    # window edges exactly on cell edges: x, y on multiples of 10 and r a multiple of 10
    e = rng.random(nq) < 0.25
    x[e] = (10 * rng.integers(0, 65, e.sum())).astype(np.float32)
    y[e] = (10 * rng.integers(0, 49, e.sum())).astype(np.float32)
    r[e] = (10 * rng.integers(1, 6, e.sum())).astype(np.float32)
    lv = np.array([LEVELS[i % len(LEVELS)] for i in range(nq)], np.int32)
    return x, y, r, lv[:, 0].copy(), lv[:, 1].copy()


@pytest.fixture(scope="module")
def mt():
    from orbslam_mapsave_amd.native import ORBmatcher
    m = ORBmatcher(0.9, True, device=0)
    yield m
    m.close()


@pytest.mark.parametrize("n", [1, 100, 1000, 8192, 8193, 9000])
@pytest.mark.parametrize("wave", [False, True])
def test_features_in_area(mt, n, wave):
    f = grid_frame(n, n)
    x, y, r, lo, hi = queries(1500, n)
    got = mt.GetFeaturesInArea(f, x, y, r, lo, hi, wave=wave)
    total = 0
    for q in range(len(x)):
        exp = oracle.features_in_area(f, float(x[q]), float(y[q]), float(r[q]), int(lo[q]),
                                      int(hi[q]))
        assert np.array_equal(got[q], exp), (q, x[q], y[q], r[q], lo[q], hi[q])
        total += len(exp)
    assert total > 0


def test_roundf_half_away_insertion(mt):
    """A keypoint at x = 5 (invW * 5 = 0.5) belongs to column 1 (roundf), not 0 (rint); one
    at x = -5 (-0.5 -> -1) is outside the grid and never returned."""
    k = np.zeros(3, KEYPOINT_DTYPE)
    k["x"] = [5.0, -5.0, 15.0]
    k["y"] = [5.0, 5.0, 25.0]
    k["class_id"] = -1
    f = Frame(k, np.zeros((3, 32), np.uint8), 640, 480, SCALE)
    # window cells: floor((0 - 6) * 0.1) = -1 -> 0 .. ceil(0.6) = 1, so columns 0 and 1
    got = mt.GetFeaturesInArea(f, [0.0], [0.0], [6.0], wave=False)[0]
    assert list(got) == list(oracle.features_in_area(f, 0.0, 0.0, 6.0)) == [0]
    # column order: kp 0 (ix 1, iy 1) before kp 2 (ix 2, iy 3)
    got = mt.GetFeaturesInArea(f, [10.0], [15.0], [30.0], wave=True)[0]
    assert list(got) == list(oracle.features_in_area(f, 10.0, 15.0, 30.0)) == [0, 2]
