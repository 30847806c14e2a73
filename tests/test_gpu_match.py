"""GPU parity of the matchers (liborbfe.so through the C ABI) against the CPU oracle.

Every output is an index, a count or a distance, so every comparison is exact: Hamming
distances, brute-force (best_idx, best, second), vnMatches12 + nmatches + updated
vbPrevMatched (SearchForInitialization), the per-keypoint MapPoint assignment +
Observations + nmatches (both SearchByProjection overloads), and isInFrustum's outputs.
"""
import numpy as np
import pytest

import oracle
import scenarios as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mt():
    from orbslam_mapsave_amd.native import ORBmatcher
    m = ORBmatcher(0.9, True, device=0)
    yield m
    m.close()


@pytest.fixture(scope="module", params=["fp4", "i8"])
def bf(request):
    """A matcher per brute-force kernel: the FP4 MFMA form (default) and the i8 MFMA form
    (ORBFE_BF_I8=1 at creation)."""
    import os
    from orbslam_mapsave_amd.native import ORBmatcher
    old = os.environ.pop("ORBFE_BF_I8", None)
    if request.param == "i8":
        os.environ["ORBFE_BF_I8"] = "1"
    try:
        m = ORBmatcher(0.9, True, device=0)
    finally:
        os.environ.pop("ORBFE_BF_I8", None)
        if old is not None:
            os.environ["ORBFE_BF_I8"] = old
    yield m
    m.close()


def test_hamming_random(mt):
    rng = np.random.Generator(np.random.PCG64(1))
    a, b = S.random_desc(rng, 5000), S.random_desc(rng, 5000)
    assert np.array_equal(mt.DescriptorDistance(a, b), oracle.hamming(a, b))
    assert mt.DescriptorDistance(a[0], a[0]) == 0
    assert mt.DescriptorDistance(a[0], ~a[0]) == 256


@pytest.mark.parametrize("nq,nr", [(1000, 2000), (1, 1), (300, 7), (513, 1500), (40, 4097), (100, 65535)])
def test_bf_match_random(bf, nq, nr):
    """(100, 65535): the largest reference set the 16-bit index field of the keys holds."""
    rng = np.random.Generator(np.random.PCG64(nq + nr))
    q, r = S.random_desc(rng, nq), S.random_desc(rng, nr)
    got = bf.bf_match(q, r)
    exp = oracle.bf_match(q, r)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)


def test_bf_match_ties(bf):
    rng = np.random.Generator(np.random.PCG64(3))
    base = S.random_desc(rng, 4)
    r = base[rng.integers(0, 4, 700)]       # many exact duplicates: first-wins ties
    q = S.flip_bits(base[rng.integers(0, 4, 300)], rng, 0.02)
    for g, e in zip(bf.bf_match(q, r), oracle.bf_match(q, r)):
        assert np.array_equal(g, e)


@pytest.mark.parametrize("nq,nr", [(257, 64), (64, 65), (31, 63), (2, 128), (700, 129)])
def test_bf_match_extremes(bf, nq, nr):
    """Partial tiles and blocks, all-zero / all-one / complementary descriptors (distances 0 and
    256: a distance-256 reference never wins), duplicates (first-wins)."""
    rng = np.random.Generator(np.random.PCG64(7 * nq + nr))
    q, r = S.random_desc(rng, nq), S.random_desc(rng, nr)
    q[0], q[-1] = 0, 255
    r[:] = np.where(rng.random((nr, 1)) < 0.2, ~q[rng.integers(0, nq, nr)], r)
    r[nr // 2], r[-1] = 0, 255
    r[nr // 3] = q[1]
    got = bf.bf_match(q, r)
    exp = oracle.bf_match(q, r)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)
    assert got[1][0] == 0 and got[1][-1] == 0                # zero / all-one references exist
    z = bf.bf_match(np.zeros((3, 32), np.uint8), np.full((5, 32), 255, np.uint8))
    assert (z[0] == -1).all() and (z[1] == 256).all() and (z[2] == 256).all()


def test_bf_match_extracted(bf):
    f1, f2 = S.extract_frame(0, 1000), S.extract_frame(1, 2000)
    for g, e in zip(bf.bf_match(f1.desc, f2.desc), oracle.bf_match(f1.desc, f2.desc)):
        assert np.array_equal(g, e)


@pytest.mark.parametrize("seed,window,check_ori", [(0, 100, True), (1, 100, True), (2, 50, False),
                                                   (3, 200, True)])
def test_search_for_initialization(mt, seed, window, check_ori):
    from orbslam_mapsave_amd.native import ORBmatcher
    m = ORBmatcher(0.9, check_ori, device=0)
    f1, f2, prev = S.sfi_case(seed)
    g12, gn, gprev = m.SearchForInitialization(f1, f2, prev, window)
    e12, en, eprev = oracle.search_for_initialization(f1, f2, prev, window, 0.9, check_ori)
    assert gn == en
    assert np.array_equal(g12, e12)
    assert np.array_equal(gprev, eprev)
    m.close()


@pytest.mark.parametrize("seed,th,stereo,prior,m", [(0, 1.0, False, False, 50000),
                                                    (1, 3.0, True, True, 20000),
                                                    (2, 5.0, False, True, 5000)])
def test_search_by_projection_local(seed, th, stereo, prior, m):
    from orbslam_mapsave_amd.native import ORBmatcher
    mt = ORBmatcher(0.8, True, device=0)
    f, mps, fmp, fobs, ids = S.sbp_local_case(seed, m, stereo=stereo, prior=prior)
    g = mt.SearchByProjection(f, mps, th, fmp, fobs, ids)
    e = oracle.search_by_projection_local(f, mps, th, 0.8, fmp, fobs, ids)
    assert g[2] == e[2]
    assert np.array_equal(g[0], e[0])
    assert np.array_equal(g[1], e[1])
    mt.close()


@pytest.mark.parametrize("seed,stereo,mono,th", [(0, False, True, 15.0), (1, False, True, 30.0),
                                                 (2, True, False, 7.0)])
def test_search_by_projection_last(mt, seed, stereo, mono, th):
    c = S.sbp_last_case(seed, stereo=stereo)
    args = (c["cur"], c["tcw_cur"], c["cam"], c["last_keys"], c["last_valid"], c["last_outlier"],
            c["last_xyz"], c["last_desc"], c["last_nobs"], c["tcw_last"])
    g = mt.SearchByProjectionLast(*args, th, mono, last_ids=c["last_ids"])
    e = oracle.search_by_projection_last(*args, th, mono, True, last_ids=c["last_ids"])
    assert g[2] == e[2]
    assert np.array_equal(g[0], e[0])
    assert np.array_equal(g[1], e[1])


def test_is_in_frustum(mt):
    fc = S.frustum_case(0)
    g = mt.is_in_frustum(**fc)
    e = oracle.is_in_frustum(**fc)
    assert np.array_equal(g[0], e[0])
    sel = e[0] == 1
    for a, b in zip(g[1:], e[1:]):
        assert np.array_equal(a[sel], b[sel])


@pytest.mark.parametrize("n_contend,check_ori", [(5, True), (24, False), (70, True), (90, False)])
def test_search_for_initialization_contended(mt, n_contend, check_ori):
    """Many F1 queries competing for the same F2 keypoints: steals (466-470) in every order of
    distances; with n_contend > 64 more acceptors of one slot in a round than the first slot
    lists hold, so the rounds rerun with lists sized for every query."""
    from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE, Frame
    from orbslam_mapsave_amd.native import ORBmatcher
    rng = np.random.Generator(np.random.PCG64(n_contend))
    scale = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    n2 = 300
    k2 = np.zeros(n2, KEYPOINT_DTYPE)
    k2["x"], k2["y"] = rng.uniform(20, 620, n2), rng.uniform(20, 460, n2)
    k2["angle"] = rng.uniform(0, 360, n2)
    k2["octave"] = rng.integers(0, 2, n2)
    k2["class_id"] = -1
    d2 = S.random_desc(rng, n2)
    hubs = rng.choice(np.flatnonzero(k2["octave"] == 0), 4, replace=False)
    q_keys, q_desc = [], []
    for h in hubs:  # n_contend near-copies of each hub, distances in random order
        for _ in range(n_contend):
            k = np.zeros(1, KEYPOINT_DTYPE)[0]
            k["x"], k["y"] = k2["x"][h] + rng.uniform(-5, 5), k2["y"][h] + rng.uniform(-5, 5)
            k["angle"] = (k2["angle"][h] + rng.choice([0.0, 1.0, 180.0])) % 360
            k["class_id"] = -1
            q_keys.append(k)
            q_desc.append(S.flip_bits(d2[h][None], rng, rng.uniform(0.0, 0.15))[0])
    n_rand = 200
    kr = np.zeros(n_rand, KEYPOINT_DTYPE)
    kr["x"], kr["y"] = rng.uniform(20, 620, n_rand), rng.uniform(20, 460, n_rand)
    kr["angle"] = rng.uniform(0, 360, n_rand)
    kr["octave"] = rng.integers(0, 3, n_rand)
    kr["class_id"] = -1
    perm = rng.permutation(len(q_keys) + n_rand)
    k1 = np.concatenate([np.array(q_keys, KEYPOINT_DTYPE), kr])[perm]
    d1 = np.concatenate([np.array(q_desc, np.uint8), S.random_desc(rng, n_rand)])[perm]
    f1, f2 = Frame(k1, d1, 640, 480, scale), Frame(k2, d2, 640, 480, scale)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    m = ORBmatcher(0.9, check_ori, device=0)
    g12, gn, gprev = m.SearchForInitialization(f1, f2, prev, 100)
    e12, en, eprev = oracle.search_for_initialization(f1, f2, prev, 100, 0.9, check_ori)
    assert en > 0
    assert gn == en
    assert np.array_equal(g12, e12)
    assert np.array_equal(gprev, eprev)
    assert m.last_rounds() > 0  # the fixed-point rounds resolved it
    m.close()


@pytest.mark.parametrize("pre", ["1", "0"])
def test_bf_match_batch_shared_refs(pre, monkeypatch):
    """orbfe_bf_match_batch_device with one reference set for the batch (r_pitch 0): expanded to
    FP4 fragments once per call (default) or by every workgroup (ORBFE_BF_PRE=0); per-entry
    reference counts that differ (partial tiles, a single row, none, the whole set) and ragged
    query counts — every (best index, best, second) triple equal to the oracle's."""
    import torch
    from orbslam_mapsave_amd.native import ORBmatcher
    monkeypatch.setenv("ORBFE_BF_PRE", pre)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(77)
    nref, cap = 2007, 300
    nrs = [2007, 65, 1, 0, 64, 1999, 130, 2007]
    nqs = [300, 17, 256, 5, 0, 299, 64, 1]
    nb = len(nrs)
    ref = rng.integers(0, 256, (nref, 32), dtype=np.uint8)
    ref[5] = ref[9]  # equal distances: the lower index wins
    q = rng.integers(0, 256, (nb, cap, 32), dtype=np.uint8)
    q[0, 3] = ref[100]
    d_r = torch.from_numpy(ref).to(dev)
    d_q = torch.from_numpy(q).to(dev)
    d_nq = torch.tensor(nqs, dtype=torch.int32, device=dev)
    d_nr = torch.tensor(nrs, dtype=torch.int32, device=dev)
    d_out = torch.full((nb, cap, 3), -7, dtype=torch.int32, device=dev)
    mt = ORBmatcher(0.9, True, device=0)
    try:
        mt.bf_match_batch_device(d_q.data_ptr(), cap * 32, d_nq.data_ptr(), cap, d_r.data_ptr(), 0,
                                 d_nr.data_ptr(), nb, d_out.data_ptr())
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
    finally:
        mt.close()
    for b in range(nb):
        if nqs[b] == 0:
            continue
        bi, bd, sd = oracle.bf_match(q[b, :nqs[b]], ref[:nrs[b]])
        got = out[b, :nqs[b]]
        assert np.array_equal(got[:, 0], bi), b
        assert np.array_equal(got[:, 1], bd), b
        assert np.array_equal(got[:, 2], sd), b


def _load_sfi_problem(path):
    from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE, Frame
    raw = open(path, "rb").read()
    o, fr = 0, []
    scale = oracle.tables(oracle.params(2000, 1.2, 8, 20, 7))["scale"]
    for _ in range(2):
        n = int(np.frombuffer(raw, np.int32, 1, o)[0])
        o += 4
        k = np.frombuffer(raw, KEYPOINT_DTYPE, n, o).copy()
        o += 28 * n
        d = np.frombuffer(raw, np.uint8, 32 * n, o).reshape(n, 32).copy()
        o += 32 * n
        fr.append(Frame(k, d, 640, 480, scale))
    return fr


@pytest.mark.parametrize("check_ori", [True, False])
def test_search_for_initialization_convergence_rounds(check_ori):
    """Two Ini frames (2000 keypoints) of tests/cpp/threads_test.cpp's images
    (tests/golden/sfi_conv3_problem.bin, written by that program with THREADS_DUMP set; oracle
    extractions): at windows 60-100 the fixed-point rounds converge at round 3 of a 6-round
    batch, where the rounds launched past convergence used to clear the converged acceptor
    lists (0 matches instead of 37-62).  Every window 20-200 bit-exact, on one matcher."""
    import os
    from orbslam_mapsave_amd.native import ORBmatcher
    f1, f2 = _load_sfi_problem(os.path.join(os.path.dirname(__file__), "golden", "sfi_conv3_problem.bin"))
    prev = np.stack([f1.keys["x"], f1.keys["y"]], 1).astype(np.float32)
    m = ORBmatcher(0.9, check_ori, device=0)
    rounds = set()
    try:
        for win in range(20, 201, 10):
            g12, gn, gprev = m.SearchForInitialization(f1, f2, prev, win)
            e12, en, eprev = oracle.search_for_initialization(f1, f2, prev, win, 0.9, check_ori)
            assert gn == en, (win, gn, en)
            assert np.array_equal(g12, e12) and np.array_equal(gprev, eprev), win
            rounds.add(m.last_rounds())
    finally:
        m.close()
    assert 4 in rounds, rounds  # the converge-at-round-3 case is exercised
