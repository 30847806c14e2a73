"""§8(f) row 4 (part) — MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:483-548): the
pairwise-Hamming + median choice of a map point's descriptor among its observations.

CPU: oracle vs a numpy restatement (full distance matrix, np.sort, index (size_t)(0.5*(N-1)),
first minimum).  GPU: distinctive_kernel (one wave per map point, bisection median) bit-exact
vs the oracle, host and device forms; N from 0 to 300 observations, duplicate descriptors for
ties, N > 64 exercises the un-staged path.
"""
import numpy as np
import pytest

import oracle


def make_case(seed=0, n_mp=2000, max_obs=40, big=(65, 130, 300)):
    rng = np.random.Generator(np.random.PCG64(seed))
    counts = rng.integers(0, max_obs + 1, n_mp)
    counts[:len(big)] = big
    counts[len(big)] = 0
    counts[len(big) + 1] = 1
    counts[len(big) + 2] = 2
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    base = rng.integers(0, 256, (n_mp, 32), dtype=np.uint8)
    desc = np.repeat(base, counts, axis=0)
    bits = np.unpackbits(desc, axis=1)
    flip = (rng.uniform(size=bits.shape) < rng.choice([0.02, 0.1, 0.3], size=(len(desc), 1))).astype(np.uint8)
    desc = np.packbits(bits ^ flip, axis=1)
    dup = rng.uniform(size=len(desc)) < 0.1  # duplicated neighbours -> equal medians
    idx = np.nonzero(dup)[0]
    idx = idx[idx > 0]
    desc[idx] = desc[idx - 1]
    return off, desc


def restated(off, desc):
    n = len(off) - 1
    best = np.full(n, -1, np.int32)
    out = np.zeros((n, 32), np.uint8)
    for i in range(n):
        d = desc[off[i]:off[i + 1]]
        N = len(d)
        if N == 0:
            continue
        dm = np.unpackbits(d[:, None, :] ^ d[None, :, :], axis=2).sum(2)
        med = np.sort(dm, axis=1)[:, int(0.5 * (N - 1))]
        best[i] = int(np.argmin(med))  # first minimum
        out[i] = d[best[i]]
    return best, out


def test_oracle_vs_restatement():
    off, desc = make_case(0, n_mp=400)
    b, o = oracle.distinctive_descriptors(off, desc)
    rb, ro = restated(off, desc)
    assert np.array_equal(b, rb)
    assert np.array_equal(o[b >= 0], ro[rb >= 0])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_gpu_distinctive(seed):
    from orbslam_mapsave_amd.native import ORBmatcher
    off, desc = make_case(seed)
    m = ORBmatcher(device=0)
    b, o = m.ComputeDistinctiveDescriptors(off, desc)
    ob, oo = oracle.distinctive_descriptors(off, desc)
    assert np.array_equal(b, ob)
    assert np.array_equal(o[b >= 0], oo[ob >= 0])
    m.close()
