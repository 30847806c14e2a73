"""The oct-tree's global-array path (orbfe_extract.hip octree_kernel): a level whose FAST list
holds more keys than the plan's LDS key capacity (oct_keys = min(4096, max(1024, 9 x the
largest level budget rounded up to 256)), orbfe_extract.hip plan) keeps its keys and node lists
in global memory instead of LDS.  These frames are built so that such a level exists — asserted
from the oracle's FAST lists before the GPU runs — and the extraction must stay bit-exact
(ORBextractor.cc:538-762 through the same list emulation)."""
import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.synth import synthetic_frame

pytestmark = pytest.mark.gpu


def oct_keys(p) -> int:
    nf = int(max(oracle.tables(p)["nfeat"]))
    return min(4096, max(1024, (9 * nf + 255) & ~255))


def noise_frame(seed, w, h):
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(0, 256, (h, w), dtype=np.uint8)


@pytest.mark.parametrize("w,h,nf,ini,kind", [(640, 480, 1000, 20, "noise"),
                                             (1920, 1080, 2000, 7, "textured"),
                                             (1280, 720, 300, 7, "textured")])
def test_octree_global_path(w, h, nf, ini, kind):
    from orbslam_mapsave_amd.native import ORBextractor
    p = oracle.params(nf, 1.2, 8, ini, 7)
    img = noise_frame(5, w, h) if kind == "noise" else synthetic_frame(6, w, h)
    cap = oct_keys(p)
    counts = [len(oracle.fast_keys(p, lv)) for lv in oracle.pyramid(p, img)]
    assert max(counts) > cap, (counts, cap)  # some level takes the global-array path
    ex = ORBextractor(nf, 1.2, 8, ini, 7, device=0, max_width=w, max_height=h)
    kps, desc = ex(img)
    okps, odesc = oracle.extract(p, img)
    assert len(kps) == len(okps) > 0
    assert kps.tobytes() == okps.tobytes()
    assert np.array_equal(desc, odesc)
    for lv, n in enumerate(counts):  # the GPU's FAST lists are the oracle's (sizes included)
        assert len(ex.get_fast_keys(lv)) == n
    ex.close()
