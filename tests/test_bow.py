"""§8(f) row 4 — bag of words: DBoW2's TemplatedVocabulary<FORB> (vendored in the reference as
Thirdparty/DBoW2) loaded from the ORBvoc.txt text format, transform -> BowVector +
FeatureVector (Frame::ComputeBoW, Frame.cc:513-520), and ORBmatcher::SearchByBoW(KeyFrame*,
Frame&) (ORBmatcher.cc:159-291).

ORBvoc.txt itself is absent from the mount, so every case runs on synthetic vocabularies
written in the same text format (synth.synthetic_vocabulary_text).  CPU: the C oracle against a
pure-Python restatement of loadFromTextFile / transform / BowVector::normalize /
FeatureVector::addFeature / SearchByBoW.  GPU: the HIP vocabulary (bow_descend_kernel,
bow_assemble_kernel, SearchByBoW through the greedy resolver) bit-exact against the oracle,
doubles compared bit for bit.
"""
import math

import numpy as np
import pytest

import oracle
import scenarios as S
from orbslam_mapsave_amd.synth import synthetic_vocabulary_text

VOCABS = {  # name: (k, L, scoring, weighting)
    "k10L4_l1_tfidf": (10, 4, 0, 0),
    "k8L3_l2_tf": (8, 3, 1, 1),
    "k10L3_dot_tfidf": (10, 3, 5, 0),
    "k6L4_l1_idf": (6, 4, 0, 2),
    "k10L3_chi_binary": (10, 3, 2, 3),
}


@pytest.fixture(scope="module")
def frames():
    f1 = S.extract_frame(0, 1000, ini=20)
    f2 = S.extract_frame(0, 1000, shift=(2, -3), ini=20)
    return f1, f2


@pytest.fixture(scope="module")
def vocab_paths(tmp_path_factory, frames):
    d = tmp_path_factory.mktemp("voc")
    out = {}
    for i, (name, (k, L, sc, wt)) in enumerate(VOCABS.items()):
        p = str(d / f"{name}.txt")
        synthetic_vocabulary_text(p, k, L, seed=i, scoring=sc, weighting=wt,
                                  anchors=frames[0].desc[::37])
        out[name] = p
    return out


def load_text(path):
    """loadFromTextFile restated (blank lines skipped)."""
    with open(path) as fh:
        lines = fh.read().split("\n")
    k, L, sc, wt = (int(x) for x in lines[0].split())
    nodes = [dict(parent=0, children=[], desc=np.zeros(32, np.uint8), weight=0.0, word=0)]
    nwords = 0
    for ln in lines[1:]:
        if not ln.strip():
            continue
        t = ln.split()
        nd = dict(parent=int(t[0]), children=[], desc=np.array([int(x) for x in t[2:34]], np.uint8),
                  weight=float(t[34]), word=0)
        if int(t[1]) > 0:
            nd["word"] = nwords
            nwords += 1
        nodes[nd["parent"]]["children"].append(len(nodes))
        nodes.append(nd)
    return dict(k=k, L=L, scoring=sc, weighting=wt, nodes=nodes, nwords=nwords)


def transform_restated(voc, desc, levelsup):
    nodes = voc["nodes"]
    nid_level = voc["L"] - levelsup
    bow, fv = {}, {}
    if voc["nwords"] == 0:
        return bow, fv
    must = voc["scoring"] != 5
    tf = voc["weighting"] in (0, 1)
    for i, d in enumerate(desc):
        node, level, nid = 0, 0, 0
        while True:
            level += 1
            ch = nodes[node]["children"]
            dist = [int(np.unpackbits(d ^ nodes[c]["desc"]).sum()) for c in ch]
            node = ch[int(np.argmin(dist))]  # first minimum = strict '<' scan
            if level == nid_level:
                nid = node
            if not nodes[node]["children"]:
                break
        w = nodes[node]["weight"]
        if w > 0:
            word = nodes[node]["word"]
            if tf:
                bow[word] = bow[word] + w if word in bow else w
            else:
                bow.setdefault(word, w)
            fv.setdefault(nid, []).append(i)
    keys = sorted(bow)
    if must:
        if voc["scoring"] == 1:
            norm = 0.0
            for kk in keys:
                norm += bow[kk] * bow[kk]
            norm = math.sqrt(norm)
        else:
            norm = 0.0
            for kk in keys:
                norm += abs(bow[kk])
        if norm > 0:
            bow = {kk: bow[kk] / norm for kk in keys}
    elif tf and bow:
        nd = float(len(bow))
        bow = {kk: bow[kk] / nd for kk in keys}
    return bow, fv


def as_arrays(bow, fv):
    wid = np.array(sorted(bow), np.int32)
    val = np.array([bow[k] for k in sorted(bow)], np.float64)
    nid = np.array(sorted(fv), np.int32)
    off = np.concatenate([[0], np.cumsum([len(fv[k]) for k in sorted(fv)])]).astype(np.int32)
    feat = np.array([i for k in sorted(fv) for i in fv[k]], np.int32)
    return wid, val, nid, off, feat


def same(a, b):
    for x, y in zip(a, b):
        assert x.shape == y.shape, (x.shape, y.shape)
        if x.dtype == np.float64:
            assert np.array_equal(x.view(np.uint64), y.view(np.uint64))
        else:
            assert np.array_equal(x, y)


@pytest.mark.parametrize("name", sorted(VOCABS))
def test_oracle_transform_vs_restatement(name, vocab_paths, frames):
    voc = load_text(vocab_paths[name])
    ov = oracle.Vocabulary(vocab_paths[name])
    assert (ov.k, ov.L, ov.nodes, ov.words) == (voc["k"], voc["L"], len(voc["nodes"]), voc["nwords"])
    desc = frames[0].desc[:300]
    for levelsup in (voc["L"] - 1, 1, voc["L"]):
        same(ov.transform(desc, levelsup), as_arrays(*transform_restated(voc, desc, levelsup)))


def search_by_bow_restated(kf, f, kf_ok, kf_fv, f_fv, nnratio=0.75, check_ori=True):
    kn, ko, kfe = kf_fv
    fn, fo, ffe = f_fv
    matches = np.full(f.n, -1, np.int32)
    hist = [[] for _ in range(30)]
    nm = 0
    a = b = 0
    F32 = np.float32
    while a < len(kn) and b < len(fn):
        if kn[a] == fn[b]:
            for ikf in kfe[ko[a]:ko[a + 1]]:
                if not kf_ok[ikf]:
                    continue
                b1, bi, b2 = 256, -1, 256
                for jf in ffe[fo[b]:fo[b + 1]]:
                    if matches[jf] >= 0:
                        continue
                    d = int(np.unpackbits(kf.desc[ikf] ^ f.desc[jf]).sum())
                    if d < b1:
                        b2, b1, bi = b1, d, jf
                    elif d < b2:
                        b2 = d
                if b1 <= 50 and F32(b1) < F32(nnratio) * F32(b2):
                    matches[bi] = ikf
                    if check_ori:
                        rot = F32(kf.keys["angle"][ikf]) - F32(f.keys["angle"][bi])
                        if rot < 0:
                            rot += F32(360)
                        bn = math.floor(float(rot * (F32(1) / F32(30))) + 0.5)
                        hist[0 if bn == 30 else bn].append(bi)
                    nm += 1
            a += 1
            b += 1
        elif kn[a] < fn[b]:
            a = int(np.searchsorted(kn, fn[b]))
        else:
            b = int(np.searchsorted(fn, kn[a]))
    if check_ori:
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i, h in enumerate(hist):
            s = len(h)
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, i
            elif s > m3:
                m3, i3 = s, i
        if m2 < F32(0.1) * F32(m1):
            i2 = i3 = -1
        elif m3 < F32(0.1) * F32(m1):
            i3 = -1
        for i in range(30):
            if i not in (i1, i2, i3):
                for bi in hist[i]:
                    matches[bi] = -1
                    nm -= 1
    return matches, nm


def bow_case(vocab_path, frames, levelsup=2, seed=0):
    ov = oracle.Vocabulary(vocab_path)
    kf, f = frames
    kf_fv = ov.transform(kf.desc, levelsup)[2:]
    f_fv = ov.transform(f.desc, levelsup)[2:]
    rng = np.random.Generator(np.random.PCG64(seed))
    kf_ok = (rng.uniform(size=kf.n) < 0.8).astype(np.uint8)
    return kf, f, kf_ok, kf_fv, f_fv


@pytest.mark.parametrize("ori", [True, False])
def test_oracle_search_by_bow_vs_restatement(ori, vocab_paths, frames):
    kf, f, kf_ok, kf_fv, f_fv = bow_case(vocab_paths["k10L4_l1_tfidf"], frames)
    m, nm = oracle.search_by_bow(kf.desc, kf.keys["angle"], kf_ok, kf_fv, f.desc, f.keys["angle"],
                                 f_fv, 0.75, ori)
    rm, rnm = search_by_bow_restated(kf, f, kf_ok, kf_fv, f_fv, 0.75, ori)
    assert nm == rnm and np.array_equal(m, rm)
    assert nm > 50


# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("zc", ["1", "0"])
@pytest.mark.parametrize("name", sorted(VOCABS))
def test_gpu_bow_transform(name, zc, vocab_paths, frames, monkeypatch):
    """The host transform (Frame::ComputeBoW): through its device-mapped pinned block (the
    kernels read the descriptors and write the vectors there) and with ORBFE_ZERO_COPY=0 through
    DMA copies; 1000, 1, 0 and then ~2000 descriptors (the pinned block grows)."""
    monkeypatch.setenv("ORBFE_ZERO_COPY", zc)
    from orbslam_mapsave_amd.native import Vocabulary
    gv = Vocabulary(vocab_paths[name], device=0)
    ov = oracle.Vocabulary(vocab_paths[name])
    assert (gv.k, gv.L, gv.nodes, gv.words) == (ov.k, ov.L, ov.nodes, ov.words)
    both = np.concatenate([frames[0].desc, frames[1].desc])
    for desc in (frames[0].desc, frames[1].desc[:1], frames[1].desc[:0], both):
        for levelsup in (1, 2, gv.L):
            same(gv.transform(desc, levelsup), ov.transform(desc, levelsup))
    gv.close()


@pytest.mark.gpu
def test_gpu_bow_transform_batch(vocab_paths):
    import torch
    from orbslam_mapsave_amd.native import Vocabulary
    path = vocab_paths["k10L4_l1_tfidf"]
    gv = Vocabulary(path, device=0)
    ov = oracle.Vocabulary(path)
    fr = [S.extract_frame(s, 1000, ini=20) for s in range(3)]
    cap = 1100
    dev = torch.device("cuda", 0)
    d = np.zeros((3, cap, 32), np.uint8)
    n = np.array([x.n for x in fr], np.int32)
    for i, x in enumerate(fr):
        d[i, :x.n] = x.desc
    D = torch.from_numpy(d).to(dev)
    N = torch.from_numpy(n).to(dev)
    wid = torch.zeros((3, cap), dtype=torch.int32, device=dev)
    val = torch.zeros((3, cap), dtype=torch.float64, device=dev)
    nid = torch.zeros((3, cap), dtype=torch.int32, device=dev)
    off = torch.zeros((3, cap + 1), dtype=torch.int32, device=dev)
    feat = torch.zeros((3, cap), dtype=torch.int32, device=dev)
    nw = torch.zeros(3, dtype=torch.int32, device=dev)
    nn = torch.zeros(3, dtype=torch.int32, device=dev)
    gv.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    gv.transform_batch_device(3, D.data_ptr(), N.data_ptr(), cap, 2, wid.data_ptr(),
                              val.data_ptr(), nw.data_ptr(), nid.data_ptr(), off.data_ptr(),
                              feat.data_ptr(), nn.data_ptr())
    torch.cuda.synchronize()
    for i, x in enumerate(fr):
        w, nnn = int(nw[i]), int(nn[i])
        o = off[i, :nnn + 1].cpu().numpy()
        got = (wid[i, :w].cpu().numpy(), val[i, :w].cpu().numpy(), nid[i, :nnn].cpu().numpy(), o,
               feat[i, :o[-1]].cpu().numpy())
        same(got, ov.transform(x.desc, 2))


@pytest.mark.gpu
@pytest.mark.parametrize("ori,ratio", [(True, 0.75), (False, 0.7), (True, 0.9)])
@pytest.mark.parametrize("zc,path", [("1", "gathered"), ("1", "general"), ("0", "general")])
def test_gpu_search_by_bow(ori, ratio, zc, path, vocab_paths, frames, monkeypatch):
    """Host SearchByBoW: the gathered path (common nodes' features gathered by the host into
    device-mapped pinned memory, one bow_search1_kernel launch writing each frame feature's
    outcome to its pinned slot, the orientation filter on the host), the general path with
    the pair's last workgroup writing the results into pinned memory (ORBFE_BOW1=0), and through
    bow_init_kernel + D2H copies (ORBFE_ZERO_COPY=0); three calls on one matcher (counters,
    histogram and staging reused)."""
    monkeypatch.setenv("ORBFE_ZERO_COPY", zc)
    monkeypatch.setenv("ORBFE_BOW1", "1" if path == "gathered" else "0")
    from orbslam_mapsave_amd.native import ORBmatcher
    kf, f, kf_ok, kf_fv, f_fv = bow_case(vocab_paths["k10L4_l1_tfidf"], frames, seed=int(ori))
    mt = ORBmatcher(ratio, ori, device=0)
    om, onm = oracle.search_by_bow(kf.desc, kf.keys["angle"], kf_ok, kf_fv, f.desc,
                                   f.keys["angle"], f_fv, ratio, ori)
    for _ in range(3):
        m, nm = mt.SearchByBoW(kf.desc, kf.keys["angle"], kf_ok, kf_fv, f.desc, f.keys["angle"],
                               f_fv)
        assert nm == onm and np.array_equal(m, om)
    mt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("levelsup", [1, 3])
def test_gpu_search_by_bow_node_levels(levelsup, vocab_paths, frames):
    """FeatureVectors at level 3 (up to 1000 nodes: more common nodes than the gathered path
    takes, so the general path runs) and level 1 (10 nodes of ~100 frame features), then a
    keyframe without any good map point (no common node has candidates: no launch), one matcher."""
    from orbslam_mapsave_amd.native import ORBmatcher
    kf, f, kf_ok, kf_fv, f_fv = bow_case(vocab_paths["k10L4_l1_tfidf"], frames, levelsup=levelsup)
    mt = ORBmatcher(0.75, True, device=0)
    for ok in (kf_ok, np.zeros_like(kf_ok), kf_ok):
        om, onm = oracle.search_by_bow(kf.desc, kf.keys["angle"], ok, kf_fv, f.desc,
                                       f.keys["angle"], f_fv, 0.75, True)
        m, nm = mt.SearchByBoW(kf.desc, kf.keys["angle"], ok, kf_fv, f.desc, f.keys["angle"], f_fv)
        assert nm == onm and np.array_equal(m, om)
    mt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ori", [True, False])
def test_gpu_search_by_bow_duplicates(ori, vocab_paths, frames):
    """Every frame descriptor twice (equal distances everywhere: ties for the best and the second,
    and a keyframe feature's best or second candidate taken by an earlier one — the gathered
    kernel's recomputation), the frame against itself and against the keyframe; bit-exact."""
    from orbslam_mapsave_amd.abi import Frame
    from orbslam_mapsave_amd.native import ORBmatcher
    ov = oracle.Vocabulary(vocab_paths["k10L4_l1_tfidf"])
    kf, f = frames
    keys = np.concatenate([f.keys, f.keys])
    keys["angle"][len(f.keys):] = np.mod(keys["angle"][len(f.keys):] + 7.0, 360.0).astype(np.float32)
    d2 = Frame(keys, np.concatenate([f.desc, f.desc]), S.W, S.H, f.scale_factors)
    mt = ORBmatcher(0.9, ori, device=0)
    for a_, b_ in ((d2, d2), (kf, d2), (d2, kf)):
        afv = ov.transform(a_.desc, 2)[2:]
        bfv = ov.transform(b_.desc, 2)[2:]
        ok = np.ones(a_.n, np.uint8)
        ok[::5] = 0
        om, onm = oracle.search_by_bow(a_.desc, a_.keys["angle"], ok, afv, b_.desc,
                                       b_.keys["angle"], bfv, 0.9, ori)
        m, nm = mt.SearchByBoW(a_.desc, a_.keys["angle"], ok, afv, b_.desc, b_.keys["angle"], bfv)
        assert nm == onm and np.array_equal(m, om)
    mt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ori", [True, False])
def test_gpu_search_by_bow_large_nodes(ori, vocab_paths, frames):
    """FeatureVectors at level 1 with the keyframe's descriptors three times over (~300 keyframe
    features per node: the gathered kernel's keyframe features in more than one chunk, later
    chunks' candidates taken by earlier ones) against the frame (~100 per node); the frame
    against the tripled keyframe (a common node of more than 256 frame features) is refused with
    ORBFE_ERR_UNSUPPORTED, as include/orbfe.h documents."""
    from orbslam_mapsave_amd.abi import ORBFE_ERR_UNSUPPORTED, Frame
    from orbslam_mapsave_amd.native import ORBmatcher, OrbfeError
    ov = oracle.Vocabulary(vocab_paths["k10L4_l1_tfidf"])
    kf, f = frames
    keys = np.concatenate([kf.keys] * 3)
    for r in (1, 2):
        sl = slice(r * len(kf.keys), (r + 1) * len(kf.keys))
        keys["angle"][sl] = np.mod(keys["angle"][sl] + 11.0 * r, 360.0).astype(np.float32)
    k3 = Frame(keys, np.concatenate([kf.desc] * 3), S.W, S.H, kf.scale_factors)
    mt = ORBmatcher(0.9, ori, device=0)
    for a_, b_ in ((k3, f), (f, k3)):
        afv = ov.transform(a_.desc, 3)[2:]
        bfv = ov.transform(b_.desc, 3)[2:]
        ok = np.ones(a_.n, np.uint8)
        ok[::7] = 0
        om, onm = oracle.search_by_bow(a_.desc, a_.keys["angle"], ok, afv, b_.desc,
                                       b_.keys["angle"], bfv, 0.9, ori)
        if np.diff(bfv[1]).max() > 256:
            with pytest.raises(OrbfeError) as e:
                mt.SearchByBoW(a_.desc, a_.keys["angle"], ok, afv, b_.desc, b_.keys["angle"], bfv)
            assert e.value.status == ORBFE_ERR_UNSUPPORTED
            continue
        m, nm = mt.SearchByBoW(a_.desc, a_.keys["angle"], ok, afv, b_.desc, b_.keys["angle"], bfv)
        assert onm > 0 and nm == onm and np.array_equal(m, om)
    mt.close()


def _flip(rng, d, nbits):
    """d with nbits distinct random bits flipped."""
    out = d.copy()
    for b in rng.choice(256, size=nbits, replace=False):
        out[b >> 3] ^= np.uint8(1 << (b & 7))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("ori", [True, False])
@pytest.mark.parametrize("bases,copies,nkf", [(6, 6, 150), (32, 8, 600)])
def test_gpu_search_by_bow_contended_node(bases, copies, nkf, ori):
    """One common node where keyframe features queue for the same frame features: frame feature
    (j, c) is base descriptor j with 4 c bits flipped, keyframe feature t is base t mod B with 2
    bits flipped, so the t of one base take copies 0, 1, 2, ... in turn (ratio 0.99).  Later t
    find three or all of their four nearest frame features taken (the gathered kernel's
    wave-parallel recomputation) and the fixed point needs one round per copy of a base; at
    (32, 8, 600) the node holds the maximum 256 frame features and 600 keyframe features (three
    chunks).  Bit-exact against the oracle (ORBmatcher.cc:211-248)."""
    from orbslam_mapsave_amd.native import ORBmatcher
    rng = np.random.Generator(np.random.PCG64(bases * 1000 + nkf))
    base = rng.integers(0, 256, size=(bases, 32), dtype=np.uint8)
    fd = np.stack([_flip(rng, base[j], 4 * c) for j in range(bases) for c in range(copies)])
    kd = np.stack([_flip(rng, base[t % bases], 2) for t in range(nkf)])
    fa = rng.uniform(0, 360, size=len(fd)).astype(np.float32)
    ka = rng.uniform(0, 360, size=nkf).astype(np.float32)
    ok = (rng.uniform(size=nkf) < 0.9).astype(np.uint8)
    one = lambda n: (np.array([7], np.int32), np.array([0, n], np.int32), np.arange(n, dtype=np.int32))
    kfv, ffv = one(nkf), one(len(fd))
    om, onm = oracle.search_by_bow(kd, ka, ok, kfv, fd, fa, ffv, 0.99, ori)
    assert onm >= bases * 2
    mt = ORBmatcher(0.99, ori, device=0)
    try:
        for _ in range(2):
            m, nm = mt.SearchByBoW(kd, ka, ok, kfv, fd, fa, ffv)
            assert nm == onm and np.array_equal(m, om)
    finally:
        mt.close()


def pack_slots(items, cap):
    """(desc, angle, ok, fv) per slot -> arrays in orbfe_bow_transform_batch_device's layout."""
    S_ = len(items)
    desc = np.zeros((S_, cap, 32), np.uint8)
    ang = np.zeros((S_, cap), np.float32)
    ok = np.zeros((S_, cap), np.uint8)
    nn = np.zeros(S_, np.int32)
    nid = np.zeros((S_, cap), np.int32)
    off = np.zeros((S_, cap + 1), np.int32)
    feat = np.zeros((S_, cap), np.int32)
    for s, (d, a, o, (ids, noff, fe)) in enumerate(items):
        desc[s, :len(d)] = d
        ang[s, :len(a)] = a
        ok[s, :len(o)] = o
        nn[s] = len(ids)
        nid[s, :len(ids)] = ids
        off[s, :len(noff)] = noff
        feat[s, :len(fe)] = fe
    return desc, ang, ok, nn, nid, off, feat


@pytest.mark.gpu
@pytest.mark.parametrize("ori,ratio", [(True, 0.75), (False, 0.7)])
def test_gpu_search_by_bow_batch(ori, ratio, vocab_paths):
    """Relocalisation's candidate loop (Tracking.cc:1636-1656) as one device call: the current
    frame against 6 candidate keyframes (one empty, one with every map point bad), plus a
    second frame, each pair bit-exact against the oracle's SearchByBoW."""
    import torch
    from orbslam_mapsave_amd.native import ORBmatcher
    path = vocab_paths["k10L4_l1_tfidf"]
    ov = oracle.Vocabulary(path)
    rng = np.random.Generator(np.random.PCG64(5))
    kfs = [S.extract_frame(s, 1000, ini=20) for s in (0, 1, 2)]
    kfs += [S.extract_frame(0, 1000, shift=(-4, 5), ini=20), S.extract_frame(3, 400, ini=20)]
    kf_items = []
    for i, k in enumerate(kfs):
        ok = (rng.uniform(size=k.n) < 0.8).astype(np.uint8) if i != 4 else np.zeros(k.n, np.uint8)
        kf_items.append((k.desc, k.keys["angle"], ok, ov.transform(k.desc, 2)[2:]))
    empty_fv = (np.zeros(0, np.int32), np.zeros(1, np.int32), np.zeros(0, np.int32))
    kf_items.append((np.zeros((0, 32), np.uint8), np.zeros(0, np.float32),
                     np.zeros(0, np.uint8), empty_fv))
    frs = [S.extract_frame(0, 1000, shift=(2, -3), ini=20), S.extract_frame(1, 1000, shift=(1, 1), ini=20)]
    f_items = [(f.desc, f.keys["angle"], np.ones(f.n, np.uint8), ov.transform(f.desc, 2)[2:]) for f in frs]
    kcap, fcap = 1100, 1050
    dev = torch.device("cuda", 0)
    K = [torch.from_numpy(x).to(dev) for x in pack_slots(kf_items, kcap)]
    F = [torch.from_numpy(x).to(dev) for x in pack_slots(f_items, fcap)]
    pairs = [(k, 0) for k in range(len(kf_items))] + [(1, 1), (3, 1), (0, 0)]
    pk = torch.tensor([p[0] for p in pairs], dtype=torch.int32, device=dev)
    pf = torch.tensor([p[1] for p in pairs], dtype=torch.int32, device=dev)
    P = len(pairs)
    out = torch.full((P, fcap), 7, dtype=torch.int32, device=dev)
    nm = torch.zeros(P, dtype=torch.int32, device=dev)
    st = torch.full((1,), 9, dtype=torch.int32, device=dev)
    mt = ORBmatcher(ratio, ori, device=0)
    mt.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    mt.search_by_bow_batch_device(
        P, pk.data_ptr(), pf.data_ptr(), kcap, K[0].data_ptr(), K[1].data_ptr(), K[2].data_ptr(),
        K[3].data_ptr(), K[4].data_ptr(), K[5].data_ptr(), K[6].data_ptr(), fcap, F[0].data_ptr(),
        F[1].data_ptr(), F[3].data_ptr(), F[4].data_ptr(), F[5].data_ptr(), F[6].data_ptr(),
        out.data_ptr(), nm.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    assert int(st[0]) == 0
    got, gnm = out.cpu().numpy(), nm.cpu().numpy()
    for p, (ki, fi) in enumerate(pairs):
        kd, ka, kok, kfv = kf_items[ki]
        fd, fa, _, ffv = f_items[fi]
        om, onm = oracle.search_by_bow(kd, ka, kok, kfv, fd, fa, ffv, ratio, ori)
        assert gnm[p] == onm, (p, gnm[p], onm)
        assert np.array_equal(got[p, :len(fd)], om), p
        assert (got[p, len(fd):] == -1).all()
    assert gnm[0] > 50 and gnm[4] == 0 and gnm[5] == 0
    mt.close()


@pytest.mark.gpu
def test_gpu_search_by_bow_rejects_repeated_feature(vocab_paths, frames):
    """A FeatureVector listing one feature index under two nodes (DBoW2 never builds one:
    FeatureVector.cpp:31-45) is refused with ORBFE_ERR_ARG instead of double-counting a match."""
    from orbslam_mapsave_amd.abi import ORBFE_ERR_ARG
    from orbslam_mapsave_amd.native import ORBmatcher, OrbfeError
    kf, f, kf_ok, kf_fv, f_fv = bow_case(vocab_paths["k10L4_l1_tfidf"], frames)
    ids, off, feat = (np.array(x, copy=True) for x in f_fv)
    feat[int(off[1])] = feat[0]  # node 1's first feature repeats node 0's first
    mt = ORBmatcher(0.75, True, device=0)
    try:
        with pytest.raises(OrbfeError) as e:
            mt.SearchByBoW(kf.desc, kf.keys["angle"], kf_ok, kf_fv, f.desc, f.keys["angle"],
                           (ids, off, feat))
        assert e.value.status == ORBFE_ERR_ARG
    finally:
        mt.close()
