"""The C ABI's concurrency promise (include/orbfe.h: distinct handles may be used from
different threads at once) in the reference's own pattern: a stereo frame's left and right
extractions on two std::threads (Frame.cc:78-81), the three Tracking extractors including the
2x-feature Ini one (Tracking.cc:208-215) and a matcher, all running concurrently from C++
(tests/cpp/threads_test.cpp), every output of every iteration bit-exact against the oracle.
A Python-thread variant (ctypes releases the GIL) adds the device-batch brute force on a
shared matcher's per-stream buffers."""
import os
import subprocess
import threading

import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.synth import synthetic_frame

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(__file__), "cpp", "build", "threads_test")


def test_cpp_threads_stereo_ini_matcher():
    assert os.path.exists(BIN), "run __graft_entry__.build() first"
    r = subprocess.run([BIN, "60"], capture_output=True, text=True, timeout=240)
    print(r.stdout[-2000:])
    assert r.returncode == 0 and "THREADS PASS" in r.stdout, r.stdout[-4000:] + r.stderr[-2000:]


def test_python_threads_handles():
    """Three extractor handles (1000, 1000, 2000 features) and a matcher, each on its own Python
    thread for 50 iterations; the matcher thread runs the batched device brute force on six
    streams in turn (more than its four per-stream reference buffers: the evicted buffer waits
    only for its own readers)."""
    import torch
    from orbslam_mapsave_amd.native import ORBextractor, ORBmatcher
    imgs = [synthetic_frame(300 + i, 640, 480) for i in range(4)]
    p1, p2 = oracle.params(1000, 1.2, 8, 20, 7), oracle.params(2000, 1.2, 8, 20, 7)
    exp1 = [oracle.extract(p1, im) for im in imgs]
    exp2 = [oracle.extract(p2, im) for im in imgs]
    q, r = exp1[0][1], exp2[1][1]
    obi, obd, osd = oracle.bf_match(q, r)
    errors = []

    def run_extractor(nf, exp, iters=50):
        try:
            e = ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=640, max_height=480)
            try:
                for i in range(iters):
                    k, d = e(imgs[i % 4])
                    ok, od = exp[i % 4]
                    if k.tobytes() != ok.tobytes() or not np.array_equal(d, od):
                        errors.append(f"extractor {nf} iteration {i}")
            finally:
                e.close()
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    def run_matcher(iters=50):
        try:
            m = ORBmatcher(0.9, True, device=0)
            streams = [torch.cuda.Stream() for _ in range(6)]
            nb = 4
            dq = torch.zeros((nb, 2048, 32), dtype=torch.uint8, device="cuda:0")
            dq[:, :len(q)] = torch.from_numpy(q).cuda()
            dnq = torch.full((nb,), len(q), dtype=torch.int32, device="cuda:0")
            dr = torch.zeros((2048, 32), dtype=torch.uint8, device="cuda:0")
            dr[:len(r)] = torch.from_numpy(r).cuda()
            dnr = torch.full((nb,), len(r), dtype=torch.int32, device="cuda:0")
            try:
                for i in range(iters):
                    s = streams[i % len(streams)]
                    out = torch.full((nb, 2048, 3), -7, dtype=torch.int32, device="cuda:0")
                    with torch.cuda.stream(s):
                        m.set_stream(s.cuda_stream)
                        m.bf_match_batch_device(dq.data_ptr(), 2048 * 32, dnq.data_ptr(), 2048, dr.data_ptr(), 0,
                                                 dnr.data_ptr(), nb, out.data_ptr())
                    s.synchronize()
                    o = out.cpu().numpy()
                    for b in range(nb):
                        if not (np.array_equal(o[b, :len(q), 0], obi) and np.array_equal(o[b, :len(q), 1], obd)
                                and np.array_equal(o[b, :len(q), 2], osd)):
                            errors.append(f"matcher iteration {i} problem {b}")
                    bi, bd, sd = m.bf_match(q, r)
                    if not (np.array_equal(bi, obi) and np.array_equal(bd, obd) and np.array_equal(sd, osd)):
                        errors.append(f"matcher host form iteration {i}")
            finally:
                m.set_stream(None)
                m.close()
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    ts = [threading.Thread(target=run_extractor, args=(1000, exp1)),
          threading.Thread(target=run_extractor, args=(1000, exp1)),
          threading.Thread(target=run_extractor, args=(2000, exp2)),
          threading.Thread(target=run_matcher)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=180)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    assert not errors, errors[:10]
