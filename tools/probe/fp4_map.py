"""Finds the FP4 operand lane map of v_mfma_scale_f32_32x32x64_f8f6f4 (build: hipcc -shared
tools/probe/fp4_map.hip -> tools/probe/build/libfp4map.so; run on the GPU box)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "build", "libfp4map.so"))
rng = np.random.default_rng(1)
# A nibbles in {0 (0.0), 2 (1.0)}, B nibbles in {2 (1.0), 10 (-1.0)}
an = rng.integers(0, 2, (64, 32)) * 2
bn = np.where(rng.integers(0, 2, (64, 32)) == 1, 10, 2)
def pack(n):
    out = np.zeros((64, 4), np.uint32)
    for j in range(32):
        out[:, j // 8] |= (n[:, j].astype(np.uint32) << (4 * (j % 8)))
    return out.view(np.int32)
a = torch.tensor(pack(an)).cuda()
b = torch.tensor(pack(bn)).cuda()
d = torch.zeros((64, 16), dtype=torch.float32).cuda()
assert lib.fp4_probe(C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), C.c_void_p(d.data_ptr())) == 0
D = d.cpu().numpy()
av = (an == 2).astype(np.float64)
bv = np.where(bn == 2, 1.0, -1.0)
def test(kmap):
    # kmap(h, j) -> k
    A = np.zeros((32, 64)); B = np.zeros((64, 32))
    for l in range(64):
        r, h = l & 31, l >> 5
        for j in range(32):
            A[r, kmap(h, j)] = av[l, j]
            B[kmap(h, j), r] = bv[l, j]
    ref = A @ B
    got = np.zeros((32, 32))
    for l in range(64):
        for e in range(16):
            got[(e & 3) + 8 * (e >> 2) + 4 * (l >> 5), l & 31] = D[l, e]
    return np.array_equal(ref, got)
hyps = {"k = 32h + j": lambda h, j: 32 * h + j,
        "k = 16h + j (j<16), 32 + 16h + j-16": lambda h, j: 16 * h + j if j < 16 else 32 + 16 * h + (j - 16),
        "k = 8h + j%8 + 16(j//8)": lambda h, j: 8 * h + (j % 8) + 16 * (j // 8)}
res = {k: test(f) for k, f in hyps.items()}
print(res)
print("D sample", D[0, :4], D[33, :4])
