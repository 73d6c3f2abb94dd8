"""The bench.py verkle line's call sequence, with every update timed: warm-up tree (full + one
update), a tree committed with per-kernel timing on (optional), the timed tree's full commitment,
then `ups` successive 1 % updates. usage: verkle_bench_seq.py [timing_tree 0/1] [ups]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg.verkle import VerkleTree  # noqa: E402

timing_tree = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ups = int(sys.argv[2]) if len(sys.argv) > 2 else 4
stream = torch.cuda.Stream()
veng = vkzg.Engine("bn254", 0)
veng.set_stream(stream.cuda_stream)
kzg = scheme.KZG(veng, 256)
rng = np.random.default_rng(91)
nk = 65536
keys = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
vals = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
veng.fixed_base_precompute(kzg.table, 8)


def tree():
    t = VerkleTree(32)
    for i in range(nk):
        t.insert_single(keys[i].tobytes(), vals[i].tobytes())
    return t


def update(t, r):
    for i in r.integers(0, nk, size=nk // 100):
        t.insert_single(keys[i].tobytes(), r.integers(0, 256, size=32, dtype=np.uint8).tobytes())
    t0 = time.perf_counter()
    t.commitment(veng, kzg.table)
    return (time.perf_counter() - t0) * 1e3


w = tree()
w.commitment(veng, kzg.table)
update(w, np.random.default_rng(17))
del w
if timing_tree:
    k = tree()
    veng.enable_timing(True)
    veng.reset_timing()
    k.commitment(veng, kzg.table)
    veng.enable_timing(False)
    del k
t = tree()
t0 = time.perf_counter()
t.commitment(veng, kzg.table)
full = (time.perf_counter() - t0) * 1e3
r = np.random.default_rng(5)
print(f"timing_tree={timing_tree} full {full:.2f} ms, updates {[round(update(t, r), 3) for _ in range(ups)]} ms", flush=True)
