"""Verkle commitment A/B (bench.py verkle line shapes): full commitment of a fresh 65,536-key tree
and the 1 % update after it, wall ms (no per-kernel events), for the path VKZG_VERKLE_DEV selects
(read per call). usage: verkle_ab.py [keys] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg.verkle import VerkleTree  # noqa: E402

nk = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
eng = vkzg.Engine("bn254", 0)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
kzg = scheme.KZG(eng, 256)
eng.fixed_base_precompute(kzg.table, int(os.environ.get("VKZG_AB_FB_C", "8")))  # window bits (A/B)
rng = np.random.default_rng(91)
keys = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
vals = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
full, upd, roots = [], [], set()
for rep in range(reps):
    t = VerkleTree(32)
    for i in range(nk):
        t.insert_single(keys[i].tobytes(), vals[i].tobytes())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = t.commitment(eng, kzg.table)
    full.append((time.perf_counter() - t0) * 1e3)
    urng = np.random.default_rng(7)
    for i in urng.integers(0, nk, size=max(1, nk // 100)):
        t.insert_single(keys[i].tobytes(), urng.integers(0, 256, size=32, dtype=np.uint8).tobytes())
    d = t.stats()["dirty"]
    t0 = time.perf_counter()
    r2 = t.commitment(eng, kzg.table)
    upd.append((time.perf_counter() - t0) * 1e3)
    roots.add((r, r2))
print(f"VKZG_VERKLE_DEV={os.environ.get('VKZG_VERKLE_DEV', '1')} keys={nk} dirty_after_update={d} "
      f"full_ms={[round(x, 2) for x in full]} update_ms={[round(x, 2) for x in upd]} "
      f"full_median_2+={sorted(full[1:])[len(full[1:]) // 2]:.2f} update_median_2+={sorted(upd[1:])[len(upd[1:]) // 2]:.2f} "
      f"same_roots={len(roots) == 1}", flush=True)
