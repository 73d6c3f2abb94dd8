"""The verkle device path's extension host stage on the CPU (no GPU): a tree of `keys` random
32-unit keys, its c1 / c2 rows built and merged (vc_verkle_debug_ext_stage), median us.
usage: verkle_host_probe.py [keys] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from vkzg.verkle import VerkleTree  # noqa: E402

nk = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 9
rng = np.random.default_rng(91)
keys = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
vals = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
t = VerkleTree(32)
t0 = time.perf_counter()
for i in range(nk):
    t.insert_single(keys[i].tobytes(), vals[i].tobytes())
print(f"insert {time.perf_counter() - t0:.3f} s, stats {t.stats()}")
for _ in range(3):
    print(f"ext stage median {t.debug_ext_stage(reps):.1f} us over {reps} reps")
