"""Where the verkle full commitment's time goes (bench.py verkle line shapes): host lap times
(VKZG_VERBOSE) and per-kernel totals of one full commitment of 65,536 random keys."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg.verkle import VerkleTree  # noqa: E402

NAMES = ("sparse_count", "sparse_expand", "sparse_rows", "sparse_count_scan", "sparse_expand_rows", "sparse_small",
         "sparse_accumulate", "msm_fixup", "sparse_store", "sparse_combine", "sparse_add_base", "normalize_out", "norm_prep",
         "norm_finish", "to_data_item", "fb_commit", "fb_combine", "fb_normalize_out", "fb_commit_small", "verkle_widen",
         "verkle_ext_rows4", "verkle_rp4", "verkle_delta", "verkle_gather", "verkle_dense", "verkle_scatter")
nk = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
eng = vkzg.Engine("bn254", 0)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
kzg = scheme.KZG(eng, 256)
rng = np.random.default_rng(91)
keys = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
vals = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
eng.fixed_base_precompute(kzg.table, 8)
reps = int(os.environ.get("REPS", "2"))
walls = []
for rep in range(reps):
    t = VerkleTree(32)
    for i in range(nk):
        t.insert_single(keys[i].tobytes(), vals[i].tobytes())
    eng.enable_timing(True)
    eng.reset_timing()
    t0 = time.perf_counter()
    t.commitment(eng, kzg.table)
    dt = time.perf_counter() - t0
    ks = {}
    for k in NAMES:
        ms, cnt = eng.kernel_time(k)
        if cnt:
            ks[k] = (round(ms, 3), cnt)
    eng.enable_timing(False)
    print(f"rep {rep}: full commitment {dt * 1e3:.2f} ms; kernels {ks}", flush=True)
    if rep > 0:
        walls.append(dt * 1e3)
if walls:
    print(f"median of reps 1..{reps - 1}: {sorted(walls)[len(walls) // 2]:.2f} ms", flush=True)
