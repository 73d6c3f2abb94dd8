"""vc_group_multiproof_prove_many with host evaluations (each member uploads its proofs' data and
proves them) on ONE card, G = 1 / 2 members: wall ms per call (median of reps) for P proofs of Q
width-256 IPA queries (the reference bench's r_j + i datasets). Run against two libraries
(VKZG_LIB) to see the upload / prove overlap of round 6 (group.cpp: sub-batches over two device
buffers, the next one's data crossing PCIe while the current one is proven).
usage: group_mp_probe.py [log_q] [P] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg.group import Group  # noqa: E402
from bench import rj_plus_i  # noqa: E402

log_q = int(sys.argv[1]) if len(sys.argv) > 1 else 14
P = int(sys.argv[2]) if len(sys.argv) > 2 else 4
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
N, Q = 256, 1 << log_q
crs = scheme.ipa_crs(N + 1, max_=512)
rng = np.random.default_rng(5)
data = np.stack([rj_plus_i(rng, Q, N).reshape(Q, N, 4) for _ in range(P)])  # [P][Q][N][4]
z = rng.integers(0, N, size=(P, Q), dtype=np.uint64)
y = np.ascontiguousarray(data[np.arange(P)[:, None], np.arange(Q)[None, :], z.astype(np.int64)])
e = vkzg.Engine("bn254")
ipa = scheme.IPA(e, N, crs)
cxy = np.zeros((P, Q, 8), dtype=np.uint64)
cinf = np.zeros((P, Q), dtype=np.uint8)
for p in range(P):
    xy, inf = e.msm_batch(ipa.table, data[p].reshape(Q * N, 4), N)
    cxy[p], cinf[p] = xy, inf
e.close()
res = {}
first = None
for G in (1, 2):
    g = Group("bn254", [0] * G)
    try:
        tid = g.upload_points(crs)
        ts, out = [], None
        for r in range(reps + 1):
            t0 = time.perf_counter()
            out = g.multiproof_prove_many(0, tid, N, data, cxy, cinf, z, y)
            if r:
                ts.append((time.perf_counter() - t0) * 1e3)
        key = [(pr["d"], pr["proof"].tip) for pr in out]
        first = first or key
        res[f"G{G}_ms"] = round(sorted(ts)[len(ts) // 2], 2)
        res[f"G{G}_same_as_G1"] = key == first
    finally:
        g.close()
print({"lib": os.path.basename(os.path.dirname(os.environ.get("VKZG_LIB", "lib/x"))), "log_q": log_q, "P": P,
       "data_MB": round(data.nbytes / 1e6), **res}, flush=True)
