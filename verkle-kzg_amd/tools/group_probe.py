"""vc_group timings on ONE card (every member on device 0, sharing it): vc_group_msm (2^20 BLS12-381,
host scalars, point split) and vc_group_kzg_prove (d = 2^20, index-range shards, in / out of the
domain) for G = 1, 2, 8 members, plus the one-context share sizes an 8-GPU node would run per GPU
(vc_msm_partial over 2^17 points of the 2^20 table). Wall ms, median of reps.
usage: group_probe.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

import vkzg  # noqa: E402
from vkzg.group import Group  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n = 1 << 20


def med(f):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(sorted(ts)[len(ts) // 2], 3)


sc = vkzg.random_scalars("bls12_381", n, np.random.default_rng(1234))
ev = vkzg.random_scalars("bls12_381", n, np.random.default_rng(44))
res = {}
for G in (1, 2, 8):
    g = Group("bls12_381", [0] * G)
    try:
        tid = g.random_bases(n, seed=2024)
        res[f"msm_G{G}"] = med(lambda: g.msm(tid, sc))
        kt, size = g.kzg_setup(n)
        res[f"kzg_in_G{G}"] = med(lambda: g.kzg_prove(kt, size, ev, n // 3))
        res[f"kzg_out_G{G}"] = med(lambda: g.kzg_prove(kt, size, ev, n + 987654321))
        print(G, {k: v for k, v in res.items() if k.endswith(f"G{G}")}, flush=True)
    finally:
        g.close()
e = vkzg.Engine("bls12_381")
try:
    tid = e.random_bases(n, seed=2024)
    share = n // 8
    res["msm_share_1of8_host_scalars"] = med(lambda: e.msm_partial(tid, sc[3 * share:4 * share], offset=3 * share))
    print("share 1/8 (one context, host scalars):", res["msm_share_1of8_host_scalars"], flush=True)
finally:
    e.close()
print(res, flush=True)
