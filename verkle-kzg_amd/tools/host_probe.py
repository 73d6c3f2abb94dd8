"""vc_msm with host scalars (the drop-in entry point) at 2^20 BLS12-381 for each
VC_OPT_MSM_HOST_CHUNKS setting, alternating settings over rounds (box clocks drift), beside the
device-scalar MSM. usage: host_probe.py [rounds] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
n = 1 << 20
e = vkzg.Engine("bls12_381", 0)
tid = e.random_bases(n, seed=2024)
k = vkzg.random_scalars("bls12_381", n, np.random.default_rng(1234))
d = torch.from_numpy(k.view(np.int64).copy()).cuda()
ref = e.msm_device(tid, d.data_ptr(), n)
# the same scalars in page-locked host memory (the runtime DMAs them without staging)
kp_t = torch.empty((n, 4), dtype=torch.int64).pin_memory()
kp_t.copy_(torch.from_numpy(k.view(np.int64)))
kp = kp_t.numpy().view(np.uint64)
src = {"pageable": k, "pinned": kp}
for _ in range(3):
    e.msm(tid, k)
res = {}
cases = [("device", 0)] + [(f"{m} chunks={c}", c) for m in ("pageable", "pinned") for c in (1, 2, 4)]
for r in range(rounds):
    for name, ch in cases:
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            if ch == 0:
                got = e.msm_device(tid, d.data_ptr(), n)
            else:
                e.set_option(e.OPT_MSM_HOST_CHUNKS, ch)
                got = e.msm(tid, src[name.split()[0]])
            ts.append((time.perf_counter() - t0) * 1e3)
            assert np.array_equal(got[0], ref[0])
        res.setdefault(name, []).append(float(np.median(ts)))
        print(f"round {r} {name}: median {np.median(ts):.3f} ms min {min(ts):.3f}", flush=True)
for name, v in res.items():
    print(f"{name}: medians {[round(x, 3) for x in v]}", flush=True)
