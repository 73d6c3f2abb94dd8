"""Adversarial scalar distributions (all-equal, few distinct) on a 2^20 BLS12-381 MSM:
timing + agreement with the same MSM split into random-order halves (linearity check)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

n = 1 << 20
e = vkzg.Engine("bls12_381", 0)
tid = e.random_bases(n, seed=7)
rng = np.random.default_rng(3)
base = vkzg.random_scalars("bls12_381", 4, rng)
cases = {"random": vkzg.random_scalars("bls12_381", n, rng),
         "all_equal": np.repeat(base[:1], n, axis=0),
         "four_values": base[rng.integers(0, 4, n)]}
for name, sc in cases.items():
    d = torch.from_numpy(np.ascontiguousarray(sc).view(np.int64)).cuda()
    e.msm_device(tid, d.data_ptr(), n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = e.msm_device(tid, d.data_ptr(), n)
    dt = (time.perf_counter() - t0) * 1e3
    h = n // 2  # linearity: MSM = partial(lo) + partial(hi)
    p1 = e.msm_device_partial(tid, d.data_ptr(), h)
    p2 = e.msm_device_partial(tid, d[h:].data_ptr(), n - h, offset=h)
    s = e.partials_sum(np.stack([p1, p2]))
    print(f"{name}: {dt:.2f} ms, split-sum agrees: {np.array_equal(s[0], r[0]) and s[1] == r[1]}", flush=True)
