"""Several MSMs over one table (vc_msm_device_many, the KZG commit + open's pipeline) against
single MSMs on the same 2^20 BLS12-381 table: wall times per call, for a rocprofv3 kernel trace /
PMC pass of the same command (per-set accumulate cost, effective clock from GRBM_GUI_ACTIVE).
usage: kset_probe.py [K ...]   (default: 1 2; K = 1 runs vc_msm_device)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

Ks = [int(x) for x in sys.argv[1:]] or [1, 2]
n = 1 << 20
reps = int(os.environ.get("KSET_REPS", "6"))
e = vkzg.Engine("bls12_381", 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
tid = e.random_bases(n, seed=2024)
rng = np.random.default_rng(1234)
d = [torch.from_numpy(vkzg.random_scalars("bls12_381", n, rng).view(np.int64).copy()).cuda() for _ in range(max(Ks))]
torch.cuda.synchronize()
for K in Ks:
    ts = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        if K == 1:
            e.msm_device(tid, d[0].data_ptr(), n)
        else:
            e.msm_device_many(tid, [x.data_ptr() for x in d[:K]], n)
        ts.append((time.perf_counter() - t0) * 1e3)
    ts = ts[1:]
    print(f"K={K}: median {np.median(ts):.3f} ms ({np.median(ts) / K:.3f} per MSM) all {[round(t, 3) for t in ts]}",
          flush=True)
