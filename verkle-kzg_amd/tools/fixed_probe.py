"""Fixed-base MSM mode (pre-shifted tables, one bucket set): 2^20 BLS12-381 MSM time vs the
window size c, beside the variable-base engine."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

n = 1 << 20
e = vkzg.Engine("bls12_381", 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
tid = e.random_bases(n, seed=2024)
sc = vkzg.random_scalars("bls12_381", n, np.random.default_rng(1234))
d = torch.from_numpy(sc.view(np.int64).copy()).cuda()


def run(label):
    for _ in range(2):
        e.msm_device(tid, d.data_ptr(), n)
    torch.cuda.synchronize()
    e.enable_timing(True)
    e.reset_timing()
    t0 = time.perf_counter()
    reps = 10
    for _ in range(reps):
        r = e.msm_device(tid, d.data_ptr(), n)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps * 1e3
    ks = {}
    for k in ("msm_sort_hist", "msm_sort_coarse", "msm_sort_fine", "msm_accumulate", "msm_fixup", "msm_segsum",
              "msm_bitsum", "msm_sumpart"):
        ms, cnt = e.kernel_time(k)
        if cnt:
            ks[k] = round(ms / cnt, 3)
    e.enable_timing(False)
    print(f"{label}: {dt:.3f} ms {ks}", flush=True)
    return r


ref = run("variable-base")
for c in (16, 17, 18, 19, 20):
    t0 = time.perf_counter()
    e.msm_fixed_base_precompute(tid, c)
    pre = time.perf_counter() - t0
    r = run(f"fixed-base c={c} (precompute {pre:.2f} s)")
    assert np.array_equal(r[0], ref[0])
    e.msm_fixed_base_precompute(tid, 0)
