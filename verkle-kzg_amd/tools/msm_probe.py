"""Where the time of one 2^k-point MSM goes: wall ms per vc_msm_device (no event timing), then
the per-kernel averages with event timing on, and the remainder (host Horner, launch gaps,
the final sync). usage: msm_probe.py [curve] [log_n]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

NAMES = ("glv_split", "glv_phi", "msm_sort_hist", "msm_scan", "msm_sort_coarse", "msm_sort_fine", "msm_accumulate",
         "msm_fixup_init", "msm_fixup_jump", "msm_fixup", "msm_fixup_long", "msm_segsum", "msm_bitsum", "msm_sumpart")

curve = sys.argv[1] if len(sys.argv) > 1 else "bls12_381"
n = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 20)
e = vkzg.Engine(curve, 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
if os.environ.get("VKZG_MSM_SHARED") == "0":  # per-window buckets, no window copies (variable base)
    e.set_option(e.OPT_MSM_SHARED_WINDOWS, 0)
tid = e.random_bases(n, seed=2024)
sc = vkzg.random_scalars(curve, n, np.random.default_rng(1234))
d = torch.from_numpy(sc.view(np.int64).copy()).cuda()
for _ in range(3):
    e.msm_device(tid, d.data_ptr(), n)
torch.cuda.synchronize()
reps = 20
t0 = time.perf_counter()
for _ in range(reps):
    e.msm_device(tid, d.data_ptr(), n)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / reps * 1e3
t0 = time.perf_counter()
for _ in range(reps):
    e.msm_device_partial(tid, d.data_ptr(), n)
torch.cuda.synchronize()
wall_part = (time.perf_counter() - t0) / reps * 1e3
e.enable_timing(True)
e.reset_timing()
for _ in range(reps):
    e.msm_device(tid, d.data_ptr(), n)
torch.cuda.synchronize()
tot = 0.0
rows = {}
for k in NAMES:
    ms, cnt = e.kernel_time(k)
    if cnt:
        rows[k] = ms / reps
        tot += ms / reps
print(f"{curve} n=2^{n.bit_length() - 1}: wall {wall:.3f} ms/MSM (partial, no normalise: {wall_part:.3f}); "
      f"kernels {tot:.3f} ms; other {wall - tot:.3f} ms")
for k, v in rows.items():
    print(f"  {k:16s} {v:.4f} ms")
