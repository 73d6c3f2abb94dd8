"""Per-rank (or per-member) cost of one 2^20 BLS12-381 MSM split G ways on this GPU, both ways:
a point range of n/G points (vc_msm_device_partial: since round 4 on the whole table's radix
shared-window copies) and a window part (vc_msm_device_window_part, 2^16-radix copies). Note: a
table keeps ONE copy layout, so the window parts rebuild their copies once after the point
ranges (untimed warm-up). usage: split_probe.py [G,G,...]"""
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
GS = [int(g) for g in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 4, 8]
KERNELS = ("glv_split", "msm_sort_coarse", "msm_sort_fine", "msm_accumulate", "msm_fixup", "msm_segsum",
           "msm_bitsum", "msm_sumpart")


def timed(f, reps=10):
    """(wall ms per call with per-kernel events OFF, per-kernel ms from a second loop with events on,
    wall ms of that instrumented loop): the events add ~0.1 ms per call, so the wall time is taken
    without them"""
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps * 1e3
    e.enable_timing(True)
    e.reset_timing()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt_ev = (time.perf_counter() - t0) / reps * 1e3
    ks = {}
    for name in KERNELS:
        ms, cnt = e.kernel_time(name)
        if cnt:
            ks[name] = round(ms / cnt, 3)
    e.enable_timing(False)
    return dt, ks, dt_ev


for mode in ("points", "windows"):
    for G in GS:
        for k in sorted({0, G - 1}):
            if mode == "points":
                lo, hi = n * k // G, n * (k + 1) // G
                f = lambda: e.msm_device_partial(tid, d.data_ptr() + lo * 32, hi - lo, offset=lo)  # noqa: E731
            else:
                f = lambda: e.msm_device_window_part(tid, d.data_ptr(), n, k, G)  # noqa: E731
            dt, ks, dt_ev = timed(f)
            plan = e.msm_last_plan()
            print(f"{mode} G={G} part={k}: {dt:.3f} ms (with per-kernel events {dt_ev:.3f}) "
                  f"radix={plan['radix_mul']}x2^{plan['window_bits']} windows={plan['windows']} {ks}", flush=True)
