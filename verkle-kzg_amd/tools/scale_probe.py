"""Per-rank cost of the window-split MSM: time one window part (k of G) of a 2^20 BLS12-381
MSM on this GPU for G = 1, 2, 4, 8 -- what each rank of bench.py --gpus G computes."""
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
for G in GS:
    for k in sorted({0, G - 1}):
        for _ in range(2):
            e.msm_device_window_part(tid, d.data_ptr(), n, k, G)
        torch.cuda.synchronize()
        e.enable_timing(True)
        e.reset_timing()
        t0 = time.perf_counter()
        reps = 10
        for _ in range(reps):
            e.msm_device_window_part(tid, d.data_ptr(), n, k, G)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps * 1e3
        ks = {}
        for name in ("msm_sort_coarse", "msm_sort_fine", "msm_accumulate", "msm_fixup", "msm_segsum", "msm_bitsum",
                     "msm_sumpart"):
            ms, cnt = e.kernel_time(name)
            if cnt:
                ks[name] = round(ms / cnt, 3)
        e.enable_timing(False)
        print(f"G={G} part={k}: {dt:.3f} ms  {ks}", flush=True)
