"""C3 probe: per-kernel times of one 10k x width-256 Bandersnatch batched commit (fixed-base
table at window c, or "c:W" for W mixed windows of c / c + 1 bits): fb_commit (chunk-major main
kernel), fb_combine, fb_normalize_out."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

dev = torch.device("cuda", 0)
e = vkzg.Engine("bandersnatch", 0)
e.set_stream(torch.cuda.current_stream(dev).cuda_stream)
tab = e.random_bases(256, seed=3)
B = int(os.environ.get("B", "10000"))
sc = vkzg.random_scalars("bandersnatch", B * 256, np.random.default_rng(5))
dcs = torch.from_numpy(sc.view(np.int64)).to(dev)
dxy = torch.zeros((B, 8), dtype=torch.int64, device=dev)
dinf = torch.zeros(B, dtype=torch.uint8, device=dev)
for arg in sys.argv[1:] or ["16"]:
    c, W = (int(v) for v in arg.split(":")) if ":" in arg else (int(arg), 0)
    t0 = time.time()
    e.fixed_base_precompute(tab, c, W)
    c = f"{c} W={e.fixed_base_geometry(tab)[1]} wide={e.fixed_base_geometry(tab)[2]}"
    torch.cuda.synchronize()
    print(f"precompute c={c}: {time.time() - t0:.2f} s", flush=True)
    e.msm_batch_device(tab, 256, dcs.data_ptr(), B, dxy.data_ptr(), dinf.data_ptr())
    torch.cuda.synchronize()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        e.msm_batch_device(tab, 256, dcs.data_ptr(), B, dxy.data_ptr(), dinf.data_ptr())
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e3
    e.enable_timing(True)
    e.reset_timing()
    for _ in range(reps):
        e.msm_batch_device(tab, 256, dcs.data_ptr(), B, dxy.data_ptr(), dinf.data_ptr())
    torch.cuda.synchronize()
    ks = {k: e.kernel_time(k) for k in ("fb_commit", "fb_combine", "fb_normalize_out", "norm_prep", "norm_finish")}
    e.enable_timing(False)
    print(f"c={c} B={B}: wall {wall:.3f} ms/batch ({B / wall * 1e3 / 1e6:.3f} M commits/s); " +
          ", ".join(f"{k} {ms / n:.3f} ms" for k, (ms, n) in ks.items() if n), flush=True)
