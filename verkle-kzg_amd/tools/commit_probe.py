"""Fixed-base commit kernel probe: per-madd rate vs table footprint (widths touching fewer bases)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

c = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda", 0)
e = vkzg.Engine("bandersnatch", 0)
e.set_stream(torch.cuda.current_stream(dev).cuda_stream)
tab = e.random_bases(256, seed=3)
t0 = time.time()
e.fixed_base_precompute(tab, c)
torch.cuda.synchronize()
print(f"precompute c={c}: {time.time() - t0:.2f} s", flush=True)
total = 10000 * 256
for width in (256, 128, 64, 32, 16):
    B = total // width
    sc = vkzg.random_scalars("bandersnatch", B * width, np.random.default_rng(5))
    dcs = torch.from_numpy(sc.view(np.int64)).to(dev)
    dxy = torch.zeros((B, 8), dtype=torch.int64, device=dev)
    dinf = torch.zeros(B, dtype=torch.uint8, device=dev)
    e.msm_batch_device(tab, width, dcs.data_ptr(), B, dxy.data_ptr(), dinf.data_ptr())
    torch.cuda.synchronize()
    e.enable_timing(True)
    e.reset_timing()
    for _ in range(3):
        e.msm_batch_device(tab, width, dcs.data_ptr(), B, dxy.data_ptr(), dinf.data_ptr())
    torch.cuda.synchronize()
    ms, n = e.kernel_time("fb_commit")
    e.enable_timing(False)
    print(f"width {width:4d} batch {B:7d}: fb_commit {ms / n:.3f} ms", flush=True)
