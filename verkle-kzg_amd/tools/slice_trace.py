"""One window slice (part 0 of G) of a 2^20 BLS12-381 MSM, repeated: run under
`rocprofv3 --kernel-trace` to see the per-rank timeline of a G-GPU run (kernels and gaps).
usage: slice_trace.py [G]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = 1 << 20
e = vkzg.Engine("bls12_381", 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
tid = e.random_bases(n, seed=2024)
sc = vkzg.random_scalars("bls12_381", n, np.random.default_rng(1234))
d = torch.from_numpy(sc.view(np.int64).copy()).cuda()
for _ in range(8):
    e.msm_device_window_part(tid, d.data_ptr(), n, 0, G)
torch.cuda.synchronize()
