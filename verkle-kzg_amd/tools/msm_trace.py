"""A 2^20 BLS12-381 MSM repeated (full vc_msm_device path): run under
`rocprofv3 --kernel-trace` and feed the CSV to gap_report.py to see launch gaps between kernels.
usage: msm_trace.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = 1 << 20
e = vkzg.Engine("bls12_381", 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
tid = e.random_bases(n, seed=2024)
sc = vkzg.random_scalars("bls12_381", n, np.random.default_rng(1234))
d = torch.from_numpy(sc.view(np.int64).copy()).cuda()
for _ in range(3 + reps):
    e.msm_device(tid, d.data_ptr(), n)
torch.cuda.synchronize()
