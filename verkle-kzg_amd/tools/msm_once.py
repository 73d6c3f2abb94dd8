"""A few 2^k-point MSMs and nothing else -- the program to run under rocprofv3 --pmc passes
(kernel-level counters of one MSM). usage: msm_once.py [curve] [log_n] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

curve = sys.argv[1] if len(sys.argv) > 1 else "bls12_381"
n = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 20)
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
e = vkzg.Engine(curve, 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
tid = e.random_bases(n, seed=2024)
sc = vkzg.random_scalars(curve, n, np.random.default_rng(1234))
d = torch.from_numpy(sc.view(np.int64).copy()).cuda()
for _ in range(reps):
    e.msm_device(tid, d.data_ptr(), n)
torch.cuda.synchronize()
print("ok")
