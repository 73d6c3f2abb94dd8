"""Phase timing of the sharded IPA multiproof at Q = 2^k (world 1): begin / accumulate / finish."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg._lib import lib  # noqa: E402

logq = int(sys.argv[1]) if len(sys.argv) > 1 else 16
N, Q = 256, 1 << logq
e = vkzg.Engine("bn254", 0)
crs = scheme.ipa_crs(N + 1, max_=512)
ipa = scheme.IPA(e, N, crs)
rng = np.random.default_rng(77)
data = rng.integers(0, 1 << 63, size=(Q * N, 4), dtype=np.uint64)
data[:, 3] &= np.uint64((1 << 60) - 1)
z = rng.integers(0, N, size=Q, dtype=np.uint64)
y = data.reshape(Q, N, 4)[np.arange(Q), z.astype(np.int64)].copy()
d_all = torch.from_numpy(data.view(np.int64)).cuda()
cxy_d = torch.zeros((Q, 8), dtype=torch.int64, device="cuda")
cinf_d = torch.zeros(Q, dtype=torch.uint8, device="cuda")
e.msm_batch_device(ipa.table, N, d_all.data_ptr(), Q, cxy_d.data_ptr(), cinf_d.data_ptr())
torch.cuda.synchronize()
cxy = cxy_d.cpu().numpy().view(np.uint64).copy()
cinf = cinf_d.cpu().numpy().copy()
e.enable_timing(True)
for it in range(5):
    e.reset_timing()
    t0 = time.perf_counter()
    tr, r, rows = scheme.multiproof_begin(N, cxy, cinf, z, y)
    t1 = time.perf_counter()
    S = torch.zeros((rows, N, 4), dtype=torch.int64, device="cuda")
    scheme.multiproof_accumulate(e, N, z, 0, Q, d_all.data_ptr(), r, S.data_ptr())
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    mp = scheme.multiproof_finish_ipa(ipa, z, S.data_ptr(), 1, tr)
    t3 = time.perf_counter()
    ms, cnt = e.kernel_time("mp_chunk")
    print(f"begin {1e3 * (t1 - t0):.2f} ms  accumulate {1e3 * (t2 - t1):.2f} ms  finish {1e3 * (t3 - t2):.2f} ms  "
          f"mp_chunk {ms / max(cnt, 1):.4f} ms ({Q * N * 32 / (ms / max(cnt, 1) * 1e-3) / 1e12:.2f} TB/s)", flush=True)
e.enable_timing(False)
# IPA prove alone (single proof)
d = scheme.LagrangeBasis([int(v) for v in range(N)])
c = ipa.commit(d)
for it in range(3):
    t0 = time.perf_counter()
    ipa.prove_point(c, 1000, d)
    print(f"ipa prove_point {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
e.enable_timing(True)
e.reset_timing()
ipa.prove_point(c, 1000, d)
for k in ("fb_commit_small", "fb_combine_small", "fb_normalize_out", "fb_commit", "fb_combine"):
    ms, n = e.kernel_time(k)
    if n:
        print(f"  {k}: {n} launches, {ms / n * 1e3:.1f} us avg", flush=True)
