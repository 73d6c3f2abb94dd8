"""configs[4] single multiproof (bench.py mp_line's step, world 1) split into its two host-visible
phases: multiproof_begin_accumulate (transcript on a helper thread beside the shard's planning and
accumulate) and multiproof_finish (quotients, D, E, inner IPA proof); and the transcript alone.
usage: mp_phase_probe.py [log_q] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg._lib import lib  # noqa: E402
from bench import rj_plus_i  # noqa: E402

logq = int(sys.argv[1]) if len(sys.argv) > 1 else 16
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
N, Q = 256, 1 << logq
e = vkzg.Engine("bn254", 0)
stream = torch.cuda.current_stream()
e.set_stream(stream.cuda_stream)
crs = scheme.ipa_crs(N + 1, max_=512)
ipa = scheme.IPA(e, N, crs)
rng = np.random.default_rng(77)
data = rj_plus_i(rng, Q, N)
z = rng.integers(0, N, size=Q, dtype=np.uint64)
y = data.reshape(Q, N, 4)[np.arange(Q), z.astype(np.int64)].copy()
d_all = torch.from_numpy(data.view(np.int64)).cuda()
cxy_d = torch.zeros((Q, 8), dtype=torch.int64, device="cuda")
cinf_d = torch.zeros(Q, dtype=torch.uint8, device="cuda")
e.msm_batch_device(ipa.table, N, d_all.data_ptr(), Q, cxy_d.data_ptr(), cinf_d.data_ptr())
torch.cuda.synchronize()
cxy = cxy_d.cpu().numpy().view(np.uint64).copy()
cinf = cinf_d.cpu().numpy().copy()
rows = scheme.multiproof_rows(N, z)
for it in range(reps):
    S = torch.empty((rows, N, 4), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr, r = scheme.multiproof_begin_accumulate(e, N, cxy, cinf, z, y, 0, Q, d_all.data_ptr(), S.data_ptr())
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    mp = scheme.multiproof_finish(ipa, z, S[None].data_ptr(), 1, tr)
    t2 = time.perf_counter()
    t3 = time.perf_counter()
    tr2, _, _ = scheme.multiproof_begin(N, cxy, cinf, z, y)
    t4 = time.perf_counter()
    lib().vc_transcript_free(tr2)
    print(f"begin+accumulate {1e3 * (t1 - t0):.2f} ms  finish {1e3 * (t2 - t1):.2f} ms  total {1e3 * (t2 - t0):.2f}  "
          f"| transcript alone {1e3 * (t4 - t3):.2f} ms", flush=True)
