"""Multiproof verification (vc_multiproof_verify_ipa) at Q = 2^k, N = 256: wall ms per call, for
a rocprofv3 kernel trace of the verifier's e-coefficient MSM. usage: mp_verify_probe.py [k] [reps]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg._lib import check, lib  # noqa: E402

logq = int(sys.argv[1]) if len(sys.argv) > 1 else 12
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
N, Q = 256, 1 << logq
e = vkzg.Engine("bn254", 0)
ipa = scheme.IPA(e, N, scheme.ipa_crs(N + 1, max_=512))
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
rows = scheme.multiproof_rows(N, z)
S = torch.empty((rows, N, 4), dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
tr, _r = scheme.multiproof_begin_accumulate(e, N, cxy, cinf, z, y, 0, Q, d_all.data_ptr(), S.data_ptr())
mp = scheme.multiproof_finish(ipa, z, S.data_ptr(), 1, tr)
b, _arrs = mp["proof"]._to()
dxy, dinf = scheme._pt_arrays([mp["d"]])


def verify():
    res = ctypes.c_int()
    check(lib().vc_multiproof_verify_ipa(e.h, ipa.table, N, Q, scheme._p(cxy), scheme._p(cinf), scheme._p(z),
                                         scheme._p(y), scheme._p(dxy), int(dinf[0]), ctypes.byref(b),
                                         ctypes.byref(res)), "multiproof_verify")
    return bool(res.value)


assert verify()
for _ in range(reps):
    t0 = time.perf_counter()
    ok = verify()
    print(f"verify Q={Q}: {1e3 * (time.perf_counter() - t0):.3f} ms ok={ok}", flush=True)
