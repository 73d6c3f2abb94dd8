"""C4 probe: 2^20 BLS12-381 KZG commit + open as one vc_kzg_commit_prove_device call (and as two
calls), a few times each, for a rocprofv3 kernel trace (tools/timeline.py prints the last call)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg._lib import check, lib  # noqa: E402

d = 1 << 20
e = vkzg.Engine("bls12_381", 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
secret = vkzg.ints_to_limbs([100])[0].copy()
tid, size = ctypes.c_int(), ctypes.c_size_t()
check(lib().vc_kzg_setup(e.h, d, ctypes.c_void_p(secret.ctypes.data), ctypes.byref(tid), ctypes.byref(size)), "setup")
tid = tid.value
ev = vkzg.random_scalars("bls12_381", d, np.random.default_rng(44))
d_ev = torch.from_numpy(ev.view(np.int64).copy()).cuda()
mode = sys.argv[1] if len(sys.argv) > 1 else "fused"
pt = vkzg.ints_to_limbs([d // 3 if "out" not in mode else d + 987654321])[0].copy()
bufs = [np.zeros(12, dtype=np.uint64), np.zeros(1, dtype=np.uint8), np.zeros(12, dtype=np.uint64),
        np.zeros(1, dtype=np.uint8), np.zeros(4, dtype=np.uint64)]
P = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731


def fused():
    check(lib().vc_kzg_commit_prove_device(e.h, tid, d, ctypes.c_void_p(d_ev.data_ptr()), d, P(pt),
                                           *[P(b) for b in bufs]), "fused")


ts = []
for _ in range(6):
    t0 = time.perf_counter()
    fused()
    ts.append((time.perf_counter() - t0) * 1e3)
print(f"{mode}: ms per call {[round(t, 3) for t in ts]}", flush=True)
