"""IPA N = 256 prove: the Python mirror's call (scheme.IPA.prove_point: marshalling the data, the
commitment and the proof buffers, converting the proof back to Python integers) against the
bare C ABI call vc_ipa_prove on inputs marshalled once -- medians of 21 calls each, alternating.
usage: ipa_abi_probe.py"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg._lib import lib, check  # noqa: E402

e = vkzg.Engine("bn254", 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
N = 256
ipa = scheme.IPA(e, N, scheme.ipa_crs(N + 1, max_=512))
r0 = 0x1234567890ABCDEF1234567890ABCDEF
data = scheme.LagrangeBasis([(r0 + i) % scheme.R_BN254 for i in range(N)])
com = ipa.commit(data)
prf = ipa.prove_point(com, 77, data)
d = np.ascontiguousarray(data.limbs(N)[:N])
cxy, cinf = scheme._pt_arrays([com])
pts = vkzg.ints_to_limbs([77], 4)
K = 8
buf, arrs = scheme.IPAProof._alloc(K)
arr = (scheme._ProofBuf * 1)(buf)


def abi():
    check(lib().vc_ipa_prove(e.h, ipa.table, N, scheme._p(d), scheme._p(cxy), scheme._p(cinf), scheme._p(pts), 1,
                             None, ctypes.cast(arr, scheme._P)), "ipa_prove")


def py():
    return ipa.prove_point(com, 77, data)


abi()
got = scheme.IPAProof._from(arr[0], arrs)
assert got.as_dict() == prf.as_dict(), "the bare call must give the same proof"
ta, tp = [], []
for _ in range(21):
    t0 = time.perf_counter()
    abi()
    ta.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    py()
    tp.append(time.perf_counter() - t0)
print(f"prove N=256: C ABI call {np.median(ta) * 1e3:.3f} ms, Python mirror call {np.median(tp) * 1e3:.3f} ms "
      f"(min {min(ta) * 1e3:.3f} / {min(tp) * 1e3:.3f})")
