"""Latency of single IPA verify calls (N = 256, BN254, the bench's ipa_line shapes)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import vkzg
from vkzg import scheme
e = vkzg.Engine("bn254", 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
N = 256
ipa = scheme.IPA(e, N, scheme.ipa_crs(N + 1, max_=512))
r0 = 0x1234567890ABCDEF1234567890ABCDEF
d = scheme.LagrangeBasis([(r0 + i) % scheme.R_BN254 for i in range(N)])
c = ipa.commit(d)
prf = ipa.prove_point(c, 77, d)
for k in range(8):
    t0 = time.perf_counter()
    ok = ipa.verify_point(c, 77, prf)
    print(f"verify {k}: {(time.perf_counter() - t0) * 1e3:.3f} ms ok={ok}", flush=True)
