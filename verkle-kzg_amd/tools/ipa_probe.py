"""Where the time of one IPA N = 256 prove / verify (BN254) goes: wall ms per call, then the
per-kernel totals per call with event timing on. usage: ipa_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg._lib import lib  # noqa: E402
import ctypes  # noqa: E402
import numpy as np  # noqa: E402

e = vkzg.Engine("bn254", 0)
e.set_stream(torch.cuda.current_stream().cuda_stream)
N = 256
ipa = scheme.IPA(e, N, scheme.ipa_crs(N + 1, max_=512))
r0 = 0x1234567890ABCDEF1234567890ABCDEF
data = scheme.LagrangeBasis([(r0 + i) % scheme.R_BN254 for i in range(N)])
com = ipa.commit(data)
prf = ipa.prove_point(com, 77, data)
reps = 20
for name, f in (("commit", lambda: ipa.commit(data)), ("prove", lambda: ipa.prove_point(com, 77, data)),
                ("verify", lambda: ipa.verify_point(com, 77, prf))):
    f()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    wall = (time.perf_counter() - t0) / reps * 1e3
    e.enable_timing(True)
    e.reset_timing()
    for _ in range(reps):
        f()
    e.enable_timing(False)
    names = ctypes.create_string_buffer(1 << 16)
    rows = []
    for k in ("fb_commit", "fb_commit_small", "fb_combine", "fb_normalize", "fb_normalize_out", "normalize_out", "norm_prep", "norm_finish", "msm_accumulate",
              "msm_sort_hist", "msm_sort_coarse", "msm_sort_fine", "msm_fixup", "msm_bitsum", "msm_sumpart",
              "msm_segsum", "to_canon", "to_mont", "glv_split", "sparse", "fb_chunk"):
        ms, cnt = e.kernel_time(k)
        if cnt:
            rows.append((k, ms / reps, cnt / reps))
    tot = sum(r[1] for r in rows)
    print(f"{name}: wall {wall:.3f} ms, timed kernels {tot:.3f} ms")
    for k, ms, c in rows:
        print(f"   {k:16s} {ms:.4f} ms  {c:.1f} launches")

# 256 independent proofs in one call (bench.py ipa_line batch_prove)
B = 256
datas = [scheme.LagrangeBasis([(r0 * (k + 1) + i) % scheme.R_BN254 for i in range(N)]) for k in range(B)]
coms = ipa.commit_batch(datas)
pts = [(31 * k) % N for k in range(B)]
ipa.prove_batch_points(coms, pts, datas)
t0 = time.perf_counter()
ipa.prove_batch_points(coms, pts, datas)
wall = (time.perf_counter() - t0) * 1e3
e.enable_timing(True)
e.reset_timing()
ipa.prove_batch_points(coms, pts, datas)
e.enable_timing(False)
rows = []
for k in ("fb_commit", "fb_commit_small", "fb_combine", "fb_normalize_out", "normalize_out", "norm_prep", "norm_finish", "fb_commit_cm"):
    ms, cnt = e.kernel_time(k)
    if cnt:
        rows.append((k, ms, cnt))
print(f"batch {B}: wall {wall:.2f} ms, timed kernels {sum(r[1] for r in rows):.3f} ms")
for k, ms, c in rows:
    print(f"   {k:16s} {ms:.4f} ms  {c} launches")
t0 = time.perf_counter()
ipa.prove_batch_points(coms, pts, datas)
print(f"batch {B} again: {(time.perf_counter() - t0) * 1e3:.2f} ms")
t0 = time.perf_counter()
d = np.concatenate([x.limbs(N)[:N] for x in datas])
print(f"python limbs of {B} datas: {(time.perf_counter() - t0) * 1e3:.2f} ms")
t0 = time.perf_counter()
cxy, cinf = scheme._pt_arrays(coms)
print(f"python commitment arrays: {(time.perf_counter() - t0) * 1e3:.2f} ms")
