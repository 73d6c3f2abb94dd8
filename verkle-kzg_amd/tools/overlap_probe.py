"""Can two window slices of one MSM overlap on one GPU? Two contexts on two streams, each
computing window part k of G of the same 2^20 BLS12-381 MSM from its own host thread (ctypes
drops the GIL), against the same parts run back to back. If the latency-bound tail of one
slice hides under the throughput-bound accumulate of the other, concurrent < sequential."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

n = 1 << 20
G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
streams = [torch.cuda.Stream() for _ in range(G)]
engs = []
for k in range(G):
    e = vkzg.Engine("bls12_381", 0)
    e.set_stream(streams[k].cuda_stream)
    engs.append((e, e.random_bases(n, seed=2024)))
sc = vkzg.random_scalars("bls12_381", n, np.random.default_rng(1234))
d = torch.from_numpy(sc.view(np.int64).copy()).cuda()
torch.cuda.synchronize()


def part(k, reps):
    e, tid = engs[k]
    for _ in range(reps):
        e.msm_device_window_part(tid, d.data_ptr(), n, k, G)


for k in range(G):
    part(k, 2)
reps = 10
t0 = time.perf_counter()
for _ in range(reps):
    for k in range(G):
        part(k, 1)
seq = (time.perf_counter() - t0) / reps * 1e3
t0 = time.perf_counter()
ths = [threading.Thread(target=part, args=(k, reps)) for k in range(G)]
for t in ths:
    t.start()
for t in ths:
    t.join()
con = (time.perf_counter() - t0) / reps * 1e3
ref = vkzg.Engine("bls12_381", 0)
rt = ref.random_bases(n, seed=2024)
for _ in range(2):
    ref.msm_device(rt, d.data_ptr(), n)
t0 = time.perf_counter()
for _ in range(reps):
    ref.msm_device(rt, d.data_ptr(), n)
whole = (time.perf_counter() - t0) / reps * 1e3
print(f"G={G}: sequential parts {seq:.3f} ms, concurrent parts {con:.3f} ms, whole MSM {whole:.3f} ms")
