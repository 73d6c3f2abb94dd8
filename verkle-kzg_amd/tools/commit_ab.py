"""configs[2] A/B: 10,000 batched width-256 Bandersnatch commits (device scalars, bench.py's
cstep) per fixed-base geometry, wall ms per batch without per-kernel events, table GB. Run under
two libraries (VKZG_LIB) to compare entry layouts. usage: commit_ab.py [reps] ["c:windows" ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
geoms = [tuple(int(x) for x in g.split(":")) for g in sys.argv[2:]] or [(16, 0), (17, 0), (18, 14)]
dev = torch.device("cuda", 0)
B = 10_000
sc = vkzg.random_scalars("bandersnatch", B * 256, np.random.default_rng(5))
dcs = torch.from_numpy(sc.view(np.int64).copy()).to(dev)
dxy = torch.zeros((B, 8), dtype=torch.int64, device=dev)
dinf = torch.zeros(B, dtype=torch.uint8, device=dev)
lib = os.path.basename(vkzg.LIB_PATH)
ref = None
for c, w in geoms:
    e = vkzg.Engine("bandersnatch", 0)
    e.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    tab = e.random_bases(256, seed=3)
    try:
        e.fixed_base_precompute(tab, c, w)
    except vkzg.VCError as ex:
        print(f"{lib} c={c} windows={w}: no table ({ex})", flush=True)
        e.close()
        continue
    for _ in range(2):
        e.msm_batch_device(tab, 256, dcs.data_ptr(), B, dxy.data_ptr(), dinf.data_ptr())
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        e.msm_batch_device(tab, 256, dcs.data_ptr(), B, dxy.data_ptr(), dinf.data_ptr())
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    out = dxy.cpu().numpy().copy()
    same = True if ref is None else bool(np.array_equal(out, ref))
    ref = out if ref is None else ref
    med = sorted(ts)[len(ts) // 2]
    print(f"{lib} c={c} windows={e.fixed_base_geometry(tab)[1]} table={e.fixed_base_table_bytes(tab) / 1e9:.1f} GB: "
          f"{med:.3f} ms per 10k ({B / med * 1e3 / 1e6:.2f} M commits/s) reps={[round(x, 3) for x in ts]} same={same}",
          flush=True)
    e.close()
