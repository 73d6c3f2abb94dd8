import sys, os, time
sys.path[:0] = ["verkle-kzg_amd", "oracle"]
import numpy as np, vkzg
rng = np.random.default_rng(1)
for curve in sys.argv[1:]:
    e = vkzg.Engine(curve)
    for n in (1, 64, 1000):
        t = e.random_bases(n, seed=n)
        print(curve, n, "bases ok", flush=True)
        r = e.msm(t, vkzg.random_scalars(curve, n, rng))
        print(curve, n, "msm ok", r[1], flush=True)
