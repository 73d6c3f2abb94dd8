"""Diagnostics: the same small tree committed on the device path and on the host path, node by
node (vc_verkle_debug_nodes): the first nodes whose items differ, with type and level."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg.verkle import VerkleTree  # noqa: E402

N, arity, n = 3, 255, 120
e = vkzg.Engine("bn254")
kzg = scheme.KZG(e, 256)
out = {}
for path in ("1", "0"):
    os.environ["VKZG_VERKLE_DEV"] = path
    rng = random.Random(7 * N + arity)
    t = VerkleTree(N)
    r0 = t.commitment(e, kzg.table)
    for _ in range(n):
        k = tuple(rng.randrange(arity) for _ in range(N))
        v = bytes(rng.randrange(256) for _ in range(32))
        try:
            t.insert_single(bytes(k), v)
        except vkzg.VCError:
            pass
    r1 = t.commitment(e, kzg.table)
    out[path] = (r0, r1, t.debug_nodes())
d, h = out["1"], out["0"]
print("roots equal:", d[0] == h[0], d[1] == h[1], "nodes", len(d[2]), len(h[2]))
bad = [(i, a, b) for i, (a, b) in enumerate(zip(d[2], h[2])) if a != b]
print("mismatching nodes:", len(bad))
for i, a, b in bad[:12]:
    print(i, "dev", a[0], a[1], hex(a[2])[:18], "host", b[0], b[1], hex(b[2])[:18])
