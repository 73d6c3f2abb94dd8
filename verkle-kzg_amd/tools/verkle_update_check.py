"""Repeated 1 % update rounds on a 32-unit-key verkle tree (the bench's shape) against fresh trees:
after every round the updated tree's root is compared with a fresh tree with the same insertion
history committed in full, on the same engine (and, informationally, with a fresh tree of the final
contents inserted once: the reference's level-skipping splits, node.rs:176-185, make the trie depend
on the insertion order, so that one may differ legitimately). Prints one line per round and exits non-zero on a mismatch.
usage: verkle_update_check.py [keys] [rounds] [seed] [distinct 0/1]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402
from vkzg.verkle import VerkleTree  # noqa: E402

nk = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 91
distinct = len(sys.argv) > 4 and sys.argv[4] == "1"
e = vkzg.Engine("bn254")
kzg = scheme.KZG(e, 256)
e.fixed_base_precompute(kzg.table, 16)
rng = np.random.default_rng(seed)
keys = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
vals = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)


def fresh(v, hist=()):
    f = VerkleTree(32)
    for i in range(nk):
        f.insert_single(keys[i].tobytes(), v[i].tobytes())
    for kv in hist:
        f.insert_single(*kv)
    return f.commitment(e, kzg.table)


t = VerkleTree(32)
for i in range(nk):
    t.insert_single(keys[i].tobytes(), vals[i].tobytes())
root0 = t.commitment(e, kzg.table)
bad = 0
print("env", {k: v for k, v in os.environ.items() if k.startswith("VKZG")}, flush=True)
print("round 0 full == fresh:", root0 == fresh(vals), flush=True)
cur = vals.copy()
history = []
for r in range(1, rounds + 1):
    idx = (rng.choice(nk, size=max(1, nk // 100), replace=False) if distinct
           else rng.integers(0, nk, size=max(1, nk // 100)))
    for i in idx:
        cur[i] = rng.integers(0, 256, size=32, dtype=np.uint8)
        history.append((keys[i].tobytes(), cur[i].tobytes()))
        t.insert_single(*history[-1])
    dirty = t.stats()["dirty"]
    got = t.commitment(e, kzg.table)
    ok = got == fresh(vals, history)
    bad += not ok
    print(f"round {r}: {len(idx)} updates ({len(set(idx.tolist()))} distinct), {dirty} dirty, "
          f"update == same-history fresh tree: {ok}, == final contents inserted once: {got == fresh(cur)}, "
          f"nodes {t.stats()}",
          flush=True)
e.close()
sys.exit(1 if bad else 0)
