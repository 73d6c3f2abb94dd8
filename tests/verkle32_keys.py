"""Key sets for the key-length-32 verkle parity tests (the bench's shape, bench.py verkle line).

At N = 32 the stem is the whole 32-byte key (lib.rs:61-67, node.rs:45) and the extension's
`stem_item = bytes_to_item(stem)` (node.rs:248-250 -> lagrange_basis.rs:175-176,
from_le_bytes_mod_order) really reduces: a random stem is >= r whenever its top byte is >= 0x31
(r = 0x30644e72... x 2^192). The engine's reduction (verkle.cpp item_of_bytes) takes one quotient
estimate q = floor(v_3 / r_3) <= 5 and one conditional add-back, so the sets below cover every
q = 0..5 and both signs of the estimate's error: k r - 1, k r, k r + 1 for k = 1..5, 2^256 - 1,
the stems straddling the top-limb boundary of each k r, and random stems >= r. The leaf unit is
the key's last byte (lib.rs:112-116), which is also the stem's top byte, so the random keys mix
units < 16 (slots in c1) and >= 16 (c2, node.rs:226-239); shared prefixes give internal nodes
below the root and the reference's level-skipping splits (node.rs:176-185).

Test data only; never shipped.
"""
import random

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def boundary_stems():
    out = []
    for k in range(1, 6):
        for d in (-1, 0, 1):
            out.append(k * R + d)
        top = (k * R) >> 192                       # stems whose top limb is k r's but below k r
        out.append(top << 192)
        out.append(((top + 1) << 192) - 1)
    out.append((1 << 256) - 1)
    out.append(0)
    return [v.to_bytes(32, "little") for v in out if 0 <= v < (1 << 256)]


def key_set(seed, n_random=300):
    """boundary stems + random keys: a third with the top byte >= 0x31 (stem >= r), a third with
    top byte < 16 (c1 slots), a third sharing 2-byte prefixes from a small alphabet (depth)"""
    rng = random.Random(seed)
    keys = boundary_stems()
    for i in range(n_random):
        b = bytearray(rng.randrange(256) for _ in range(32))
        kind = i % 3
        if kind == 0:
            b[31] = rng.randrange(0x31, 256)
        elif kind == 1:
            b[31] = rng.randrange(16)
        else:
            b[0], b[1] = rng.randrange(4), rng.randrange(3)
        keys.append(bytes(b))
    rng.shuffle(keys)
    return keys


def quirk_keys():
    """A, B, C in this order, then A again: A and B share units 0-1, so their split puts an
    internal node at root slot 200 keyed by unit 2 (the reference's level-skipping split,
    node.rs:176-185); C (unit 1 = A's unit 2) then reaches A's extension through that node at depth
    1 and splits it; re-inserting A walks slot 200 -> unit A[1] = 7, finds nothing and adds a second
    extension for A's stem. Returned as (first-round keys, the key to re-insert later)."""
    a = bytes([200, 7, 1]) + bytes(range(3, 32))
    b = bytes([200, 7, 2]) + bytes(range(3, 32))
    c = bytes([200, 1, 9]) + bytes(range(40, 69))
    return [a, b, c], a


def value(rng):
    return bytes(rng.randrange(256) for _ in range(32))
