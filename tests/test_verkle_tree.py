"""Verkle tree (include/vc_verkle.h, C++ in libvkzg.so) against the oracle restatement of
/root/reference/verkle-tree/src (oracle/pyoracle/verkle.py): insert / get / path_to_stem
semantics on CPU (host code, no GPU), including the reference's own tests restated
(lib.rs:261-350) and its panic case; the level-batched commitments on the GPU
(tests/test_gpu_verkle.py)."""
import random

import pytest


def _key(rng, N, arity=255, prefix=()):
    return tuple(prefix) + tuple(rng.randrange(arity) for _ in range(N - len(prefix)))


def _val(rng):
    return bytes(rng.randrange(256) for _ in range(32))


def test_reference_insert_get_leaves():
    """lib.rs:261-297 test_insert_get_leaves (50 leaves, 1/4 sharing a stem), two insertion orders"""
    from vkzg.verkle import VerkleTree
    rng = random.Random(1)
    N = 3
    stem = _key(rng, N)
    kvs = {}
    for _ in range(50 // 4):
        kvs[_key(rng, N, prefix=stem)] = _val(rng)
    while len(kvs) < 50:
        kvs[_key(rng, N)] = _val(rng)
    keys = list(kvs)
    keys2 = keys[:]
    rng.shuffle(keys2)
    t1, t2 = VerkleTree(N), VerkleTree(N)
    for k1, k2 in zip(keys, keys2):
        t1.insert_single(k1, kvs[k1])
        t2.insert_single(k2, kvs[k2])
    for k in kvs:
        assert t1.get_single(k) == t2.get_single(k) == kvs[k]


def test_reference_overwrite():
    """lib.rs:299-311 test_overwrite"""
    from vkzg.verkle import VerkleTree
    rng = random.Random(2)
    t = VerkleTree(3)
    k = _key(rng, 3)
    v1, v2 = _val(rng), _val(rng)
    t.insert_single(k, v1)
    t.insert_single(k, v2)
    assert t.get_single(k) == v2


def test_reference_path_to_stem():
    """lib.rs:327-349 test_path_to_stem"""
    from vkzg.verkle import VerkleTree
    rng = random.Random(3)
    t = VerkleTree(3)
    k = _key(rng, 3)
    t.insert_single(k, _val(rng))
    t.insert_single(_key(rng, 3, prefix=(k[0],)), _val(rng))
    for i, p in enumerate(t.path_to_stem(k)):
        assert p[0] == tuple(k[:i + 1]) and p[1] == k[i]


@pytest.mark.parametrize("N,arity,n", [(3, 255, 300), (3, 4, 40), (4, 3, 60), (5, 2, 30)])
def test_tree_semantics_match_oracle(N, arity, n):
    """random trees with heavy prefix sharing (small arity): every insert (or its rejection,
    where the reference panics), get and path agree with the oracle restatement"""
    from pyoracle import verkle as ov
    from vkzg._lib import VCError
    from vkzg.verkle import VerkleTree
    rng = random.Random(N * 100 + arity)
    t, o = VerkleTree(N), ov.VerkleTree(N)
    keys, rejected = [], 0
    for _ in range(n):
        k = _key(rng, N, arity)
        v = _val(rng)
        try:
            o.insert_single(k, v)
            ok = True
        except ov.VerklePanic:
            ok = False
        if ok:
            t.insert_single(k, v)
            keys.append(k)
        else:
            rejected += 1
            with pytest.raises(VCError):
                t.insert_single(k, v)
    for k in keys + [_key(rng, N, arity) for _ in range(20)]:
        assert t.get_single(k) == o.get_single(k), k
        try:
            want = o.path_to_stem(k)
        except KeyError:
            with pytest.raises(VCError):
                t.path_to_stem(k)
            continue
        assert t.path_to_stem(k) == want
    if arity <= 4:
        assert rejected > 0   # the panic path is exercised


def test_key32_sets_reach_every_reduction():
    """tests/verkle32_keys.py (the key-length-32 GPU parity tests' stems) reaches stems >= r with
    every quotient 0..5 of bytes_to_item's reduction (lagrange_basis.rs:175-176), leaf units on
    both sides of N / 2 = 16 (c1 / c2, node.rs:226-239), and the oracle tree inserts them all
    without the reference's panic"""
    from verkle32_keys import R, key_set, value
    from pyoracle import verkle as ov
    keys = key_set(11)
    assert {int.from_bytes(k, "little") // R for k in keys} >= {0, 1, 2, 3, 4, 5}
    assert any(k[-1] < 16 for k in keys) and any(k[-1] >= 16 for k in keys)
    o, rng = ov.VerkleTree(32), random.Random(3)
    for k in keys:
        o.insert_single(k, value(rng))


def test_key32_quirk_update_adds_an_extension():
    """the reference's level-skipping split (node.rs:176-185) makes a later re-insert of a key add a
    second extension for its stem: the oracle and the engine's host trie agree on the shape"""
    from verkle32_keys import quirk_keys, value
    from pyoracle import verkle as ov
    from vkzg.verkle import VerkleTree
    first, again = quirk_keys()
    o, t, rng = ov.VerkleTree(32), VerkleTree(32), random.Random(4)
    for k in first:
        v = value(rng)
        o.insert_single(k, v)
        t.insert_single(k, v)
    n_before = t.stats()["extension"]
    v = value(rng)
    o.insert_single(again, v)
    t.insert_single(again, v)
    assert t.stats()["extension"] == n_before + 1 == 4

    def exts(node):
        return 1 if node.ext else sum(exts(c) for c in node.children.values())
    assert exts(o.root) == 4
