"""CPU tests of the host side of the boundary (no GPU): transcript / hash_to_field /
compressed encoding / IPA CRS from libvkzg.so against the golden fixtures and the oracle."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def load(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)


def P(h):
    return None if h is None else (int(h[0], 16), int(h[1], 16))


def test_hash_to_field_golden():
    from vkzg import scheme
    for h in load("transcript.json")["hash_to_field"]:
        assert hex(scheme.hash_to_field(bytes.fromhex(h["msg"]), h["dst"].encode())) == h["out"]


def test_transcript_golden():
    from vkzg import scheme
    t = scheme.TranscriptHasher("ipa")
    t.append_point((1, 2), "C")
    t.append_fr(5, "input point")
    t.append_fr(7, "output point")
    assert hex(t.digest("w")) == load("transcript.json")["transcript_ipa_w"]


def test_transcript_matches_oracle_multistep():
    from pyoracle import arkser
    from vkzg import scheme
    a, b = arkser.TranscriptHasher("multiproof"), scheme.TranscriptHasher("multiproof")
    pts = [P(c["point"]) for c in load("transcript.json")["compressed"]]
    for i, p in enumerate(pts):
        for t in (a, b):
            t.append_point(p, "C")
            t.append_usize(i * 977, "z")
            t.append_fr(i * 12345678901234567, "y")
        if i % 3 == 2:
            assert a.digest("r") == b.digest("r")
    assert a.digest("t") == b.digest("t")


def test_multiproof_transcript_matches_oracle():
    """vc_multiproof_begin's challenge r (multiproof.rs:106-114) over Q = 9000 queries -- the
    records are serialised on several host threads at this size -- against the oracle's
    transcript fed query by query; identity commitments included."""
    import numpy as np
    import vkzg
    from pyoracle import arkser
    from vkzg import scheme
    from vkzg._lib import lib
    gold = [P(c["point"]) for c in load("transcript.json")["compressed"]]
    Q, N = 9000, 256
    pts = [None if i % 97 == 5 else gold[i % len(gold)] for i in range(Q)]
    z = np.array([(i * 37) % N for i in range(Q)], dtype=np.uint64)
    ys = [(i * 0x9E3779B97F4A7C15 + 11) % (1 << 250) for i in range(Q)]
    a = arkser.TranscriptHasher("multiproof")
    for p, zi, yi in zip(pts, z, ys):
        a.append_point(p, "C")
        a.append_usize(int(zi), "z")
        a.append_fr(yi, "y")
    want = a.digest("r")
    cxy, cinf = vkzg.points_to_arrays("bn254", pts)
    tr, r, rows = scheme.multiproof_begin(N, cxy, cinf, z, vkzg.ints_to_limbs(ys))
    try:
        assert sum(int(v) << (64 * k) for k, v in enumerate(r)) == want
        assert rows == len(set(int(v) for v in z))
        # the state after the digest (the records stream into the hash, never stored): the next
        # challenge t after D (multiproof.rs:152-155) agrees with the oracle's
        d = gold[3]
        a.append_point(d, "D")
        want_t = a.digest("t")
        dxy, dinf = vkzg.points_to_arrays("bn254", [d])
        lib().vc_transcript_append_point(tr, scheme._p(dxy), int(dinf[0]), b"D")
        t = np.zeros(4, dtype=np.uint64)
        assert lib().vc_transcript_digest(tr, b"t", scheme._p(t)) == 0
        assert sum(int(v) << (64 * k) for k, v in enumerate(t)) == want_t
    finally:
        lib().vc_transcript_free(tr)


def test_compress_and_to_data_item_golden():
    from pyoracle import arkser
    from vkzg import scheme
    for c in load("transcript.json")["compressed"]:
        assert scheme.point_compress(P(c["point"])).hex() == c["bytes"]


def test_ipa_crs_golden():
    import pytest
    import vkzg
    from vkzg import scheme
    want = [P(h) for h in load("ipa_crs_bn254.json")["points"]]
    assert scheme.ipa_crs(257, max_=512) == want
    with pytest.raises(vkzg.VCError):          # OutOfBounds: default max 256 < 257
        scheme.ipa_crs(257)


def test_multiproof_rows_host():
    """vc_multiproof_rows (host only): the distinct query points, VC_E_DOMAIN for z >= N (the
    reference indexes the Lagrange evaluations with z and panics), VC_E_INVALID for a width that is
    not a power of two -- the checks vc_multiproof_begin_accumulate runs before anything else."""
    import numpy as np
    from vkzg import scheme
    from vkzg._lib import lib
    VC_E_INVALID, VC_E_DOMAIN = -1, -8  # include/vc_msm.h
    z = np.array([3, 3, 0, 255, 7, 3], dtype=np.uint64)
    assert scheme.multiproof_rows(256, z) == 4
    import ctypes
    rows = ctypes.c_size_t()
    bad = np.array([1, 256], dtype=np.uint64)
    assert lib().vc_multiproof_rows(256, 2, scheme._p(bad), ctypes.byref(rows)) == VC_E_DOMAIN
    assert lib().vc_multiproof_rows(255, 2, scheme._p(z), ctypes.byref(rows)) == VC_E_INVALID
