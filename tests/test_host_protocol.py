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
