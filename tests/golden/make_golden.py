#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/ from the Python oracle (oracle/pyoracle).

The reference (Rust/arkworks, /root/reference) cannot be built or run in this image (no
cargo/rustc, no arkworks sources) and its tests hold no golden vectors (all random
round-trips). So these fixtures are the oracle's outputs on fixed seeds:
group/field results are mathematically unique (pinned by the curve KATs and by the
reference's round-trip/tamper tests restated in tests/test_oracle.py); byte conventions
(transcript, CRS hashing, compressed flags) are "parity unpinned vs arkworks".

    python tests/golden/make_golden.py        # rewrites tests/golden/*.json (deterministic)
    python tests/golden/make_golden.py multiproof_256   # only multiproof_256.json
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))

from pyoracle import arkser, protocol  # noqa: E402
from pyoracle.curves import BANDERSNATCH, BLS12_381, BN254, CURVES, random_points  # noqa: E402


def hexs(x):
    return hex(int(x))


def pt(P):
    if P is None:
        return None
    return [hexs(P[0]), hexs(P[1])]


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


def msm_cases():
    out = []
    rng = random.Random(0x5EED)
    for C, sizes in ((BN254, (1, 2, 7, 256)), (BLS12_381, (1, 7, 64)), (BANDERSNATCH, (1, 7, 64))):
        for n in sizes:
            pts = random_points(C, n, rng)
            sc = [rng.randrange(C.r) for _ in range(n)]
            if n >= 7:
                sc[0] = 0
                sc[1] = C.r - 1
                pts[3] = pts[2]          # repeated base
                sc[3] = sc[2]            # P + P
                pts[4] = C.neg(pts[5])   # P + (-P) with equal scalars
                sc[4] = sc[5]
                if C.kind == "sw":
                    pts[6] = None        # identity base
            out.append({"curve": C.name, "n": n, "bases": [pt(P) for P in pts],
                        "scalars": [hexs(s) for s in sc], "expected": pt(C.msm(pts, sc))})
    return out


def main():
    dump("msm.json", {"source": "oracle/pyoracle curves.msm (utils.rs:16-19 restated)", "cases": msm_cases()})

    # transcript / hash_to_field / serialisation (parity unpinned vs arkworks)
    t = arkser.TranscriptHasher("ipa")
    t.append_point(BN254.g, "C")
    t.append_fr(5, "input point")
    t.append_fr(7, "output point")
    w = t.digest("w")
    h2f = [{"msg": m.hex(), "dst": d.decode(), "out": hexs(arkser.hash_to_field(m, d, BN254.r))}
           for m, d in ((b"", b"ipa"), (b"abc", b"multiproof"), (bytes(range(100)), b"ipa"))]
    rng = random.Random(11)
    pts = random_points(BN254, 6, rng) + [BN254.neg(BN254.g), BN254.g, None]
    dump("transcript.json", {
        "hash_to_field": h2f,
        "transcript_ipa_w": hexs(w),
        "compressed": [{"point": pt(P), "bytes": arkser.ser_point_compressed(P).hex(),
                        "to_data_item": hexs(arkser.to_data_item(P))} for P in pts],
        "note": "DefaultFieldHasher<Sha256> with ExpanderXmd z_pad = 48 bytes; parity unpinned vs arkworks",
    })

    # IPA CRS (ipa_point_generator.rs) -- first 257 points (N = 256 + q)
    crs = protocol.ipa_gen_points(257, max_=512)
    dump("ipa_crs_bn254.json", {"seed": "eth_verkle_oct_2021", "points": [pt(P) for P in crs],
                                "note": "from_random_bytes quirk per SURVEY A.6; parity unpinned vs arkworks"})

    # IPA N=256: commit of r+i data (benches/ipa.rs:54-62) and proofs in/out of domain
    N = 256
    ipa = protocol.IPA(N, points=crs)
    r0 = random.Random(21).randrange(BN254.r)
    data = protocol.LagrangeBasis.from_vec([(r0 + i) % BN254.r for i in range(N)])
    com = ipa.commit(data)
    pin = ipa.prove(com, 77, data)
    pout = ipa.prove(com, 1000, data)
    pcom = ipa.prove_commitment(com, data)                              # ipa/mod.rs:199-234
    assert ipa.verify_commitment_proof(com, pcom)
    ser = lambda p: {"l": [pt(x) for x in p["l"]], "r": [pt(x) for x in p["r"]], "tip": hexs(p["tip"]),
                     "y": hexs(p["y"])}
    dump("ipa_256.json", {"N": N, "data": [hexs(x) for x in data.evals], "commitment": pt(com),
                          "proof_in_domain": {"point": 77, **ser(pin)},
                          "proof_out_domain": {"point": 1000, **ser(pout)},
                          "commitment_proof": ser({**pcom, "y": 0})})

    # KZG d=256 (s = 100): Lagrange SRS scalars, commit, openings in/boundary/out of domain
    kz = protocol.KZG(256)
    rng = random.Random(31)
    ev = [rng.randrange(BN254.r) for _ in range(200)]
    kd = protocol.LagrangeBasis(ev, 256)
    kc = kz.commit(kd)
    opens = []
    for z in (3, 199, 200, 255, 256, 123456789):
        if z == kz.max_size():
            # prove_point tests `<=` but vanishing_at(size) is out of bounds: the reference panics
            opens.append({"point": z, "error": "out of bounds (Appendix B.4)"})
            continue
        q, y = kz.quotient(z, kd)
        pr = kz.prove_point(kc, z, kd)
        opens.append({"point": z, "y": hexs(y), "q_head": [hexs(v) for v in q[:4]],
                      "q_sum": hexs(sum(q) % BN254.r), "proof": pt(pr["proof"])})
    dump("kzg_256.json", {"max_items": 256, "secret": 100, "lagrange_scalars": [hexs(c) for c in kz.lagrange_scalars],
                          "evals": [hexs(x) for x in ev], "commitment": pt(kc), "openings": opens})

    # multiproof: 20 queries, N = 32, IPA and KZG (multiproof.rs:261-357)
    mp = {}
    for name, vc in (("ipa", protocol.IPA(32, points=crs[:33])), ("kzg", protocol.KZG(32))):
        rng = random.Random(41)
        qs = []
        for _ in range(20):
            r0 = rng.randrange(BN254.r)
            d = protocol.LagrangeBasis.from_vec([(r0 + i) % BN254.r for i in range(32)])
            z = rng.randrange(32)
            qs.append((d, vc.commit(d), z, d[z]))
        proof = protocol.prove_multiproof(vc, qs)
        ent = {"queries": [{"data": [hexs(x) for x in q[0].evals], "commit": pt(q[1]), "z": q[2], "y": hexs(q[3])}
                           for q in qs], "d": pt(proof["d"])}
        if name == "ipa":
            ent["proof"] = ser(proof["proof"])
        else:
            ent["proof"] = {"proof": pt(proof["proof"]["proof"]), "y": hexs(proof["proof"]["y"])}
        mp[name] = ent
    dump("multiproof_32.json", mp)
    multiproof_256(crs)
    print("golden fixtures written to", HERE)


def multiproof_256(crs=None):
    """multiproof at the reference's width N = 256 (benches/ipa.rs:18, data r_j + i as :38-49),
    Q = 64 queries: 20 on z = 5 and 20 on z = 200 (more than one 16-query chunk of the engine's
    per-point sums on a row), the rest random; IPA and KZG (multiproof.rs:99-176). Data are stored
    as r_j (f_j[i] = r_j + i). Query commitments by msm_fast (the same group elements as the naive
    commit, which prove_multiproof itself runs for D and E)."""
    if crs is None:
        crs = protocol.ipa_gen_points(257, max_=512)
    N, Q = 256, 64
    rng = random.Random(61)
    zs = [5] * 20 + [200] * 20 + [rng.randrange(N) for _ in range(Q - 40)]
    rng.shuffle(zs)
    r0s = [rng.randrange(BN254.r) for _ in range(Q)]
    out = {"N": N, "Q": Q, "data_rule": "f_j[i] = r0_j + i mod r", "r0": [hexs(x) for x in r0s], "z": zs}
    for name, vc in (("ipa", protocol.IPA(N, points=crs)), ("kzg", protocol.KZG(N))):
        bases = vc.g if name == "ipa" else vc.lagrange
        qs = []
        for r0, z in zip(r0s, zs):
            d = protocol.LagrangeBasis.from_vec([(r0 + i) % BN254.r for i in range(N)])
            qs.append((d, BN254.msm_fast(bases, d.evals), z, d[z]))
        proof = protocol.prove_multiproof(vc, qs)
        ent = {"commits": [pt(q[1]) for q in qs], "d": pt(proof["d"])}
        if name == "ipa":
            p = proof["proof"]
            ent["proof"] = {"l": [pt(x) for x in p["l"]], "r": [pt(x) for x in p["r"]], "tip": hexs(p["tip"]),
                            "y": hexs(p["y"])}
        else:
            ent["proof"] = {"proof": pt(proof["proof"]["proof"]), "y": hexs(proof["proof"]["y"])}
        out[name] = ent
    dump("multiproof_256.json", out)


if __name__ == "__main__":
    if sys.argv[1:] == ["multiproof_256"]:
        multiproof_256()
    else:
        main()
