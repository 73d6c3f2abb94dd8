"""ORACLE (test infrastructure only) -- prove_multiproof (multiproof.rs:99-176) at the reference's
bench shape: N = 256 and up to 2^16 queries (benches/ipa.rs:18-19, 111-131). Same algorithm as
protocol.prove_multiproof, assembled from the oracle's pieces so Q = 2^16 finishes in seconds:

  transcript over (C, z, y) -> r        arkser.TranscriptHasher            transcript.rs:28-62, :105-115
  g = sum_z divide_by_vanishing(...)    cref.mp_g (oracle/c/ref_multiproof.c)        :117-150
  D = commit(g)                         cref.msm_arrays, naive inner_product         utils.rs:16-19
  append D -> t                                                                      :152-153
  h = sum_i inv[z_i] r^i f_i            cref.mp_h                                    :155-165
  E = commit(h), append E                                                            :167-170
  proof = prove_point(E - D, t, h - g)  protocol.low_level_ipa / KZG.prove_point     :172-175
                                        (ipa/mod.rs:137-154, 268-319; kzg/mod.rs:136-154)

Every intermediate (r, g, D, t, h, E) is returned so a test can say which one differs.
"""
import numpy as np

from . import arkser, cref, protocol
from .curves import BN254


def _ints(rows):
    return [cref.limbs_to_int(r) for r in rows]


def commitments_from_arrays(cxy, cinf):
    """(Q, 8) canonical u64 affine + (Q,) identity flags -> affine tuples (None = identity)."""
    out = []
    for k in range(cxy.shape[0]):
        out.append(None if cinf[k] else (cref.limbs_to_int(cxy[k, :4]), cref.limbs_to_int(cxy[k, 4:])))
    return out


def multiproof(vc, N, data, cxy, cinf, z, nthreads=1):
    """vc: protocol.IPA(N) or protocol.KZG(N) over BN254. data (Q*N, 4) or (Q, N, 4) canonical u64
    evaluations, cxy / cinf the query commitments, z (Q,) point indices (< N); y_i = f_i(z_i) is
    read from data, as the reference's bench does (benches/ipa.rs:38-49)."""
    C = BN254
    data = np.ascontiguousarray(data, dtype=np.uint64).reshape(-1, N, 4)
    Q = data.shape[0]
    z = np.ascontiguousarray(z, dtype=np.uint64)
    ys = data[np.arange(Q), z.astype(np.int64)]
    coms = commitments_from_arrays(cxy, cinf)
    tr = arkser.TranscriptHasher("multiproof", C)                     # multiproof.rs:108
    for k in range(Q):                                                # :109-113
        tr.append_point(coms[k], "C")
        tr.append_usize(int(z[k]), "z")
        tr.append_fr(cref.limbs_to_int(ys[k]), "y")
    r = tr.digest("r", True)                                          # :115
    omega = protocol.group_gen(N, C)
    st, g_l = cref.mp_g(N, data, z, r, omega, nthreads)
    try:
        ipa = isinstance(vc, protocol.IPA)
        bases = vc.g if ipa else vc.lagrange
        bxy, binf = cref.points_to_array("bn254", bases[:N])
        d = cref.array_to_point("bn254", *cref.msm_arrays("bn254", bxy, binf, g_l, nthreads))
        tr.append_point(d, "D")                                       # :152
        t = tr.digest("t", True)                                      # :153
        h_l = cref.mp_h(st, N, t)
    finally:
        cref.mp_free(st)
    e = cref.array_to_point("bn254", *cref.msm_arrays("bn254", bxy, binf, h_l, nthreads))
    tr.append_point(e, "E")                                           # :170
    g, h = _ints(g_l), _ints(h_l)
    hmg = protocol.LagrangeBasis([(a - b) % C.r for a, b in zip(h, g)], protocol.domain_size(N), C)
    mcom = C.add(e, C.neg(d))
    proof = vc.prove_point(mcom, t, hmg, tr)                          # :172-175
    return {"r": r, "t": t, "g": g, "h": h, "d": d, "e": e, "proof": proof}
