"""Reference-shaped VectorCommitment API over the HIP engine (include/vc_scheme.h).

Mirrors /root/reference/vector-commit/src: `IPA` (ipa/mod.rs), `KZG` (kzg/mod.rs),
`LagrangeBasis` (lagrange_basis.rs), `TranscriptHasher` (transcript.rs),
`prove_multiproof` / `verify_multiproof` (multiproof.rs), `to_data_item` (lib.rs:56-67).
Same names, argument meaning and error behaviour (errors raise `VCError` where the Rust
returns Err or panics). Curve: BN254 G1 (the reference's only instantiation).
Points are canonical affine (x, y) tuples, the identity is None; field elements are ints.
All arithmetic runs in libvkzg.so; this module only marshals.
"""
import ctypes

import numpy as np

from ._lib import VCError, check, lib
from .engine import Engine, ints_to_limbs, limbs_to_int

R_BN254 = 21888242871839275222246405745257275088548364400416034343698204186575808495617
_P = ctypes.c_void_p


def _p(a):
    # data_as keeps a reference to the array in the pointer object: callers pass temporaries
    # (e.g. _p(_fr(point))), and a bare c_void_p(a.ctypes.data) let the array be freed before the
    # foreign call read it -- harmless single-threaded by luck, garbage once another thread
    # reused the memory (tests/test_gpu_threads.py found it)
    return a.ctypes.data_as(ctypes.c_void_p)


def _fr(x):
    return ints_to_limbs([int(x) % R_BN254], 4)[0].copy()


_M256 = (1 << 256) - 1


def _pt_arrays(pts):
    """[(x, y) | None] -> ((n, 8) u64 limbs, (n,) identity flags): one bytes buffer for all points
    (per-point numpy assignments cost ~10 us per call of the IPA prover's Python mirror)"""
    n = len(pts)
    buf = bytearray(64 * n)
    inf = np.zeros(n, dtype=np.uint8)
    for i, P in enumerate(pts):
        if P is None:
            inf[i] = 1
        else:
            buf[64 * i:64 * i + 32] = (int(P[0]) & _M256).to_bytes(32, "little")
            buf[64 * i + 32:64 * i + 64] = (int(P[1]) & _M256).to_bytes(32, "little")
    xy = np.frombuffer(buf, dtype="<u8").reshape(n, 8).astype(np.uint64)
    return xy, inf


def _pt(xy, inf):
    if inf:
        return None
    return (limbs_to_int(xy[:4]), limbs_to_int(xy[4:8]))


# ---------------------------------------------------------------- transcript.rs
class TranscriptHasher:
    def __init__(self, label, _h=None):
        self.h = _h if _h is not None else lib().vc_transcript_new(label.encode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().vc_transcript_free(self.h)
            self.h = None

    def clone(self):
        return TranscriptHasher(None, lib().vc_transcript_clone(self.h))

    def append_point(self, P, label):
        xy, inf = _pt_arrays([P])
        check(lib().vc_transcript_append_point(self.h, _p(xy), int(inf[0]), label.encode()), "append_point")

    def append_fr(self, x, label):
        check(lib().vc_transcript_append_fr(self.h, _p(_fr(x)), label.encode()), "append_fr")

    def append_usize(self, z, label):
        check(lib().vc_transcript_append_u64(self.h, int(z), label.encode()), "append_usize")

    def digest(self, label, clear=True):
        out = np.zeros(4, dtype=np.uint64)
        check(lib().vc_transcript_digest(self.h, label.encode(), _p(out)), "digest")
        return limbs_to_int(out)


def hash_to_field(msg, dst):
    m = np.frombuffer(bytes(msg) or b"\0", dtype=np.uint8).copy()
    d = np.frombuffer(bytes(dst) or b"\0", dtype=np.uint8).copy()
    out = np.zeros(4, dtype=np.uint64)
    check(lib().vc_hash_to_field(_p(m), len(msg), _p(d), len(dst), _p(out)), "hash_to_field")
    return limbs_to_int(out)


def point_compress(P):
    xy, inf = _pt_arrays([P])
    out = np.zeros(32, dtype=np.uint8)
    check(lib().vc_point_compress(_p(xy), int(inf[0]), _p(out)), "point_compress")
    return out.tobytes()


def to_data_item(engine, pts):
    """VCCommitment::to_data_item for a batch of points (device)."""
    xy, inf = _pt_arrays(pts)
    out = np.zeros((len(pts), 4), dtype=np.uint64)
    check(lib().vc_to_data_item_batch(engine.h, _p(xy), _p(inf), len(pts), _p(out)), "to_data_item")
    return [limbs_to_int(r) for r in out]


def ipa_crs(num, seed=b"eth_verkle_oct_2021", max_=256):
    """IPAPointGenerator::gen (ipa_point_generator.rs:51-67); VCError(VC_E_RANGE) = OutOfBounds."""
    s = np.frombuffer(seed, dtype=np.uint8).copy()
    out = np.zeros((max(num, 1), 8), dtype=np.uint64)
    check(lib().vc_ipa_crs(_p(s), len(seed), max_, num, _p(out)), "ipa_crs")
    return [_pt(out[i], 0) for i in range(num)]


# ---------------------------------------------------------------- lagrange_basis.rs
class LagrangeBasis:
    """Evaluations over a radix-2 domain (possibly shorter than it: `max`)."""

    def __init__(self, evals, domain_size=None):
        # a tuple: the limbs below are cached per padded length, so the values must not change
        self.evals = tuple(int(e) % R_BN254 for e in evals)
        self._limbs = {}
        ds = 1
        while ds < len(self.evals):
            ds <<= 1
        self.dsize = domain_size if domain_size is not None else ds

    @classmethod
    def from_vec(cls, data):
        return cls(data)

    def __getitem__(self, i):
        return self.evals[i]

    def max(self):
        return len(self.evals) - 1

    def limbs(self, n=None):
        """(max(len, n), 4) canonical u64 limbs, converted once per n (read-only array)."""
        arr = self._limbs.get(n)
        if arr is None:
            arr = ints_to_limbs(self.evals, 4)
            if n is not None and arr.shape[0] < n:
                arr = np.vstack([arr, np.zeros((n - arr.shape[0], 4), dtype=np.uint64)])
            arr = np.ascontiguousarray(arr)
            arr.flags.writeable = False
            self._limbs[n] = arr
        return arr


# ---------------------------------------------------------------- proofs
class _ProofBuf(ctypes.Structure):
    _fields_ = [("rounds", ctypes.c_size_t), ("l_xy", _P), ("l_inf", _P), ("r_xy", _P), ("r_inf", _P),
                ("tip", ctypes.c_uint64 * 4), ("y", ctypes.c_uint64 * 4)]


class IPAProof:
    def __init__(self, l, r, tip, y):
        self.l, self.r, self.tip, self.y = l, r, tip, y

    def as_dict(self):
        return {"l": self.l, "r": self.r, "tip": self.tip, "y": self.y}

    @staticmethod
    def _alloc(rounds):
        # one buffer, four views (the caller keeps `arrs`, hence the buffer, alive while the struct's
        # raw pointers are in use): four allocations and four data_as pointers cost ~19 us a call
        k = rounds
        raw = np.zeros(128 * k + 2 * k, dtype=np.uint8)
        base = raw.ctypes.data
        arrs = {"lxy": raw[:64 * k].view(np.uint64).reshape(k, 8), "rxy": raw[64 * k:128 * k].view(np.uint64).reshape(k, 8),
                "linf": raw[128 * k:128 * k + k], "rinf": raw[128 * k + k:], "_raw": raw}
        b = _ProofBuf(k, base, base + 128 * k, base + 64 * k, base + 128 * k + k)
        return b, arrs

    @staticmethod
    def _from(b, arrs):
        k = b.rounds
        fb = int.from_bytes

        def pts(xy, inf):  # whole arrays to bytes once, then one int.from_bytes per coordinate
            raw, flags = np.ascontiguousarray(xy[:k], dtype="<u8").tobytes(), inf[:k].tolist()
            return [None if flags[i] else (fb(raw[64 * i:64 * i + 32], "little"), fb(raw[64 * i + 32:64 * i + 64], "little"))
                    for i in range(k)]
        return IPAProof(pts(arrs["lxy"], arrs["linf"]), pts(arrs["rxy"], arrs["rinf"]),
                        fb(bytes(b.tip), "little"), fb(bytes(b.y), "little"))

    def _to(self):
        k = len(self.l)
        b, arrs = IPAProof._alloc(k)
        xy, inf = _pt_arrays(self.l)
        arrs["lxy"][:] = xy
        arrs["linf"][:] = inf
        xy, inf = _pt_arrays(self.r)
        arrs["rxy"][:] = xy
        arrs["rinf"][:] = inf
        b.tip[:] = [int(v) for v in _fr(self.tip)]
        b.y[:] = [int(v) for v in _fr(self.y)]
        return b, arrs


def _log2(n):
    k = 0
    while (1 << k) < n:
        k += 1
    return k


# ---------------------------------------------------------------- ipa/mod.rs
class IPA:
    """IPA<N, G1(BN254), DefaultFieldHasher<Sha256>, GeneralEvaluationDomain>."""

    def __init__(self, engine, N, points):
        if engine.curve != "bn254":
            raise ValueError("the protocol layer is instantiated for BN254")
        assert len(points) == N + 1
        self.engine, self.N = engine, N
        self.g, self.q = points[:N], points[N]
        self.table = engine.upload_points(points)          # IPAUniversalParams::new_from_vec

    @classmethod
    def setup(cls, engine, max_items, gen_max=256, seed=b"eth_verkle_oct_2021"):
        """IPA::setup (:121-128): N + 1 generator points (fails OutOfBounds, Appendix B.1)."""
        return cls(engine, max_items, ipa_crs(max_items + 1, seed, gen_max))

    def max_size(self):
        return self.N

    def commit(self, data):
        return self.commit_batch([data])[0]

    def commit_batch(self, datas):
        sc = np.concatenate([d.limbs(self.N)[: self.N] for d in datas])
        xy, inf = self.engine.msm_batch(self.table, sc, self.N)
        return [_pt(xy[i], inf[i]) for i in range(len(datas))]

    def prove_point(self, commitment, point, data, transcript=None):
        return self.prove_batch_points([commitment], [point], [data], [transcript])[0]

    def prove_batch_points(self, commitments, points, datas, transcripts=None):
        B = len(datas)
        d = datas[0].limbs(self.N)[: self.N] if B == 1 else np.concatenate([x.limbs(self.N)[: self.N] for x in datas])
        cxy, cinf = _pt_arrays(commitments)
        pts = ints_to_limbs([int(p) % R_BN254 for p in points], 4)
        K = _log2(self.N)
        bufs = [IPAProof._alloc(K) for _ in range(B)]
        arr = (_ProofBuf * B)(*[b for b, _ in bufs])
        trs = None
        if transcripts is not None and any(t is not None for t in transcripts):
            trs = (_P * B)(*[(t.h if t is not None else None) for t in transcripts])
        check(lib().vc_ipa_prove(self.engine.h, self.table, self.N, _p(d), _p(cxy), _p(cinf), _p(pts), B,
                                 ctypes.cast(trs, _P) if trs is not None else None, ctypes.cast(arr, _P)),
              "ipa_prove")
        return [IPAProof._from(arr[i], bufs[i][1]) for i in range(B)]

    def prove(self, commitment, index, data):
        return self.prove_point(commitment, index, data)

    def verify_point(self, commitment, point, proof, transcript=None):
        cxy, cinf = _pt_arrays([commitment])
        b, arrs = proof._to()
        res = ctypes.c_int()
        check(lib().vc_ipa_verify(self.engine.h, self.table, self.N, _p(cxy), int(cinf[0]), _p(_fr(point)),
                                  ctypes.byref(b), transcript.h if transcript is not None else None,
                                  ctypes.byref(res)), "ipa_verify")
        return bool(res.value)

    def verify(self, commitment, index, proof):
        return self.verify_point(commitment, index, proof)

    def prove_commitment(self, commitment, data):
        """:199-234 -> IPAProof with l, r, tip (y = 0)."""
        return self.prove_commitment_batch([commitment], [data])[0]

    def prove_commitment_batch(self, commitments, datas):
        n = datas[0].max() + 1
        if any(d.max() + 1 != n for d in datas):
            raise ValueError("one batch proves data of one length")
        B = len(datas)
        d = np.concatenate([x.limbs(n)[:n] for x in datas])
        cxy, cinf = _pt_arrays(commitments)
        K = _log2(n)
        bufs = [IPAProof._alloc(K) for _ in range(B)]
        arr = (_ProofBuf * B)(*[b for b, _ in bufs])
        check(lib().vc_ipa_prove_commitment(self.engine.h, self.table, n, _p(d), _p(cxy), _p(cinf), B,
                                            ctypes.cast(arr, _P)), "ipa_prove_commitment")
        return [IPAProof._from(arr[i], bufs[i][1]) for i in range(B)]

    def verify_commitment_proof(self, commitment, proof):
        """:237-265."""
        cxy, cinf = _pt_arrays([commitment])
        b, arrs = proof._to()
        res = ctypes.c_int()
        check(lib().vc_ipa_verify_commitment_proof(self.engine.h, self.table, _p(cxy), int(cinf[0]), ctypes.byref(b),
                                                   ctypes.byref(res)), "ipa_verify_commitment_proof")
        return bool(res.value)


# ---------------------------------------------------------------- kzg/mod.rs
class KZG:
    """KZG<Bn254, ...> prover side (pairing verification is out of scope: see DESIGN.md)."""

    def __init__(self, engine, max_items, secret=100):
        self.engine = engine
        tid = ctypes.c_int()
        size = ctypes.c_size_t()
        check(lib().vc_kzg_setup(engine.h, max_items, _p(_fr(secret)), ctypes.byref(tid), ctypes.byref(size)),
              "kzg_setup")
        self.table, self.size, self.secret = tid.value, size.value, secret

    def max_size(self):
        return self.size

    def lagrange_points(self):
        xy, inf = self.engine.download_bases(self.table)
        return [_pt(xy[i], inf[i]) for i in range(self.size)]

    def commit(self, data):
        """:126-134 inner_product(lagrange_commitments, evals) (zip-truncating)."""
        sc = data.limbs()
        xy, inf = self.engine.msm(self.table, sc)
        return _pt(xy, inf)

    def prove_point(self, commitment, point, data, transcript=None):
        ev = data.limbs()
        pxy = np.zeros(8, dtype=np.uint64)
        pinf = np.zeros(1, dtype=np.uint8)
        y = np.zeros(4, dtype=np.uint64)
        check(lib().vc_kzg_prove(self.engine.h, self.table, self.size, _p(ev), len(data.evals), _p(_fr(point)),
                                 _p(pxy), _p(pinf), _p(y)), "kzg_prove")
        return {"proof": _pt(pxy, pinf[0]), "y": limbs_to_int(y)}

    def prove(self, commitment, index, data):
        return self.prove_point(commitment, index, data)

    def prove_all_points(self, data, mode=0):
        """KZG::prove_all_points (kzg/mod.rs:200-235) -- mode 0: the reference's computation
        exactly (its h_hat values, y = data[i]); mode 1: the FK opening proofs at every domain
        point (== prove at each index). Returns a list of {"proof", "y"}."""
        ev = data.limbs() if data.evals else np.zeros((0, 4), dtype=np.uint64)
        n_out = self.size if mode == 1 else max(1, len(data.evals))
        xy = np.zeros((n_out, 8), dtype=np.uint64)
        inf = np.zeros(n_out, dtype=np.uint8)
        ys = np.zeros((n_out, 4), dtype=np.uint64)
        cnt = ctypes.c_size_t()
        check(lib().vc_kzg_prove_all_points(self.engine.h, self.table, self.size, _p(ev), len(data.evals), mode,
                                            _p(xy), _p(inf), _p(ys), ctypes.byref(cnt)), "kzg_prove_all_points")
        return [{"proof": _pt(xy[i], inf[i]), "y": limbs_to_int(ys[i])} for i in range(cnt.value)]

    def quotient(self, point, data):
        ev = data.limbs()
        q = np.zeros((self.size, 4), dtype=np.uint64)
        y = np.zeros(4, dtype=np.uint64)
        check(lib().vc_kzg_quotient(self.engine.h, self.size, _p(ev), len(data.evals), _p(_fr(point)), _p(q),
                                    _p(y)), "kzg_quotient")
        return [limbs_to_int(r) for r in q], limbs_to_int(y)


# ---------------------------------------------------------------- multiproof.rs
def _queries(queries, N):
    Q = len(queries)
    data = np.concatenate([q[0].limbs(N)[:N] for q in queries])
    cxy, cinf = _pt_arrays([q[1] for q in queries])
    z = np.array([int(q[2]) for q in queries], dtype=np.uint64)
    y = ints_to_limbs([int(q[3]) % R_BN254 for q in queries], 4)
    return Q, data, cxy, cinf, z, y


def prove_multiproof(vc, queries):
    """queries: list of (LagrangeBasis data, commitment, z, y). Returns {"proof", "d"}."""
    N = vc.N if isinstance(vc, IPA) else vc.size
    Q, data, cxy, cinf, z, y = _queries(queries, N)
    dxy = np.zeros(8, dtype=np.uint64)
    dinf = np.zeros(1, dtype=np.uint8)
    if isinstance(vc, IPA):
        b, arrs = IPAProof._alloc(_log2(N))
        check(lib().vc_multiproof_prove(vc.engine.h, 0, vc.table, N, Q, _p(data), _p(cxy), _p(cinf), _p(z), _p(y),
                                        _p(dxy), _p(dinf), ctypes.byref(b), None, None, None), "multiproof_prove")
        return {"proof": IPAProof._from(b, arrs), "d": _pt(dxy, dinf[0])}
    kxy = np.zeros(8, dtype=np.uint64)
    kinf = np.zeros(1, dtype=np.uint8)
    ky = np.zeros(4, dtype=np.uint64)
    check(lib().vc_multiproof_prove(vc.engine.h, 1, vc.table, N, Q, _p(data), _p(cxy), _p(cinf), _p(z), _p(y),
                                    _p(dxy), _p(dinf), None, _p(kxy), _p(kinf), _p(ky)), "multiproof_prove")
    return {"proof": {"proof": _pt(kxy, kinf[0]), "y": limbs_to_int(ky)}, "d": _pt(dxy, dinf[0])}


def verify_multiproof(vc, vqueries, mp):
    """IPA: full verification. KZG: returns the (E - D, t) claim for an external pairing check."""
    N = vc.N if isinstance(vc, IPA) else vc.size
    Q = len(vqueries)
    cxy, cinf = _pt_arrays([q[0] for q in vqueries])
    z = np.array([int(q[1]) for q in vqueries], dtype=np.uint64)
    y = ints_to_limbs([int(q[2]) % R_BN254 for q in vqueries], 4)
    dxy, dinf = _pt_arrays([mp["d"]])
    if isinstance(vc, IPA):
        b, arrs = mp["proof"]._to()
        res = ctypes.c_int()
        check(lib().vc_multiproof_verify_ipa(vc.engine.h, vc.table, N, Q, _p(cxy), _p(cinf), _p(z), _p(y), _p(dxy),
                                             int(dinf[0]), ctypes.byref(b), ctypes.byref(res)), "multiproof_verify")
        return bool(res.value)
    oxy = np.zeros(8, dtype=np.uint64)
    oinf = np.zeros(1, dtype=np.uint8)
    t = np.zeros(4, dtype=np.uint64)
    check(lib().vc_multiproof_kzg_claim(vc.engine.h, N, Q, _p(cxy), _p(cinf), _p(z), _p(y), _p(dxy), int(dinf[0]),
                                        _p(oxy), _p(oinf), _p(t)), "multiproof_kzg_claim")
    return {"commitment": _pt(oxy, oinf[0]), "t": limbs_to_int(t)}


class MultiproofSet:
    """Output buffers of P multiproofs (vc_multiproof_prove_many / _sharded / _gather): D points,
    and P IPA proofs (scheme 0) or P KZG (proof, y) pairs (scheme 1)."""

    def __init__(self, scheme_id, N, P):
        self.scheme, self.N, self.P = scheme_id, N, P
        self.d_xy = np.zeros((max(P, 1), 8), dtype=np.uint64)
        self.d_inf = np.zeros(max(P, 1), dtype=np.uint8)
        self.bufs, self.arrs = None, []
        self.kxy = self.kinf = self.ky = None
        if scheme_id == 0:
            self.bufs = (_ProofBuf * max(P, 1))()
            for p in range(P):
                b, arrs = IPAProof._alloc(_log2(N))
                self.bufs[p] = b
                self.arrs.append(arrs)
        else:
            self.kxy = np.zeros((max(P, 1), 8), dtype=np.uint64)
            self.kinf = np.zeros(max(P, 1), dtype=np.uint8)
            self.ky = np.zeros((max(P, 1), 4), dtype=np.uint64)

    def args(self):
        """(d_xy, d_inf, ipa_proofs, kzg_xy, kzg_inf, kzg_y) pointers of the C ABI"""
        if self.scheme == 0:
            return _p(self.d_xy), _p(self.d_inf), ctypes.cast(self.bufs, ctypes.c_void_p), None, None, None
        return _p(self.d_xy), _p(self.d_inf), None, _p(self.kxy), _p(self.kinf), _p(self.ky)

    def proofs(self):
        out = []
        for p in range(self.P):
            if self.scheme == 0:
                pr = IPAProof._from(self.bufs[p], self.arrs[p])
            else:
                pr = {"proof": _pt(self.kxy[p], self.kinf[p]), "y": limbs_to_int(self.ky[p])}
            out.append({"proof": pr, "d": _pt(self.d_xy[p], self.d_inf[p])})
        return out


def prove_multiproof_many(vc, cxy, cinf, z, y, d_data_ptr):
    """P independent multiproofs at once on one GPU (vc_multiproof_prove_many): cxy [P][Q][8],
    cinf [P][Q], z [P][Q], y [P][Q][4] host arrays; d_data_ptr -> [P][Q][N] canonical evaluations
    on the device. Returns P {"proof", "d"} as prove_multiproof does."""
    ipa = isinstance(vc, IPA)
    N = vc.N if ipa else vc.size
    P, Q = z.shape
    out = MultiproofSet(0 if ipa else 1, N, P)
    cxy, cinf, z, y = (np.ascontiguousarray(a) for a in (cxy, cinf, z, y))
    check(lib().vc_multiproof_prove_many(vc.engine.h, out.scheme, vc.table, N, Q, P, ctypes.c_void_p(d_data_ptr),
                                         _p(cxy), _p(cinf), _p(z), _p(y), *out.args()), "multiproof_prove_many")
    return out.proofs()


# ---------------------------------------------------------------- sharded multiproof
def multiproof_begin(N, cxy, cinf, z, y):
    """Phase 1 (host, every rank): transcript over all queries -> (transcript handle, r limbs, rows)."""
    Q = len(z)
    tr = ctypes.c_void_p()
    r = np.zeros(4, dtype=np.uint64)
    rows = ctypes.c_size_t()
    check(lib().vc_multiproof_begin(N, Q, _p(cxy), _p(cinf), _p(z), _p(y), ctypes.byref(tr), _p(r),
                                    ctypes.byref(rows)), "multiproof_begin")
    return tr, r, rows.value


def multiproof_accumulate(engine, N, z, first, count, d_data_ptr, r, d_S_ptr):
    """Phase 2 (device): this shard's rows x N per-point sums into d_S (canonical u64 x 4)."""
    check(lib().vc_multiproof_accumulate(engine.h, N, len(z), _p(z), first, count, ctypes.c_void_p(d_data_ptr),
                                         _p(r), ctypes.c_void_p(d_S_ptr)), "multiproof_accumulate")


def multiproof_rows(N, z):
    """The number of distinct query points (rows of the per-point sums S)."""
    rows = ctypes.c_size_t()
    check(lib().vc_multiproof_rows(N, len(z), _p(z), ctypes.byref(rows)), "multiproof_rows")
    return rows.value


def multiproof_begin_accumulate(engine, N, cxy, cinf, z, y, first, count, d_data_ptr, d_S_ptr):
    """Phases 1 + 2 in one call (the transcript overlapped with the shard's planning and uploads)
    -> (transcript handle, r limbs); S of the shard into d_S (multiproof_rows(N, z) x N x 4 u64)."""
    tr = ctypes.c_void_p()
    r = np.zeros(4, dtype=np.uint64)
    check(lib().vc_multiproof_begin_accumulate(engine.h, N, len(z), _p(cxy), _p(cinf), _p(z), _p(y), first, count,
                                               ctypes.c_void_p(d_data_ptr), ctypes.c_void_p(d_S_ptr),
                                               ctypes.byref(tr), _p(r)), "multiproof_begin_accumulate")
    return tr, r


def multiproof_finish(vc, z, d_S_parts_ptr, G, tr):
    """Phase 3: sum the G shards' S, then D, t, E and the inner proof -- an IPA proof or the KZG
    (proof, y) of prove_point at t (multiproof.rs:129-175). Frees `tr`."""
    if isinstance(vc, IPA):
        return multiproof_finish_ipa(vc, z, d_S_parts_ptr, G, tr)
    N = vc.size
    dxy = np.zeros(8, dtype=np.uint64)
    dinf = np.zeros(1, dtype=np.uint8)
    kxy = np.zeros(8, dtype=np.uint64)
    kinf = np.zeros(1, dtype=np.uint8)
    ky = np.zeros(4, dtype=np.uint64)
    try:
        check(lib().vc_multiproof_finish(vc.engine.h, 1, vc.table, N, len(z), _p(z), ctypes.c_void_p(d_S_parts_ptr),
                                         G, tr, _p(dxy), _p(dinf), None, _p(kxy), _p(kinf), _p(ky)),
              "multiproof_finish")
    finally:
        lib().vc_transcript_free(tr)
    return {"proof": {"proof": _pt(kxy, kinf[0]), "y": limbs_to_int(ky)}, "d": _pt(dxy, dinf[0])}


def multiproof_finish_ipa(ipa, z, d_S_parts_ptr, G, tr):
    """Phase 3: sum the G shards' S, then D, t, E and the inner IPA proof. Frees `tr`."""
    N = ipa.N
    dxy = np.zeros(8, dtype=np.uint64)
    dinf = np.zeros(1, dtype=np.uint8)
    b, arrs = IPAProof._alloc(_log2(N))
    try:
        check(lib().vc_multiproof_finish(ipa.engine.h, 0, ipa.table, N, len(z), _p(z), ctypes.c_void_p(d_S_parts_ptr),
                                         G, tr, _p(dxy), _p(dinf), ctypes.byref(b), None, None, None),
              "multiproof_finish")
    finally:
        lib().vc_transcript_free(tr)
    return {"proof": IPAProof._from(b, arrs), "d": _pt(dxy, dinf[0])}
