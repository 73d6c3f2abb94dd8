"""One process, several GPUs (include/vc_group.h): a thin ctypes handle on vc_group -- one vc_ctx
and one host worker per member; every call splits its work over the members and returns the
whole result, so a single-process caller (the reference's stateless VectorCommitment trait,
vector-commit/src/lib.rs:70-174) uses a whole node with no SPMD code."""
import ctypes

import numpy as np

from ._lib import check, lib
from .engine import CURVE_IDS, NL, ints_to_limbs, limbs_to_int

SPLIT_AUTO, SPLIT_WINDOWS, SPLIT_POINTS = 0, 1, 2


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Group:
    def __init__(self, curve, devices):
        self.curve, self.cid, self.nl = curve, CURVE_IDS[curve], NL[curve]
        devs = np.asarray(devices, dtype=np.int32)
        h = ctypes.c_void_p()
        check(lib().vc_group_create(self.cid, len(devs), _p(devs), ctypes.byref(h)), "vc_group_create")
        self.h = h

    def close(self):
        if self.h:
            lib().vc_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def size(self):
        return lib().vc_group_size(self.h)

    def peer_path(self, a, b):
        """how copies from member a to member b travel: 0 one device, 1 peer access (xGMI), 2 staged"""
        r = lib().vc_group_peer_path(self.h, a, b)
        check(min(r, 0), "vc_group_peer_path")
        return r

    def member(self, k):
        """member k's vc_ctx handle (ctypes.c_void_p)"""
        return ctypes.c_void_p(lib().vc_group_member(self.h, k))

    def member_table(self, table, k):
        out = ctypes.c_int()
        check(lib().vc_group_member_table(self.h, table, k, ctypes.byref(out)), "vc_group_member_table")
        return out.value

    def set_msm_split(self, split):
        check(lib().vc_group_set_msm_split(self.h, split), "vc_group_set_msm_split")

    # -------------------------------------------------------------- tables
    def upload_points(self, pts):
        xy = np.zeros((len(pts), 2 * self.nl), dtype=np.uint64)
        inf = np.zeros(len(pts), dtype=np.uint8)
        for i, P in enumerate(pts):
            if P is None:
                inf[i] = 1
            else:
                xy[i, :self.nl] = ints_to_limbs([P[0]], self.nl)[0]
                xy[i, self.nl:] = ints_to_limbs([P[1]], self.nl)[0]
        return self.upload(xy, inf)

    def upload(self, xy, inf=None):
        xy = np.ascontiguousarray(xy, dtype=np.uint64)
        inf = None if inf is None else np.ascontiguousarray(inf, dtype=np.uint8)
        tid = ctypes.c_int()
        check(lib().vc_group_bases_upload(self.h, _p(xy), _p(inf), xy.shape[0], ctypes.byref(tid)),
              "vc_group_bases_upload")
        return tid.value

    def random_bases(self, n, seed):
        tid = ctypes.c_int()
        check(lib().vc_group_bases_random(self.h, seed, n, ctypes.byref(tid)), "vc_group_bases_random")
        return tid.value

    def kzg_setup(self, max_items, secret=100):
        tid, size = ctypes.c_int(), ctypes.c_size_t()
        s = ints_to_limbs([secret])[0].copy()
        check(lib().vc_group_kzg_setup(self.h, max_items, _p(s), ctypes.byref(tid), ctypes.byref(size)),
              "vc_group_kzg_setup")
        return tid.value, size.value

    def fixed_base_precompute(self, table, window_bits, windows=0):
        check(lib().vc_group_fixed_base_precompute(self.h, table, window_bits, windows),
              "vc_group_fixed_base_precompute")

    # -------------------------------------------------------------- MSMs
    def msm(self, table, scalars, offset=0, mont=False):
        sc = np.ascontiguousarray(scalars, dtype=np.uint64)
        xy = np.zeros(2 * self.nl, dtype=np.uint64)
        inf = np.zeros(1, dtype=np.uint8)
        check(lib().vc_group_msm(self.h, table, offset, _p(sc), sc.shape[0], int(mont), _p(xy), _p(inf)),
              "vc_group_msm")
        return xy, int(inf[0])

    def msm_batch(self, table, scalars, width, mont=False):
        sc = np.ascontiguousarray(scalars, dtype=np.uint64)
        batch = sc.shape[0] // width
        xy = np.zeros((batch, 2 * self.nl), dtype=np.uint64)
        inf = np.zeros(batch, dtype=np.uint8)
        check(lib().vc_group_msm_batch(self.h, table, width, _p(sc), batch, int(mont), _p(xy), _p(inf)),
              "vc_group_msm_batch")
        return xy, inf

    def kzg_prove(self, table, size, evals, point):
        ev = np.ascontiguousarray(evals, dtype=np.uint64)
        pt = ints_to_limbs([point])[0].copy()
        xy = np.zeros(2 * self.nl, dtype=np.uint64)
        inf = np.zeros(1, dtype=np.uint8)
        y = np.zeros(4, dtype=np.uint64)
        check(lib().vc_group_kzg_prove(self.h, table, size, _p(ev), ev.shape[0], _p(pt), _p(xy), _p(inf), _p(y)),
              "vc_group_kzg_prove")
        return xy, int(inf[0]), limbs_to_int(y)

    # -------------------------------------------------------------- multiproofs
    def multiproof_prove(self, scheme_id, table, N, data, cxy, cinf, z, y):
        """one multiproof (vc_group_multiproof_prove); returns {"proof", "d"} like
        scheme.prove_multiproof."""
        from . import scheme
        Q = z.shape[0]
        data, cxy, cinf, z, y = (np.ascontiguousarray(a) for a in (data, cxy, cinf, z, y))
        out = scheme.MultiproofSet(scheme_id, N, 1)
        check(lib().vc_group_multiproof_prove(self.h, scheme_id, table, N, Q, _p(data), _p(cxy), _p(cinf), _p(z),
                                              _p(y), *out.args()), "vc_group_multiproof_prove")
        return out.proofs()[0]

    def multiproof_prove_many(self, scheme_id, table, N, data, cxy, cinf, z, y):
        """P multiproofs, member k proving its share (vc_group_multiproof_prove_many): data
        [P][Q][N] x 4, cxy [P][Q][8], cinf [P][Q], z [P][Q], y [P][Q][4] host arrays."""
        from . import scheme
        P, Q = z.shape
        data, cxy, cinf, z, y = (np.ascontiguousarray(a) for a in (data, cxy, cinf, z, y))
        out = scheme.MultiproofSet(scheme_id, N, P)
        check(lib().vc_group_multiproof_prove_many(self.h, scheme_id, table, N, Q, P, _p(data), _p(cxy), _p(cinf),
                                                   _p(z), _p(y), *out.args()), "vc_group_multiproof_prove_many")
        return out.proofs()

    def verkle_commitment(self, tree, table):
        from .scheme import _pt
        xy = np.zeros(8, dtype=np.uint64)
        inf = np.zeros(1, dtype=np.uint8)
        check(lib().vc_group_verkle_commitment(self.h, table, tree.h, _p(xy), _p(inf)), "vc_group_verkle_commitment")
        return _pt(xy, inf[0])
