"""VerkleTree over the engine (include/vc_verkle.h), mirroring /root/reference/verkle-tree/src
(lib.rs VerkleTree<N, u8, VC, U256>; node.rs Node). Keys: N bytes; values: 32 bytes.
The tree lives in libvkzg.so (C++); commitments are level-batched on the GPU against any
BN254 table (KZG Lagrange SRS from KZG(...).table, or an IPA CRS from IPA(...).table)."""
import ctypes

import numpy as np

from ._lib import VCError, check, lib
from .engine import limbs_to_int


def _b(x):
    a = np.frombuffer(bytes(x), dtype=np.uint8).copy()
    return a, a.ctypes.data_as(ctypes.c_void_p)


class VerkleTree:
    def __init__(self, key_len):
        self.N = key_len
        self.h = lib().vc_verkle_new(key_len)
        if not self.h:
            raise VCError(-1, "vc_verkle_new")

    def __del__(self):
        if getattr(self, "h", None):
            try:
                lib().vc_verkle_free(self.h)
            except TypeError:  # interpreter shutdown: module globals already cleared
                pass
            self.h = None

    def insert_single(self, key, value):
        """lib.rs:112-116; VCError(VC_E_INVALID) where the reference panics."""
        assert len(key) == self.N and len(value) == 32
        k, kp = _b(key)
        v, vp = _b(value)
        check(lib().vc_verkle_insert(self.h, kp, vp), "vc_verkle_insert")

    def get_single(self, key):
        k, kp = _b(key)
        out = np.zeros(32, dtype=np.uint8)
        found = ctypes.c_int()
        check(lib().vc_verkle_get(self.h, kp, ctypes.c_void_p(out.ctypes.data), ctypes.byref(found)), "vc_verkle_get")
        return out.tobytes() if found.value else None

    def path_to_stem(self, key):
        """[(prefix, unit)] as node.rs:97-120; VCError for InvalidPath."""
        k, kp = _b(key)
        units = np.zeros(self.N, dtype=np.uint8)
        n = ctypes.c_size_t()
        check(lib().vc_verkle_path(self.h, kp, self.N, ctypes.c_void_p(units.ctypes.data), ctypes.byref(n)),
              "vc_verkle_path")
        return [(tuple(key[:d + 1]), key[d]) for d in range(n.value)]

    def debug_ext_stage(self, reps=5):
        """median us of the device path's extension host stage over every extension (no GPU)"""
        us = ctypes.c_double()
        check(lib().vc_verkle_debug_ext_stage(self.h, reps, ctypes.byref(us)), "vc_verkle_debug_ext_stage")
        return us.value

    def debug_nodes(self):
        """per node id: (type 0 internal / 1 extension, level, committed item as int)"""
        n = ctypes.c_size_t()
        check(lib().vc_verkle_debug_nodes(self.h, 0, None, None, None, ctypes.byref(n)), "vc_verkle_debug_nodes")
        m = n.value
        ty = np.zeros(m, dtype=np.uint8)
        lv = np.zeros(m, dtype=np.int32)
        it = np.zeros((m, 4), dtype=np.uint64)
        check(lib().vc_verkle_debug_nodes(self.h, m, ctypes.c_void_p(ty.ctypes.data), ctypes.c_void_p(lv.ctypes.data),
                                          ctypes.c_void_p(it.ctypes.data), ctypes.byref(n)), "vc_verkle_debug_nodes")
        return [(int(ty[i]), int(lv[i]), limbs_to_int(it[i])) for i in range(m)]

    def stats(self):
        a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        check(lib().vc_verkle_stats(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "vc_verkle_stats")
        return {"internal": a.value, "extension": b.value, "dirty": c.value}

    def commitment(self, engine, table):
        """lib.rs:127-129: root commitment (canonical affine (x, y) or None)."""
        xy = np.zeros(8, dtype=np.uint64)
        inf = np.zeros(1, dtype=np.uint8)
        check(lib().vc_verkle_commitment(engine.h, table, self.h, ctypes.c_void_p(xy.ctypes.data),
                                         ctypes.c_void_p(inf.ctypes.data)), "vc_verkle_commitment")
        return None if inf[0] else (limbs_to_int(xy[:4]), limbs_to_int(xy[4:]))
