"""Multi-GPU through the C ABI (include/vc_comm.h): a vc_comm rank with an all-gather -- RCCL
over xGMI, or a host callback -- and the sharded workloads that run this rank's share on its
engine and exchange once per step. A Rust caller of libvkzg.so gets the same entry points
without Python; this module only marshals.

Transports:
  Comm.rccl(device, rank, world, uid): RCCL, uid from unique_id() on rank 0, handed to the other
      ranks by the caller (torch.distributed broadcast, a file, ...).
  Comm.host(rank, world, fn): fn(send: bytes) -> bytes of world * len(send) (rank order), e.g.
      torch_allgather() over a torch.distributed group (gloo on CPU tests), or an in-process
      exchange between threads (GPU tests: G ranks as G threads on one GPU).
"""
import ctypes

import numpy as np

from ._lib import ALLGATHER_FN, check, lib  # noqa: F401 (ALLGATHER_FN re-exported)

ID_BYTES = 128


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def unique_id():
    """RCCL unique id (bytes) for vc_comm_init_rccl, made on rank 0."""
    buf = (ctypes.c_uint8 * ID_BYTES)()
    check(lib().vc_comm_unique_id(buf), "vc_comm_unique_id")
    return bytes(buf)


def torch_allgather(group=None):
    """Host all-gather over torch.distributed (any backend that all-gathers CPU tensors: gloo)."""
    import torch
    import torch.distributed as dist

    def fn(send):
        t = torch.frombuffer(bytearray(send), dtype=torch.uint8) if send else torch.zeros(0, dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
        dist.all_gather(outs, t, group=group)
        return b"".join(o.numpy().tobytes() for o in outs)
    return fn


class Comm:
    def __init__(self, handle, keep=None):
        self.h = handle
        self._keep = keep  # the ctypes callback must outlive the comm

    @classmethod
    def rccl(cls, device, rank, world, uid):
        h = ctypes.c_void_p()
        idb = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(uid)
        check(lib().vc_comm_init_rccl(device, rank, world, idb, ctypes.byref(h)), "vc_comm_init_rccl")
        return cls(h)

    @classmethod
    def host(cls, rank, world, fn):
        def tramp(_user, send, nbytes, recv):
            try:
                data = ctypes.string_at(send, nbytes) if nbytes else b""
                out = fn(data)
                if len(out) != nbytes * world:
                    return 1
                if nbytes:
                    ctypes.memmove(recv, out, len(out))
                return 0
            except Exception:  # reported to the caller as VC_E_COMM
                return 1
        cb = ALLGATHER_FN(tramp)
        h = ctypes.c_void_p()
        check(lib().vc_comm_init_host(rank, world, cb, None, ctypes.byref(h)), "vc_comm_init_host")
        return cls(h, keep=cb)

    def close(self):
        if self.h:
            lib().vc_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def rank(self):
        return lib().vc_comm_rank(self.h)

    @property
    def world(self):
        return lib().vc_comm_world(self.h)

    @property
    def is_rccl(self):
        return bool(lib().vc_comm_is_rccl(self.h))

    def allgather(self, send, engine=None):
        """bytes -> bytes (world * len), through vc_comm_allgather (RCCL needs the engine)."""
        src = np.frombuffer(send, dtype=np.uint8).copy() if send else np.zeros(1, np.uint8)
        out = np.zeros(max(1, len(send) * self.world), dtype=np.uint8)
        check(lib().vc_comm_allgather(self.h, engine.h if engine else None, _p(src), len(send), _p(out)),
              "vc_comm_allgather")
        return out[:len(send) * self.world].tobytes()

    # ---------------------------------------------------------------- sharded workloads
    SPLIT_WINDOWS, SPLIT_POINTS = 1, 2

    def set_msm_split(self, split):
        """how vc_msm_sharded splits one MSM: SPLIT_WINDOWS (default) or SPLIT_POINTS (same on every rank)"""
        check(lib().vc_comm_set_msm_split(self.h, split), "vc_comm_set_msm_split")

    def msm(self, engine, table, d_scalars_ptr, n, offset=0, mont=False):
        """whole MSM of n device-resident scalars; rank k computes its window slice (or, after
        set_msm_split(SPLIT_POINTS), the MSM of its point range)."""
        from .engine import NL
        xy = np.zeros(2 * NL[engine.curve], dtype=np.uint64)
        inf = np.zeros(1, dtype=np.uint8)
        check(lib().vc_msm_sharded(engine.h, self.h, table, offset, ctypes.c_void_p(d_scalars_ptr), n, int(mont),
                                   _p(xy), _p(inf)), "vc_msm_sharded")
        return xy, int(inf[0])

    def msm_batch(self, engine, table, width, d_scalars_ptr, batch, mont=False):
        """all `batch` width-`width` commitments; rank k commits its contiguous batch slice."""
        from .engine import NL
        xy = np.zeros((batch, 2 * NL[engine.curve]), dtype=np.uint64)
        inf = np.zeros(batch, dtype=np.uint8)
        check(lib().vc_msm_batch_sharded(engine.h, self.h, table, width, ctypes.c_void_p(d_scalars_ptr), batch,
                                         int(mont), _p(xy), _p(inf)), "vc_msm_batch_sharded")
        return xy, inf

    def kzg_prove(self, kzg, d_evals_ptr, max_items, point):
        """KZG::prove_point with the proof MSM window-split over the ranks -> (proof point, y)."""
        from .engine import limbs_to_int
        from .scheme import _pt
        pt = np.array([(int(point) >> (64 * j)) & 0xFFFFFFFFFFFFFFFF for j in range(4)], dtype=np.uint64)
        xy = np.zeros(8, dtype=np.uint64)
        inf = np.zeros(1, dtype=np.uint8)
        y = np.zeros(4, dtype=np.uint64)
        check(lib().vc_kzg_prove_sharded(kzg.engine.h, self.h, kzg.table, kzg.size, ctypes.c_void_p(d_evals_ptr),
                                         max_items, _p(pt), _p(xy), _p(inf), _p(y)), "vc_kzg_prove_sharded")
        return {"proof": _pt(xy, inf[0]), "y": limbs_to_int(y)}

    def multiproof(self, vc, cxy, cinf, z, y, d_data_slice_ptr):
        """prove_multiproof over the ranks (IPA or KZG `vc`); d_data_slice_ptr: this rank's
        shard_range(Q) slice of the evaluations on its device."""
        from . import scheme
        from .engine import limbs_to_int
        ipa = isinstance(vc, scheme.IPA)
        N = vc.N if ipa else vc.size
        dxy = np.zeros(8, dtype=np.uint64)
        dinf = np.zeros(1, dtype=np.uint8)
        if ipa:
            b, arrs = scheme.IPAProof._alloc(scheme._log2(N))
            check(lib().vc_multiproof_prove_sharded(vc.engine.h, self.h, 0, vc.table, N, len(z),
                                                    ctypes.c_void_p(d_data_slice_ptr), _p(cxy), _p(cinf), _p(z),
                                                    _p(y), _p(dxy), _p(dinf), ctypes.byref(b), None, None, None),
                  "vc_multiproof_prove_sharded")
            return {"proof": scheme.IPAProof._from(b, arrs), "d": scheme._pt(dxy, dinf[0])}
        kxy = np.zeros(8, dtype=np.uint64)
        kinf = np.zeros(1, dtype=np.uint8)
        ky = np.zeros(4, dtype=np.uint64)
        check(lib().vc_multiproof_prove_sharded(vc.engine.h, self.h, 1, vc.table, N, len(z),
                                                ctypes.c_void_p(d_data_slice_ptr), _p(cxy), _p(cinf), _p(z), _p(y),
                                                _p(dxy), _p(dinf), None, _p(kxy), _p(kinf), _p(ky)),
              "vc_multiproof_prove_sharded")
        return {"proof": {"proof": scheme._pt(kxy, kinf[0]), "y": limbs_to_int(ky)}, "d": scheme._pt(dxy, dinf[0])}

    def multiproof_many(self, vc, cxy, cinf, z, y, d_data_mine_ptr):
        """proof-parallel multiproofs over the ranks (vc_multiproof_prove_many_sharded): all P
        proofs' queries on the host ([P][Q] layouts), this rank's proofs' evaluations at
        d_data_mine_ptr ([P_k][Q][N], device); every rank returns all P proofs."""
        from . import scheme
        ipa = isinstance(vc, scheme.IPA)
        N = vc.N if ipa else vc.size
        P, Q = z.shape
        out = scheme.MultiproofSet(0 if ipa else 1, N, P)
        cxy, cinf, z, y = (np.ascontiguousarray(a) for a in (cxy, cinf, z, y))
        check(lib().vc_multiproof_prove_many_sharded(vc.engine.h, self.h, out.scheme, vc.table, N, Q, P,
                                                     ctypes.c_void_p(d_data_mine_ptr), _p(cxy), _p(cinf), _p(z),
                                                     _p(y), *out.args()), "vc_multiproof_prove_many_sharded")
        return out.proofs()

    def multiproof_gather(self, out, status=0, engine=None):
        """the proof-parallel exchange alone (vc_multiproof_gather) on a scheme.MultiproofSet whose
        shard_range(P, rank, world) entries this rank filled; status = this rank's share's status"""
        check(lib().vc_multiproof_gather(self.h, engine.h if engine is not None else None, status, out.scheme, out.N,
                                         out.P, *out.args()), "vc_multiproof_gather")
        return out

    def verkle_commitment(self, tree, engine, table):
        """root commitment of a verkle tree every rank holds identically; each level's dirty
        nodes are cut into rank slices and all-gathered."""
        from .scheme import _pt
        xy = np.zeros(8, dtype=np.uint64)
        inf = np.zeros(1, dtype=np.uint8)
        check(lib().vc_verkle_commitment_sharded(engine.h, self.h, table, tree.h, _p(xy), _p(inf)),
              "vc_verkle_commitment_sharded")
        return _pt(xy, inf[0])


class ThreadGroup:
    """In-process all-gather for G ranks run as G threads (GPU tests on one card): every rank
    deposits its bytes, the last one to arrive releases them all."""

    def __init__(self, world):
        import threading
        self.world = world
        self.cv = threading.Condition()
        self.slots = [None] * world
        self.gen = 0
        self.result = None

    def fn(self, rank):
        def allgather(send):
            with self.cv:
                gen = self.gen
                self.slots[rank] = send
                if all(s is not None for s in self.slots):
                    self.result = b"".join(self.slots)
                    self.slots = [None] * self.world
                    self.gen += 1
                    self.cv.notify_all()
                else:
                    if not self.cv.wait_for(lambda: self.gen != gen, timeout=60):
                        raise TimeoutError("all-gather peer missing")
                return self.result
        return allgather
