"""Multi-GPU sharding of one MSM: one process per GPU, one exchange step.

Two splits, both ending in one all-gather of un-normalised projective partials
(torch.distributed: RCCL over xGMI with the "nccl" backend, gloo on CPU in tests) that are
added on the host (vc_partials_sum); the message is world x 128-192 bytes, latency-bound,
so a single all-gather is the right collective:

  split="windows" (default): rank k computes Pippenger windows [kW/G, (k+1)W/G) of ALL n
      terms (vc_msm_device_window_part). Accumulation work is n*W/G per rank as with a point
      split, but the bucket reduction -- W * 2^(c-1) buckets, independent of n -- is divided
      by G too. Every rank streams all n bases (resident on each GPU; 100 MB at 2^20); the
      MSM is VALU-bound, not HBM-bound, so re-reading them is free.
  split="points": rank k takes the contiguous slice [kn/G, (k+1)n/G) of bases and scalars
      (vc_msm_device_partial) and runs a full Pippenger on it.
"""
import numpy as np

BASE_P = {
    "bn254": 21888242871839275222246405745257275088696311157297823662689037894645226208583,
    "bls12_381": int("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eab"
                     "fffeb153ffffb9feffffffffaaab", 16),
    "bandersnatch": 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
}
WORDS = {"bn254": 32, "bls12_381": 48, "bandersnatch": 32}


def shard_range(n, rank, world):
    """Contiguous near-equal split of [0, n)."""
    return n * rank // world, n * (rank + 1) // world


def affine_to_acc_words(curve, P):
    """Canonical affine point -> the engine's accumulator words (Montgomery XYZZ / extended,
    Z = 1). Used to feed externally computed partials (e.g. from another engine) to
    vc_partials_sum."""
    p = BASE_P[curve]
    limbs = WORDS[curve] // 4
    R = 1 << (32 * limbs)
    if curve == "bandersnatch":
        x, y = P if P is not None else (0, 1)
        vals = [x * R % p, y * R % p, x * y % p * R % p, R % p]      # X, Y, T, Z
    elif P is None:
        vals = [R % p, R % p, 0, 0]                                    # XYZZ zero: ZZ = 0
    else:
        vals = [P[0] * R % p, P[1] * R % p, R % p, R % p]
    out = np.zeros(WORDS[curve], dtype=np.uint32)
    for k, v in enumerate(vals):
        for j in range(limbs):
            out[k * limbs + j] = (v >> (32 * j)) & 0xFFFFFFFF
    return out


def all_gather_partials(part_words, world, device=None):
    """All-gather one partial accumulator per rank. `device` None -> CPU tensors (gloo)."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(part_words).view(np.int32).copy())
    if device is not None:
        t = t.to(device)
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return torch.stack(outs).cpu().numpy().view(np.uint32)


def window_count(curve, n, with_terms=False):
    """(window bits c, window count W[, terms per point]) the engine picks for an n-term MSM
    (vc_msm_windows); terms per point = 2 when the GLV split applies."""
    import ctypes
    from ._lib import check, lib
    from .engine import CURVE_IDS
    c, w, t = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    check(lib().vc_msm_windows(CURVE_IDS[curve], n, ctypes.byref(c), ctypes.byref(w), ctypes.byref(t)),
          "vc_msm_windows")
    return (c.value, w.value, t.value) if with_terms else (c.value, w.value)


def all_gather_commitments(xy, inf, total, world):
    """Batched commits sharded by contiguous batch slices (shard_range): all-gather every
    rank's (xy, inf) slice so each rank holds all `total` commitments in batch order.
    xy: (b_k, 2*NL) int64 tensor, inf: (b_k,) uint8 tensor on this rank's device (or CPU
    with gloo). Slices differ in length by at most one, so they are padded to the largest."""
    import torch
    import torch.distributed as dist
    bmax = (total + world - 1) // world
    pad_xy = torch.zeros((bmax, xy.shape[1]), dtype=xy.dtype, device=xy.device)
    pad_inf = torch.zeros((bmax,), dtype=inf.dtype, device=inf.device)
    pad_xy[:xy.shape[0]] = xy
    pad_inf[:inf.shape[0]] = inf
    outs_xy = [torch.zeros_like(pad_xy) for _ in range(world)]
    outs_inf = [torch.zeros_like(pad_inf) for _ in range(world)]
    dist.all_gather(outs_xy, pad_xy)
    dist.all_gather(outs_inf, pad_inf)
    parts_xy, parts_inf = [], []
    for r in range(world):
        lo, hi = shard_range(total, r, world)
        parts_xy.append(outs_xy[r][:hi - lo])
        parts_inf.append(outs_inf[r][:hi - lo])
    return torch.cat(parts_xy), torch.cat(parts_inf)


def msm_sharded(engine, table, d_scalars_ptr, n, rank, world, device, split="windows"):
    """Whole-MSM result on every rank: local partial -> all-gather -> host sum.
    split="windows": d_scalars_ptr points at ALL n scalars (4 u64 each) in device memory;
    split="points": at this rank's shard [lo, hi) only."""
    if split == "windows":
        part = engine.msm_device_window_part(table, d_scalars_ptr, n, rank, world)
    elif split == "points":
        lo, hi = shard_range(n, rank, world)
        part = engine.msm_device_partial(table, d_scalars_ptr, hi - lo, offset=lo)
    else:
        raise ValueError(f"unknown split {split!r}")
    parts = all_gather_partials(part, world, device) if world > 1 else part[None, :]
    return partials_sum(engine.curve, parts)


def partials_sum(curve, parts):
    """Host-side sum of projective partials -> ((2*NL,) uint64 canonical affine, inf)."""
    from .engine import partials_sum as _ps
    return _ps(curve, parts)


def kzg_open_sharded(engine, table, size, d_evals_ptr, max_items, point, rank, world, device):
    """KZG open (kzg/mod.rs:136-154) across ranks: every rank computes the
    quotient (elementwise, ~10 % of the open) and window slice `rank` of the proof MSM
    (vc_kzg_prove_device_part); one all-gather of partials, host sum.
    Returns ((2*NL,) uint64 canonical affine proof, inf, y limbs)."""
    import ctypes
    from ._lib import check, lib
    pt = np.array([(int(point) >> (64 * j)) & 0xFFFFFFFFFFFFFFFF for j in range(4)], dtype=np.uint64)
    acc = np.zeros(engine.point_words(), dtype=np.uint32)
    y = np.zeros(4, dtype=np.uint64)
    check(lib().vc_kzg_prove_device_part(engine.h, table, size, ctypes.c_void_p(d_evals_ptr), max_items,
                                         ctypes.c_void_p(pt.ctypes.data), rank, world,
                                         ctypes.c_void_p(acc.ctypes.data), ctypes.c_void_p(y.ctypes.data)),
          "vc_kzg_prove_device_part")
    parts = all_gather_partials(acc, world, device) if world > 1 else acc[None, :]
    xy, inf = partials_sum(engine.curve, parts)
    return xy, inf, y


def multiproof_prove_sharded(vc, cxy, cinf, z, y, d_data_ptr, rank, world, device=None):
    """Multiproof (multiproof.rs:99-176) over ranks, IPA or KZG (`vc` is a
    scheme.IPA or scheme.KZG): every rank runs the host transcript over all queries (challenge
    r), accumulates the per-point sums S of its query slice [lo, hi) = shard_range(Q)
    (d_data_ptr: that slice's evaluations, Qs x N canonical u64x4 on this rank's device), the S
    matrices (rows x N x 32 B, <= 2 MiB at N = 256) are all-gathered over RCCL -- the one
    exchange -- and every rank finishes (quotients, D, E, inner proof) on the summed S."""
    import torch
    import torch.distributed as dist
    from . import scheme
    from ._lib import lib
    N = vc.N if isinstance(vc, scheme.IPA) else vc.size
    rows = scheme.multiproof_rows(N, z)
    lo, hi = shard_range(len(z), rank, world)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    # every element of S is written by the accumulate (on the engine's stream, which is
    # synchronised before it returns): no fill on torch's stream that could race with it
    S = torch.empty((rows, N, 4), dtype=torch.int64, device=dev)
    torch.cuda.current_stream(dev).synchronize()
    # the host transcript (phase 1) overlapped with this shard's planning (phase 2)
    tr, r = scheme.multiproof_begin_accumulate(vc.engine, N, cxy, cinf, z, y, lo, hi - lo, d_data_ptr, S.data_ptr())
    try:
        if world > 1:
            outs = [torch.empty_like(S) for _ in range(world)]
            dist.all_gather(outs, S)
            parts = torch.stack(outs).contiguous()
        else:
            parts = S[None]
        torch.cuda.current_stream(dev).synchronize()
    except BaseException:
        lib().vc_transcript_free(tr)
        raise
    return scheme.multiproof_finish(vc, z, parts.data_ptr(), world, tr)
