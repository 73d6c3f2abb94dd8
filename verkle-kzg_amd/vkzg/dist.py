"""Multi-GPU sharding of one MSM: one process per GPU, point-range shards,
one exchange step.

Each rank runs the Pippenger engine on its contiguous slice [lo, hi) of the bases and
scalars (it streams only n/world of them from its own HBM), producing an un-normalised
projective partial sum (vc_msm_device_partial). The partials are all-gathered
(torch.distributed: RCCL over xGMI with the "nccl" backend, gloo on CPU in tests) and
added on the host (vc_partials_sum). The message is world x 128-192 bytes: latency-bound,
nowhere near the xGMI link rate, so a single all-gather is the right collective.
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


def msm_sharded(engine, table, d_scalars_ptr, n, rank, world, device):
    """Whole-MSM result on every rank: local shard partial -> all-gather -> host sum.
    d_scalars_ptr points at this rank's shard scalars (4 u64 each) in device memory."""
    lo, hi = shard_range(n, rank, world)
    part = engine.msm_device_partial(table, d_scalars_ptr, hi - lo, offset=lo)
    parts = all_gather_partials(part, world, device) if world > 1 else part[None, :]
    return partials_sum(engine.curve, parts)


def partials_sum(curve, parts):
    """Host-side sum of projective partials -> ((2*NL,) uint64 canonical affine, inf)."""
    from .engine import partials_sum as _ps
    return _ps(curve, parts)
