"""world_size-2 gloo test (CPU) of the multi-GPU MSM exchange: point-range shards or window
slices, all-gather of projective partials, host sum (vkzg.dist) == the whole MSM. Shard
partials come from the oracle here (no GPU in this container); on the GPU box bench.py runs
the same path with the HIP partials over RCCL (tests/test_gpu_msm.py checks the HIP window
parts against the same oracle)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, curve, q, split="points"):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "verkle-kzg_amd"), os.path.join(ROOT, "oracle")]
    import random
    import torch.distributed as dist
    from pyoracle import cref
    from pyoracle import pippenger
    from pyoracle.curves import CURVES, random_points
    from vkzg import dist as vdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    C = CURVES[curve]
    rng = random.Random(17)
    n = 37
    pts = random_points(C, n, rng)
    sc = [rng.randrange(C.r) for _ in range(n)]
    if split == "points":
        lo, hi = vdist.shard_range(n, rank, world)
        part = cref.msm(curve, pts[lo:hi], sc[lo:hi], 1)
    else:  # window slice `rank` of `world` over all n terms
        part = cref.msm(curve, pts, pippenger.part_scalars(curve, sc, rank, world, C.r), 1)
    words = vdist.affine_to_acc_words(curve, part)
    parts = vdist.all_gather_partials(words, world, None)
    xy, inf = vdist.partials_sum(curve, parts)
    full = cref.msm(curve, pts, sc, 1)
    nl = len(xy) // 2
    got = None if inf else (sum(int(v) << (64 * j) for j, v in enumerate(xy[:nl])),
                            sum(int(v) << (64 * j) for j, v in enumerate(xy[nl:])))
    if curve == "bandersnatch" and inf:
        got = (0, 1)
    q.put((rank, got == full, parts.shape))
    dist.destroy_process_group()


@pytest.mark.parametrize("split", ["points", "windows"])
@pytest.mark.parametrize("curve", ["bn254", "bls12_381", "bandersnatch"])
def test_sharded_msm_gloo_world2(curve, split, oracle_c):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, curve, q, split)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(ok for _, ok, _ in res), res
    assert all(shape[0] == 2 for _, _, shape in res)


def test_shard_range_covers():
    from vkzg import dist as vdist
    for n in (0, 1, 7, 1 << 20):
        for w in (1, 2, 3, 8):
            parts = [vdist.shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))


def _commit_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "verkle-kzg_amd")]
    import torch
    import torch.distributed as dist
    from vkzg import dist as vdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 7
    lo, hi = vdist.shard_range(B, rank, world)
    # stand-in commitments: row j = (j, j^2, ...) so the gathered order is checkable
    xy = torch.tensor([[j * 10 + k for k in range(8)] for j in range(lo, hi)], dtype=torch.int64)
    inf = torch.tensor([j % 2 for j in range(lo, hi)], dtype=torch.uint8)
    gxy, ginf = vdist.all_gather_commitments(xy, inf, B, world)
    ok = (gxy.shape == (B, 8) and all(int(gxy[j, k]) == j * 10 + k for j in range(B) for k in range(8))
          and [int(v) for v in ginf] == [j % 2 for j in range(B)])
    q.put((rank, ok))
    dist.destroy_process_group()


def test_batched_commit_gather_gloo_world2():
    """the batch-sliced commit path's all-gather (bench.py secondary)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_commit_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(ok for _, ok in res), res


def _mp_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "verkle-kzg_amd")]
    import random
    import torch
    import torch.distributed as dist
    from vkzg import dist as vdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    rng = random.Random(3)
    N, Q = 8, 13
    f = [[rng.randrange(R) for _ in range(N)] for _ in range(Q)]
    z = [rng.randrange(N) for _ in range(Q)]
    r = rng.randrange(R)
    rows = sorted(set(z))

    def sums(lo, hi):  # restatement of k_mp_chunk + k_mp_chunk_reduce: S[row][k] = sum r^i f_i[k]
        S = [[0] * N for _ in rows]
        for i in range(lo, hi):
            for k in range(N):
                S[rows.index(z[i])][k] = (S[rows.index(z[i])][k] + pow(r, i, R) * f[i][k]) % R
        return S

    lo, hi = vdist.shard_range(Q, rank, world)
    mine = sums(lo, hi)
    t = torch.tensor([[[(v >> (64 * j)) & 0xFFFFFFFFFFFFFFFF for j in range(4)] for v in row] for row in mine],
                     dtype=torch.uint64).view(torch.int64)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    got = [[0] * N for _ in rows]
    for o in outs:
        u = o.numpy().view("uint64")
        for a in range(len(rows)):
            for k in range(N):
                got[a][k] = (got[a][k] + sum(int(u[a, k, j]) << (64 * j) for j in range(4))) % R
    q.put((rank, got == sums(0, Q)))
    dist.destroy_process_group()


def test_multiproof_sums_exchange_gloo_world2():
    """the sharded multiproof's one exchange: per-rank per-point sums over query slices,
    all-gathered and added mod r, equal the whole query set's sums."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(ok for _, ok in res), res


def _comm_worker(rank, world, port, q):
    """the C ABI's host-callback transport (vc_comm_init_host + vc_comm_allgather, include/
    vc_comm.h) over a gloo group: what a non-RCCL caller of libvkzg.so plugs in."""
    import sys
    sys.path[:0] = [os.path.join(ROOT, "verkle-kzg_amd")]
    import torch.distributed as dist
    from vkzg import comm as vcomm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = vcomm.Comm.host(rank, world, vcomm.torch_allgather())
    ok = c.rank == rank and c.world == world and not c.is_rccl
    for size in (1, 13, 4096, 100_003):
        send = bytes((rank * 31 + i) % 251 for i in range(size))
        got = c.allgather(send)
        want = b"".join(bytes((r * 31 + i) % 251 for i in range(size)) for r in range(world))
        ok = ok and got == want
    c.close()
    q.put((rank, ok))
    dist.destroy_process_group()


def test_comm_host_transport_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(60)
    assert sorted(res) == [(0, True), (1, True)]


def test_comm_world_one_and_bad_args():
    import sys
    sys.path[:0] = [os.path.join(ROOT, "verkle-kzg_amd")]
    import ctypes
    from vkzg import comm as vcomm
    from vkzg import lib
    c = vcomm.Comm.host(0, 1, None)
    assert c.allgather(b"xyz") == b"xyz" and c.world == 1
    c.close()
    h = ctypes.c_void_p()
    assert lib().vc_comm_init_host(0, 2, ctypes.cast(None, vcomm.ALLGATHER_FN), None, ctypes.byref(h)) == -1
    assert lib().vc_comm_init_host(2, 2, vcomm.ALLGATHER_FN(lambda *a: 0), None, ctypes.byref(h)) == -1


def _mp_gather_worker(rank, world, port, q):
    """vc_multiproof_gather (the proof-parallel multiproof exchange, include/vc_comm.h) over the
    host-callback transport on a gloo group: every rank fills its shard_range(P) proofs, all ranks
    end with all P; a failed share makes every rank fail (its status / VC_E_PEER)."""
    import sys
    sys.path[:0] = [os.path.join(ROOT, "verkle-kzg_amd")]
    import numpy as np
    import torch.distributed as dist
    import vkzg
    from vkzg import comm as vcomm
    from vkzg import dist as vdist
    from vkzg import scheme
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = vcomm.Comm.host(rank, world, vcomm.torch_allgather())
    ok = True
    N, P = 8, 5

    def fill(out, p, rng):
        out.d_xy[p] = rng.integers(0, 1 << 63, size=8, dtype=np.uint64)
        out.d_inf[p] = p % 2
        if out.scheme == 0:
            a = out.arrs[p]
            a["lxy"][:] = rng.integers(0, 1 << 63, size=a["lxy"].shape, dtype=np.uint64)
            a["rxy"][:] = rng.integers(0, 1 << 63, size=a["rxy"].shape, dtype=np.uint64)
            a["linf"][:] = rng.integers(0, 2, size=a["linf"].shape, dtype=np.uint8)
            a["rinf"][:] = rng.integers(0, 2, size=a["rinf"].shape, dtype=np.uint8)
            out.bufs[p].tip[:] = [int(v) for v in rng.integers(0, 1 << 63, size=4, dtype=np.uint64)]
            out.bufs[p].y[:] = [int(v) for v in rng.integers(0, 1 << 63, size=4, dtype=np.uint64)]
        else:
            out.kxy[p] = rng.integers(0, 1 << 63, size=8, dtype=np.uint64)
            out.kinf[p] = 1 - p % 2
            out.ky[p] = rng.integers(0, 1 << 63, size=4, dtype=np.uint64)

    def snapshot(out, p):
        s = [out.d_xy[p].tolist(), int(out.d_inf[p])]
        if out.scheme == 0:
            a = out.arrs[p]
            s += [a["lxy"].tolist(), a["rxy"].tolist(), a["linf"].tolist(), a["rinf"].tolist(),
                  list(out.bufs[p].tip), list(out.bufs[p].y)]
        else:
            s += [out.kxy[p].tolist(), int(out.kinf[p]), out.ky[p].tolist()]
        return s

    for sid in (0, 1):
        want = scheme.MultiproofSet(sid, N, P)
        for p in range(P):
            fill(want, p, np.random.default_rng(100 * sid + p))
        out = scheme.MultiproofSet(sid, N, P)
        lo, hi = vdist.shard_range(P, rank, world)
        for p in range(lo, hi):
            fill(out, p, np.random.default_rng(100 * sid + p))
        c.multiproof_gather(out)
        ok = ok and all(snapshot(out, p) == snapshot(want, p) for p in range(P))
        # rank 1's share failed (VC_E_OOM): it returns that, its peer VC_E_PEER -- nobody hangs
        try:
            c.multiproof_gather(scheme.MultiproofSet(sid, N, P), status=-3 if rank == 1 else 0)
            ok = False
        except vkzg.VCError as ex:
            ok = ok and ex.status == (-3 if rank == 1 else -10)
        # rank 1's output buffers are unusable (an IPA proof with too few rounds, a NULL KZG y):
        # it fails with VC_E_INVALID inside the exchange, its peer gets VC_E_PEER, and neither
        # rank's outputs are written (no partial copy-out before the group agrees)
        bad = scheme.MultiproofSet(sid, N, P)
        for p in range(lo, hi):
            fill(bad, p, np.random.default_rng(100 * sid + p))
        before = [snapshot(bad, p) for p in range(P)]
        args = list(bad.args())
        if rank == 1:
            if sid == 0:
                bad.bufs[P - 1].rounds = 1
            else:
                args[5] = None
        from vkzg._lib import lib
        st = lib().vc_multiproof_gather(c.h, None, 0, sid, N, P, *args)
        ok = ok and st == (-1 if rank == 1 else -10)
        if sid == 0 and rank == 1:
            bad.bufs[P - 1].rounds = 3
        ok = ok and [snapshot(bad, p) for p in range(P)] == before
    c.close()
    q.put((rank, ok))
    dist.destroy_process_group()


def test_multiproof_gather_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mp_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(60)
    assert sorted(res) == [(0, True), (1, True)]
