#!/usr/bin/env python3
"""Benchmark: single 2^20-point BLS12-381 G1 MSM (BASELINE.json configs[1]) on N MI355X.

A step = one 2^20-point MSM over synthetic inputs already resident in HBM (bases uploaded
once, scalars on the device). With N ranks the MSM is split (AUTO_SPLIT below, from the
one-card split probe): into point ranges on the shared radix copies for 2-3 ranks, into
Pippenger window parts from 4 (rank k computes windows [kW/N, (k+1)W/N) of all n terms);
the per-rank projective partial sums are all-gathered over RCCL and added on the host: one
exchange step, so scaling is "strong" (total work fixed).

Secondary line items (same JSON object): 10k batched width-256 Bandersnatch commits/s
(config 3; the batch split across the N ranks, results all-gathered), and the CPU baseline:
the reference's naive MSM restated in C (oracle/c/ref_curve.c) timed on a bounded sample on
this host.

    python bench.py [--gpus N --steps K --warmup W]

--gpus N > 1 starts N rank processes itself (torch.distributed.run on 127.0.0.1) unless a launcher
already set WORLD_SIZE (then --gpus must equal it); --rehearse-one-gpu puts every rank on device 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "verkle-kzg_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import vkzg  # noqa: E402
from vkzg import dist as vdist  # noqa: E402

METRIC = "width-256 commits/sec + 2^20-pt MSM ms at 1/2/4/8 GPU; achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# algorithmic bytes per 2^20 BLS12-381 MSM: n*(96 B affine + 32 B scalar) + 96 B out
BYTES_PER_POINT = {"bls12_381": 96 + 32, "bn254": 64 + 32, "bandersnatch": 64 + 32}
OUT_BYTES = {"bls12_381": 96, "bn254": 64, "bandersnatch": 64}
# VALU roofline: field multiplies per mixed add in the accumulate kernel
# (XYZZ 8M+2S; extended Edwards 8M) x 2 N^2 v_mad_u64_u32 per N-limb Montgomery multiply
CURVE_TAG = {"bls12_381": "BLS381Fq", "bn254": "BN254Fq", "bandersnatch": "BandD"}  # kernel-name match
SCALAR_BITS = {"bls12_381": 255, "bn254": 254, "bandersnatch": 253}
# HBM bytes of the dominant kernel from rocprofv3 PMC passes of this same command
# (scripts/bench_profile.sh -> verkle-kzg_amd/tools/prof_summary.py), refreshed each profiling round
PMC_SUMMARY = next((p for p in (os.path.join(ROOT, "profiles", r, "pmc_summary.json") for r in ("r06", "r05", "r04", "r03", "r02", "r01"))
                    if os.path.exists(p)), os.path.join(ROOT, "profiles", "r04", "pmc_summary.json"))
# the headline's accumulate instantiation in the PMC summary: the shared-window copies in the pair
# layout (AffP, the default), else the (x, y, -y) records (AffN), else the packed tables


def _acc_key_rank(k):
    return 0 if "::AffP" in k else 1 if "::AffN" in k else 2


def progress(msg):
    """one stderr line per finished bench stage (rank 0): long runs show they are alive"""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); N > 1 without a launcher's WORLD_SIZE starts N ranks itself")
    ap.add_argument("--steps", type=int, default=20)
    # 20 untimed steps (~55 ms) before the timed region: measured 2.58-2.60 ms per step after 3,
    # 2.56 after 20, 2.53-2.55 after 100 on one box (the clock settles; profiles/r05/warmup/)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--curve", default="bls12_381")
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--commit-batch", type=int, default=10000)
    ap.add_argument("--commit-window", type=int, default=19,
                    help="fixed-base window bits of the config-3 table (19 with --commit-windows 13: 13 windows of "
                         "19 / 20 bits, 172 GB of 128-B entries, the speed of a c = 20 table; falls back to 16)")
    ap.add_argument("--commit-windows", type=int, default=13,
                    help="windows of the config-3 table (0: uniform c-bit windows)")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kzg", action="store_true", help="skip the KZG commit+open line (configs[3])")
    ap.add_argument("--kzg-log-d", type=int, default=20)
    ap.add_argument("--no-mp", action="store_true", help="skip the IPA multiproof line (configs[4])")
    ap.add_argument("--mp-log-q", type=int, default=16)
    ap.add_argument("--no-verkle", action="store_true", help="skip the verkle-tree commitment line (8(f) rank 1)")
    ap.add_argument("--no-ipa", action="store_true", help="skip the single IPA prove/verify line (benches/ipa.rs)")
    ap.add_argument("--verkle-keys", type=int, default=1 << 16)
    ap.add_argument("--verkle-reps", type=int, default=5, help="fresh trees / 1 % update rounds timed (medians)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads of the Pippenger CPU baseline (0: min(16, cpu_count), one GPU's CPU share)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 16, help="terms of the CPU naive MSM sample (~15 s)")
    ap.add_argument("--no-variable-base", action="store_true",
                    help="skip the variable-base (no shared-window copies) MSM sub-line")
    ap.add_argument("--no-check", action="store_true", help="skip the one-time 2^20 result check")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="multi-rank rehearsal on a 1-GPU box: every rank on device 0, gloo process group, "
                         "vc_comm host-callback exchange (RCCL refuses two ranks on one device); timings are "
                         "not scaling numbers")
    ap.add_argument("--launch-check", action="store_true",
                    help="rank bookkeeping only (gloo, no GPU): rank 0 prints the world it ran in")
    ap.add_argument("--comm", choices=["capi", "torch"], default="capi",
                    help="N > 1 exchange: vc_comm (C ABI, RCCL) or torch.distributed all-gather")
    ap.add_argument("--msm-split", choices=["auto", "windows", "points"], default="auto",
                    help="N > 1: how one MSM splits over the ranks (auto: by N, from the one-card split probe)")
    return ap.parse_args()


# N > 1 split of the headline MSM, chosen per N from the one-card per-rank probe
# (verkle-kzg_amd/tools/split_probe.py: the slowest rank's share of a 2^20 MSM, point range vs
# window part, wall time without per-kernel events; profiles/r05/split_walltime/: G = 2 points
# 1.41-1.42 ms against windows 1.54-1.58, G = 8 windows 0.60-0.62 against points 0.70-0.71 -- an
# eighth of the points still pays the radix copies' whole bucket tail; G = 4 a tie in round 4)
AUTO_SPLIT = {2: "points", 3: "points"}


def msm_split(a, world):
    if a.msm_split != "auto":
        return a.msm_split
    return AUTO_SPLIT.get(world, "windows")


def kernel_table(eng):
    """mean device ms per launch of the MSM pipeline's kernels (HIP events on the launch stream)"""
    out = {}
    for k in ("glv_split", "glv_phi", "msm_sort_hist", "msm_scan", "msm_sort_coarse", "msm_sort_fine",
              "msm_accumulate", "msm_fixup", "msm_segsum", "msm_bitsum", "msm_sumpart"):
        ms, cnt = eng.kernel_time(k)
        if cnt:
            out[k] = round(ms / cnt, 4)
    return out


def cpu_baseline(curve, n_full, sample, reps=3):
    """Reference algorithm (naive per-term double-and-add + sequential sum, utils.rs:16-19)
    restated in C (oracle/), 1 thread: `reps` disjoint slices of `sample` terms, each timed, the
    median per-term time extrapolated linearly to n_full (median of the runs)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import cref  # CPU baseline leg only (checker/baseline, never the measured path)
    if not os.path.exists(cref.LIB_PATH):
        import subprocess
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")], stdout=subprocess.DEVNULL)
    rng = np.random.default_rng(7)
    e = vkzg.Engine(curve, 0)
    tid = e.random_bases(sample, seed=77)
    xy, inf = e.download_bases(tid)
    e.close()
    sc = vkzg.random_scalars(curve, sample, rng)
    part = sample // reps
    ts = []
    for k in range(reps):
        lo = k * part
        t0 = time.perf_counter()
        cref.msm_arrays(curve, xy[lo:lo + part], inf[lo:lo + part], sc[lo:lo + part], 1)
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    per_msm_s = dt * n_full / part
    return {"value": 1.0 / per_msm_s, "unit": "MSM/s", "cores": 1, "kind": "port",
            "sample": f"{reps} slices of {part} of {n_full} terms of the naive {curve} MSM (reference utils.rs:16-19 "
                      f"restated in C, oracle/c/ref_curve.c), 1 thread, {[round(t, 2) for t in ts]} s, the median "
                      f"extrapolated linearly",
            "ms_per_msm": per_msm_s * 1e3, "host_cpus": os.cpu_count()}


def provenance():
    """What ran the line: the host CPU model, the SHA-256 rounds the host
    transcript used, and the hash of the libvkzg.so this process loaded."""
    import hashlib
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        so = open(vkzg.LIB_PATH, "rb").read()
        lib_sha = hashlib.sha256(so).hexdigest()
    except OSError:
        lib_sha = None
    sha = vkzg.lib().vc_host_sha256_path()
    return {"host_cpu": model, "host_cpus": host_cpu_share(),
            "sha256_path": "SHA-NI" if sha == 1 else "portable",
            "libvkzg_sha256": lib_sha, "libvkzg": os.path.relpath(vkzg.LIB_PATH, ROOT),
            "device": torch.cuda.get_device_name(torch.cuda.current_device())}


def host_cpu_share():
    """What the process may actually run on: the CPUs it reports, its affinity mask and the cgroup
    v2 CPU quota (cpu.max "quota period"; None when unlimited or unreadable). On the GPU boxes the
    OS reports 256 CPUs while the quota is one GPU's share, so a 256-thread run time-slices."""
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"reported": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota}


def cpu_pippenger(curve, xy, inf, scalars, want, threads, reps=3):
    """The fair all-core CPU bound: the same 2^20 MSM by the bucket method in C
    (oracle/c/ref_curve.c pip_msm: per-thread point chunks, signed windows, mixed bucket adds),
    on `threads` host threads, the whole workload `reps` times (no extrapolation), the median;
    its result is checked against the GPU's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import cref  # CPU baseline leg only
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        got = cref.pip_msm_arrays(curve, xy, inf, scalars, threads)
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    return {"value": 1.0 / dt, "unit": "MSM/s", "cores": threads, "kind": "pippenger",
            "sample": f"the full {scalars.shape[0]}-term {curve} MSM of the bench (bases and scalars of the timed "
                      f"step), Pippenger in C on {threads} threads (oracle/c/ref_curve.c pip_msm), "
                      f"{[round(t, 2) for t in ts]} s, the median",
            "ms_per_msm": dt * 1e3, "same_result_as_gpu": bool(got[1] == int(want[1]) and np.array_equal(got[0], np.asarray(want[0])))}


def cpu_pippenger_commits(batch, threads):
    """configs[2] on the CPU: `batch` width-256 Bandersnatch commits, one Pippenger per commit in C,
    commits split over `threads` host threads."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import cref  # CPU baseline leg only
    e = vkzg.Engine("bandersnatch", 0)
    tid = e.random_bases(256, seed=3)
    xy, inf = e.download_bases(tid)
    e.close()
    sc = vkzg.random_scalars("bandersnatch", 256 * batch, np.random.default_rng(9))
    t0 = time.perf_counter()
    cref.pip_msm_batch_arrays("bandersnatch", xy, inf, sc, 256, threads)
    dt = time.perf_counter() - t0
    return {"value": batch / dt, "unit": "commits/s", "cores": threads, "kind": "pippenger",
            "sample": f"{batch} width-256 bandersnatch commits, Pippenger per commit in C "
                      f"(oracle/c/ref_curve.c pip_msm_batch) on {threads} threads, {dt:.2f} s"}


def cpu_commit_baselines(reps=8):
    """The reference's commit (IPA/KZG::commit = naive inner_product, utils.rs:16-19) restated in
    C, 1 thread: one width-256 commit on BN254 (configs[0], the reference's own curve) and on
    Bandersnatch (configs[2]); `reps` commits each."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import cref  # CPU baseline leg only
    out = {}
    for name, curve in (("C1_width256_commit_bn254", "bn254"), ("C3_width256_commit_bandersnatch", "bandersnatch")):
        e = vkzg.Engine(curve, 0)
        tid = e.random_bases(256, seed=3)
        xy, inf = e.download_bases(tid)
        e.close()
        sc = vkzg.random_scalars(curve, 256 * reps, np.random.default_rng(9))
        t0 = time.perf_counter()
        for r in range(reps):
            cref.msm_arrays(curve, xy, inf, sc[r * 256:(r + 1) * 256], 1)
        dt = (time.perf_counter() - t0) / reps
        out[name] = {"value": 1.0 / dt, "unit": "commits/s", "cores": 1, "kind": "port",
                     "sample": f"{reps} naive width-256 {curve} commits (utils.rs:16-19 in C), 1 thread",
                     "ms_per_commit": dt * 1e3}
    return out


def kzg_line(a, rank, world, local, dev, stream):
    """configs[3]: KZG commit + open at d = 2^kzg_log_d on BLS12-381 (the north_star's KZG
    curve): commit = MSM over the Lagrange SRS, open = quotient + MSM (kzg/mod.rs:126-154),
    at an in-domain index m = d/3 and at an out-of-domain point; both MSMs window-split
    across ranks. The SRS (L_j = l_j(100) G, Appendix A.7) is built on the GPU once, untimed."""
    import ctypes
    from vkzg._lib import check, lib
    d = 1 << a.kzg_log_d
    keng = vkzg.Engine("bls12_381", local)
    keng.set_stream(stream.cuda_stream)
    secret = vkzg.ints_to_limbs([100])[0].copy()
    tid, size = ctypes.c_int(), ctypes.c_size_t()
    t0 = time.perf_counter()
    check(lib().vc_kzg_setup(keng.h, d, ctypes.c_void_p(secret.ctypes.data), ctypes.byref(tid), ctypes.byref(size)),
          "vc_kzg_setup")
    setup_s = time.perf_counter() - t0
    tid = tid.value
    ev = vkzg.random_scalars("bls12_381", d, np.random.default_rng(44))
    d_ev = torch.from_numpy(ev.view(np.int64).copy()).to(dev)
    g = dev if world > 1 else None
    pts = {"in_domain": d // 3, "outside": d + 987654321}

    def step(point):
        com = vdist.msm_sharded(keng, tid, d_ev.data_ptr(), d, rank, world, g, split="windows")
        prf = vdist.kzg_open_sharded(keng, tid, d, d_ev.data_ptr(), d, point, rank, world, g)
        return com, prf

    res = {}
    for name, point in pts.items():
        step(point)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        keng.enable_timing(True)
        keng.reset_timing()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            step(point)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        dt = (time.perf_counter() - t0) / reps
        if world > 1:
            tt = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        keng.enable_timing(False)
        qk = {}
        for k in ("kzg_den", "binv_prep", "binv_finish", "kzg_q_in", "kzg_q_out", "kzg_bary", "kzg_fold",
                  "kzg_inv_shift", "powers", "to_mont"):
            ms, cnt = keng.kernel_time(k)
            if cnt:
                qk[k] = round(ms / cnt, 4)
        res[name] = {"ms_per_commit_open": dt * 1e3, "quotient_kernels_ms": qk}
        if world == 1:  # commit + open as one call: both SRS MSMs in one batched pipeline
            pt = vkzg.ints_to_limbs([point])[0].copy()
            bufs = [np.zeros(12, dtype=np.uint64), np.zeros(1, dtype=np.uint8), np.zeros(12, dtype=np.uint64),
                    np.zeros(1, dtype=np.uint8), np.zeros(4, dtype=np.uint64)]
            P = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731

            def fused():
                check(lib().vc_kzg_commit_prove_device(keng.h, tid, d, ctypes.c_void_p(d_ev.data_ptr()), d, P(pt),
                                                       *[P(b) for b in bufs]), "vc_kzg_commit_prove_device")
            fused()
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                fused()
                ts.append((time.perf_counter() - t0) * 1e3)
            com_s, prf_s = step(point)
            pts = lambda xy, inf: vkzg.arrays_to_points("bls12_381", np.asarray(xy)[None, :],  # noqa: E731
                                                        np.array([inf], np.uint8))[0]
            same_c = pts(bufs[0], bufs[1][0]) == pts(com_s[0], com_s[1])
            same_p = pts(bufs[2], bufs[3][0]) == pts(prf_s[0], prf_s[1])
            same_y = bool(np.array_equal(bufs[4], np.asarray(prf_s[2], dtype=np.uint64)))
            res[name]["separate_calls_ms"] = res[name]["ms_per_commit_open"]
            res[name]["fused_ms_all"] = [round(t, 3) for t in ts]
            res[name]["fused_same_commitment"] = bool(same_c)
            res[name]["fused_same_proof_and_y"] = bool(same_p and same_y)
            # the C4 number on one GPU is the one-call commit + open (vc_kzg_commit_prove_device)
            # when its commitment, proof and y all equal the two separate calls' (commit MSM, then
            # open); otherwise the separate-call number stays and the mismatch is flagged
            if same_c and same_p and same_y:
                res[name]["ms_per_commit_open"] = float(np.median(ts))
            else:
                res[name]["fused_mismatch"] = True
    keng.close()
    fused_bytes = d * (96 + 32) + 2 * 96  # SURVEY 8(d) C4 fused minimum
    return {"workload": f"KZG commit + open, d = 2^{a.kzg_log_d}, BLS12-381 (configs[3]), MSMs window-split "
                        f"over {world} rank(s)", "srs_setup_s": setup_s, **res,
            "algorithmic_bytes_per_unit": fused_bytes,
            "achieved_GBps_in_domain": fused_bytes / (res["in_domain"]["ms_per_commit_open"] * 1e-3) / 1e9}


def rj_plus_i(rng, Q, N):
    """Q datasets of N evaluations f_j[i] = r_j + i (benches/ipa.rs gen_data, :54-62), r_j random
    BN254 Fr: (Q * N, 4) canonical u64 limbs. r_j's top limb is drawn below r's, so r_j + i < r
    for every i < 2^64 (no reduction)."""
    from vkzg import scheme
    r3 = scheme.R_BN254 >> 192
    rj = rng.integers(0, 1 << 63, size=(Q, 4), dtype=np.uint64) * np.uint64(2) + \
        rng.integers(0, 2, size=(Q, 4), dtype=np.uint64)
    rj[:, 3] = rng.integers(0, r3, size=Q, dtype=np.uint64)
    i = np.arange(N, dtype=np.uint64)
    out = np.empty((Q, N, 4), dtype=np.uint64)
    out[:, :, 0] = rj[:, None, 0] + i[None, :]
    carry = (out[:, :, 0] < rj[:, None, 0]).astype(np.uint64)
    for k in (1, 2, 3):
        out[:, :, k] = rj[:, None, k] + carry
        carry = carry & (out[:, :, k] == 0).astype(np.uint64)
    return out.reshape(Q * N, 4)


def mp_line(a, rank, world, local, dev, stream, comm=None):
    """configs[4]: IPA multiproof (multiproof.rs:99-176) over Q = 2^mp_log_q width-256 queries
    on BN254 (the reference's curve), the query set sharded over the ranks (vkzg.dist
    .multiproof_prove_sharded: host transcript on every rank, per-point sums of the local
    slice on the GPU, one all-gather of the 256 x 256 sums, finish on every rank). Inputs: the
    reference bench's datasets f_j[i] = r_j + i (benches/ipa.rs:38-62, rj_plus_i), their
    commitments (batched fixed-base commits, untimed), uniform points z in [0, 256), y = f(z)."""
    from vkzg import scheme
    N, Q = 256, 1 << a.mp_log_q
    meng = vkzg.Engine("bn254", local)
    meng.set_stream(stream.cuda_stream)
    crs = scheme.ipa_crs(N + 1, max_=512)
    ipa = scheme.IPA(meng, N, crs)
    rng = np.random.default_rng(77)
    lo, hi = vdist.shard_range(Q, rank, world)
    data = rj_plus_i(rng, Q, N)
    z = rng.integers(0, N, size=Q, dtype=np.uint64)
    y = data.reshape(Q, N, 4)[np.arange(Q), z.astype(np.int64)].copy()
    # commitments of all queries (every rank needs all of them for the transcript), untimed
    d_all = torch.from_numpy(data.view(np.int64)).to(dev)
    cxy_d = torch.zeros((Q, 8), dtype=torch.int64, device=dev)
    cinf_d = torch.zeros(Q, dtype=torch.uint8, device=dev)
    meng.msm_batch_device(ipa.table, N, d_all.data_ptr(), Q, cxy_d.data_ptr(), cinf_d.data_ptr())
    torch.cuda.synchronize(dev)
    cxy = cxy_d.cpu().numpy().view(np.uint64).copy()
    cinf = cinf_d.cpu().numpy().copy()
    d_slice = d_all[lo * N:hi * N]
    g = dev if world > 1 else None

    def step():
        return vdist.multiproof_prove_sharded(ipa, cxy, cinf, z, y, d_slice.data_ptr(), rank, world, g)

    step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    # each proof timed alone, without per-kernel events (the median of 5: one host hiccup in a
    # 4-ms proof moved a 3-rep mean by 2 ms); then one pass with events for the kernel times
    reps = 5
    mp_ms = []
    for _ in range(reps):
        t0 = time.perf_counter()
        mp = step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        mp_ms.append((time.perf_counter() - t0) * 1e3)
    dt = float(np.median(mp_ms)) / 1e3
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    meng.enable_timing(True)
    meng.reset_timing()
    step()
    torch.cuda.synchronize(dev)
    kms = {}
    for k in ("mp_rpow", "mp_chunk", "mp_chunk_reduce", "mp_sum_parts", "mp_quot", "fb_commit"):
        ms, cnt = meng.kernel_time(k)
        if cnt:
            kms[k] = round(ms / cnt, 4)
    meng.enable_timing(False)
    # host transcript alone (the serial part every rank repeats)
    t0 = time.perf_counter()
    tr, _, _ = scheme.multiproof_begin(N, cxy, cinf, z, y)
    t_begin = time.perf_counter() - t0
    from vkzg._lib import lib
    lib().vc_transcript_free(tr)
    pipe = mp_pipelined(ipa, N, cxy, cinf, z, y, d_all, dev, mp) if world == 1 else None
    par = mp_proof_parallel(ipa, N, cxy, cinf, z, y, d_all, dev, rank, world, comm, mp) \
        if (world == 1 or comm is not None) else {"skipped": "no vc_comm for the proof exchange"}
    cpu = ({"data": data, "crs": crs, "threads": a.cpu_threads or min(16, os.cpu_count() or 1)}
           if (rank == 0 and world == 1 and not a.no_cpu_baseline) else None)
    ref_shapes = mp_reference_shapes(ipa, N, cxy, cinf, z, y, d_all, dev, cpu=cpu) if rank == 0 else None
    meng.close()
    alg = Q * N * 32 + Q * 64 + Q * 40
    out = {"workload": f"IPA multiproof, Q = 2^{a.mp_log_q} width-256 queries, BN254 (configs[4]), query set "
                       f"split over {world} rank(s)", "ms_per_multiproof": dt * 1e3,
           "ms_per_multiproof_all": [round(x, 3) for x in mp_ms],
           "host_transcript_ms": t_begin * 1e3, "kernel_ms": kms, "algorithmic_bytes_per_unit": alg,
           "achieved_GBps": alg / dt / 1e9, "d_inf": mp["d"] is None}
    if pipe is not None:
        out["pipelined"] = pipe
    if ref_shapes is not None:
        out["reference_bench_shapes"] = ref_shapes
    out["proof_parallel"] = par
    out["sliced_bound"] = ("the query-sliced single multiproof repeats the host transcript "
                           f"({t_begin * 1e3:.2f} ms) and the finish on every rank: at most ~1.15x on 8 GPUs "
                           "(DESIGN.md 6); proof_parallel scales with the ranks")
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_multiproof(N, data, z, cxy, cinf, crs, a.cpu_threads or min(16, os.cpu_count() or 1),
                                             mp["d"])
    return out


def mp_reference_shapes(ipa, N, cxy, cinf, z, y, d_all, dev, reps=5, cpu=None):
    """The reference's multiproof benches (vector-commit/benches/ipa.rs:111-159): prove_multiproof
    and verify_multiproof at Q = MAX_MULTIPROOF/8 x {1, 4, 8} = 4096, 16384, 32768 width-256 queries
    (the first Q of this line's query set; evaluations device-resident). Prove = the three phases
    (host transcript, per-point sums, finish with D, E and the inner IPA proof); verify =
    vc_multiproof_verify_ipa (transcript, the e-coefficient MSM over the Q commitments -- 8(f) rank
    2 -- and the inner IPA verification). Median of `reps` after a warm-up, each proof verified."""
    import ctypes
    from vkzg import scheme
    from vkzg._lib import check, lib
    out = {}
    for q in (4096, 16384, 32768):
        if q > z.shape[0]:
            break
        cq, ciq, zq, yq = (np.ascontiguousarray(v[:q]) for v in (cxy, cinf, z, y))

        def prove():  # phases 1 + 2 in one call: the transcript overlapped with the planning
            rows = scheme.multiproof_rows(N, zq)
            S = torch.empty((rows, N, 4), dtype=torch.int64, device=dev)
            torch.cuda.current_stream(dev).synchronize()
            tr, _r = scheme.multiproof_begin_accumulate(ipa.engine, N, cq, ciq, zq, yq, 0, q, d_all.data_ptr(),
                                                        S.data_ptr())
            return scheme.multiproof_finish(ipa, zq, S.data_ptr(), 1, tr)

        def verify(mp):
            b, _arrs = mp["proof"]._to()
            dxy, dinf = scheme._pt_arrays([mp["d"]])
            res = ctypes.c_int()
            check(lib().vc_multiproof_verify_ipa(ipa.engine.h, ipa.table, N, q, scheme._p(cq), scheme._p(ciq),
                                                 scheme._p(zq), scheme._p(yq), scheme._p(dxy), int(dinf[0]),
                                                 ctypes.byref(b), ctypes.byref(res)), "multiproof_verify")
            return bool(res.value)

        mp = prove()
        ok = verify(mp)
        tp, tv = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            mp = prove()
            tp.append((time.perf_counter() - t0) * 1e3)
            t0 = time.perf_counter()
            ok = verify(mp) and ok
            tv.append((time.perf_counter() - t0) * 1e3)
        out[str(q)] = {"prove_ms_median": float(np.median(tp)), "verify_ms_median": float(np.median(tv)),
                       "prove_ms": [round(x, 3) for x in tp], "verify_ms": [round(x, 3) for x in tv],
                       "verified": ok}
        if cpu is not None:  # the CPU restatement of the same prove and verify, real challenges
            data_q = cpu["data"][:q * N]
            pr = cpu_multiproof(N, data_q, zq, cq, ciq, cpu["crs"], cpu["threads"], mp["d"])
            vf = cpu_multiproof_verify(N, cq, ciq, zq, yq, cpu["crs"][:N])
            out[str(q)]["cpu_baseline"] = {"prove_ms": pr["ms_per_multiproof"], "prove_cores": pr["cores"],
                                           "prove_same_d_as_gpu": pr["same_d_as_gpu"],
                                           "prove_parts_ms": pr["parts_ms"], "verify_ms": vf["ms"],
                                           "verify_cores": vf["cores"], "verify_parts_ms": vf["parts_ms"],
                                           "kind": "port", "sample": pr["sample"] + "; verify: " + vf["sample"]}
    return out


def mp_proof_parallel(ipa, N, cxy, cinf, z, y, d_all, dev, rank, world, comm, want, per_rank=4, reps=3):
    """Proof-parallel multiproofs (the throughput mode of configs[4] on N GPUs): P = per_rank x N
    independent multiproofs of the line's Q queries; rank k proves its shard_range(P) proofs end
    to end (vc_multiproof_prove_many: transcripts on host threads beside the GPU sums, D / E commits
    and inner IPA proofs batched over its proofs) and one all-gather of the finished proofs
    (vc_multiproof_prove_many_sharded) gives every rank all P. Every proof is the same query set
    (the cost does not depend on the values); each is checked against the single-proof result."""
    from vkzg import scheme
    P = per_rank * world
    lo, hi = vdist.shard_range(P, rank, world)
    mine = hi - lo
    tile = lambda a: np.ascontiguousarray(np.broadcast_to(a, (P,) + a.shape))  # noqa: E731
    cx, ci, zz, yy = tile(cxy), tile(cinf), tile(z), tile(y)
    d_mine = d_all.repeat(mine, 1) if mine > 0 else None
    torch.cuda.synchronize(dev)

    def step():
        if world == 1:
            return scheme.prove_multiproof_many(ipa, cx, ci, zz, yy, d_mine.data_ptr())
        return comm.multiproof_many(ipa, cx, ci, zz, yy, d_mine.data_ptr() if d_mine is not None else 0)

    first = step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        got = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = (time.perf_counter() - t0) / reps
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    same = len(got) == P and all(g["d"] == want["d"] and g["proof"].as_dict() == want["proof"].as_dict()
                                 for g in got + first)
    del d_mine
    return {"proofs": P, "proofs_per_rank": per_rank, "ms_per_batch": dt * 1e3, "multiproofs_per_s": P / dt,
            "ms_per_multiproof_amortised": dt / P * 1e3, "same_proofs_as_single": same,
            "exchange": "vc_multiproof_prove_many_sharded (vc_comm all-gather of finished proofs)" if world > 1
            else "one GPU: vc_multiproof_prove_many"}


def mp_pipelined(ipa, N, cxy, cinf, z, y, d_all, dev, want, P=9):
    """A stream of P multiproofs through the three-phase ABI: phase 1 (the host transcript over all
    queries, vc_multiproof_begin -- pure host code, ctypes drops the GIL) of proof k + 1 runs on a
    second host thread while proof k's accumulate and finish (GPU, then the IPA rounds) run: what a
    caller proving several multiproofs (several blocks) gets from the library as it is. Same query
    set every time (the cost does not depend on the values); every proof is checked against the
    unpipelined one."""
    from concurrent.futures import ThreadPoolExecutor
    from vkzg import scheme
    Q = z.shape[0]

    def back(begun):
        tr, r, rows = begun
        S = torch.empty((rows, N, 4), dtype=torch.int64, device=dev)
        torch.cuda.current_stream(dev).synchronize()
        scheme.multiproof_accumulate(ipa.engine, N, z, 0, Q, d_all.data_ptr(), r, S.data_ptr())
        return scheme.multiproof_finish(ipa, z, S.data_ptr(), 1, tr)

    def run(depth):
        # up to `depth` transcripts in flight on host threads (the serial SHA-256 of one transcript
        # is longer than one proof's GPU phases) while the main thread runs proof k's phases 2 + 3
        with ThreadPoolExecutor(depth) as pool:
            back(pool.submit(scheme.multiproof_begin, N, cxy, cinf, z, y).result())  # warm
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            futs = [pool.submit(scheme.multiproof_begin, N, cxy, cinf, z, y) for _ in range(min(depth, P))]
            ok = True
            for k in range(P):
                begun = futs.pop(0).result()
                if k + depth < P:
                    futs.append(pool.submit(scheme.multiproof_begin, N, cxy, cinf, z, y))
                got = back(begun)
                ok = ok and got["d"] == want["d"] and got["proof"].as_dict() == want["proof"].as_dict()
            torch.cuda.synchronize(dev)
            return (time.perf_counter() - t0) / P, ok

    depths = {d: run(d) for d in (1, 2, 3)}
    best = min(depths, key=lambda d: depths[d][0])
    dt = depths[best][0]
    return {"proofs": P, "ms_per_multiproof": dt * 1e3, "multiproofs_per_s": 1.0 / dt, "transcripts_in_flight": best,
            "same_proofs": all(ok for _, ok in depths.values()),
            "ms_per_multiproof_by_transcripts_in_flight": {str(d): v[0] * 1e3 for d, v in depths.items()},
            "note": "phase 1 (host transcript) of proofs k+1 .. k+d on d host threads, overlapped with proof k's "
                    "GPU phases and IPA rounds; ms_per_multiproof at the best d of 1, 2, 3 (all three listed)"}


BN254_P = 21888242871839275222246405745257275088696311157297823662689037894645226208583  # base field


def _mp_records(cxy, cinf, z, y):
    """The multiproof transcript's per-query bytes (multiproof.rs:109-113, transcript.rs:28-49):
    "C" ++ compressed(C_i) ++ "z" ++ le64(z_i) ++ "y" ++ le(y_i), 75 B each, with the compressed
    point's flags (x LE, 0x80 in the last byte when y is the larger root, 0x40 for the identity:
    SURVEY Appendix A.3) -- vectorised, so the baseline pays SHA-256 and not Python."""
    Q = z.shape[0]
    half = (BN254_P - 1) // 2
    hl = [(half >> (64 * k)) & ((1 << 64) - 1) for k in range(4)]
    yl = cxy[:, 4:8]
    gt = np.zeros(Q, dtype=bool)
    eq = np.ones(Q, dtype=bool)
    for k in (3, 2, 1, 0):
        gt |= eq & (yl[:, k] > np.uint64(hl[k]))
        eq &= yl[:, k] == np.uint64(hl[k])
    rec = np.zeros((Q, 75), dtype=np.uint8)
    rec[:, 0], rec[:, 33], rec[:, 42] = ord("C"), ord("z"), ord("y")
    rec[:, 1:33] = np.ascontiguousarray(cxy[:, :4]).view(np.uint8).reshape(Q, 32)
    rec[gt, 32] |= 0x80
    inf = cinf.astype(bool)
    rec[inf, 1:33] = 0
    rec[inf, 32] = 0x40
    rec[:, 34:42] = np.ascontiguousarray(z).view(np.uint8).reshape(Q, 8)
    rec[:, 43:75] = np.ascontiguousarray(y).view(np.uint8).reshape(Q, 32)
    return rec


def cpu_multiproof(N, data, z, cxy, cinf, crs, threads, gpu_d=None):
    """configs[4] on the CPU, the reference's prove_multiproof (multiproof.rs:99-176) restated with
    its real challenges: the transcript over the Q (C, z, y) records and hash_to_field -> r
    (oracle/pyoracle/arkser.py, transcript.rs:28-62), the field phases in C with the reference's
    thread structure (oracle/c/ref_multiproof.c: scaling par_iter over queries, grouped quotients
    par_bridge over points, g and h serial) on `threads` threads, D = commit(g) by the naive
    inner_product in C (utils.rs:16-19, what IPA::commit runs), t from the transcript, h, E =
    commit(h), and the inner IPA proof as its 8 rounds of L / R commits and generator folds (naive
    per-term scalar multiplications of the same sizes; work-equivalent). D is compared with the
    GPU's D of the same inputs (`same_d_as_gpu`)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import arkser, cref  # CPU baseline leg only
    from pyoracle import protocol
    Q = z.shape[0]
    r_mod = vkzg.SCALAR_R["bn254"]
    crs_xy, crs_inf = cref.points_to_array("bn254", crs)
    omega = protocol.group_gen(N)
    y = data.reshape(Q, N, 4)[np.arange(Q), z.astype(np.int64)]
    t0 = time.perf_counter()
    state = _mp_records(cxy, cinf, z, y).tobytes() + b"r"
    r = arkser.hash_to_field(state, b"multiproof", r_mod)
    t_tr = time.perf_counter() - t0
    t0 = time.perf_counter()
    st, g = cref.mp_g(N, data, z, r, omega, threads)
    t_field = time.perf_counter() - t0
    t0 = time.perf_counter()
    dxy, dinf = cref.msm_arrays("bn254", crs_xy[:N], crs_inf[:N], g, 1)
    t_commit = time.perf_counter() - t0
    t0 = time.perf_counter()
    d = cref.array_to_point("bn254", dxy, dinf)
    t = arkser.hash_to_field(arkser.ser_fr(r) + b"r" + b"D" + arkser.ser_point_compressed(d) + b"t",
                             b"multiproof", r_mod)
    h = cref.mp_h(st, N, t)
    cref.mp_free(st)
    t_field += time.perf_counter() - t0
    t0 = time.perf_counter()
    cref.msm_arrays("bn254", crs_xy[:N], crs_inf[:N], h, 1)
    t_commit += time.perf_counter() - t0
    t0 = time.perf_counter()
    m = N
    sc = np.asarray(g, dtype=np.uint64)
    while m > 1:                                      # L, R and the fold of G each round
        for _ in range(3):
            cref.msm_arrays("bn254", crs_xy[:m // 2], crs_inf[:m // 2], sc[:m // 2], 1)
        m //= 2
    t_ipa = time.perf_counter() - t0
    total = t_tr + t_field + t_commit + t_ipa
    return {"value": 1.0 / total, "unit": "multiproofs/s", "ms_per_multiproof": total * 1e3, "cores": threads,
            "kind": "port", "parts_ms": {"transcript_hash_to_field": t_tr * 1e3, "field_phases": t_field * 1e3,
                                         "d_e_commits_naive": t_commit * 1e3, "inner_ipa_naive": t_ipa * 1e3},
            "same_d_as_gpu": (d == gpu_d) if gpu_d is not None else None,
            "sample": f"the full Q = {Q} x N = {N} workload once with the transcript's own r and t: field phases "
                      f"in C on {threads} threads with the reference's rayon structure (oracle/c/ref_multiproof.c), "
                      "naive D / E commits and IPA rounds in C (1 thread, as the reference's serial IPA; the "
                      "rounds are work-equivalent), SHA-256 transcript and hash_to_field"}


def _naive_ms(cref, xy, inf, sc):
    """one naive MSM (utils.rs:16-19 restated in C, 1 thread): wall ms"""
    t0 = time.perf_counter()
    cref.msm_arrays("bn254", xy, inf, sc, 1)
    return (time.perf_counter() - t0) * 1e3


def cpu_multiproof_verify(N, cxy, cinf, z, y, crs, sample=512):
    """verify_multiproof (multiproof.rs:178-215) on the CPU, restated: the transcript over the Q
    (C, z, y) records + hash_to_field (r), t, the e-coefficient MSM over the Q commitments as the
    naive inner_product (utils.rs:16-19; timed on `sample` terms and extrapolated linearly to Q),
    and the inner IPA verification (low_level_verify_ipa, ipa/mod.rs:321-360: 2 scalar
    multiplications per round and the 256-point naive MSM <g, s>)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import arkser, cref  # CPU baseline leg only
    Q = z.shape[0]
    r_mod = vkzg.SCALAR_R["bn254"]
    t0 = time.perf_counter()
    arkser.hash_to_field(_mp_records(cxy, cinf, z, y).tobytes() + b"r", b"multiproof", r_mod)
    t_tr = (time.perf_counter() - t0) * 1e3
    m = min(sample, Q)
    sc = vkzg.random_scalars("bn254", m, np.random.default_rng(6))
    t_e = _naive_ms(cref, cxy[:m], cinf[:m], sc) * Q / m
    crs_xy, crs_inf = cref.points_to_array("bn254", crs)
    K = N.bit_length() - 1
    s2 = vkzg.random_scalars("bn254", max(N, 2), np.random.default_rng(8))
    t_ipa = sum(_naive_ms(cref, crs_xy[:2], crs_inf[:2], s2[:2]) for _ in range(K))
    t_ipa += _naive_ms(cref, crs_xy[:N], crs_inf[:N], s2[:N])
    total = t_tr + t_e + t_ipa
    return {"ms": total, "cores": 1, "kind": "port",
            "parts_ms": {"transcript_hash_to_field": t_tr, "e_msm_naive": t_e, "inner_ipa_verify_naive": t_ipa},
            "sample": f"transcript over all {Q} queries; the e-coefficient naive MSM timed on {m} of the {Q} "
                      "commitments and extrapolated linearly; the inner IPA verification's scalar multiplications "
                      "and 256-point MSM in C, 1 thread"}


def cpu_ipa_single(crs, N=256):
    """benches/ipa.rs:85-109 on the CPU (1 thread, the reference's serial prover/verifier), work-
    equivalent in C: prove = low_level_ipa's log2 N rounds, each two half-size naive MSMs (L, R), a
    generator fold of m/2 scalar multiplications (vec_add_and_distribute on points) and two
    multiplications by q' (ipa/mod.rs:268-319); verify = 2 scalar multiplications per round and the
    N-point naive MSM <g, s> (:321-360). Median of 3."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import cref  # CPU baseline leg only
    xy, inf = cref.points_to_array("bn254", crs)
    sc = vkzg.random_scalars("bn254", N, np.random.default_rng(10))

    def prove():
        t, m = 0.0, N
        while m > 1:
            h = m // 2
            t += 3 * _naive_ms(cref, xy[:h], inf[:h], sc[:h]) + _naive_ms(cref, xy[:2], inf[:2], sc[:2])
            m = h
        return t

    def verify():
        K = N.bit_length() - 1
        return sum(_naive_ms(cref, xy[:2], inf[:2], sc[:2]) for _ in range(K)) + _naive_ms(cref, xy[:N], inf[:N], sc)

    p = float(np.median([prove() for _ in range(3)]))
    v = float(np.median([verify() for _ in range(3)]))
    return {"prove_ms": p, "verify_ms": v, "cores": 1, "kind": "port",
            "sample": f"N = {N}: the rounds' naive MSMs and scalar multiplications in C (oracle/c/ref_curve.c), "
                      "1 thread, median of 3 (work-equivalent: the same MSM sizes and scalar multiplications)"}


def kzg_reference_shapes(local, stream, cpu=True):
    """The reference's KZG benches (vector-commit/benches/kzg.rs:45-75) on BN254: KZG::setup at
    32 / 2048 / 4096 / 16384 (vc_kzg_setup: the Lagrange SRS on the GPU), commit of 20 values over a
    32-point CRS, and a single proof at an in-range index; GPU medians, and beside them the CPU port:
    setup = max_items scalar multiplications (s^i G, kzg_point_generator.rs:32-43) + the G1 iFFT's
    n/2 log2 n twiddle multiplications (kzg/mod.rs:119-121), timed on a sample and extrapolated;
    commit = the 20-term naive MSM; proof = divide_by_vanishing in C (lagrange_basis.rs:91-119) +
    the 32-term naive MSM."""
    import ctypes
    from vkzg import scheme
    from vkzg._lib import check, lib
    e = vkzg.Engine("bn254", local)
    e.set_stream(stream.cuda_stream)
    out = {"workload": "KZG on BN254, benches/kzg.rs shapes (DATA_SIZE 20, MAX_CRS 32; setup 32..16384)"}
    secret = vkzg.ints_to_limbs([100])[0].copy()

    def med(f, reps=7):
        f()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            f()
            ts.append((time.perf_counter() - t0) * 1e3)
        return float(np.median(ts))

    def setup_once(size):
        tid, sz = ctypes.c_int(), ctypes.c_size_t()
        check(lib().vc_kzg_setup(e.h, size, ctypes.c_void_p(secret.ctypes.data), ctypes.byref(tid), ctypes.byref(sz)),
              "vc_kzg_setup")

    out["setup_ms"] = {str(sz): med(lambda: setup_once(sz), reps=3) for sz in (32, 2048, 4096, 16384)}
    kz = scheme.KZG(e, 32)
    rng = np.random.default_rng(12)
    data = scheme.LagrangeBasis([int(v) for v in rng.integers(0, 1 << 62, size=20)], 32)
    com = kz.commit(data)
    out["commit_ms_pippenger"] = med(lambda: kz.commit(data))
    out["single_proof_ms_pippenger"] = med(lambda: kz.prove(com, 7, data))
    prf = kz.prove(com, 7, data)
    # the SRS's fixed-base windows (setup, untimed -- a fixed CRS): vc_msm's small commits then take
    # the fixed-base latency path
    e.fixed_base_precompute(kz.table, 8)
    out["commit_ms"] = med(lambda: kz.commit(data))
    out["commit_same_result"] = kz.commit(data) == com
    out["single_proof_ms"] = med(lambda: kz.prove(com, 7, data))
    out["single_proof_same_result"] = kz.prove(com, 7, data) == prf
    e.close()
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from pyoracle import cref, protocol  # CPU baseline leg only
        ceng = vkzg.Engine("bn254", local)
        try:
            tid = ceng.random_bases(512, seed=21)
            xy, inf = ceng.download_bases(tid)
        finally:
            ceng.close()
        sc = vkzg.random_scalars("bn254", 512, np.random.default_rng(13))
        per_mul = _naive_ms(cref, xy, inf, sc) / 512          # one naive scalar multiplication (+ add)
        setup = {}
        for sz in (32, 2048, 4096, 16384):
            setup[str(sz)] = per_mul * (sz + sz // 2 * (sz.bit_length() - 1))
        dl = vkzg.ints_to_limbs([int(v) for v in data.evals] + [0] * 12)
        omega = protocol.group_gen(32)

        def proof():
            st, _g = cref.mp_g(32, dl, np.array([7], dtype=np.uint64), 1, omega, 1)
            cref.mp_free(st)
            cref.msm_arrays("bn254", xy[:32], inf[:32], sc[:32], 1)

        t_c = float(np.median([_naive_ms(cref, xy[:20], inf[:20], sc[:20]) for _ in range(5)]))
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            proof()
            ts.append((time.perf_counter() - t0) * 1e3)
        out["cpu_baseline"] = {"setup_ms": setup, "commit_ms": t_c, "single_proof_ms": float(np.median(ts)),
                               "cores": 1, "kind": "port",
                               "sample": f"setup: {per_mul * 1e3:.1f} us per naive scalar multiplication (a 512-term "
                                         "naive MSM in C) x (max_items + n/2 log2 n iFFT twiddles), extrapolated; "
                                         "commit: the 20-term naive MSM; proof: divide_by_vanishing in C "
                                         "(oracle/c/ref_multiproof.c) + the 32-term naive MSM; 1 thread, medians"}
    return out


def _log2_int(n):
    k = 0
    while (1 << k) < n:
        k += 1
    return k


def ipa_line(local, stream, batch=256, cpu=False):
    """The reference's IPA bench shapes (vector-commit/benches/ipa.rs:79-109, N = 256, BN254,
    data r + i): single commit, prove in / out of domain, verify in domain -- latency of one
    call each -- and a batch of independent proofs in one vc_ipa_prove call (proofs/s)."""
    from vkzg import scheme
    ieng = vkzg.Engine("bn254", local)
    ieng.set_stream(stream.cuda_stream)
    N = 256
    ipa = scheme.IPA(ieng, N, scheme.ipa_crs(N + 1, max_=512))
    r0 = 0x1234567890ABCDEF1234567890ABCDEF
    datas = [scheme.LagrangeBasis([(r0 * (k + 1) + i) % scheme.R_BN254 for i in range(N)]) for k in range(batch)]
    coms = ipa.commit_batch(datas)

    def timed(f, reps=7):  # the median of single calls: one preempted call (a 2.8 ms verify seen once
        f()                # against 0.27-0.33 in every other run) must not move a latency line
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = f()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3, r

    out = {"workload": "IPA N = 256 on BN254 (benches/ipa.rs shapes, data r + i)"}
    out["commit_ms"], _ = timed(lambda: ipa.commit(datas[0]))
    out["prove_in_domain_ms"], prf = timed(lambda: ipa.prove_point(coms[0], 77, datas[0]))
    # the same proof through the bare C ABI (vc_ipa_prove on inputs marshalled once): the library's
    # latency without the Python mirror's conversions (tools/ipa_abi_probe.py)
    import ctypes
    from vkzg._lib import lib as _lib, check as _check
    d0 = np.ascontiguousarray(datas[0].limbs(N)[:N])
    cxy0, cinf0 = scheme._pt_arrays([coms[0]])
    pt0 = vkzg.ints_to_limbs([77], 4)
    pbuf, parrs = scheme.IPAProof._alloc(_log2_int(N))
    parr = (scheme._ProofBuf * 1)(pbuf)

    def abi_prove():
        _check(_lib().vc_ipa_prove(ieng.h, ipa.table, N, scheme._p(d0), scheme._p(cxy0), scheme._p(cinf0),
                                   scheme._p(pt0), 1, None, ctypes.cast(parr, scheme._P)), "ipa_prove")
    out["prove_in_domain_ms_c_abi"], _ = timed(abi_prove)
    if scheme.IPAProof._from(parr[0], parrs).as_dict() != prf.as_dict():
        raise SystemExit("bench: the bare vc_ipa_prove call gave a different proof")
    out["prove_out_domain_ms"], _ = timed(lambda: ipa.prove_point(coms[0], N * 7 + 3, datas[0]))
    out["verify_in_domain_ms"], ok = timed(lambda: ipa.verify_point(coms[0], 77, prf))
    assert ok
    pts = [(31 * k) % N for k in range(batch)]
    ms, _ = timed(lambda: ipa.prove_batch_points(coms, pts, datas), reps=2)
    out["batch_prove"] = {"proofs": batch, "ms": ms, "proofs_per_s": batch / ms * 1e3}
    out["concurrent_contexts"] = ipa_concurrent(N, datas, coms)
    ieng.close()
    if cpu:
        out["cpu_baseline"] = cpu_ipa_single(scheme.ipa_crs(N + 1, max_=512)[:N])
    return out


def ipa_concurrent(N, datas, coms, per=16):
    """Single prove_point calls from T host threads, each with its own context (own stream, own
    CRS copy) -- the overlap a rayon caller gets with one vc_ctx per worker (one shared context
    serialises its calls on the context mutex): proofs/s at T = 1, 2, 4."""
    import threading
    from vkzg import scheme
    crs = scheme.ipa_crs(N + 1, max_=512)
    res = {}
    for T in (1, 2, 4):
        engs = [vkzg.Engine("bn254", torch.cuda.current_device()) for _ in range(T)]
        try:
            ipas = [scheme.IPA(e, N, crs) for e in engs]
            for k in range(T):  # warm-up (workspaces, fixed-base tables)
                ipas[k].prove_point(coms[k], 77, datas[k])

            def worker(k):
                for j in range(per):
                    i = k * per + j
                    ipas[k].prove_point(coms[i % len(coms)], (31 * i) % N, datas[i % len(datas)])

            th = [threading.Thread(target=worker, args=(k,)) for k in range(T)]
            t0 = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            dt = time.perf_counter() - t0
            res[str(T)] = {"proofs": T * per, "ms": dt * 1e3, "proofs_per_s": T * per / dt}
        finally:
            for e in engs:
                e.close()
    res["note"] = ("one vc_ctx per host thread; each thread proves its share with single "
                   "prove_point calls (latency-bound dependent rounds)")
    return res


def verkle_line(a, local, stream):
    """verkle-tree commitment (lib.rs:127-129 / node.rs:205-277) over a
    KZG(256) Lagrange SRS on BN254, 32-unit keys (Ethereum-style 31-byte stem + suffix), random
    32-byte values: the median full commitment of --verkle-reps fresh trees (after an untimed
    warm-up commitment of an identical tree) and the median of --verkle-reps rounds of 1 % key
    updates (only the dirty nodes of each level recommitted, one batched launch per level); every
    root checked (result_check)."""
    from vkzg import scheme
    from vkzg.verkle import VerkleTree
    veng = vkzg.Engine("bn254", local)
    veng.set_stream(stream.cuda_stream)
    kzg = scheme.KZG(veng, 256)
    rng = np.random.default_rng(91)
    nk = a.verkle_keys
    keys = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
    vals = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
    # the SRS fixed-base tables, untimed (setup): 16-bit windows (16 per scalar, 17.2 GB for the 256
    # Lagrange points) -- half the table points per non-zero of c = 8's 32 windows: full commitment
    # 3.47-3.60 -> 3.03-3.07 ms (profiles/r05/verkle/fb_c/)
    veng.fixed_base_precompute(kzg.table, 16)
    # warm-up: one full commitment of an identical tree and one 1 % update of it (first-use
    # workspace and page-locked staging allocations of both paths; other keys than the timed update's)
    w = VerkleTree(32)
    for i in range(nk):
        w.insert_single(keys[i].tobytes(), vals[i].tobytes())
    w.commitment(veng, kzg.table)
    wrng = np.random.default_rng(17)
    for i in wrng.integers(0, nk, size=max(1, nk // 100)):
        w.insert_single(keys[i].tobytes(), wrng.integers(0, 256, size=32, dtype=np.uint8).tobytes())
    w.commitment(veng, kzg.table)
    del w
    # the kernel totals of a full commitment: an identical tree committed with per-kernel events;
    # its root is the reference every timed commitment below is checked against
    k = VerkleTree(32)
    for i in range(nk):
        k.insert_single(keys[i].tobytes(), vals[i].tobytes())
    veng.enable_timing(True)
    veng.reset_timing()
    root_k = k.commitment(veng, kzg.table)
    veng.enable_timing(False)
    del k
    kms = {}
    # every launch name the verkle paths time (csrc VK_LAUNCH names; the fused sparse kernels and the
    # latency path's sparse_small were missing before round 6's last rehearsal, which overstated the
    # host share by their ~0.1 ms)
    for kn in ("sparse_count", "sparse_expand", "sparse_rows", "sparse_count_scan", "sparse_expand_rows",
               "sparse_small", "sparse_accumulate", "msm_fixup_init", "msm_fixup_jump", "msm_fixup", "sparse_store",
               "sparse_combine", "sparse_add_base", "norm_prep", "norm_finish", "fb_normalize", "fb_commit",
               "fb_combine", "fb_commit_small", "to_data_item", "sparse_iota", "verkle_widen", "verkle_ext_rows4",
               "verkle_rp4", "verkle_delta", "verkle_gather", "verkle_dense", "verkle_scatter"):
        ms, cnt = veng.kernel_time(kn)
        if cnt:
            kms[kn] = round(ms, 3)
    gpu_ms = sum(kms.values())
    # full commitments: FRESH trees (nothing committed yet), timed without per-kernel events, each
    # root compared with tree k's
    fulls, t_ins, st, same_full = [], [], None, True
    for _ in range(a.verkle_reps):
        t = VerkleTree(32)
        t0 = time.perf_counter()
        for i in range(nk):
            t.insert_single(keys[i].tobytes(), vals[i].tobytes())
        t_ins.append(time.perf_counter() - t0)
        st = t.stats()
        t0 = time.perf_counter()
        root = t.commitment(veng, kzg.table)
        fulls.append(time.perf_counter() - t0)
        same_full &= root == root_k
        del t
    # 1 % updates: rounds of nk / 100 rewritten keys on one tree (dirty nodes only, delta rows)
    t = VerkleTree(32)
    for i in range(nk):
        t.insert_single(keys[i].tobytes(), vals[i].tobytes())
    t.commitment(veng, kzg.table)
    upd = max(1, nk // 100)
    upds, dirty, history = [], [], []
    for _ in range(a.verkle_reps):
        for i in rng.choice(nk, size=upd, replace=False):
            history.append((keys[i].tobytes(), rng.integers(0, 256, size=32, dtype=np.uint8).tobytes()))
            t.insert_single(*history[-1])
        dirty.append(t.stats()["dirty"])
        t0 = time.perf_counter()
        root_u = t.commitment(veng, kzg.table)
        upds.append(time.perf_counter() - t0)
    # the last update's root == a fresh tree with the same insertion history committed in full
    # (untimed). Not the final contents inserted once: the reference's level-skipping splits
    # (node.rs:176-185) make the trie depend on the order, and re-inserting a key below such a
    # split can add a second extension for it (an oracle replay of this bench's first round: 65,537
    # extensions against 65,536), so that tree may have another shape and root
    f = VerkleTree(32)
    for i in range(nk):
        f.insert_single(keys[i].tobytes(), vals[i].tobytes())
    for kv in history:
        f.insert_single(*kv)
    same_upd = f.commitment(veng, kzg.table) == root_u
    del f, t
    veng.close()
    if not (same_full and same_upd):
        raise SystemExit(f"bench: verkle result check FAILED (full {same_full}, update {same_upd})")
    full_med = float(np.median(fulls))
    return {"workload": f"verkle tree, {nk} random 32-unit keys, KZG(256) BN254 (8(f) rank 1)",
            "srs_fixed_base": "16-bit windows, 16 per scalar, 17.2 GB (setup, untimed)",
            "nodes": st, "insert_s": float(np.median(t_ins)),
            "reps": a.verkle_reps,
            "full_commitment_ms": full_med * 1e3,
            "full_commitment_ms_all": [round(x * 1e3, 3) for x in fulls],
            "nodes_per_s_full": st["dirty"] / full_med, "full_kernel_ms_total": kms,
            "full_split_ms": {"gpu_kernels": gpu_ms, "host_and_transfers": full_med * 1e3 - gpu_ms,
                              "host_and_transfers_frac": 1 - gpu_ms / (full_med * 1e3),
                              "note": "kernels from one commitment with per-kernel events; wall = median of the fresh trees"},
            "updated_keys": upd, "dirty_nodes": int(np.median(dirty)),
            "update_commitment_ms": float(np.median(upds)) * 1e3,
            "update_commitment_ms_all": [round(x * 1e3, 3) for x in upds],
            "result_check": {"ok": True,
                             "method": "every fresh tree's root == tree k's (committed with events); the last "
                                       "update's root == a fresh tree with the same insertion history "
                                       "committed in full"}}


def launch_ranks(a, argv):
    """`--gpus N` (N > 1) without a launcher: start N rank processes under torch.distributed.run
    (127.0.0.1, a free port) running this same command line, and return their exit status. Runs
    BEFORE anything touches HIP in this process (no vkzg.lib(), no torch.cuda call): the ranks are
    children, never an exec of a process that initialised the GPU. Rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    progress(f"--gpus {a.gpus} without WORLD_SIZE: launching {a.gpus} ranks ({' '.join(cmd[1:7])} ...)")
    return subprocess.call(cmd)


def launch_check(a):
    """--launch-check: the rank bookkeeping alone (gloo, no GPU): rank 0 prints the world and the
    ranks that reported (tests/test_bench_launch.py runs `bench.py --gpus 2 --launch-check`)"""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
        got = [None] * world
        dist.all_gather_object(got, {"rank": rank, "pid": os.getpid()})
        dist.destroy_process_group()
    else:
        got = [{"rank": rank, "pid": os.getpid()}]
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "gpus_flag": a.gpus, "ranks": got}), flush=True)


def world_from_env(a):
    """the world this process belongs to; refuses a --gpus that disagrees with a launcher's WORLD_SIZE"""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in os.environ and a.gpus != world:
        raise SystemExit(f"bench: --gpus {a.gpus} disagrees with WORLD_SIZE={world} set by the launcher")
    if not a.rehearse_one_gpu and not a.launch_check and world > 1:
        ndev = torch.cuda.device_count()  # (counting devices does not initialise HIP on this image)
        if world > ndev:
            raise SystemExit(f"bench: {world} ranks but {ndev} visible GPU(s); --rehearse-one-gpu puts every rank on device 0")
    return world


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a, sys.argv[1:]))
    world = world_from_env(a)
    if a.launch_check:
        launch_check(a)
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.rehearse_one_gpu:  # every rank on device 0, gloo + host-callback exchange (see --help)
        local = 0
        a.commit_window = 16  # the ranks share one card's HBM: no 188 GB c = 20 table per rank
    if world > 1:
        dist.init_process_group("gloo" if a.rehearse_one_gpu else "nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)

    curve, n = a.curve, 1 << a.log_n
    eng = vkzg.Engine(curve, local)
    eng.set_stream(stream.cuda_stream)
    # identical synthetic inputs on every rank (same seeds); each rank keeps its shard
    table = eng.random_bases(n, seed=2024)
    rng = np.random.default_rng(1234)
    scalars = vkzg.random_scalars(curve, n, rng)
    d_sc = torch.from_numpy(scalars.view(np.int64).copy()).to(dev)

    # N > 1: the exchange goes through the C ABI (include/vc_comm.h: vc_msm_sharded over a
    # vc_comm on RCCL, the path a Rust caller of libvkzg.so uses); the unique id travels over
    # the torch.distributed group. --comm torch keeps the Python all-gather (vkzg.dist).
    comm, comm_kind = None, "none" if world == 1 else a.comm
    if world > 1 and a.rehearse_one_gpu:
        from vkzg import comm as vcomm
        comm, comm_kind = vcomm.Comm.host(rank, world, vcomm.torch_allgather()), "vc_comm host callback (gloo)"
    elif world > 1 and a.comm == "capi":
        from vkzg import comm as vcomm
        obj = [vcomm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        try:
            comm = vcomm.Comm.rccl(local, rank, world, obj[0])
        except Exception as ex:  # no usable RCCL through the C ABI: torch's all-gather instead
            print(f"[bench] vc_comm_init_rccl failed ({ex}); using the torch.distributed exchange",
                  file=sys.stderr, flush=True)
            comm_kind = "torch (vc_comm init failed)"
        ok = torch.tensor([0 if comm is None else 1], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0 and comm is not None:  # every rank must take the same path
            comm.close()
            comm, comm_kind = None, "torch (vc_comm init failed on a peer)"
    split = msm_split(a, world)
    if comm is not None:
        comm.set_msm_split(comm.SPLIT_POINTS if split == "points" else comm.SPLIT_WINDOWS)
    plo, _phi = vdist.shard_range(n, rank, world)

    def step():
        if world == 1:  # one call: vc_msm_device (sort .. reduction, host fold, affine result)
            return eng.msm_device(table, d_sc.data_ptr(), n)
        if comm is not None:  # window slice or point range (HIP) -> vc_comm RCCL all-gather -> host sum, all in C
            return comm.msm(eng, table, d_sc.data_ptr(), n)
        # partial (HIP) -> torch RCCL all-gather of projective partials -> host sum
        return vdist.msm_sharded(eng, table, d_sc.data_ptr() + (plo * 32 if split == "points" else 0), n, rank, world,
                                 dev if world > 1 else None, split=split)

    for _ in range(a.warmup):
        res = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # the timed region runs WITHOUT per-kernel HIP events: an event recorded between two kernels
    # of one stream holds the next dispatch ~10 us (profiles/r05/event_gaps/), i.e. ~0.1 ms of the
    # ~11-kernel pipeline; the kernel durations come from a second pass below
    step_ms = []  # every step returns its host result (the call is synchronous): per-step times
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ts = time.perf_counter()
        res = step()
        step_ms.append((time.perf_counter() - ts) * 1e3)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    plan = eng.msm_last_plan()  # the geometry the timed MSMs ran (before the 1-term result check)
    # kernel-timing pass: the same K steps with HIP events around every launch (on the stream the
    # kernels run on); its wall time is reported beside the headline as ms_per_step_with_events
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    eng.enable_timing(True)
    eng.reset_timing()
    t0e = time.perf_counter()
    for _ in range(a.steps):
        res_e = step()
    torch.cuda.synchronize(dev)
    dt_events = time.perf_counter() - t0e
    eng.enable_timing(False)
    if not (int(res_e[1]) == int(res[1]) and np.array_equal(np.asarray(res_e[0]), np.asarray(res[0]))):
        raise SystemExit("bench: the kernel-timing pass gave a different MSM result")
    acc_mhz, acc_clk_n = eng.accumulate_clock()
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        tm = torch.tensor(step_ms, dtype=torch.float64, device=dev)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)  # per-step max over ranks
        step_ms = tm.cpu().tolist()
    ms_per_step = dt / a.steps * 1e3

    # dominant kernel (bucket accumulation) device time, HIP events on the launch stream
    acc_ms, acc_n = eng.kernel_time("msm_accumulate")
    kernels = kernel_table(eng)

    # one-time result check, outside the timed region: the bases are P_i = s_i G with s_i
    # re-derived on the host (vkzg.random_base_scalars), so sum k_i P_i = t P_0 with
    # t = (sum k_i s_i) / s_0 mod r -- a 1-term MSM on the same table (tests/test_gpu_fullsize.py
    # pins the same identity against the oracle's group law)
    check = None
    if not a.no_check:
        r_mod = vkzg.SCALAR_R[curve]
        s_all = vkzg.random_base_scalars(curve, 2024, n)
        t = vkzg.dot_mod(scalars, s_all, r_mod) * pow(vkzg.limbs_to_int(s_all[0]), -1, r_mod) % r_mod
        want = eng.msm(table, vkzg.ints_to_limbs([t]), offset=0)
        ok = bool(int(res[1]) == want[1] and np.array_equal(np.asarray(res[0]), want[0]))
        check = {"ok": ok, "method": "sum k_i P_i == ((sum k_i s_i) / s_0 mod r) P_0, P_i = s_i G (host-derived s_i)"}
        if not ok:
            raise SystemExit(f"bench: 2^{a.log_n} MSM result check FAILED: {res} vs {want}")

    progress(f"headline: {ms_per_step:.3f} ms per MSM")
    # variable-base sub-line: the same MSM without the per-table shifted window copies
    # (VC_OPT_MSM_SHARED_WINDOWS = 0): plain Pippenger, W bucket sets, no precomputation
    variable = None
    if not a.no_variable_base and curve == "bls12_381":
        eng.set_option(eng.OPT_MSM_SHARED_WINDOWS, 0)
        for _ in range(max(1, a.warmup)):
            vres = step()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        eng.reset_timing()
        eng.enable_timing(True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            vres = step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        vdt = time.perf_counter() - t0
        eng.enable_timing(False)
        if world > 1:
            tt = torch.tensor([vdt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            vdt = float(tt.item())
        vacc_ms, vacc_n = eng.kernel_time("msm_accumulate")
        eng.set_option(eng.OPT_MSM_SHARED_WINDOWS, 1)
        vsame = bool(int(vres[1]) == int(res[1]) and np.array_equal(np.asarray(vres[0]), np.asarray(res[0])))
        vk_ms = vacc_ms / vacc_n if vacc_n else None
        variable = {"ms_per_msm": vdt / a.steps * 1e3, "value": a.steps / vdt, "unit": "2^20-pt MSM/s",
                    "precomputed_bases": None, "same_result": vsame,
                    "kernel_ms": kernel_table(eng),
                    "roofline": {"kernel": "msm_accumulate", "kernel_ms": vk_ms,
                                 "achieved": (n * BYTES_PER_POINT[curve] + OUT_BYTES[curve]) / world / (vk_ms * 1e-3) / 1e9
                                 if vk_ms else None, "peak": HBM_PEAK_GBS, "unit": "GB/s"}}
        if variable["roofline"]["achieved"]:
            variable["roofline"]["frac"] = variable["roofline"]["achieved"] / HBM_PEAK_GBS

    # host-scalar latency: vc_msm with the scalars in (pageable) host memory -- the entry point
    # INTEGRATION.md's Rust binding calls; adds the 32 MB H2D copy over PCIe to every MSM
    host_line = None
    if world == 1:
        eng.msm(table, scalars)
        t0 = time.perf_counter()
        hreps = 5
        for _ in range(hreps):
            eng.msm(table, scalars)
        hdt = (time.perf_counter() - t0) / hreps
        host_line = {"ms_per_msm": hdt * 1e3, "h2d_bytes": int(scalars.nbytes),
                     "note": "vc_msm, scalars in pageable host memory (PCIe copy inside the call); not `value`"}
    acc_s = acc_ms / acc_n * 1e-3 if acc_n else None
    # algorithmic bytes of this rank's share of the MSM (n*(96+32) + 96 per MSM)
    shard_bytes = (n * BYTES_PER_POINT[curve] + OUT_BYTES[curve]) / world
    achieved = shard_bytes / acc_s / 1e9 if acc_s else None
    # VALU roofline: the accumulate's executed VALU instructions (PMC SQ_INSTS_VALU per launch,
    # wave-level, from the committed profile of this same command) x 64 lanes / its live time,
    # against the live issue peak of 4-cycle VALU work (v_mad_u64_u32; VCC adds issue the same,
    # plain 32-bit adds in half: tools/issueprobe.hip), i.e. lanes x SIMDs x clock / 4
    c_bits, w_total, terms = plan["window_bits"], plan["windows"], plan["terms_per_point"]
    w_rank = (rank + 1) * w_total // world - rank * w_total // world
    madds = terms * n * w_rank if (world == 1 or split == "windows") else terms * (_phi - plo) * w_total
    mad_peak = eng.device_mad_rate()
    pmc = json.load(open(PMC_SUMMARY)) if os.path.exists(PMC_SUMMARY) else None
    # the committed counters count only if they were taken on this geometry (same n, windows, radix)
    pmc_match = bool(pmc) and all(pmc.get("config", {}).get(k) == v for k, v in
                                  (("log_n", a.log_n), ("windows", w_total), ("radix", plan["radix_mul"] << c_bits)))
    insts = None
    if pmc_match and world == 1:
        # the headline's instantiation (the radix copies' limb records)
        key = [k for k in pmc["kernels"] if k.startswith("vk::k_msm_accumulate") and CURVE_TAG[curve] in k]
        key = sorted(key, key=_acc_key_rank)
        if key:
            ke = pmc["kernels"][key[0]]
            # the headline's launch class (one bucket set; the KZG line's two-set launches share
            # the kernel instance: prof_summary.py by_class)
            insts = ke.get("by_class", {}).get("1", ke).get("SQ_INSTS_VALU_per_launch")
    ach = insts * 64 / acc_s / 1e12 if (insts and acc_s) else None
    valu = {"achieved": ach, "peak": mad_peak, "unit": "T VALU lane-instructions/s",
            "frac": (ach / mad_peak) if ach else None,
            "work": f"{madds} mixed adds ({'signed radix-2^30, 13 limbs' if curve == 'bls12_381' else 'radix-2^29'} XYZZ: "
                    f"8 products + 2 squares, 9 Montgomery reductions -- Y3 is one lazy sum of two products); "
                    f"{insts / madds * 64 if insts else float('nan'):.0f} VALU lane-instructions per mixed add (PMC)",
            "madds_per_s": madds / acc_s if acc_s else None,
            "peak_source": "vc_device_mad_rate: v_mad_u64_u32 issue rate measured live on this GPU (v_mad_i64_i32 issues the same)",
            "insts_source": os.path.relpath(PMC_SUMMARY, ROOT) if insts else None}
    traffic, traffic_src = None, None
    if world == 1 and pmc_match:
        key = sorted([k for k in pmc.get("kernels", {}) if "k_msm_accumulate<vk::SWCurve<vk::BLS381Fq" in k],
                     key=_acc_key_rank)
        if key and curve == "bls12_381":
            ke = pmc["kernels"][key[0]]
            traffic = ke.get("by_class", {}).get("1", ke).get("hbm_bytes_per_launch")
            traffic_src = os.path.relpath(PMC_SUMMARY, ROOT)

    prov = provenance()
    out = {
        "metric": METRIC,
        "value": a.steps / dt,
        "unit": "2^20-pt MSM/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "ms_per_step_median": float(np.median(step_ms)),
        "ms_per_step_min": float(np.min(step_ms)),
        "ms_per_step_with_events": dt_events / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (random subgroup bases s_i*G generated on device, uniform scalars < r)",
        "config": {"workload": f"single 2^{a.log_n}-point {curve} G1 Pippenger MSM (configs[1])",
                   "n_points": n, "curve": curve,
                   "parallelism": (f"Pippenger-window slices x{world}" if split == "windows" else
                                   f"point ranges x{world}") if world > 1 else "one GPU",
                   "msm_split": split if world > 1 else None,
                   "exchange": comm_kind,
                   "window_bits": c_bits, "windows": w_total, "radix": plan["radix_mul"] << c_bits,
                   "radix_form": f"{plan['radix_mul']} * 2^{c_bits}", "terms_per_point": terms,
                   "precomputed_bases": (f"{w_total} x 2n window copies B^w P_i, B^w phi(P_i) with B = "
                                         f"{plan['radix_mul']} * 2^{c_bits}, each signed copy (+-) one aligned "
                                         f"128-B record of signed radix-2^30 limbs (x, y) "
                                         f"({w_total * 2 * n * 2 * 128 / 1e9:.2f} GB), built once per base table "
                                         "(a fixed CRS), untimed; `variable_base` is the same MSM without them")
                   if plan["shared_windows"] else None},
        "roofline": {"bound": "valu", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": "msm_accumulate",
                     "kernel_ms": (acc_ms / acc_n) if acc_n else None,
                     "algorithmic_bytes_per_launch": shard_bytes,
                     "valu": valu,
                     "note": "EC MSM is VALU integer-multiply bound, not HBM bound (SURVEY 8(d)): achieved/peak/"
                             "frac are the algorithmic-HBM figures BASELINE.json's metric asks for; the "
                             "valu object is the binding roofline"},
        "kernel_ms": kernels,
        "kernel_timing": ("a second pass of the same K steps with HIP events around every launch on the "
                          "launch stream (ms_per_step_with_events); the headline pass runs without them"),
        "accumulate_clock_mhz": acc_mhz or None,
        "accumulate_clock_source": (f"s_memtime / s_memrealtime stamps around one lane's loop, {acc_clk_n} "
                                    "timed launches (vc_ctx_accumulate_clock)") if acc_clk_n else None,
        "provenance": prov,
        "pmc_libvkzg_sha256": (pmc or {}).get("libvkzg_sha256"),
        "pmc_same_library": bool(pmc) and (pmc or {}).get("libvkzg_sha256") == prov.get("libvkzg_sha256"),
        "result_inf": int(res[1]),
        "result_check": check,
        "variable_base": variable,
        "host_scalars": host_line,
    }

    progress("variable-base / host-scalar lines done")
    if not a.no_secondary:
        # config 3: batched width-256 commits (fixed-base tables), batch split across ranks; timed
        # on the commit_window / commit_windows table (172 GB at 19 / 13), the c = 16 one (17.2 GB), the c = 18 x 14
        # one (68.7 GB) and the deployable 15-window one (31.1 GB)
        cstate = {}

        def cengine():  # (re)create: closing the engine frees a table a peer rank could not fit
            if "eng" in cstate:
                cstate["eng"].close()
            cstate["eng"] = vkzg.Engine("bandersnatch", local)
            cstate["eng"].set_stream(stream.cuda_stream)
            cstate["tab"] = cstate["eng"].random_bases(256, seed=3)

        cengine()
        B = a.commit_batch
        blo, bhi = vdist.shard_range(B, rank, world)
        Bl = bhi - blo
        csc = vkzg.random_scalars("bandersnatch", B * 256, np.random.default_rng(5))[blo * 256:bhi * 256]
        dcs = torch.from_numpy(np.ascontiguousarray(csc).view(np.int64)).to(dev)
        dxy = torch.zeros((max(Bl, 1), 8), dtype=torch.int64, device=dev)
        dinf = torch.zeros(max(Bl, 1), dtype=torch.uint8, device=dev)

        def cstep():
            ceng, ctab = cstate["eng"], cstate["tab"]
            ceng.msm_batch_device(ctab, 256, dcs.data_ptr(), Bl, dxy.data_ptr(), dinf.data_ptr())
            if world > 1:  # every rank ends with all B commitments (RCCL all-gather)
                return vdist.all_gather_commitments(dxy[:Bl], dinf[:Bl], B, world)
            return dxy, dinf

        def ctime(cw, windows=0):
            ceng, ctab = cstate["eng"], cstate["tab"]
            fits = True
            try:
                ceng.fixed_base_precompute(ctab, cw, windows)
            except vkzg.VCError:  # table does not fit next to the rest
                fits = False
            if world > 1:  # every rank takes the same branch (a lone skip would hang the barriers)
                ok = torch.tensor([1 if fits else 0], device=dev)
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                fits = bool(int(ok.item()))
            if not fits:
                cengine()
                return None
            for _ in range(2):
                cstep()
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            reps = 5
            for _ in range(reps):  # no per-kernel events in the timed passes
                cstep()
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            cdt = (time.perf_counter() - t0) / reps
            ceng.reset_timing()
            ceng.enable_timing(True)  # one more pass for the kernel time
            cstep()
            torch.cuda.synchronize(dev)
            ceng.enable_timing(False)
            if world > 1:
                tt = torch.tensor([cdt], dtype=torch.float64, device=dev)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                cdt = float(tt.item())
            fb_ms, fb_n = ceng.kernel_time("fb_commit")
            gc, gw, gbig = ceng.fixed_base_geometry(ctab)
            return {"window_bits": cw, "windows": gw, "wide_windows": gbig, "commits_per_s": B / cdt,
                    "ms_per_batch": cdt * 1e3,
                    "fb_commit_kernel_ms": fb_ms / fb_n if fb_n else None,
                    "achieved_GBps": (Bl * 8256) / (fb_ms / fb_n * 1e-3) / 1e9 if fb_n else None,
                    "table_bytes": ceng.fixed_base_table_bytes(ctab)}

        big = ctime(a.commit_window, a.commit_windows if a.commit_window != 16 else 0)
        small = ctime(16) if a.commit_window != 16 else big
        # the <= 70 GB table: 14 windows (12 of 18 bits, 2 of 19), 68.7 GB (not when more than two
        # rehearsal ranks share one card: four of them do not fit its HBM beside the rest)
        mixed = ctime(18, 14) if not (a.rehearse_one_gpu and world > 2) else None
        # the deployable <= 32 GB table: 15 windows (14 of 17 bits, one of 16), 31.1 GB -- the adds
        # of c = 17's 15 windows from a smaller table (c = 17 x 15 is 32.2 GB)
        deploy = ctime(16, 15)
        # the headline is the deployable <= 32 GB table: a 256-point CRS served
        # from ~11 % of the card; the larger tables are named sub-lines
        head = deploy or small or big
        if head is None:  # no table fits beside the rest on every rank
            out["secondary"] = {"workload": f"{B} batched width-256 Bandersnatch commits (configs[2])",
                                "skipped": "no fixed-base table fits on every rank"}
        else:
            out["secondary"] = {
                "workload": f"{B} batched width-256 Bandersnatch commits (configs[2]), fixed-base "
                            f"c={head['window_bits']} ({head['windows']} windows, {head['wide_windows']} of them "
                            f"{head['window_bits'] + 1} bits, {head['table_bytes'] / 1e9:.1f} GB table), "
                            f"batch split over {world} rank(s)",
                **head,
                "table_choice": "the deployable table (<= 32 GB) leads; larger tables below as sub-lines",
                "c16": small,
                "mixed_c18_w14": mixed,
                f"large_c{a.commit_window}_w{a.commit_windows}": big if big is not small else None,
            }
        cstate["eng"].close()

    progress("commit lines done")
    if not a.no_kzg:
        out["kzg"] = kzg_line(a, rank, world, local, dev, stream)
        progress("kzg line done")

    if not a.no_mp:
        out["multiproof"] = mp_line(a, rank, world, local, dev, stream, comm)
        progress("multiproof line done")

    if rank == 0 and not a.no_ipa:
        out["ipa"] = ipa_line(local, stream, cpu=(world == 1 and not a.no_cpu_baseline))
        progress("ipa line done")
        out["kzg_reference_shapes"] = kzg_reference_shapes(local, stream, cpu=(world == 1 and not a.no_cpu_baseline))
        progress("kzg reference shapes done")

    if rank == 0 and not a.no_verkle:
        out["verkle"] = verkle_line(a, local, stream)
        progress("verkle line done")

    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(curve, n, a.cpu_sample)
        progress("cpu naive baseline done")
        out["cpu_baselines_other"] = cpu_commit_baselines()
        # the all-core bound beside the 1-core naive port: the CPU share of one GPU on the box
        thr = a.cpu_threads or min(16, os.cpu_count() or 1)
        bxy, binf = eng.download_bases(table)
        out["cpu_baseline_pippenger"] = cpu_pippenger(curve, bxy, binf, scalars, res, thr)
        # and on every host core the box reports ("Pippenger on all host cores")
        allc = cpu_pippenger(curve, bxy, binf, scalars, res, os.cpu_count() or 1)
        share = host_cpu_share()
        allc["host_cpu_share"] = share
        if share["cgroup_quota_cpus"] is not None and share["cgroup_quota_cpus"] < allc["cores"]:
            allc["note"] = (f"{allc['cores']} threads time-slice a cgroup quota of {share['cgroup_quota_cpus']} CPUs: "
                            f"slower than the {thr}-thread line; the true all-core figure of a whole host is not "
                            f"measurable from this box")
        out["cpu_baseline_pippenger_allcores"] = allc
        del bxy, binf
        out["cpu_baselines_other"]["C3_width256_commits_pippenger"] = cpu_pippenger_commits(a.commit_batch, thr)
        if "kzg" in out:  # configs[3] on the CPU: its two 2^20 MSMs alone (quotient not counted)
            out["cpu_baselines_other"]["C4_kzg_commit_open_lower_bound"] = {
                "value": 2 * out["cpu_baseline"]["ms_per_msm"], "unit": "ms", "cores": 1, "kind": "port",
                "sample": "2 x the naive 2^20 BLS12-381 MSM above (commit + proof MSM); the reference's "
                          "per-element inversions of the quotient are not counted, so this is a lower bound"}
            pip = out["cpu_baseline_pippenger"]
            out["cpu_baselines_other"]["C4_kzg_commit_open_lower_bound_pippenger"] = {
                "value": 2 * pip["ms_per_msm"], "unit": "ms", "cores": pip["cores"], "kind": "pippenger",
                "sample": "2 x the all-core Pippenger 2^20 BLS12-381 MSM above (commit + proof MSM); quotient "
                          "not counted (lower bound)"}

    if comm is not None:
        comm.close()
    eng.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
