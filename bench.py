#!/usr/bin/env python3
"""Benchmark: single 2^20-point BLS12-381 G1 MSM (BASELINE.json configs[1]) on N MI355X.

A step = one 2^20-point MSM over synthetic inputs already resident in HBM (bases uploaded
once, scalars on the device). With N ranks the MSM is split by point range (each rank
streams only its n/N bases and scalars), the per-rank projective partial sums are
all-gathered over RCCL and added on the host: one exchange step, so
scaling is "strong" (total work fixed).

Secondary line items (same JSON object): 10k batched width-256 Bandersnatch commits/s on
this rank (config 3), and the CPU baseline: the reference's naive MSM restated in C
(oracle/c/ref_curve.c) timed on a bounded sample on this host.

    python bench.py [--gpus N --steps K --warmup W]
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--curve", default="bls12_381")
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--commit-batch", type=int, default=10000)
    ap.add_argument("--commit-window", type=int, default=16)
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1 << 14, help="terms of the CPU naive MSM sample")
    return ap.parse_args()


def cpu_baseline(curve, n_full, sample):
    """Reference algorithm (naive per-term double-and-add + sequential sum, utils.rs:16-19)
    restated in C (oracle/), 1 thread, on `sample` terms; extrapolated linearly to n_full."""
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
    t0 = time.perf_counter()
    cref.msm_arrays(curve, xy, inf, sc, 1)
    dt = time.perf_counter() - t0
    per_msm_s = dt * n_full / sample
    return {"value": 1.0 / per_msm_s, "unit": "MSM/s", "cores": 1, "kind": "port",
            "sample": f"{sample} of {n_full} terms of the naive {curve} MSM (reference utils.rs:16-19 "
                      f"restated in C, oracle/c/ref_curve.c), 1 thread, {dt:.2f} s, extrapolated linearly",
            "ms_per_msm": per_msm_s * 1e3, "host_cpus": os.cpu_count()}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
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
    lo, hi = vdist.shard_range(n, rank, world)
    d_sc = torch.from_numpy(scalars[lo:hi].view(np.int64).copy()).to(dev)

    def step():
        # shard partial (HIP) -> RCCL all-gather of projective partials -> host sum
        return vdist.msm_sharded(eng, table, d_sc.data_ptr(), n, rank, world, dev if world > 1 else None)

    for _ in range(a.warmup):
        res = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    eng.enable_timing(True)
    eng.reset_timing()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    eng.enable_timing(False)
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_per_step = dt / a.steps * 1e3

    # dominant kernel (bucket accumulation) device time, HIP events on the launch stream
    acc_ms, acc_n = eng.kernel_time("msm_accumulate")
    kernels = {}
    for k in ("msm_sort_hist", "msm_scan", "msm_sort_coarse", "msm_sort_fine", "msm_accumulate", "msm_fixup", "msm_segsum",
              "msm_bitsum", "msm_sumpart"):
        ms, cnt = eng.kernel_time(k)
        if cnt:
            kernels[k] = round(ms / cnt, 4)
    shard_bytes = (hi - lo) * BYTES_PER_POINT[curve] + OUT_BYTES[curve]
    achieved = shard_bytes / (acc_ms / acc_n * 1e-3) / 1e9 if acc_n else None

    out = {
        "metric": METRIC,
        "value": a.steps / dt,
        "unit": "2^20-pt MSM/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (random subgroup bases s_i*G generated on device, uniform scalars < r)",
        "config": {"workload": f"single 2^{a.log_n}-point {curve} G1 Pippenger MSM (configs[1])",
                   "n_points": n, "curve": curve, "parallelism": f"point-range shards x{world}",
                   "window_bits": 16 if n >= (1 << 19) else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": None,
                     "kernel": "msm_accumulate",
                     "kernel_ms": (acc_ms / acc_n) if acc_n else None,
                     "algorithmic_bytes_per_launch": shard_bytes,
                     "note": "EC MSM is VALU integer-multiply bound, not HBM bound (SURVEY 8(d))"},
        "kernel_ms": kernels,
        "result_inf": int(res[1]),
    }

    if rank == 0 and not a.no_secondary:
        # config 3: batched width-256 commits (fixed-base tables), this rank only
        ceng = vkzg.Engine("bandersnatch", local)
        ceng.set_stream(stream.cuda_stream)
        ctab = ceng.random_bases(256, seed=3)
        ceng.fixed_base_precompute(ctab, a.commit_window)
        B = a.commit_batch
        csc = vkzg.random_scalars("bandersnatch", B * 256, np.random.default_rng(5))
        dcs = torch.from_numpy(csc.view(np.int64)).to(dev)
        dxy = torch.zeros((B, 8), dtype=torch.int64, device=dev)
        dinf = torch.zeros(B, dtype=torch.uint8, device=dev)
        for _ in range(2):
            ceng.msm_batch_device(ctab, 256, dcs.data_ptr(), B, dxy.data_ptr(), dinf.data_ptr())
        torch.cuda.synchronize(dev)
        ceng.enable_timing(True)
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            ceng.msm_batch_device(ctab, 256, dcs.data_ptr(), B, dxy.data_ptr(), dinf.data_ptr())
        torch.cuda.synchronize(dev)
        cdt = (time.perf_counter() - t0) / reps
        fb_ms, fb_n = ceng.kernel_time("fb_commit")
        out["secondary"] = {
            "workload": f"{B} batched width-256 Bandersnatch commits (configs[2]), fixed-base c={a.commit_window}",
            "commits_per_s": B / cdt, "ms_per_batch": cdt * 1e3,
            "fb_commit_kernel_ms": fb_ms / fb_n if fb_n else None,
            "achieved_GBps": (B * 8256) / (fb_ms / fb_n * 1e-3) / 1e9 if fb_n else None,
        }
        ceng.close()

    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(curve, n, a.cpu_sample)

    eng.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
