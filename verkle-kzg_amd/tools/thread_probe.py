"""Diagnose order / concurrency dependence of calls on one shared vc_ctx (tests/test_gpu_threads.py).

Runs the same job list serially in order, serially in a shuffled order, and from 8 threads, and
prints which jobs (by kind) disagree with the in-order serial results, and whether their proofs
verify. Usage: python tools/thread_probe.py [--kinds msm,batch,prove]
"""
import argparse
import os
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE)]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime: torch's)

import vkzg  # noqa: E402
from vkzg import scheme  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="msm,batch,prove")
    ap.add_argument("--jobs", type=int, default=48)
    ap.add_argument("--lock", default="", help="serialise these phases under one Python lock: commit,prove,verify")
    a = ap.parse_args()
    kinds = a.kinds.split(",")
    eng = vkzg.Engine("bn254")
    N = 64
    ipa = scheme.IPA(eng, N, scheme.ipa_crs(N + 1, max_=512))
    big = eng.random_bases(20000, seed=8)
    rng = np.random.default_rng(3)
    jobs = []
    for j in range(a.jobs):
        kind = kinds[j % len(kinds)]
        if kind == "msm":
            jobs.append((kind, vkzg.random_scalars("bn254", int(rng.integers(100, 20000)), rng)))
        elif kind == "batch":
            jobs.append((kind, vkzg.random_scalars("bn254", 5 * N, rng)))
        else:
            vals = [int(v) for v in rng.integers(0, 1 << 62, size=N)]
            jobs.append((kind, (scheme.LagrangeBasis(vals), int(rng.integers(0, 4 * N)))))

    lk = threading.Lock()
    locked = set(a.lock.split(",")) if a.lock else set()

    def maybe(phase, f):
        if phase in locked:
            with lk:
                return f()
        return f()

    def run(job):
        kind, arg = job
        if kind == "msm":
            xy, inf = eng.msm(big, arg)
            return (xy.tobytes(), inf)
        if kind == "batch":
            xy, inf = eng.msm_batch(ipa.table, arg, N)
            return (xy.tobytes(), inf.tobytes())
        data, pt = arg
        com = maybe("commit", lambda: ipa.commit(data))
        pr = maybe("prove", lambda: ipa.prove_point(com, pt, data))
        ok = maybe("verify", lambda: ipa.verify_point(com, pt, pr))
        ok2 = maybe("verify", lambda: ipa.verify_point(com, pt, pr))
        return (com, str(pr.as_dict()), ok, pt, ok2)

    ref = [run(j) for j in jobs]
    bad = [i for i, r in enumerate(ref) if len(r) == 5 and not r[2]]
    print("serial in-order: proofs failing verify:", bad, flush=True)
    again = [run(j) for j in jobs]
    print("serial repeat mismatches:", [i for i in range(len(jobs)) if again[i] != ref[i]], flush=True)
    order = np.random.default_rng(1).permutation(len(jobs))
    shuf = [None] * len(jobs)
    for i in order:
        shuf[i] = run(jobs[i])
    print("serial shuffled mismatches:", [(i, jobs[i][0]) for i in range(len(jobs)) if shuf[i] != ref[i]],
          flush=True)
    res = [None] * len(jobs)

    def worker(k):
        for i in range(k, len(jobs), 8):
            res[i] = run(jobs[i])

    th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    mm = [i for i in range(len(jobs)) if res[i] != ref[i]]
    print("threaded mismatches:", [(i, jobs[i][0]) for i in mm], flush=True)
    for i in mm:
        r, s = res[i], ref[i]
        if len(r) == 5:
            print(f"  job {i} prove pt={r[3]}: commit equal {r[0] == s[0]}, proof equal {r[1] == s[1]}, "
                  f"verify threaded={r[2]},{r[4]} serial={s[2]}", flush=True)
        else:
            print(f"  job {i} {jobs[i][0]}: inf {r[1]!r} vs {s[1]!r}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
