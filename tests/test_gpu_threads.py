"""GPU: one vc_ctx shared by 8 host threads (the reference's multiproof bound requires
UniversalParams: Sync, multiproof.rs:96, and callers may invoke commit / prove_point from rayon
workers). Interleaved vc_msm, vc_msm_batch and vc_ipa_prove calls from the threads must give
exactly the results of the same calls run serially. ctypes releases the GIL around each foreign
call, so the threads really are inside libvkzg.so concurrently; the context's mutex serialises
them."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_shared_ctx_eight_threads():
    import vkzg
    from vkzg import scheme
    eng = vkzg.Engine("bn254")
    try:
        N = 64
        ipa = scheme.IPA(eng, N, scheme.ipa_crs(N + 1, max_=512))
        big = eng.random_bases(20000, seed=8)
        rng = np.random.default_rng(3)
        jobs = []
        for j in range(48):
            kind = ("msm", "batch", "prove")[j % 3]
            if kind == "msm":
                n = int(rng.integers(100, 20000))
                jobs.append((kind, vkzg.random_scalars("bn254", n, rng)))
            elif kind == "batch":
                jobs.append((kind, vkzg.random_scalars("bn254", 5 * N, rng)))
            else:
                vals = [int(v) for v in rng.integers(0, 1 << 62, size=N)]
                jobs.append((kind, (scheme.LagrangeBasis(vals), int(rng.integers(0, 4 * N)))))

        def run(job):
            kind, arg = job
            if kind == "msm":
                xy, inf = eng.msm(big, arg)
                return (xy.tobytes(), inf)
            if kind == "batch":
                xy, inf = eng.msm_batch(ipa.table, arg, N)
                return (xy.tobytes(), inf.tobytes())
            data, pt = arg
            com = ipa.commit(data)
            pr = ipa.prove_point(com, pt, data)
            return (com, str(pr.as_dict()), ipa.verify_point(com, pt, pr))

        serial = [run(j) for j in jobs]
        results = [None] * len(jobs)
        errors = []

        def worker(k):
            try:
                for i in range(k, len(jobs), 8):
                    results[i] = run(jobs[i])
            except Exception as ex:  # surfaced below
                errors.append(ex)

        for _ in range(2):
            th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=120)
            assert not errors, errors
            assert results == serial
            for r in results:
                if len(r) == 3:
                    assert r[2] is True
    finally:
        eng.close()


def test_context_per_thread():
    """The overlap pattern for rayon-style callers: one vc_ctx per worker
    thread, each with its own stream and its own copy of the CRS, so latency-bound calls (the IPA
    prover's dependent rounds) from different threads run on the GPU at the same time instead of
    queueing on one context's mutex. Proofs must equal the single-context ones."""
    import vkzg
    from vkzg import scheme
    N, T, per = 256, 4, 6
    crs = scheme.ipa_crs(N + 1, max_=512)
    rng = np.random.default_rng(12)
    jobs = [(scheme.LagrangeBasis([int(v) for v in rng.integers(0, 1 << 62, size=N)]), int(rng.integers(0, 4 * N)))
            for _ in range(T * per)]
    engs = [vkzg.Engine("bn254") for _ in range(T)]
    try:
        ipas = [scheme.IPA(e, N, crs) for e in engs]
        want = []
        for data, pt in jobs:
            com = ipas[0].commit(data)
            want.append((com, str(ipas[0].prove_point(com, pt, data).as_dict())))
        got = [None] * len(jobs)
        errors = []

        def worker(k):
            try:
                for i in range(k, len(jobs), T):
                    data, pt = jobs[i]
                    com = ipas[k].commit(data)
                    got[i] = (com, str(ipas[k].prove_point(com, pt, data).as_dict()))
            except Exception as ex:  # surfaced below
                errors.append(ex)

        th = [threading.Thread(target=worker, args=(k,)) for k in range(T)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not errors, errors
        assert got == want
    finally:
        for e in engs:
            e.close()
