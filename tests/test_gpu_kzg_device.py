"""GPU: KZG open with device-resident evaluations and its multi-GPU window-part form
(vc_kzg_prove_device[_part]) on BN254 and BLS12-381 (the north_star's KZG curve):
device == host-input proof, parts sum to the proof, and the proof satisfies the trapdoor
identity pi*(s - z) == C - y*G (s = 100 is the reference's public test secret,
kzg/mod.rs:115-124 + Appendix A.7), checked with the oracle's group law."""
import ctypes
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GEN = {"bn254": 5, "bls12_381": 7}


@pytest.mark.parametrize("curve", ["bn254", "bls12_381"])
@pytest.mark.parametrize("where", ["in_domain", "outside"])
def test_kzg_device_parts_trapdoor(curve, where):
    import torch
    import vkzg
    from pyoracle.curves import CURVES
    from vkzg._lib import check, lib
    C = CURVES[curve]
    r = C.r
    e = vkzg.Engine(curve)
    n = 1024
    secret = vkzg.ints_to_limbs([100])[0].copy()
    tid, size = ctypes.c_int(), ctypes.c_size_t()
    check(lib().vc_kzg_setup(e.h, n, ctypes.c_void_p(secret.ctypes.data), ctypes.byref(tid), ctypes.byref(size)),
          "setup")
    tid, size = tid.value, size.value
    assert size == n
    rng = random.Random(5)
    ev_int = [rng.randrange(r) for _ in range(n)]
    ev = vkzg.ints_to_limbs(ev_int)
    if where == "in_domain":
        m = n // 3
        point_int = m
        zval = pow(GEN[curve], (r - 1) // n, r)
        zval = pow(zval, m, r)
    else:
        point_int = n + 12345
        zval = point_int
    point = vkzg.ints_to_limbs([point_int])[0].copy()
    P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    nl = vkzg.NL[curve]
    pxy = np.zeros(2 * nl, dtype=np.uint64)
    pinf = np.zeros(1, dtype=np.uint8)
    y = np.zeros(4, dtype=np.uint64)
    check(lib().vc_kzg_prove(e.h, tid, size, P(ev), n, P(point), P(pxy), P(pinf), P(y)), "prove")
    d_ev = torch.from_numpy(ev.view(np.int64).copy()).cuda()
    pxy2 = np.zeros_like(pxy)
    pinf2 = np.zeros_like(pinf)
    y2 = np.zeros_like(y)
    check(lib().vc_kzg_prove_device(e.h, tid, size, ctypes.c_void_p(d_ev.data_ptr()), n, P(point), P(pxy2),
                                    P(pinf2), P(y2)), "prove_device")
    assert np.array_equal(pxy, pxy2) and pinf[0] == pinf2[0] and np.array_equal(y, y2)
    parts = 3
    accs = []
    for k in range(parts):
        acc = np.zeros(e.point_words(), dtype=np.uint32)
        yk = np.zeros(4, dtype=np.uint64)
        check(lib().vc_kzg_prove_device_part(e.h, tid, size, ctypes.c_void_p(d_ev.data_ptr()), n, P(point), k,
                                             parts, P(acc), P(yk)), "prove_part")
        assert np.array_equal(yk, y)
        accs.append(acc)
    sxy, sinf = e.partials_sum(np.stack(accs))
    assert np.array_equal(sxy, pxy) and sinf == pinf[0]
    # trapdoor identity with the oracle group law
    com_xy, com_inf = e.msm(tid, ev)
    com = vkzg.arrays_to_points(curve, com_xy[None, :], np.array([com_inf], dtype=np.uint8))[0]
    proof = vkzg.arrays_to_points(curve, pxy[None, :], pinf)[0]
    yv = vkzg.limbs_to_int(y)
    lhs = C.mul(proof, (100 - zval) % r)
    rhs = C.add(com, C.neg(C.mul(C.g, yv)))
    assert lhs == rhs
    e.close()
