"""GPU: KZG::prove_all_points (kzg/mod.rs:200-235, SURVEY 8(f) row 4, FK amortised openings) through
vc_kzg_prove_all_points.
  mode 0 -- the reference's computation exactly: == the oracle's restatement
    (oracle/pyoracle/protocol.py kzg_prove_all_points) on the inputs where the reference returns
    (interpolant degree d with D::new(2 d) <= len(data)), VC_E_DOMAIN where it panics (all-zero
    data, a domain longer than the data).
  mode 1 -- the FK opening proofs the reference's disabled test expects: == prove at every index
    (itself golden-pinned, tests/test_gpu_scheme.py) and the trapdoor identity pi (s - w^i) = C - y G.
"""
import random

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import vkzg
    e = vkzg.Engine("bn254")
    yield e
    e.close()


def _low_degree(rng, m, d, r, omega):
    coeffs = [rng.randrange(r) for _ in range(d + 1)]
    return [sum(c * pow(omega, i * k, r) for k, c in enumerate(coeffs)) % r for i in range(m)]


@pytest.mark.parametrize("m,d", [(8, 0), (8, 1), (8, 2), (8, 4), (16, 3), (16, 8), (32, 5), (32, 16)])
def test_mode0_matches_oracle(eng, m, d):
    from pyoracle import protocol
    from pyoracle.curves import BN254
    from vkzg import scheme
    r = BN254.r
    kz = scheme.KZG(eng, 32)
    okz = protocol.KZG(32)
    rng = random.Random(31 * m + d)
    evals = _low_degree(rng, m, d, r, protocol.group_gen(m))
    want = protocol.kzg_prove_all_points(okz, protocol.LagrangeBasis(evals, m))
    got = kz.prove_all_points(scheme.LagrangeBasis(evals), mode=0)
    assert [(g["proof"], g["y"]) for g in got] == want


@pytest.mark.parametrize("evals", [[0] * 8, "deg5_len8", "random_len16"])
def test_mode0_reference_panics_are_domain_errors(eng, evals):
    import vkzg
    from pyoracle import protocol
    from pyoracle.curves import BN254
    from vkzg import scheme
    r = BN254.r
    rng = random.Random(5)
    if evals == "deg5_len8":
        evals = _low_degree(rng, 8, 5, r, protocol.group_gen(8))    # D::new(10) = 16 > 8
    elif evals == "random_len16":
        evals = [rng.randrange(r) for _ in range(16)]              # degree 15: domain 32 > 16
    with pytest.raises(protocol.ReferencePanic):
        protocol.kzg_prove_all_points(protocol.KZG(32), protocol.LagrangeBasis(evals, len(evals)))
    with pytest.raises(vkzg.VCError) as ex:
        scheme.KZG(eng, 32).prove_all_points(scheme.LagrangeBasis(evals), mode=0)
    assert ex.value.status == -8


@pytest.mark.parametrize("size,n", [(32, 32), (32, 20), (256, 256)])
def test_mode1_fk_proofs_equal_single_openings(eng, size, n):
    from pyoracle import protocol
    from pyoracle.curves import BN254
    from vkzg import scheme
    C, r = BN254, BN254.r
    kz = scheme.KZG(eng, size)
    rng = random.Random(size + n)
    data = scheme.LagrangeBasis([rng.randrange(r) for _ in range(n)], size)
    com = kz.commit(data)
    allp = kz.prove_all_points(data, mode=1)
    assert len(allp) == size
    w = protocol.group_gen(size)
    for i in list(range(0, size, max(1, size // 16))) + [size - 1]:
        single = kz.prove(com, i, data)
        assert allp[i]["proof"] == single["proof"] and allp[i]["y"] == single["y"]
        # trapdoor identity (s = 100 public in the reference's setup)
        lhs = C.mul(allp[i]["proof"], (100 - pow(w, i, r)) % r)
        rhs = C.add(com, C.neg(C.mul(C.g, allp[i]["y"])))
        assert lhs == rhs
