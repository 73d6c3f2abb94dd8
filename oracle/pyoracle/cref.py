"""ORACLE (test infrastructure only) -- ctypes binding of oracle/_build/libref_oracle.so (C restatement)."""
import ctypes
import os

import numpy as np

from .curves import CURVES

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_build", "libref_oracle.so")
NL = {"bn254": 4, "bls12_381": 6, "bandersnatch": 4}
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle C library missing: run `make -C oracle`")
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def ints_to_limbs(vals, nl):
    out = np.zeros((len(vals), nl), dtype=np.uint64)
    for i, v in enumerate(vals):
        v = int(v)
        for j in range(nl):
            out[i, j] = (v >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
    return out


def limbs_to_int(row):
    return sum(int(x) << (64 * j) for j, x in enumerate(row))


def points_to_array(curve_name, pts):
    nl = NL[curve_name]
    arr = np.zeros((len(pts), 2 * nl), dtype=np.uint64)
    inf = np.zeros(len(pts), dtype=np.uint8)
    for i, P in enumerate(pts):
        if P is None:
            inf[i] = 1
            continue
        arr[i, :nl] = ints_to_limbs([P[0]], nl)[0]
        arr[i, nl:] = ints_to_limbs([P[1]], nl)[0]
    return arr, inf


def array_to_point(curve_name, xy, inf):
    nl = NL[curve_name]
    c = CURVES[curve_name]
    if inf:
        return c.identity()
    return (limbs_to_int(xy[:nl]), limbs_to_int(xy[nl:]))


def msm_arrays(curve_name, bases, inf, scalars, nthreads=1):
    """bases: (n, 2*NL) uint64 canonical; scalars: (n, 4) uint64 canonical. Returns (xy, inf)."""
    nl = NL[curve_name]
    n = scalars.shape[0]
    bases = np.ascontiguousarray(bases, dtype=np.uint64)
    scalars = np.ascontiguousarray(scalars, dtype=np.uint64)
    infp = None
    if inf is not None:
        inf = np.ascontiguousarray(inf, dtype=np.uint8)
        infp = inf.ctypes.data_as(ctypes.c_void_p)
    out = np.zeros(2 * nl, dtype=np.uint64)
    oinf = np.zeros(1, dtype=np.uint8)
    fn = getattr(lib(), curve_name + "_ref_msm")
    fn.restype = ctypes.c_int
    fn(bases.ctypes.data_as(ctypes.c_void_p), infp, scalars.ctypes.data_as(ctypes.c_void_p),
       ctypes.c_size_t(n), ctypes.c_int(nthreads), out.ctypes.data_as(ctypes.c_void_p),
       oinf.ctypes.data_as(ctypes.c_void_p))
    return out, int(oinf[0])


def msm(curve_name, pts, scalars, nthreads=1):
    arr, inf = points_to_array(curve_name, pts)
    sc = ints_to_limbs(scalars, 4)
    xy, oi = msm_arrays(curve_name, arr, inf, sc, nthreads)
    return array_to_point(curve_name, xy, oi)


def on_curve(curve_name, bases):
    bases = np.ascontiguousarray(bases, dtype=np.uint64)
    fn = getattr(lib(), curve_name + "_ref_on_curve")
    return bool(fn(bases.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(bases.shape[0])))


def pip_msm_arrays(curve_name, bases, inf, scalars, nthreads=1):
    """Pippenger baseline (bucket method on `nthreads` threads, point chunks): same result as
    msm_arrays. bases: (n, 2*NL) uint64 canonical; scalars: (n, 4) uint64 canonical."""
    nl = NL[curve_name]
    n = scalars.shape[0]
    bases = np.ascontiguousarray(bases, dtype=np.uint64)
    scalars = np.ascontiguousarray(scalars, dtype=np.uint64)
    infp = None
    if inf is not None:
        inf = np.ascontiguousarray(inf, dtype=np.uint8)
        infp = inf.ctypes.data_as(ctypes.c_void_p)
    out = np.zeros(2 * nl, dtype=np.uint64)
    oinf = np.zeros(1, dtype=np.uint8)
    fn = getattr(lib(), curve_name + "_pip_msm")
    fn.restype = ctypes.c_int
    fn(bases.ctypes.data_as(ctypes.c_void_p), infp, scalars.ctypes.data_as(ctypes.c_void_p),
       ctypes.c_size_t(n), ctypes.c_int(nthreads), out.ctypes.data_as(ctypes.c_void_p),
       oinf.ctypes.data_as(ctypes.c_void_p))
    return out, int(oinf[0])


def pip_msm_batch_arrays(curve_name, bases, inf, scalars, width, nthreads=1):
    """`batch` commits of `width` terms over bases[:width] (scalars (batch*width, 4)), commits
    split over threads. Returns ((batch, 2*NL) xy, (batch,) inf)."""
    nl = NL[curve_name]
    batch = scalars.shape[0] // width
    bases = np.ascontiguousarray(bases, dtype=np.uint64)
    scalars = np.ascontiguousarray(scalars, dtype=np.uint64)
    infp = None
    if inf is not None:
        inf = np.ascontiguousarray(inf, dtype=np.uint8)
        infp = inf.ctypes.data_as(ctypes.c_void_p)
    out = np.zeros((batch, 2 * nl), dtype=np.uint64)
    oinf = np.zeros(batch, dtype=np.uint8)
    fn = getattr(lib(), curve_name + "_pip_msm_batch")
    fn.restype = ctypes.c_int
    fn(bases.ctypes.data_as(ctypes.c_void_p), infp, scalars.ctypes.data_as(ctypes.c_void_p),
       ctypes.c_size_t(width), ctypes.c_size_t(batch), ctypes.c_int(nthreads),
       out.ctypes.data_as(ctypes.c_void_p), oinf.ctypes.data_as(ctypes.c_void_p))
    return out, oinf


def mp_field_phases(N, data, z, r, t, omega, nthreads=1):
    """C restatement of prove_multiproof's field phases over BN254 Fr (oracle/c/ref_multiproof.c):
    data (Q, N, 4) or (Q*N, 4) uint64 canonical, z (Q,) point indices, r / t / omega ints.
    Returns (g, h): (N, 4) uint64 canonical each."""
    data = np.ascontiguousarray(data, dtype=np.uint64)
    z = np.ascontiguousarray(z, dtype=np.uint64)
    Q = z.shape[0]
    limbs = [ints_to_limbs([int(v)], 4)[0] for v in (r, t, omega)]
    g = np.zeros((N, 4), dtype=np.uint64)
    h = np.zeros((N, 4), dtype=np.uint64)
    fn = lib().bn254fr_mp_field_phases
    fn.restype = ctypes.c_int
    st = fn(ctypes.c_size_t(N), ctypes.c_size_t(Q), data.ctypes.data_as(ctypes.c_void_p),
            z.ctypes.data_as(ctypes.c_void_p), limbs[0].ctypes.data_as(ctypes.c_void_p),
            limbs[1].ctypes.data_as(ctypes.c_void_p), limbs[2].ctypes.data_as(ctypes.c_void_p),
            ctypes.c_int(nthreads), g.ctypes.data_as(ctypes.c_void_p), h.ctypes.data_as(ctypes.c_void_p))
    if st != 0:
        raise ValueError("bn254fr_mp_field_phases: bad argument")
    return g, h


def mp_g(N, data, z, r, omega, nthreads=1):
    """prove_multiproof's first field phase (multiproof.rs:117-150: scaling, grouped quotients,
    g) in C. Returns (state, g (N, 4) uint64 canonical); pass the state to mp_h, then mp_free."""
    data = np.ascontiguousarray(data, dtype=np.uint64)
    z = np.ascontiguousarray(z, dtype=np.uint64)
    limbs = [ints_to_limbs([int(v)], 4)[0] for v in (r, omega)]
    g = np.zeros((N, 4), dtype=np.uint64)
    fn = lib().bn254fr_mp_g
    fn.restype = ctypes.c_void_p
    st = fn(ctypes.c_size_t(N), ctypes.c_size_t(z.shape[0]), data.ctypes.data_as(ctypes.c_void_p),
            z.ctypes.data_as(ctypes.c_void_p), limbs[0].ctypes.data_as(ctypes.c_void_p),
            limbs[1].ctypes.data_as(ctypes.c_void_p), ctypes.c_int(nthreads), g.ctypes.data_as(ctypes.c_void_p))
    if not st:
        raise ValueError("bn254fr_mp_g: bad argument")
    return ctypes.c_void_p(st), g


def mp_h(state, N, t):
    """The second field phase (multiproof.rs:155-165: invert_domain_at(t), h) on mp_g's state."""
    tl = ints_to_limbs([int(t)], 4)[0]
    h = np.zeros((N, 4), dtype=np.uint64)
    fn = lib().bn254fr_mp_h
    fn.restype = ctypes.c_int
    if fn(state, tl.ctypes.data_as(ctypes.c_void_p), h.ctypes.data_as(ctypes.c_void_p)) != 0:
        raise ValueError("bn254fr_mp_h: t - i = 0")
    return h


def mp_free(state):
    lib().bn254fr_mp_free(state)
