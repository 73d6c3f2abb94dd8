"""Python handle on the HIP MSM engine (thin wrapper over include/vc_msm.h).

Layouts follow the C ABI: field elements are canonical little-endian u64 limbs, affine
points are (x limbs, y limbs) rows plus a u8 identity flag, scalars are 4 u64 limbs.
"""
import ctypes

import numpy as np

from ._lib import check, lib

CURVE_IDS = {"bn254": 0, "bls12_381": 1, "bandersnatch": 2}
NL = {"bn254": 4, "bls12_381": 6, "bandersnatch": 4}
# scalar-field moduli (for synthetic data generation and range checks)
SCALAR_R = {
    "bn254": 21888242871839275222246405745257275088548364400416034343698204186575808495617,
    "bls12_381": 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
    "bandersnatch": 13108968793781547619861935127046491459309155893440570251786403306729687672801,
}


def _ptr(a):
    # the pointer object keeps `a` alive for the duration of the call (see scheme._p)
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def ints_to_limbs(vals, nl=4):
    """Python ints -> (len, nl) little-endian u64 limbs (values taken mod 2^(64 nl), two's
    complement for negatives). One to_bytes per value: ~10x faster than per-limb shifts, which
    dominated the Python side of batched calls (256 x 256 scalars: 20 ms)."""
    nb = 8 * nl
    mask = (1 << (64 * nl)) - 1
    buf = b"".join((int(v) & mask).to_bytes(nb, "little") for v in vals)
    return np.frombuffer(buf, dtype="<u8").reshape(len(vals), nl).astype(np.uint64)


def limbs_to_int(row):
    if isinstance(row, np.ndarray):
        return int.from_bytes(np.ascontiguousarray(row, dtype="<u8").tobytes(), "little")
    return sum(int(x) << (64 * j) for j, x in enumerate(row))


def points_to_arrays(curve, pts):
    """[(x, y) | None] -> ((n, 2*NL) uint64, (n,) uint8). Edwards identity may be (0, 1)."""
    nl = NL[curve]
    arr = np.zeros((len(pts), 2 * nl), dtype=np.uint64)
    inf = np.zeros(len(pts), dtype=np.uint8)
    for i, P in enumerate(pts):
        if P is None:
            inf[i] = 1
            continue
        arr[i, :nl] = ints_to_limbs([P[0]], nl)[0]
        arr[i, nl:] = ints_to_limbs([P[1]], nl)[0]
    return arr, inf


def arrays_to_points(curve, xy, inf):
    nl = NL[curve]
    out = []
    for i in range(xy.shape[0]):
        if inf[i]:
            out.append((0, 1) if curve == "bandersnatch" else None)
        else:
            out.append((limbs_to_int(xy[i, :nl]), limbs_to_int(xy[i, nl:])))
    return out


def random_scalars(curve, n, rng):
    """n scalars below r (top limb drawn below r's top limb): (n, 4) uint64."""
    r = SCALAR_R[curve]
    top = r >> 192
    s = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64, endpoint=False)
    s[:, 3] = rng.integers(0, top, size=n, dtype=np.uint64)
    return s


SCALAR_BITS = {"bn254": 254, "bls12_381": 255, "bandersnatch": 253}


def random_base_scalars(curve, seed, n):
    """The discrete logs of vc_bases_random(seed, n): P_i = s_i * G with s_i from splitmix64 of
    (seed, i) (bases.hip k_random) -- the host mirror of that derivation, so callers can check an
    MSM over synthetic bases by linearity: sum k_i P_i = (sum k_i s_i mod r) * G. Returns (n, 4)
    uint64 limbs."""
    M1, M2, G = np.uint64(0xbf58476d1ce4e5b9), np.uint64(0x94d049bb133111eb), np.uint64(0x9e3779b97f4a7c15)
    with np.errstate(over="ignore"):
        st = np.uint64(seed) * np.uint64(0x100000001b3) + np.arange(n, dtype=np.uint64)
        out = np.zeros((n, 4), dtype=np.uint64)
        for k in range(4):
            st = st + G
            z = st.copy()
            z = (z ^ (z >> np.uint64(30))) * M1
            z = (z ^ (z >> np.uint64(27))) * M2
            out[:, k] = z ^ (z >> np.uint64(31))
    top = SCALAR_BITS[curve] - 2 - 192
    out[:, 3] &= np.uint64((1 << top) - 1)
    out[:, 0] |= np.uint64(1)
    return out


def limb_rows_to_ints(a):
    """(n, k) uint64 limbs -> list of Python ints."""
    a = np.ascontiguousarray(a, dtype="<u8")
    k = a.shape[1]
    b = a.tobytes()
    return [int.from_bytes(b[8 * k * i:8 * k * (i + 1)], "little") for i in range(a.shape[0])]


def dot_mod(a, b, r):
    """sum a_i b_i mod r over two (n, 4) limb arrays (host, exact)."""
    s = 0
    for x, y in zip(limb_rows_to_ints(a), limb_rows_to_ints(b)):
        s += x * y
    return s % r


def partials_sum(curve, accs):
    """vc_partials_sum: add projective accumulators on the host (no device needed)."""
    accs = np.ascontiguousarray(accs, dtype=np.uint32)
    nl = NL[curve]
    out = np.zeros(2 * nl, dtype=np.uint64)
    oinf = np.zeros(1, dtype=np.uint8)
    check(lib().vc_partials_sum(CURVE_IDS[curve], _ptr(accs), accs.shape[0], _ptr(out), _ptr(oinf)),
          "vc_partials_sum")
    return out, int(oinf[0])


class Engine:
    """One vc_ctx: a curve on one device."""

    def __init__(self, curve, device=0):
        self.curve = curve
        self.cid = CURVE_IDS[curve]
        self.nl = NL[curve]
        h = ctypes.c_void_p()
        check(lib().vc_ctx_create(self.cid, device, ctypes.byref(h)), "vc_ctx_create")
        self.h = h

    def close(self):
        if self.h:
            lib().vc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- streams / timing
    def set_stream(self, stream_handle):
        check(lib().vc_ctx_set_stream(self.h, ctypes.c_void_p(stream_handle)), "vc_ctx_set_stream")

    # vc_ctx_set_option knobs (include/vc_msm.h)
    OPT_MSM_SHARED_WINDOWS = 1
    OPT_MSM_CHUNK_POINTS = 2
    OPT_MSM_HOST_CHUNKS = 3

    def set_option(self, option, value):
        check(lib().vc_ctx_set_option(self.h, option, int(value)), "vc_ctx_set_option")

    def get_option(self, option):
        v = ctypes.c_int64()
        check(lib().vc_ctx_get_option(self.h, option, ctypes.byref(v)), "vc_ctx_get_option")
        return v.value

    def enable_timing(self, on=True):
        check(lib().vc_ctx_enable_timing(self.h, 1 if on else 0), "vc_ctx_enable_timing")

    def reset_timing(self):
        check(lib().vc_ctx_reset_timing(self.h), "vc_ctx_reset_timing")

    def accumulate_clock(self):
        """mean effective shader clock (MHz) of the accumulate launches timed since the last reset,
        and their count (vc_ctx_accumulate_clock: s_memtime / s_memrealtime stamps)"""
        mhz = ctypes.c_double()
        cnt = ctypes.c_long()
        check(lib().vc_ctx_accumulate_clock(self.h, ctypes.byref(mhz), ctypes.byref(cnt)), "vc_ctx_accumulate_clock")
        return mhz.value, cnt.value

    def kernel_time(self, name):
        ms = ctypes.c_double()
        cnt = ctypes.c_long()
        check(lib().vc_ctx_kernel_time(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(cnt)),
              "vc_ctx_kernel_time")
        return ms.value, cnt.value

    # -------------------------------------------------------------- bases
    def upload_bases(self, xy, inf=None):
        xy = np.ascontiguousarray(xy, dtype=np.uint64)
        assert xy.ndim == 2 and xy.shape[1] == 2 * self.nl
        if inf is not None:
            inf = np.ascontiguousarray(inf, dtype=np.uint8)
            assert inf.shape == (xy.shape[0],)
        tid = ctypes.c_int()
        check(lib().vc_bases_upload(self.h, _ptr(xy), _ptr(inf), xy.shape[0], ctypes.byref(tid)),
              "vc_bases_upload")
        return tid.value

    def upload_points(self, pts):
        xy, inf = points_to_arrays(self.curve, pts)
        return self.upload_bases(xy, inf)

    def random_bases(self, n, seed=0):
        tid = ctypes.c_int()
        check(lib().vc_bases_random(self.h, seed, n, ctypes.byref(tid)), "vc_bases_random")
        return tid.value

    def bases_count(self, table):
        n = ctypes.c_size_t()
        check(lib().vc_bases_count(self.h, table, ctypes.byref(n)), "vc_bases_count")
        return n.value

    def download_bases(self, table):
        n = self.bases_count(table)
        xy = np.zeros((n, 2 * self.nl), dtype=np.uint64)
        inf = np.zeros(n, dtype=np.uint8)
        check(lib().vc_bases_download(self.h, table, _ptr(xy), _ptr(inf)), "vc_bases_download")
        return xy, inf

    def fixed_base_precompute(self, table, window_bits=8, windows=0):
        """Fixed-base window tables; windows > 0 mixes window_bits / window_bits + 1 bit windows."""
        if windows:
            check(lib().vc_fixed_base_precompute_windows(self.h, table, window_bits, windows),
                  "vc_fixed_base_precompute_windows")
        else:
            check(lib().vc_fixed_base_precompute(self.h, table, window_bits), "vc_fixed_base_precompute")

    def fixed_base_table_bytes(self, table):
        """HBM bytes of the table's fixed-base window tables (vc_fixed_base_table_bytes)"""
        b = ctypes.c_size_t()
        check(lib().vc_fixed_base_table_bytes(self.h, table, ctypes.byref(b)), "vc_fixed_base_table_bytes")
        return b.value

    def fixed_base_geometry(self, table):
        """(window_bits, windows, wide_windows) of the table's fixed-base tables (0s if none)."""
        c, w, b = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        check(lib().vc_fixed_base_geometry(self.h, table, ctypes.byref(c), ctypes.byref(w), ctypes.byref(b)),
              "vc_fixed_base_geometry")
        return c.value, w.value, b.value

    # -------------------------------------------------------------- MSM
    def msm(self, table, scalars, offset=0, mont=False):
        """scalars: (n, 4) uint64 (or list of ints). Returns ((2*NL,) uint64, inf)."""
        if not isinstance(scalars, np.ndarray):
            scalars = ints_to_limbs(scalars, 4)
        sc = np.ascontiguousarray(scalars, dtype=np.uint64)
        out = np.zeros(2 * self.nl, dtype=np.uint64)
        oinf = np.zeros(1, dtype=np.uint8)
        check(lib().vc_msm(self.h, table, offset, _ptr(sc), sc.shape[0], 1 if mont else 0, _ptr(out),
                           _ptr(oinf)), "vc_msm")
        return out, int(oinf[0])

    def msm_point(self, table, scalars, offset=0, mont=False):
        xy, inf = self.msm(table, scalars, offset, mont)
        return arrays_to_points(self.curve, xy[None, :], np.array([inf]))[0]

    def msm_device(self, table, d_scalars_ptr, n, offset=0, mont=False):
        # ctypes buffers passed as they are (two numpy arrays and two data_as pointers cost a few us
        # per call: the bench's timed step); the result is a numpy view of the output buffer
        out = (ctypes.c_uint64 * (2 * self.nl))()
        oinf = ctypes.c_uint8(0)
        check(lib().vc_msm_device(self.h, table, offset, ctypes.c_void_p(d_scalars_ptr), n,
                                  1 if mont else 0, out, ctypes.byref(oinf)), "vc_msm_device")
        return np.frombuffer(out, dtype=np.uint64), int(oinf.value)

    def msm_device_many(self, table, d_scalars_ptrs, n, mont=None):
        """len(d_scalars_ptrs) MSMs over one table (vc_msm_device_many): one batched pipeline on
        the radix shared-window geometry -> list of (xy, inf)"""
        K = len(d_scalars_ptrs)
        ptrs = (ctypes.c_void_p * max(K, 1))(*[ctypes.c_void_p(p) for p in d_scalars_ptrs])
        mt = np.array([1 if (mont and mont[k]) else 0 for k in range(K)] or [0], dtype=np.int32)
        out = np.zeros((max(K, 1), 2 * self.nl), dtype=np.uint64)
        oinf = np.zeros(max(K, 1), dtype=np.uint8)
        check(lib().vc_msm_device_many(self.h, table, ptrs, _ptr(mt), n, K, _ptr(out), _ptr(oinf)),
              "vc_msm_device_many")
        return [(out[k], int(oinf[k])) for k in range(K)]

    def device_mad_rate(self):
        """Measured v_mad_u64_u32 throughput of this device (tera-ops/s)."""
        v = ctypes.c_double(0)
        check(lib().vc_device_mad_rate(self.h, ctypes.byref(v)), "vc_device_mad_rate")
        return v.value

    def point_words(self):
        return lib().vc_point_words(self.cid)

    def msm_device_partial(self, table, d_scalars_ptr, n, offset=0, mont=False):
        acc = np.zeros(self.point_words(), dtype=np.uint32)
        check(lib().vc_msm_device_partial(self.h, table, offset, ctypes.c_void_p(d_scalars_ptr), n,
                                          1 if mont else 0, _ptr(acc)), "vc_msm_device_partial")
        return acc

    def msm_partial(self, table, scalars, offset=0, mont=False):
        """un-normalised accumulator of the MSM over table[offset, offset + n) from host scalars"""
        sc = np.ascontiguousarray(scalars, dtype=np.uint64)
        acc = np.zeros(self.point_words(), dtype=np.uint32)
        check(lib().vc_msm_partial(self.h, table, offset, _ptr(sc), len(sc), 1 if mont else 0, _ptr(acc)),
              "vc_msm_partial")
        return acc

    def msm_last_plan(self):
        """geometry of the last MSM on this engine (vc_msm_last_plan): window bits, windows, terms
        per point, radix multiplier (radix = mul * 2^bits), shared windows"""
        v = [ctypes.c_int() for _ in range(5)]
        check(lib().vc_msm_last_plan(self.h, *[ctypes.byref(x) for x in v]), "vc_msm_last_plan")
        c, W, terms, mul, shared = (x.value for x in v)
        return {"window_bits": c, "windows": W, "terms_per_point": terms, "radix_mul": mul,
                "shared_windows": bool(shared)}

    def msm_device_window_part(self, table, d_scalars_ptr, n, part, parts, offset=0, mont=False):
        """Accumulator of Pippenger windows [part*W/parts, (part+1)*W/parts) of the whole MSM."""
        acc = np.zeros(self.point_words(), dtype=np.uint32)
        check(lib().vc_msm_device_window_part(self.h, table, offset, ctypes.c_void_p(d_scalars_ptr), n,
                                              1 if mont else 0, part, parts, _ptr(acc)),
              "vc_msm_device_window_part")
        return acc

    def partials_sum(self, accs):
        return partials_sum(self.curve, accs)

    def msm_batch(self, table, scalars, width, mont=False):
        """scalars: (batch*width, 4) uint64. Returns ((batch, 2*NL) uint64, (batch,) uint8)."""
        sc = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        assert sc.shape[0] % width == 0
        batch = sc.shape[0] // width
        out = np.zeros((batch, 2 * self.nl), dtype=np.uint64)
        oinf = np.zeros(batch, dtype=np.uint8)
        check(lib().vc_msm_batch(self.h, table, width, _ptr(sc), batch, 1 if mont else 0, _ptr(out),
                                 _ptr(oinf)), "vc_msm_batch")
        return out, oinf

    def msm_batch_sparse(self, table, row_ptr, cols, scalars, mont=False):
        """CSR batched commits: row g = sum over j in [row_ptr[g], row_ptr[g+1]) of
        scalars[j] * bases[cols[j]]. Returns ((batch, 2*NL) uint64, (batch,) uint8)."""
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint64)
        cols = np.ascontiguousarray(cols, dtype=np.uint32)
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        batch = len(row_ptr) - 1
        xy = np.zeros((max(batch, 1), 2 * NL[self.curve]), dtype=np.uint64)
        inf = np.zeros(max(batch, 1), dtype=np.uint8)
        check(lib().vc_msm_batch_sparse(self.h, table, batch, _ptr(row_ptr), _ptr(cols), _ptr(scalars),
                                        1 if mont else 0, _ptr(xy), _ptr(inf)), "vc_msm_batch_sparse")
        return xy[:batch], inf[:batch]

    def msm_batch_device(self, table, width, d_scalars_ptr, batch, d_out_xy_ptr, d_out_inf_ptr, mont=False):
        check(lib().vc_msm_batch_device(self.h, table, width, ctypes.c_void_p(d_scalars_ptr), batch,
                                        1 if mont else 0, ctypes.c_void_p(d_out_xy_ptr),
                                        ctypes.c_void_p(d_out_inf_ptr)), "vc_msm_batch_device")
