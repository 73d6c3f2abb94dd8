"""Per-wave timeline of the MSM tail kernels, from the diagnostic build
(make EXTRA=-DVKZG_TAIL_TRACE LIBOUT=lib_trace/libvkzg.so BUILD=build_trace; run with
VKZG_LIB=<that library>): every lane of k_msm_fixup_own / walk_q (kernel 0), k_msm_segr_q (1),
k_msm_bitsum (2) and k_msm_sumpart_q (3) stamps entry and exit on s_memrealtime (100 MHz), its
HW_ID / XCC_ID and a kernel word (fix-up: chain length; bit sums: kind << 24 | items per lane;
final sums: partial count). One traced 2^20 BLS12-381 MSM after warm-up (the bench's headline
call), then the G = 8 window parts 0 and 7 (the per-rank share of the 8-GPU split).
Per kernel: waves, span (first entry to last exit), wave entry offsets and lifetimes
(percentiles), active waves over time, the longest waves with their words and slots.
usage: tail_trace.py [out.json]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import vkzg  # noqa: E402
from vkzg._lib import lib  # noqa: E402

TT_KERNELS, TT_MAXT = 4, 1 << 18
NAMES = ["fixup", "segr_q", "bitsum", "sumpart_q"]
TICK_US = 0.01  # s_memrealtime: 100 MHz


def fetch():
    buf = np.zeros(TT_KERNELS * TT_MAXT * 4, dtype=np.uint64)
    fn = lib().vkzg_tail_trace_fetch
    fn.restype = ctypes.c_int
    rc = fn(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.size))
    assert rc == 0, rc
    return buf.reshape(TT_KERNELS, TT_MAXT, 4)


def pct(a, qs=(0, 10, 50, 90, 99, 100)):
    return {f"p{q}": round(float(np.percentile(a, q)), 2) for q in qs} if len(a) else {}


def analyse(tr):
    out, t_first = {}, None
    for k in range(TT_KERNELS):
        rec = tr[k]
        valid = (rec[:, 3] >> np.uint64(63)) == 1
        if not valid.any():
            continue
        gid = np.nonzero(valid)[0]
        t0, t1 = rec[gid, 0].astype(np.int64), rec[gid, 1].astype(np.int64)
        info = (rec[gid, 3] & np.uint64(0xffffffff)).astype(np.int64)
        hw = (rec[gid, 2] & np.uint64(0xffffffff)).astype(np.int64)
        xcc = (rec[gid, 2] >> np.uint64(32)).astype(np.int64) & 0xf
        wave = gid // 64
        uw, inv = np.unique(wave, return_inverse=True)
        ws = np.full(len(uw), np.iinfo(np.int64).max)
        we = np.zeros(len(uw), dtype=np.int64)
        wi = np.zeros(len(uw), dtype=np.int64)
        np.minimum.at(ws, inv, t0)
        np.maximum.at(we, inv, t1)
        np.maximum.at(wi, inv, info)
        whw = np.zeros(len(uw), dtype=np.int64)
        wx = np.zeros(len(uw), dtype=np.int64)
        whw[inv] = hw
        wx[inv] = xcc
        k0 = ws.min()
        t_first = k0 if t_first is None else min(t_first, k0)
        life = (we - ws) * TICK_US
        start = (ws - k0) * TICK_US
        end = (we - k0) * TICK_US
        span = (we.max() - k0) * TICK_US
        # active waves in 2-us bins
        nb = int(span / 2) + 1
        act = np.zeros(nb)
        for s_, e_ in zip(start, end):
            act[int(s_ / 2):int(e_ / 2) + 1] += 1
        order = np.argsort(-life)[:10]
        simd = (whw >> 4) & 3
        cu = (whw >> 8) & 0xf
        se = (whw >> 13) & 0x7
        per_xcc_end = {int(x): round(float(end[wx == x].max()), 2) for x in np.unique(wx)}
        out[NAMES[k]] = {
            "waves": int(len(uw)), "lanes": int(len(gid)), "span_us": round(float(span), 2),
            "entry_offset_us": pct(start), "lifetime_us": pct(life), "exit_us": pct(end),
            "waves_entered_by_us": {f"{x}us": int((start <= x).sum()) for x in (1, 2, 5, 10, 20, 40)},
            "active_waves_per_2us": [int(a) for a in act[:60]],
            "info_max_per_wave": pct(wi),
            "longest": [{"wave": int(uw[i]), "life_us": round(float(life[i]), 2), "start_us": round(float(start[i]), 2),
                         "info": int(wi[i]), "xcc": int(wx[i]), "se": int(se[i]), "cu": int(cu[i]),
                         "simd": int(simd[i])} for i in order],
            "exit_by_xcc_us": per_xcc_end,
            "waves_per_simd_slot_max": int(np.bincount(wx * 4096 + se * 512 + cu * 8 + simd * 2).max()),
        }
    for k in out.values():
        k["_note"] = "times in us from the kernel's first wave entry"
    return out


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else None
    curve, n = "bls12_381", 1 << 20
    e = vkzg.Engine(curve)
    table = e.random_bases(n, seed=2024)
    sc = vkzg.random_scalars(curve, n, np.random.default_rng(1234))
    d_sc = torch.from_numpy(sc.view(np.int64).copy()).cuda()
    torch.cuda.synchronize()
    res = {}
    for _ in range(10):
        e.msm_device(table, d_sc.data_ptr(), n)
    fetch()
    e.msm_device(table, d_sc.data_ptr(), n)
    res["msm_2e20"] = analyse(fetch())
    print("msm_2e20", json.dumps({k: {kk: v[kk] for kk in ("waves", "span_us", "entry_offset_us", "lifetime_us")}
                                  for k, v in res["msm_2e20"].items()}), flush=True)
    for part in (0, 7):
        for _ in range(5):
            e.msm_device_window_part(table, d_sc.data_ptr(), n, part, 8)
        fetch()
        e.msm_device_window_part(table, d_sc.data_ptr(), n, part, 8)
        res[f"window_part_{part}_of_8"] = analyse(fetch())
        print(f"part {part}", json.dumps({k: {kk: v[kk] for kk in ("waves", "span_us", "entry_offset_us", "lifetime_us")}
                                          for k, v in res[f"window_part_{part}_of_8"].items()}), flush=True)
    e.close()
    if path:
        with open(path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
