"""TEST INFRASTRUCTURE ONLY (never shipped, never measured).

Restatement of the engine's signed-window scalar decomposition
(verkle-kzg_amd/csrc/msm.hip: choose_window, for_each_digit, msm_run_t's window slices), used
to check the window-sliced multi-GPU split (vc_msm_device_window_part): the part-k MSM equals
sum_i s_i^(k) P_i with s_i^(k) = sum_{w in [kW/G, (k+1)W/G)} d_iw 2^(c w), and the parts add
up to the reference inner_product (vector-commit/src/utils.rs:16-19).
"""

SCALAR_BITS = {"bn254": 254, "bls12_381": 255, "bandersnatch": 253}


def choose_window(n):
    for lim, c in ((1 << 19, 16), (1 << 17, 15), (1 << 15, 13), (1 << 12, 11), (1 << 9, 9), (64, 7)):
        if n >= lim:
            return c
    return 5


def signed_digits(s, c, W):
    """W signed c-bit digits d_w in (-2^(c-1), 2^(c-1)] with s = sum d_w 2^(c w)."""
    half, out, carry = 1 << (c - 1), [], 0
    for _ in range(W):
        raw = (s & ((1 << c) - 1)) + carry
        s >>= c
        if raw > half:
            out.append(raw - (1 << c))
            carry = 1
        else:
            out.append(raw)
            carry = 0
    return out


def window_slice(curve, n, part, parts):
    c = choose_window(n)
    W = (SCALAR_BITS[curve] + 1 + c - 1) // c
    return c, W, part * W // parts, (part + 1) * W // parts


def part_scalars(curve, scalars, part, parts, r):
    """Per-term scalars (mod r) of window slice `part` of `parts`."""
    c, W, wb, we = window_slice(curve, len(scalars), part, parts)
    out = []
    for s in scalars:
        d = signed_digits(s, c, W)
        out.append(sum(d[w] << (c * w) for w in range(wb, we)) % r)
    return out
