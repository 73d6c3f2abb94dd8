"""TEST INFRASTRUCTURE ONLY (never shipped, never measured).

Restatement of the engine's signed-window scalar decomposition
(verkle-kzg_amd/csrc/msm.hip: choose_window, for_each_digit, k_glv_split, msm_run_t's window
slices), used to check the window-sliced multi-GPU split (vc_msm_device_window_part): the
part-k MSM equals sum_i s_i^(k) P_i with s_i^(k) = sum_{w in [kW/G, (k+1)W/G)} d_iw 2^(c w)
(with the GLV split on BLS12-381: the digits of both halves, the k2 half weighted by lambda),
and the parts add up to the reference inner_product (vector-commit/src/utils.rs:16-19).
"""

SCALAR_BITS = {"bn254": 254, "bls12_381": 255, "bandersnatch": 253}
# BLS12-381: lambda = z^2 - 1 with r = lambda^2 + lambda + 1 (phi(x, y) = (beta x, y) = [lambda])
GLV_LAMBDA = 0xac45a4010001a40200000000ffffffff
GLV_MIN_N = 4096
GLV_BITS = 128


def glv_active(curve, n):
    return curve == "bls12_381" and GLV_MIN_N <= n < (1 << 30)


def glv_split(k, r):
    """k_glv_split: k mod r = k1 + lambda k2 with |k1|, |k2| <= lambda/2 + 1; returns the
    signed halves (k1, k2)."""
    lam = GLV_LAMBDA
    k %= r
    q, rem = divmod(k, lam)
    half = lam >> 1
    if q > half:                      # (rem - 1) + lambda (q - lambda - 1) = k - r
        q, rem = q - lam - 1, rem - 1
    if rem > half:                    # (rem - lambda) + lambda (q + 1)
        rem, q = rem - lam, q + 1
    return rem, q


def top_shortfall(c, total):
    """bits the top window of `total` digit bits in c-bit windows lacks (msm.hip top_shortfall)"""
    W = (total + c - 1) // c
    return c - (total - c * (W - 1))


def choose_window(n, total):
    """msm.hip choose_window: the size rule, unless its top window is short by more than 2 bits;
    then the cheapest c in c0 - 5 .. c0 + 2 (W n + 2 W 2^(c-1)) whose top window is not."""
    c0 = 5
    for lim, c in ((1 << 19, 16), (1 << 17, 15), (1 << 15, 13), (1 << 12, 11), (1 << 9, 9), (64, 7)):
        if n >= lim:
            c0 = c
            break
    if top_shortfall(c0, total) <= 2:
        return c0
    best, best_cost = c0, None
    for c in range(max(4, c0 - 5), min(16, c0 + 2) + 1):
        if top_shortfall(c, total) > 2:
            continue
        W = (total + c - 1) // c
        cost = W * n + 2 * W * (1 << (c - 1))
        if best_cost is None or cost < best_cost:
            best, best_cost = c, cost
    return best


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


def glv_window(nv):
    return 16 if nv >= 1 << 19 else (13 if nv >= 1 << 15 else 10)


def window_slice(curve, n, part, parts):
    if glv_active(curve, n):
        c = glv_window(2 * n)
        W = (GLV_BITS + c - 1) // c
    else:
        c = choose_window(n, SCALAR_BITS[curve] + 1)
        W = (SCALAR_BITS[curve] + 1 + c - 1) // c
    return c, W, part * W // parts, (part + 1) * W // parts


def _part(v, c, W, wb, we):
    """digits of |v| in windows [wb, we), with v's sign"""
    d = signed_digits(abs(v), c, W)
    t = sum(d[w] << (c * w) for w in range(wb, we))
    return -t if v < 0 else t


def part_scalars(curve, scalars, part, parts, r):
    """Per-term scalars (mod r) of window slice `part` of `parts`."""
    c, W, wb, we = window_slice(curve, len(scalars), part, parts)
    glv = glv_active(curve, len(scalars))
    out = []
    for s in scalars:
        if glv:
            k1, k2 = glv_split(s, r)
            assert abs(k1) < 1 << 127 and abs(k2) < 1 << 127
            out.append((_part(k1, c, W, wb, we) + GLV_LAMBDA * _part(k2, c, W, wb, we)) % r)
        else:
            d = signed_digits(s, c, W)
            out.append(sum(d[w] << (c * w) for w in range(wb, we)) % r)
    return out


# Radix-B shared windows (msm.hip k_glv_radix / radix_digits, the one-GPU whole-table GLV MSM):
# B = 5 * 2^16, 7 windows (B^7 / 2 > 2^127), B / 2 = 5 * 2^15 buckets in one set.
RADIX_MUL, RADIX_C0, RADIX_W = 5, 16, 7


def radix_digits(k, mul=RADIX_MUL, c0=RADIX_C0, W=RADIX_W):
    """W signed digits d_w in (-B/2, B/2] of 0 <= k < 2^127 with k = sum d_w B^w, B = mul 2^c0
    (radix_digits: low c0 bits, then (k >> c0) mod mul, carry recoding as signed_digits)."""
    B = mul << c0
    out, carry = [], 0
    for _ in range(W):
        raw = (k % B) + carry
        k //= B
        if raw > B // 2:
            out.append(raw - B)
            carry = 1
        else:
            out.append(raw)
            carry = 0
    assert k == 0 and carry == 0, "scalar too wide for the radix"
    return out


def radix_bucket_sum(buckets, lseg):
    """Host fold of the radix reduction (msm.hip slice_finish, msm_tail.hip segsum / bitsum):
    V = sum_b (b + 1) B_b = A + lseg * sum_j 2^j T_j with segments of lseg buckets,
    A = sum_s acc_s, acc_s = sum_k (k + 1) B_{s lseg + k}, T_j = sum_{s: bit j of s} R_s.
    Works on any additive group given as numbers (integers mod anything)."""
    S = len(buckets) // lseg
    R = [sum(buckets[s * lseg:(s + 1) * lseg]) for s in range(S)]
    A = sum((k + 1) * buckets[s * lseg + k] for s in range(S) for k in range(lseg))
    J = max(1, (S - 1).bit_length())
    T = [sum(R[s] for s in range(S) if (s >> j) & 1) for j in range(J)]
    return A + lseg * sum(t << j for j, t in enumerate(T))


def radix_bucket_sum_residue(buckets, lseg):
    """The residue form of the same reduction (msm_tail.hip k_msm_segr + the U sums of
    k_msm_bitsum, msm.hip shared_set_sum): with b = lseg s + r,
    V = lseg * sum_j 2^j T_j + sum_r (r + 1) U_r,  U_r = sum_s B_{lseg s + r},
    and sum_r (r + 1) U_r taken as the host does it, by suffix sums."""
    S = len(buckets) // lseg
    R = [sum(buckets[s * lseg:(s + 1) * lseg]) for s in range(S)]
    U = [sum(buckets[s * lseg + r] for s in range(S)) for r in range(lseg)]
    J = max(1, (S - 1).bit_length())
    T = [sum(R[s] for s in range(S) if (s >> j) & 1) for j in range(J)]
    v = lseg * sum(t << j for j, t in enumerate(T))
    suf = 0
    for r in range(lseg - 1, -1, -1):
        suf += U[r]
        v += suf
    return v


def bit_sums_marginal(R, h):
    """T_j = sum_{s: bit j of s} R_s by the marginal form of msm_tail.hip k_msm_bitsum /
    PartLoc (msm_tail.hpp msm_tail_plan): with s = G hi + lo (G = 2^h), the column sums
    L_lo = sum_hi R_{G hi + lo} and row sums H_hi = sum_lo R_{G hi + lo}; T_j is the sum of the
    L_lo with bit j of lo (j < h) or of the H_hi with bit j - h of hi (j >= h)."""
    S = len(R)
    J = max(1, (S - 1).bit_length())
    assert S == 1 << J and 0 < h < J
    G, Hn = 1 << h, 1 << (J - h)
    Lc = [sum(R[hi * G + lo] for hi in range(Hn)) for lo in range(G)]
    Hr = [sum(R[hi * G + lo] for lo in range(G)) for hi in range(Hn)]
    return [sum(Lc[lo] for lo in range(G) if (lo >> j) & 1) if j < h else
            sum(Hr[hi] for hi in range(Hn) if (hi >> (j - h)) & 1) for j in range(J)]


def bit_sums_marginal_urow(R, h, pL):
    """The row-derived total of the marginal form (msm_tail.hpp TailPlan::urow, msm_tail.hip
    PartLoc, msm.hip slice_finish), for Lseg = 1 where the total U = sum_s R_s is wanted beside the
    T_j: every column sum L_lo is made as pL partials (pL waves over Hn / pL rows each); T_j (j < h)
    sums the partials of the columns with bit j of lo, T_j (j >= h) the row sums H_hi with bit j - h
    of hi; the final stage's U slot holds X = the row sums of even hi, and the host adds T_h.
    Returns (T, U)."""
    S = len(R)
    J = max(1, (S - 1).bit_length())
    G, Hn = 1 << h, 1 << (J - h)
    assert S == 1 << J and 0 < h < J and pL >= 1 and Hn % pL == 0
    part = [[sum(R[hi * G + lo] for hi in range(p * Hn // pL, (p + 1) * Hn // pL)) for p in range(pL)]
            for lo in range(G)]
    Hr = [sum(R[hi * G + lo] for lo in range(G)) for hi in range(Hn)]
    T = [sum(x for lo in range(G) if (lo >> j) & 1 for x in part[lo]) if j < h else
         sum(Hr[hi] for hi in range(Hn) if (hi >> (j - h)) & 1) for j in range(J)]
    X = sum(Hr[hi] for hi in range(0, Hn, 2))
    return T, X + T[h]

