"""ORACLE (test infrastructure only) -- arkworks 0.4 byte conventions for BN254, restated.

Parity at this boundary is UNPINNED against arkworks: the reference's tests hold no
golden bytes; these follow SURVEY.md Appendix A.3-A.6 and the
arkworks 0.4 source as published (ark-serialize / ark-ff / ark-ec 0.4.2).

  * compressed SW point  (lib.rs:63, transcript.rs:66)          -> ser_point_compressed
  * Fr canonical LE bytes (transcript.rs:66)                     -> ser_fr
  * usize as u64 LE (multiproof.rs:111)                          -> ser_usize
  * VCCommitment::to_data_item (lib.rs:56-67)                    -> to_data_item
  * DefaultFieldHasher<Sha256>/ExpanderXmd (transcript.rs:55)    -> hash_to_field
  * Affine::from_random_bytes (ipa_point_generator.rs:104)       -> from_random_bytes
"""
import hashlib

from .curves import BN254, sqrt_mod

SEC_PARAM = 128
# switch kept visible: ark-ff 0.4 DefaultFieldHasher::new sets block_size = len_per_base_elem
XMD_ZPAD_LEN = None  # None -> len_per_base_elem (48 for BN254 Fr); 64 would be RFC 9380 SHA-256


def ser_fr(x, nbytes=32):
    return int(x).to_bytes(nbytes, "little")


def ser_usize(z):
    return int(z).to_bytes(8, "little")


def ser_point_compressed(P, curve=BN254):
    """SW affine compressed: x LE, byte[-1] |= 0x80 if y is the larger root, 0x40 for infinity."""
    n = curve.fbytes
    if P is None:
        b = bytearray(n)
        b[-1] |= 0x40
        return bytes(b)
    x, y = P
    b = bytearray(int(x).to_bytes(n, "little"))
    neg_y = (-y) % curve.p
    if not (y <= neg_y):  # SWFlags::from_y_coordinate: YIsNegative iff !(y <= -y)
        b[-1] |= 0x80
    return bytes(b)


def to_data_item(P, curve=BN254):
    """lib.rs:56-67: identity -> 0 else from_le_bytes_mod_order(compressed(P)) (flags included)."""
    if P is None:
        return 0
    return int.from_bytes(ser_point_compressed(P, curve), "little") % curve.r


def _len_per_elem(modulus):
    return (modulus.bit_length() + SEC_PARAM + 7) // 8


def expand_message_xmd(msg, dst, n, block_size):
    """ark-ff 0.4 ExpanderXmd::expand with z_pad of `block_size` bytes."""
    b_len = 32
    ell = (n + b_len - 1) // b_len
    assert ell <= 255
    dst_prime = bytes(dst) + bytes([len(dst)])
    z_pad = bytes(block_size)
    lib_str = n.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + bytes(msg) + lib_str + b"\x00" + dst_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bytearray(bi)
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(a ^ b for a, b in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return bytes(out[:n])


def hash_to_field(msg, dst, modulus):
    """DefaultFieldHasher<Sha256,128>::hash_to_field(msg, 1)[0]: big-endian bytes mod r."""
    L = _len_per_elem(modulus)
    blk = L if XMD_ZPAD_LEN is None else XMD_ZPAD_LEN
    u = expand_message_xmd(msg, dst, L, blk)
    return int.from_bytes(u, "big") % modulus


def from_random_bytes(b, curve=BN254):
    """Affine::from_random_bytes for a 32-byte SW base field with 2 spare bits (BN254 Fq)."""
    assert len(b) == 32 and curve.fbytes == 32
    flags = b[31] & 0xC0
    xb = bytearray(b)
    xb[31] &= 0x3F
    x = int.from_bytes(bytes(xb), "little")
    if x >= curve.p:
        return "reject"
    x_sign = bool(flags & 0x80)
    is_inf = bool(flags & 0x40)
    if x_sign and is_inf:
        return "reject"
    if is_inf:
        return None if x == 0 else "reject"  # identity only for x == 0
    rhs = (x * x * x + curve.b) % curve.p
    y = sqrt_mod(rhs, curve.p)
    if y is None:
        return "reject"
    ny = (-y) % curve.p
    smaller, larger = (y, ny) if y <= ny else (ny, y)
    greatest = not x_sign  # YIsPositive -> get_point_from_x_unchecked(x, true) -> larger
    return (x, larger if greatest else smaller)


class TranscriptHasher:
    """transcript.rs:28-62: byte-buffer transcript, hash_to_field with DST = label given at new()."""

    def __init__(self, label, curve=BN254):
        self.state = bytearray()
        self.dst = label.encode()
        self.curve = curve

    def clone(self):
        t = TranscriptHasher.__new__(TranscriptHasher)
        t.state = bytearray(self.state)
        t.dst = self.dst
        t.curve = self.curve
        return t

    def append_bytes(self, raw, label):
        self.state += label.encode()
        self.state += raw

    def append_point(self, P, label):
        self.append_bytes(ser_point_compressed(P, self.curve), label)

    def append_fr(self, x, label):
        self.append_bytes(ser_fr(x), label)

    def append_usize(self, z, label):
        self.append_bytes(ser_usize(z), label)

    def digest(self, label, clear=True):
        self.state += label.encode()
        res = hash_to_field(bytes(self.state), self.dst, self.curve.r)
        if clear:
            self.state = bytearray(ser_fr(res)) + label.encode()
        return res
