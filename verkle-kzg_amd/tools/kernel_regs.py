"""Register use of the kernels in the built libvkzg.so (no GPU needed): unbundles the gfx950 code
object from the .hip_fatbin section and reads each kernel's AMDGPU metadata note (llvm-readelf).
usage: kernel_regs.py [lib] [name-substring]  -> "name vgpr_count agpr_count spills" lines.
Used by tests/test_abi.py to pin the occupancy of the hot kernels (k_msm_accumulate must stay at
<= 256 VGPRs + AGPRs: two waves per SIMD; a variant at 268 ran at one wave and 15 % slower)."""
import os
import re
import struct
import subprocess
import sys
import tempfile

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def _section(path, name):
    data = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sh(i):
        return struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize)
    stro = sh(shstrndx)[4]
    for i in range(shnum):
        h = sh(i)
        nm = data[stro + h[0]:data.index(b"\0", stro + h[0])].decode()
        if nm == name:
            return data[h[4]:h[4] + h[5]]
    raise KeyError(name)


def code_objects(lib):
    """gfx950 code objects of every offload bundle in the fat binary section"""
    blob = _section(lib, ".hip_fatbin")
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out, pos = [], 0
    while True:
        b = blob.find(magic, pos)
        if b < 0:
            break
        n, = struct.unpack_from("<Q", blob, b + 24)
        p = b + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple:
                out.append(blob[b + off:b + off + size])
        pos = b + 1
    return out


def kernel_regs(lib, sub=""):
    rows = []
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".hsaco", delete=False) as f:
            f.write(co)
            tmp = f.name
        try:
            txt = subprocess.run([READELF, "--notes", tmp], capture_output=True, text=True).stdout
        finally:
            os.unlink(tmp)
        for blk in txt.split("  - .agpr_count:")[1:]:
            def g(key):
                m = re.search(r"\." + key + r":\s+(\S+)", blk)
                return m.group(1) if m else None
            agpr = int(re.match(r"\s*(\d+)", blk).group(1))
            name = g("name")
            if name and sub in name:
                rows.append((name, int(g("vgpr_count")), agpr, int(g("vgpr_spill_count") or 0)))
    return rows


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "lib", "libvkzg.so")
    for r in kernel_regs(lib, sys.argv[2] if len(sys.argv) > 2 else ""):
        print(*r)
