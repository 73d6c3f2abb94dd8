"""Static instruction mix of the headline accumulate kernel (k_msm_accumulate on the BLS12-381
pair-layout radix copies) in the built libvkzg.so: disassembles the gfx950 code object and counts
the kernel's instructions by class, whole kernel and inside its main loop (the basic blocks
between the loop head and its back edge are taken as the body of the add). No GPU needed.
usage: acc_breakdown.py [lib] [kernel-substring]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_regs import code_objects  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
CLASSES = [
    ("mad64 (v_mad_i64_i32 / v_mad_u64_u32)", r"^v_mad_(i64_i32|u64_u32)"),
    ("mul32 (v_mul_lo / v_mul_hi)", r"^v_mul_(lo|hi)_"),
    ("64-bit shift", r"^v_(ashrrev|lshrrev|lshlrev)_(b|i)64"),
    ("64-bit add (v_lshl_add_u64 / v_add_co + v_addc)", r"^v_(lshl_add_u64|add_co_u32|addc_co_u32|add_co_ci|sub_co_u32|subb_co_u32|subrev_co_u32|sub_co_ci)"),
    ("32-bit add / sub / add3", r"^v_(add|sub|subrev)_(u32|i32|nc_u32)|^v_add3_u32|^v_add_u32|^v_sub_u32"),
    ("bitfield / shift 32 (bfe, alignbit, lshl_or, shifts)", r"^v_(bfe|bfi|alignbit|alignbyte|lshl_or|lshl_add_u32|and_or|or3|lshlrev_b32|lshrrev_b32|ashrrev_i32)"),
    ("logic 32 (and / or / xor / not)", r"^v_(and|or|xor|not)_b32"),
    ("select / compare", r"^v_(cndmask|cmp|cmpx)"),
    ("move", r"^v_(mov|readfirstlane|readlane|writelane)"),
    ("vector memory", r"^(global|buffer|flat|scratch)_"),
    ("scalar", r"^s_"),
    ("lds / dpp", r"^ds_"),
]


def classify(op):
    for name, pat in CLASSES:
        if re.match(pat, op):
            return name
    return "other VALU" if op.startswith("v_") else "other"


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "lib", "libvkzg.so")
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_msm_accumulateINS_7SWCurveINS_8BLS381FqELi4ELb0EEENS_4SW30IS3_NS_11F30BLS381FqEE4AffP"
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".hsaco", delete=False) as f:
            f.write(co)
            tmp = f.name
        try:
            txt = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", tmp], capture_output=True, text=True).stdout
        finally:
            os.unlink(tmp)
        start = None
        lines = txt.splitlines()
        for i, l in enumerate(lines):
            if re.match(r"^[0-9a-f]+ <.*" + re.escape(sub) + r".*>:", l):
                start = i
                break
        if start is None:
            continue
        body = []
        for l in lines[start + 1:]:
            if re.match(r"^[0-9a-f]+ <", l):
                break
            m = re.match(r"\s+(\S+)", l)
            if m and not l.strip().startswith(";"):
                body.append(l.strip())
        ops = [b.split()[0] for b in body if b and not b.endswith(":")]
        tot = collections.Counter(classify(o) for o in ops)
        print(f"kernel {lines[start].split('<')[1][:100]}...: {len(ops)} instructions")
        valu = sum(v for k, v in tot.items() if k not in ("scalar", "vector memory", "other"))
        for k, v in tot.most_common():
            print(f"  {k:55s} {v:6d}  {100 * v / max(valu, 1):5.1f} % of VALU" if k not in ("scalar", "vector memory", "other")
                  else f"  {k:55s} {v:6d}")
        print(f"  VALU total {valu}")
        return
    print("kernel not found")


if __name__ == "__main__":
    main()
