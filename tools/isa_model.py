"""Issue-cycle model of a kernel from its gfx950 ISA:
    python tools/isa_model.py <file.hip> <kernel-substring> [extra hipcc flags]
Compiles with -save-temps into a temp dir, counts the VALU instructions of the
kernel body and prices them with the per-wave64 issue costs measured by
tools/ubench_ops.hip: VOP3-encoded instructions (v_mad_u64_u32, v_add3_u32,
v_lshl_add_u64, v_lshrrev_b64, v_mul_lo_u32, v_alignbit_b32, *_e64, ...)
~4.2 cycles, VOP1/VOP2 (*_e32, v_mov_b32, ...) ~2.2 cycles per SIMD.
For k_accumulate29 the body is one mixed addition plus the per-piece
bookkeeping, so the total approximates the issue cycles of one addition per
wave (bench.py MADD_ISSUE_CYCLES)."""
import collections
import os
import re
import subprocess
import sys
import tempfile

VOP3 = ("v_mad_", "v_mul_lo", "v_mul_hi", "v_add3", "v_lshl_add", "v_lshl_or", "v_or3", "v_and_or",
        "v_alignbit", "v_bfe", "v_bfi", "v_lshrrev_b64", "v_lshlrev_b64", "v_ashrrev_i64", "v_xad",
        "v_perm", "v_mov_b64", "v_cmp_gt_u64", "v_cmp_eq_u64", "v_cmp_lt_u64", "v_cmp_ne_u64")


def cost(op):
    if op.endswith("_e64") or op.startswith(VOP3):
        return 4.2
    return 2.2


def main():
    src, kname = sys.argv[1], sys.argv[2]
    extra = sys.argv[3:]
    d = tempfile.mkdtemp()
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-save-temps", "-c", os.path.abspath(src), "-o", "k.o"] + extra, cwd=d,
                          stderr=subprocess.DEVNULL)
    s = open(os.path.join(d, [f for f in os.listdir(d) if f.endswith("gfx950.s")][0])).read()
    names = [m for m in re.findall(r"^(_Z\w+):", s, re.M) if kname in m]
    for nm in names:
        b = s.index(nm + ":")
        body = s[b:s.index(".Lfunc_end", b)]
        ops = collections.Counter()
        for line in body.split("\n"):
            t = line.strip()
            if t.startswith("v_"):
                ops[t.split()[0]] += 1
        cyc = sum(n * cost(o) for o, n in ops.items())
        print(f"{nm}: {sum(ops.values())} VALU instructions, {cyc:.0f} issue cycles")
        for o, n in ops.most_common(12):
            print(f"    {o:28s} {n:6d}  x {cost(o)}")


if __name__ == "__main__":
    main()
