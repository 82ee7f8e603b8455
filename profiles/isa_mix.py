#!/usr/bin/env python3
"""Instruction mix of the bucket-accumulation add (k_accumulate<3>) from the compiled gfx950 ISA:
the production build, and a count-only copy whose add_aff has its rare-case branch (the exact
P == 0 test that leads to doubling / infinity) removed, so that the common path is one basic block.
Prints, per build, the hot blocks' instruction counts and, for the common path, the opcode classes
per bucket entry. Evidence for DESIGN.md §3 (why the XYZZ add sits at ~2,200 VALU instructions per
entry: 1,467 mads + the per-product reduction / carry overhead), next to the dynamic counts of the
counter pass (profiles/r02/clock_valu_issue.txt: 2,296 per entry including loop control).
usage: python profiles/isa_mix.py [out.txt]"""
import collections
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "kzg-grandsums-study_amd", "csrc")
SYM = "_ZN3kgs12k_accumulateILi3EEEvPjS1_S1_PKjS3_jS3_jS1_j"


def compile_asm(src_dir, out):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                           "-S", os.path.join(src_dir, "msm.hip"), "-o", out], stderr=subprocess.DEVNULL)


def blocks_of(asm):
    lines = open(asm).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.startswith(SYM + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    blocks, cur = [], ("entry", [])
    for ln in lines[start:end]:
        s = ln.strip()
        if re.match(r"^\.LBB\d+_\d+:", s):
            blocks.append(cur)
            cur = (s.split(":")[0], [])
        elif s and not s.startswith(";") and not s.startswith("."):
            cur[1].append(s.split()[0])
    blocks.append(cur)
    return blocks


CLASSES = [("v_mad_u64_u32", "mad 32x32+64 (partial products)"),
           ("v_mul_lo_u32", "mul_lo (CIOS m = t0 * q')"),
           ("v_and_b32", "and (m mask, limb mask)"),
           ("v_lshrrev_b64", "64-bit shift (column carry)"),
           ("v_lshl_add_u64", "64-bit add (carry into next column)"),
           ("v_add", "32-bit add/add3 (limb-wise sums)"),
           ("v_sub", "32-bit sub (limb-wise differences)"),
           ("v_alignbit_b32", "funnel shift (unpack)"),
           ("v_cndmask", "select (sign, special cases)"),
           ("v_", "other VALU"),
           ("s_", "scalar / branch"),
           ("global_", "memory"),
           ("", "other")]


# measured issue cost per wave64 instruction, SIMD cycles at the nominal clock
# (profiles/ubench/issue_rates2.hip -> profiles/ubench/issue_rates2_r03.txt); VOP2 32-bit ops ~2.3-2.8,
# every VOP3 / 64-bit op ~4.2-4.4 (v_cndmask_b32's 22.9 there is its benchmark's VCC dependency, not
# the op: priced as a VOP2 op)
ISSUE = {"v_mad_u64_u32": 4.16, "v_mul_lo_u32": 4.28, "v_and_b32_e32": 2.49, "v_lshrrev_b64": 4.16,
         "v_lshl_add_u64": 4.40, "v_ashrrev_i64": 4.16, "v_sub_u32_e32": 2.47, "v_add_u32_e32": 2.82,
         "v_alignbit_b32": 4.16, "v_lshrrev_b32_e32": 2.28, "v_lshlrev_b32_e32": 2.28, "v_add3_u32": 4.20,
         "v_lshl_add_u32": 4.18, "v_or3_b32": 4.17, "v_or_b32_e32": 2.47, "v_cndmask_b32_e32": 2.49,
         "v_mov_b32_e32": 2.24, "v_bfe_u32": 4.15, "v_lshl_or_b32": 4.17}


def issue_cycles(ops):
    """(total SIMD cycles, cycles by opcode) of a straight-line instruction list: VALU at the measured
    per-opcode cost (unlisted VOP3 forms 4.2, unlisted 32-bit VOP2 forms 2.4); scalar / memory not
    counted (they issue on other ports)"""
    by = collections.Counter()
    for op in ops:
        if not op.startswith("v_"):
            continue
        c = ISSUE.get(op)
        if c is None:
            c = 2.4 if op.endswith("_e32") else 4.2
        by[op] += c
    return sum(by.values()), by


def classify(op):
    for pre, name in CLASSES:
        if op.startswith(pre):
            return name
    return "other"


def main():
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else sys.stdout
    tmp = tempfile.mkdtemp()
    try:
        prod = os.path.join(tmp, "prod.s")
        compile_asm(CSRC, prod)
        cdir = os.path.join(tmp, "csrc")
        shutil.copytree(CSRC, cdir)
        f29 = os.path.join(cdir, "field29.hpp")
        s = open(f29).read()
        a = s.index("    if (PP.maybe_zero8()) {  // rare: decide exactly")
        b = s.index("    // ordered so that P, PP, ZZ, ZZZ and Qv die early")
        open(f29, "w").write(s[:a] + s[b:])
        cnt = os.path.join(tmp, "count.s")
        compile_asm(cdir, cnt)
        for label, asm in (("production", prod), ("count-only (rare branch removed)", cnt)):
            bl = blocks_of(asm)
            big = [(n, ins) for n, ins in bl if len(ins) >= 30]
            print(f"== k_accumulate<3>, {label}: blocks of >= 30 instructions", file=out)
            for n, ins in big:
                print(f"   {n:12s} {len(ins):5d} instr, {sum(1 for x in ins if x == 'v_mad_u64_u32'):5d} v_mad_u64_u32",
                      file=out)
        hot = max(blocks_of(cnt), key=lambda b: len(b[1]))[1]
        c = collections.Counter(classify(x) for x in hot)
        print(f"\n== common path of one bucket add (count-only build, hot block: {len(hot)} instructions)", file=out)
        for _, name in CLASSES:
            if c.get(name):
                print(f"   {name:40s} {c[name]:5d}", file=out)
        mads = c.get(CLASSES[0][1], 0)
        print(f"   non-mad VALU: {sum(v for k, v in c.items() if k not in (CLASSES[0][1], 'scalar / branch', 'memory', 'other')) }",
              file=out)
        print(f"   per 254-bit product (10 product-equivalents: 6 mul + 2 sqr + 1 lazily reduced double product"
              f" counted as 1.5 + ...): mads {mads} = 6 x 162 + 2 x 126 + 243", file=out)
        tot, by = issue_cycles(hot)
        print(f"\n== issue cycles of the common path per bucket entry (measured per-opcode costs): {tot:.0f} SIMD cycles",
              file=out)
        for op, cyc in by.most_common(12):
            print(f"   {op:22s} {cyc:7.0f}  ({100 * cyc / tot:4.1f} %)", file=out)
        print(f"   non-mad: {tot - by['v_mad_u64_u32']:.0f} cycles ({100 * (tot - by['v_mad_u64_u32']) / tot:.1f} %)",
              file=out)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
