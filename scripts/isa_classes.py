#!/usr/bin/env python3
"""Per-phase instruction-class histogram of one kernel from its gfx950 assembly.

usage: isa_classes.py <file.s> <kernel symbol or a unique prefix of it> [phase names...]

The kernel body (symbol .. .Lfunc_end) is cut at every s_barrier into phases (the
guide stage's phases are separated by barriers, vip_texture.hip). Each instruction is
counted in one class:
  valu_fast   f32 add/sub/mul/fma/fmac, integer add/sub, and/or/xor, mov, not: ~1.2 ns per
              wave-instruction per SIMD back to back (microbench/valu_rates.hip)
  valu_slow   sad, shifts-with-op (lshl_or/add), bfe, cvt, min/max/med3, cndmask, compares,
              mad_u32_u24/mad_legacy, perm, alignbit, dot2, packed (v_pk_*): 1.55-2.1 ns back to back
              (they interleave with fast ops at the fast rate up to about 1:1)
  valu_shift  plain shifts (lshlrev/lshrrev/ashrrev)
  valu_trans  transcendental/quarter-rate (exp, log, rcp, rsq, sqrt, sin, cos)
  valu_f64    double-precision ops (v_*_f64, v_div_*, v_trig_preop, v_frexp/ldexp on f64)
  lds         ds_* ; vmem: global_/buffer_/flat_ loads and stores
  salu        s_* other than waits, barriers and branches; wait: s_waitcnt; branch: s_cbranch/s_branch
Static counts: the phases the guide stage runs are straight-line code, except the loops
this script reports (a backward branch inside a phase), whose bodies run more than once.
"""
import collections
import re
import sys

FAST = re.compile(r"^v_(add|sub|subrev|mul|fma|fmac|mac)_f32|^v_(add|sub|subrev)_(co_)?(u32|i32|nc_u32)|"
                  r"^v_(and|or|xor|not)_b32|^v_mov_b32|^v_(add|sub)_co_ci_u32|^v_(add|sub)c_")
SLOW = re.compile(r"^v_(sad|lshl_or|lshl_add|add_lshl|and_or|or3|xor3|add3|bfe|bfi|cvt|min|max|med3|cndmask|cmp|"
                  r"mad_u32|mad_i32|mad_legacy|mad_u16|mad_u64|mul_lo|mul_hi|mul_u32|mul_i32|perm|alignbit|alignbyte|"
                  r"dot2|pk_|readfirstlane|readlane|writelane|lerp|msad|sad_|bcnt|ffbh|ffbl|mbcnt|sat_pk)")
SHIFT = re.compile(r"^v_(lshlrev|lshrrev|ashrrev)_b(16|32|64)")
TRANS = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_(f32|f16|legacy)")
F64 = re.compile(r"_f64|^v_div_(scale|fmas|fixup)|^v_trig_preop")


def classify(op: str) -> str:
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if F64.search(op):
            return "valu_f64"
        if TRANS.search(op):
            return "valu_trans"
        if SHIFT.search(op):
            return "valu_shift"
        if FAST.search(op):
            return "valu_fast"
        if SLOW.search(op):
            return "valu_slow"
        return "valu_other"
    return "other"


def body(path: str, sym: str) -> list:
    lines, inside, name = [], False, None
    with open(path) as fh:
        for ln in fh:
            if not inside:
                m = re.match(r"^([A-Za-z_0-9.$]+):", ln)
                if m and m.group(1).startswith(sym) and not m.group(1).startswith(".L"):
                    inside, name = True, m.group(1)
                continue
            if ln.startswith(".Lfunc_end"):
                break
            lines.append(ln.rstrip("\n"))
    if not inside:
        raise SystemExit(f"{sym}: not found in {path}")
    return name, lines


def main():
    path, sym = sys.argv[1], sys.argv[2]
    names = sys.argv[3:]
    name, lines = body(path, sym)
    phases = [collections.Counter()]
    ops = [collections.Counter()]
    labels = {}
    loops = []
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(phases) - 1
            continue
        op = s.split()[0]
        if op == "s_barrier":
            phases.append(collections.Counter())
            ops.append(collections.Counter())
            continue
        c = classify(op)
        phases[-1][c] += 1
        ops[-1][op] += 1
        if op.startswith(("s_cbranch", "s_branch")):
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] == len(phases) - 1:
                loops.append((len(phases) - 1, tgt))
    cols = ["valu_fast", "valu_slow", "valu_shift", "valu_trans", "valu_f64", "valu_other", "lds", "vmem", "salu",
            "wait", "branch"]
    print(f"# {name}")
    print("| phase | " + " | ".join(cols) + " | VALU total | slow-class share |")
    print("|---|" + "---|" * (len(cols) + 2))
    tot = collections.Counter()
    for i, p in enumerate(phases):
        tot.update(p)
        valu = sum(v for k, v in p.items() if k.startswith("valu"))
        slow = p["valu_slow"] + p["valu_shift"] + p["valu_trans"] + p["valu_f64"] + p["valu_other"]
        label = names[i] if i < len(names) else f"after barrier {i}" if i else "entry"
        print(f"| {label} | " + " | ".join(str(p[c]) for c in cols) + f" | {valu} | {slow / max(valu, 1):.2f} |")
    valu = sum(v for k, v in tot.items() if k.startswith("valu"))
    slow = valu - tot["valu_fast"]
    print("| **total** | " + " | ".join(str(tot[c]) for c in cols) + f" | {valu} | {slow / max(valu, 1):.2f} |")
    if loops:
        print("\nloops (backward branches inside a phase): " + ", ".join(f"phase {p} -> {t}" for p, t in loops))
    print("\ntop VALU ops per phase:")
    for i, o in enumerate(ops):
        top = [(k, v) for k, v in o.most_common() if k.startswith("v_")][:12]
        label = names[i] if i < len(names) else f"phase {i}"
        print(f"  {label}: " + ", ".join(f"{k} {v}" for k, v in top))


if __name__ == "__main__":
    main()
