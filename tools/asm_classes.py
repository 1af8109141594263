"""Instruction classes of one k_trace step slot in an hipcc -S listing (development tool).

The 8 radial-form slots of the 8-step kernel are unrolled copies; each ends with the wait for
its kappa load (`s_waitcnt vmcnt(0)` at the top of the next slot's step).  This prints, for the
listing lines of one slot (between two consecutive such waits), the count of each instruction
class -- FP64 arithmetic, transcendental seeds, v_cndmask (two per double select), compares,
integer / bit work, moves, lane-mask (SALU) work -- per basic block and in total.

usage: python tools/asm_classes.py <kernel.s> [slot index, default 2]
"""
import re
import sys
from collections import Counter, OrderedDict

CLASSES = OrderedDict([
    ("fp64 arith", re.compile(r"^v_(fma|mul|add|fmac|min|max|ldexp|frexp|div_fixup|div_fmas|div_scale|trig_preop|fract)_f64")),
    ("transcendental", re.compile(r"^v_(rcp|rsq|sqrt)_f64|^v_(exp|log|sin|cos|rcp|rsq|sqrt)_f32")),
    ("v_cndmask", re.compile(r"^v_cndmask")),
    ("v_cmp", re.compile(r"^v_cmp")),
    ("64-bit move", re.compile(r"^v_mov_b64|^v_pk_mov_b32")),
    ("32-bit move", re.compile(r"^v_mov_b32")),
    ("int / bit", re.compile(r"^v_(add|sub|subrev|mul|mad|lshl|lshr|ashr|and|or|xor|bfe|bfi|alignbit|bcnt|mbcnt|bitop3|lshl_add|add3|lshl_or|and_or|or3|not|max_i|min_i|max_u|min_u|cvt)")),
    ("lane (readlane etc.)", re.compile(r"^v_(readlane|readfirstlane|writelane)")),
    ("other VALU", re.compile(r"^v_")),
    ("SALU", re.compile(r"^s_(?!waitcnt|nop|cbranch|branch)")),
    ("branch / wait / nop", re.compile(r"^s_")),
    ("memory (VMEM / LDS)", re.compile(r"^(global|buffer|ds|scratch|flat)_")),
])


def classify(op):
    for name, rx in CLASSES.items():
        if rx.match(op):
            return name
    return "other"


def main():
    lines = open(sys.argv[1]).read().split("\n")
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    waits = [i for i, l in enumerate(lines) if l.strip() == "s_waitcnt vmcnt(0)"]
    # the slot boundaries: the kappa waits of the steps, each followed at once by the optical
    # depth's FMA (tau_cell = best * kappa, the first use of the loaded kappa)
    marks = [i for i in waits if any(lines[j].strip().startswith("v_fma_f64") for j in range(i + 1, min(i + 3, len(lines))))]
    if len(marks) < k + 2:
        sys.exit(f"found {len(marks)} slot marks")
    a, b = marks[k], marks[k + 1]
    total = Counter()
    blocks = []
    cur_name, cur = "(start)", Counter()
    for l in lines[a:b]:
        t = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", t) or t.startswith("; %bb."):
            blocks.append((cur_name, cur))
            cur_name, cur = t.split(":")[0].split(";")[-1].strip(), Counter()
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        c = classify(t.split()[0])
        cur[c] += 1
        total[c] += 1
    blocks.append((cur_name, cur))
    cols = list(CLASSES.keys())
    print(f"listing lines {a + 1}-{b} (slot {k})")
    print("| block | " + " | ".join(cols) + " |")
    print("|---|" + "---|" * len(cols))
    for name, cnt in blocks:
        if sum(cnt.values()):
            print(f"| {name} | " + " | ".join(str(cnt[c]) for c in cols) + " |")
    print("| **total** | " + " | ".join(str(total[c]) for c in cols) + " |")
    v = sum(total[c] for c in cols if c not in ("SALU", "branch / wait / nop", "memory (VMEM / LDS)"))
    print(f"\nVALU {v}, SALU {total['SALU']}, v_cndmask {total['v_cndmask']} ({100.0 * total['v_cndmask'] / max(v, 1):.0f} % of VALU)")


if __name__ == "__main__":
    main()
