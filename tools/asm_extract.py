"""Extract one kernel's listing from an hipcc -S file (development tool).
usage: python tools/asm_extract.py <listing.s> <mangled-name-prefix> <out.s>"""
import sys

s = open(sys.argv[1]).read().split("\n")
i = [k for k, l in enumerate(s) if l.startswith(sys.argv[2]) and (l.rstrip().endswith(":") or ": ;" in l)][0]
j = [k for k in range(i, len(s)) if s[k].startswith(".Lfunc_end")][0]
open(sys.argv[3], "w").write("\n".join(s[i:j]))
print(s[i].split(":")[0], j - i, "lines")
