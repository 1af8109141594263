#!/bin/bash
# Extract one kernel from artes_amd/csrc/transport.s (make asm) and print its basic-block
# counts (development tool).  usage: bash tools/asm_kernel.sh <mangled-name-prefix> <out.s>
set -e
python3 - "$1" "$2" <<'PY'
import sys
s = open('artes_amd/csrc/transport.s').read().split('\n')
i = [k for k, l in enumerate(s) if l.startswith(sys.argv[1]) and l.rstrip().endswith(':') or (l.startswith(sys.argv[1]) and ': ;' in l)][0]
j = [k for k in range(i, len(s)) if s[k].startswith('.Lfunc_end')][0]
open(sys.argv[2], 'w').write('\n'.join(s[i:j]))
print(s[i].split(':')[0], j - i, 'lines')
PY
python3 tools/asm_blocks.py "$2" > "$2.blocks"
