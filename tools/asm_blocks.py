"""Basic-block instruction counts of one kernel in an hipcc -S listing (development tool).
usage: python tools/asm_blocks.py <kernel.s>"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
blocks, cur = [], None
for i, l in enumerate(lines):
    if re.match(r'^\.LBB\d+_\d+:', l) or l.startswith('; %bb.'):
        cur = {'name': l.split(':')[0].split(';')[-1].strip(), 'line': i + 1, 'v': 0, 's': 0, 'o': 0, 'br': [], 'tags': set()}
        blocks.append(cur)
        continue
    if cur is None:
        continue
    t = l.strip()
    if not t or t.startswith(';') or t.startswith('.'):
        continue
    op = t.split()[0]
    if op.startswith('v_'):
        cur['v'] += 1
    elif op.startswith('s_'):
        cur['s'] += 1
        if 'branch' in op:
            cur['br'].append(op.replace('s_cbranch_', '').replace('s_branch', 'jmp') + ' ' + t.split()[-1])
    else:
        cur['o'] += 1
    for tag in ['v_rcp_f64', 'v_rsq_f64', 'v_div_scale', 'scratch', 'global_load', 'global_store', 'ds_read', 'ds_write',
                'global_atomic', 'v_exp', 'v_log', 'vmcnt', 'lgkmcnt', 'v_readlane', 's_sleep']:
        if tag in t:
            cur['tags'].add(tag)
for b in blocks:
    print(f"{b['line']:5d} {b['name']:14s} v={b['v']:4d} s={b['s']:3d} o={b['o']:3d} {','.join(sorted(b['tags']))} {b['br']}")
