"""Instruction mix of one kernel in a hipcc --save-temps .s file (diagnostic).
usage: python diag/isa_stats.py FILE.s KERNEL_SUBSTRING"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
m = None
for mm in re.finditer(r'^(\S+):\s*(?:;.*)?$', s, re.M):
    if pat in mm.group(1) and not mm.group(1).startswith('.'):
        m = mm
        break
body = s[m.end():]
body = body[:body.index('.Lfunc_end')]
c = collections.Counter()
for line in body.split('\n'):
    t = line.strip().split()
    if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'):
        continue
    op = t[0]
    if op.startswith('v_mfma'):
        c['#MFMA'] += 1
    elif op.startswith(('v_exp', 'v_rcp', 'v_log', 'v_sqrt', 'v_rsq')):
        c['#TRANS'] += 1
    elif op.startswith('v_'):
        c['#VALU'] += 1
    elif op.startswith('ds_'):
        c['#DS'] += 1
    elif op.startswith(('scratch_', 'buffer_store', 'buffer_load')):
        c['#SCRATCH/BUF'] += 1
    elif op.startswith('s_'):
        c['#SALU'] += 1
    elif op.startswith('global_'):
        c['#GLOBAL'] += 1
    c[op] += 1
print(m.group(1))
for k, v in sorted(c.items(), key=lambda kv: (not kv[0].startswith('#'), -kv[1]))[:45]:
    print(f"{v:6d} {k}")
