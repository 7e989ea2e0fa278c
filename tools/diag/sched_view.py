#!/usr/bin/env python3
"""Compact instruction-class view of the blocks of one kernel between two labels (development).
M=MFMA e=v_exp v=other VALU a=accvgpr d=DS read/write B=buffer/global w=s_waitcnt n=s_nop
|=s_barrier >=branch s=other SALU.  Usage: sched_view.py file.s kernel_substring first_label last_label"""
import re
import sys

s = open(sys.argv[1]).read()
name = [n for n in re.findall(r'^(_Z\S+):', s, re.M) if sys.argv[2] in n][0]
i = s.index(name + ':')
body = s[i:s.index('.Lfunc_end', i)].split('\n')
a = [k for k, l in enumerate(body) if l.startswith(sys.argv[3] + ':')][0]
b = [k for k, l in enumerate(body) if l.startswith(sys.argv[4] + ':')][0]
out = []
for l in body[a:b]:
    t = l.strip()
    if not t or t.startswith(';'):
        continue
    if t.startswith('.LBB'):
        out.append('\n' + t.split(':')[0] + ' ')
        continue
    op = t.split()[0]
    if op.startswith('v_mfma'): c = 'M'
    elif op.startswith('v_exp'): c = 'e'
    elif op.startswith('v_accvgpr'): c = 'a'
    elif op.startswith('v_'): c = 'v'
    elif op.startswith('ds_'): c = 'd'
    elif op.startswith('buffer') or op.startswith('global'): c = 'B'
    elif op == 's_waitcnt': c = 'w'
    elif op == 's_nop': c = 'n'
    elif op == 's_barrier': c = '|'
    elif op.startswith('s_cbranch') or op == 's_branch': c = '>'
    elif op.startswith('s_'): c = 's'
    else: continue
    out.append(c)
print(''.join(out))
