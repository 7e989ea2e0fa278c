#!/usr/bin/env python3
"""Instruction statistics of kernels in a device .s file, per basic-block loop (development).
Usage: isa_stats.py file.s kernel_substring..."""
import re
import sys


def body(s, name):
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    return s[i:j]


def main():
    s = open(sys.argv[1]).read()
    names = re.findall(r'^(_Z\S+):', s, re.M)
    for pat in sys.argv[2:]:
        for n in names:
            if pat not in n:
                continue
            b = body(s, n)
            lines = [l.strip() for l in b.split('\n') if (l.startswith('\t') and not l.startswith('\t.')) or l.startswith('.LBB')]
            cnt = lambda k: sum(k in l for l in lines)
            print(n[:90])
            print('  total', len(lines), 'mfma', cnt('v_mfma'), 'readlane', cnt('v_readlane'),
                  'writelane', cnt('v_writelane'), 'scratch', cnt('scratch_'), 'exp', cnt('v_exp_f32'),
                  'waitcnt', cnt('s_waitcnt'), 'barrier', cnt('s_barrier'), 'ds_read', cnt('ds_read'),
                  'accvgpr', cnt('v_accvgpr'))
            # loops: labels that are targets of backward branches
            labels = {}
            for k, l in enumerate(lines):
                m = re.match(r'^(\.LBB\S+):', l)
                if m:
                    labels[m.group(1)] = k
            for k, l in enumerate(lines):
                m = re.match(r'^s_cbranch_\w+ (\.LBB\S+)|^s_branch (\.LBB\S+)', l)
                if m:
                    tgt = m.group(1) or m.group(2)
                    if tgt in labels and labels[tgt] < k:
                        seg = lines[labels[tgt]:k + 1]
                        c2 = lambda key: sum(key in x for x in seg)
                        print(f'  loop {tgt}: {len(seg)} instr, mfma {c2("v_mfma")}, valu-ish '
                              f'{sum(x.startswith("v_") and "mfma" not in x for x in seg)}, salu '
                              f'{sum(x.startswith("s_") for x in seg)}, ds {c2("ds_")}, '
                              f'readlane {c2("v_readlane")}, writelane {c2("v_writelane")}, '
                              f'waitcnt {c2("s_waitcnt")}, buffer {c2("buffer_")}')


if __name__ == '__main__':
    main()
