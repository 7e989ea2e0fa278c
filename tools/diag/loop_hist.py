#!/usr/bin/env python3
"""Mnemonic histogram of one loop (label .. backward branch) of a kernel in a device .s file
(development).  Usage: loop_hist.py file.s kernel_substring loop_label"""
import collections
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    names = re.findall(r'^(_Z\S+):', s, re.M)
    name = [n for n in names if sys.argv[2] in n][0]
    i = s.index(name + ':')
    body = s[i:s.index('.Lfunc_end', i)].split('\n')
    lab = sys.argv[3]
    start = [k for k, l in enumerate(body) if l.startswith(lab + ':')][0]
    end = max(k for k, l in enumerate(body) if re.search(r's_c?branch\w* ' + re.escape(lab) + r'$', l))
    ins = [l.strip().split()[0] for l in body[start:end + 1] if l.startswith('\t') and not l.startswith('\t.') and not l.strip().startswith(';')]
    c = collections.Counter(ins)
    print(len(ins), 'instructions')
    for k, v in c.most_common():
        print(f'{v:5d} {k}')


if __name__ == '__main__':
    main()
