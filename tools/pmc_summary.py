#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc csv outputs under a directory: per kernel, mean per dispatch."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if not name.startswith("void mfa::") and not name.startswith("mfa::"):
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, ctr in sorted(acc.items()):
    print("==", name[:110])
    for k in sorted(ctr):
        v = ctr[k]
        print(f"   {k:28s} {sum(v) / len(v):12.4g}  (n={len(v)})")
    c = {k: sum(v) / len(v) for k, v in ctr.items()}
    if "SQ_INSTS_MFMA" in c and "SQ_INSTS_VALU" in c:
        print(f"   -> VALU per MFMA {c['SQ_INSTS_VALU'] / max(c['SQ_INSTS_MFMA'], 1):.2f}")
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c:
                print(f"   -> {k}/WAVE_CYCLES {c[k] / w:.3f}")
    if "FETCH_SIZE" in c:
        print(f"   -> HBM read bytes (2 x FETCH_SIZE KB) {2 * c['FETCH_SIZE'] * 1024 / 1e6:.1f} MB")
    if "WRITE_SIZE" in c:
        print(f"   -> HBM write bytes {c['WRITE_SIZE'] * 1024 / 1e6:.1f} MB")
