#!/usr/bin/env python3
"""HBM bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/pmc.sh output):
2 x FETCH_SIZE + WRITE_SIZE (KB), the gfx950 correction of MI355X_MICROARCH.md §HBM; and the
MFMA busy fraction SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) per launch.
Usage: python tools/pmc_traffic.py gpurun_out/TAG > profiles/rNN_pmc_traffic.json"""
import collections
import csv
import glob
import json
import os
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] not in ("FETCH_SIZE", "WRITE_SIZE", "SQ_VALU_MFMA_BUSY_CYCLES",
                                     "GRBM_GUI_ACTIVE"):
            continue
        if "mfa::" not in r["Kernel_Name"]:
            continue
        name = re.sub(r"^void ", "", r["Kernel_Name"])
        name = re.sub(r"^mfa::", "", name)
        name = re.sub(r"\(.*\)$", "", name).replace("mfa::", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for name, c in sorted(acc.items()):
    if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        continue
    fk = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
    wk = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
    out[name] = {"fetch_kb": fk, "write_kb": wk, "hbm_bytes": (2 * fk + wk) * 1024}
    if c.get("SQ_VALU_MFMA_BUSY_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
        busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(c["SQ_VALU_MFMA_BUSY_CYCLES"])
        gui = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"])
        out[name]["mfma_busy"] = busy / (gui / 8 * 1024)
print(json.dumps(out, indent=1))
