"""Summarise rocprofv3 --pmc counter CSVs (gpurun_out/pmc_*/run_counter_collection.csv) per
kernel: mean counter value per dispatch, and the HBM traffic per launch with the gfx950
corrections of MI355X_MICROARCH.md (FETCH_SIZE is in KiB and reads 1/2 of the bytes of wide
coalesced loads -> x2; WRITE_SIZE in KiB, exact).

    python tools/pmc_summary.py gpurun_out > profiles/r01_pmc_summary.json
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "pmc_*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in agg.items():
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    d["dispatches"] = max(len(v) for v in cs.values())
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        d["hbm_bytes_per_launch_corrected"] = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
    if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
        d["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
    out[k] = d
json.dump(out, sys.stdout, indent=1)
print()
