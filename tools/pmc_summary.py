"""Summarise rocprofv3 --pmc counter CSVs per workload and kernel: mean counter value per
dispatch, HBM bytes per launch with the gfx950 corrections of MI355X_MICROARCH.md (FETCH_SIZE in
KiB, reads 1/2 of the bytes of wide coalesced loads -> x2; WRITE_SIZE in KiB, exact), VALU
instructions per wave, and the issue-stall / MFMA fractions.

    python tools/pmc_summary.py gpurun_out/r02_pmc > profiles/r02_pmc_summary.json
Input layout: <root>/<workload>_<pass>/.../run_counter_collection.csv (tools/profile_round.sh).
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True)):
    workload = os.path.relpath(f, root).split(os.sep)[0].rsplit("_", 1)[0]
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mpccbf::dev::", "")
        agg[(workload, name)][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = collections.defaultdict(dict)
for (w, k), cs in agg.items():
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    d["dispatches"] = max(len(v) for v in cs.values())
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        d["hbm_bytes_per_launch_corrected"] = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
    if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d and d["SQ_WAVES"] > 0:
        d["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
    if "SQ_WAIT_INST_ANY" in d and "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"] > 0:
        d["issue_stall_frac"] = d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]
        d["valu_active_frac"] = d.get("SQ_ACTIVE_INST_VALU", 0.0) / d["SQ_WAVE_CYCLES"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "SQ_BUSY_CYCLES" in d and d["SQ_BUSY_CYCLES"] > 0:
        d["mfma_busy_per_busy_cycle"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / d["SQ_BUSY_CYCLES"]
    out[w][k] = d
json.dump(out, sys.stdout, indent=1)
print()
