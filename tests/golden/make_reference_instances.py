"""Transcribe the reference's own experiment instances as data (mpc-cbf_amd/mpccbf/data/reference_instances.json).

Source: /root/reference/workspace/experiments/config/baseline/{2r,3r,5r,6r,8r}/*.json (the 16
instances the example reads, MPCCBFFormationControl_example.cpp:43-44,97-117; CI runs 2r/line.json,
.github/workflows/ci.yml:112-114) and experiments/config/base_config.json, whose sections replace every
section of an instance except "tasks" before a run (experiments/python/preprocess.py:21). Only data is
kept: each instance's tasks.so / tasks.sf arrays and its own (unused after the overlay) parameter
sections, and the base config. Run here (the reference is not on the GPU box):

    python tests/golden/make_reference_instances.py
"""
import glob
import json
import os

REF = "/root/reference/workspace/experiments/config"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mpc-cbf_amd", "mpccbf", "data",
                   "reference_instances.json")


def main():
    base = json.load(open(os.path.join(REF, "base_config.json")))
    inst = {}
    for f in sorted(glob.glob(os.path.join(REF, "baseline", "*", "*.json"))):
        name = os.path.relpath(f, os.path.join(REF, "baseline"))[:-5]
        js = json.load(open(f))
        inst[name] = {"tasks": {"so": js["tasks"]["so"], "sf": js["tasks"]["sf"]},
                      "own_params": {k: v for k, v in js.items() if k != "tasks"}}
    out = {"source": "workspace/experiments/config/{base_config.json, baseline/*/*.json}",
           "base_config": base, "instances": inst}
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"wrote {len(inst)} instances to {OUT}")


if __name__ == "__main__":
    main()
