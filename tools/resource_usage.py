"""Per-kernel resource usage of libmpccbf's HIP kernels (hipcc -Rpass-analysis=kernel-resource-usage):
VGPRs, AGPRs, scratch bytes per lane, LDS bytes per block and occupancy (waves per SIMD), as a table
(profiles/<tag>_resource_usage.txt). Runs on the CPU (cross-compile only).

    python tools/resource_usage.py [out.txt]
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mpc-cbf_amd")
SRCS = ["csrc/kernels/impc_kernel.hip", "csrc/kernels/impc_fov.hip", "csrc/kernels/cbf_control.hip",
        "csrc/kernels/connectivity_control.hip", "csrc/kernels/neighbors.hip", "csrc/dense_qp.hip"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-function",
         "-munsafe-fp-atomics", "-mllvm", "-amdgpu-mfma-vgpr-form"]
KEYS = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch",
        "Occupancy [waves/SIMD]": "occupancy", "LDS Size [bytes/block]": "lds"}


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True)
    return out.stdout.splitlines() if out.returncode == 0 else names


def usage():
    rows = []
    for src in SRCS:
        r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-c", src, "-o", os.devnull,
                            "-Rpass-analysis=kernel-resource-usage"], cwd=PKG, capture_output=True, text=True)
        cur = None
        for ln in r.stderr.splitlines():
            m = re.search(r"remark:\s+(Function Name|[A-Za-z ]+(?:\[[^\]]*\])?):\s*(\S+)", ln)
            if not m:
                continue
            k, v = m.group(1).strip(), m.group(2)
            if k == "Function Name":
                cur = {"kernel": v, "src": src}
                rows.append(cur)
            elif cur is not None and k in KEYS:
                cur[KEYS[k]] = int(v)
    names = demangle([r["kernel"] for r in rows])
    for r, n in zip(rows, names):
        r["kernel"] = n.replace("mpccbf::dev::", "").split("(")[0].replace("void ", "")
    return rows


def main():
    rows = usage()
    lines = [f"{'kernel':58s} {'VGPR':>5s} {'AGPR':>5s} {'scratch B/lane':>14s} {'LDS B/block':>11s} {'waves/SIMD':>10s}"]
    for r in rows:
        lines.append(f"{r['kernel'][:58]:58s} {r.get('vgpr', 0):5d} {r.get('agpr', 0):5d} {r.get('scratch', 0):14d} "
                     f"{r.get('lds', 0):11d} {r.get('occupancy', 0):10d}")
    txt = "\n".join(lines) + "\n"
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(txt)
    print(txt, end="")


if __name__ == "__main__":
    main()
