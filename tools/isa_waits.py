"""The global-memory round trips of one kernel as the compiler scheduled them: compiles a HIP source
for gfx950 to assembly with line tables and prints, in program order, every vector memory load /
store, scratch access and `s_waitcnt vmcnt` with the source line it belongs to. A load followed by
a wait for it before the next load issues is a serialised round trip; scratch lines are spills.

    python tools/isa_waits.py <src.hip> <kernel-name-substring> [max-lines] [-D...]
e.g.  python tools/isa_waits.py csrc/kernels/impc_kernel.hip impc_sep_kernelILi1ELi1ELb0ELi256ELb0ELb0E
(paths relative to mpc-cbf_amd/)"""
import os
import re
import subprocess
import sys
import tempfile

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpc-cbf_amd")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function", "-munsafe-fp-atomics",
         "-mllvm", "-amdgpu-mfma-vgpr-form", "-gline-tables-only", "--cuda-device-only", "-S"]


def main():
    src, want = sys.argv[1], sys.argv[2]
    mx = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3].isdigit() else 10 ** 9
    extra = [a for a in sys.argv[3:] if a.startswith("-D")]
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, src, "-o", out], cwd=PKG, check=True,
                       stderr=subprocess.DEVNULL)
        lines = open(out).read().split("\n")
    files = {}
    for ln in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
    on, loc, cnt = False, None, 0
    for ln in lines:
        if re.match(r"^_ZN\S*:", ln):
            on, cnt = want in ln.split(":")[0], 0
        if not on:
            continue
        cnt += 1
        if cnt > mx:
            break
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
        if m:
            loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        t = ln.strip()
        if t.startswith(("global_load", "global_store", "scratch_", "flat_")) or (
                t.startswith("s_waitcnt") and "vmcnt" in t):
            print(cnt, loc, t[:72])


if __name__ == "__main__":
    main()
