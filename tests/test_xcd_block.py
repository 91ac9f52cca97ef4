"""The XCD-aware block order of the IMPC kernels (impc_common.hpp xcd_block) is a bijection of the
grid for every grid size, and gives each XCD (block b runs on XCD b % 8) one contiguous range of
logical blocks. Compiled for the host from the kernel header itself (hipcc, no GPU needed)."""
import os
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(REPO, "mpc-cbf_amd", "csrc", "kernels")

SRC = r"""
#include "impc_common.hpp"
#include <cstdio>
#include <vector>
int main() {
    for (int nb = 1; nb <= 4096; nb++) {
        std::vector<int> seen(nb, 0);
        std::vector<int> lo(8, 1 << 30), hi(8, -1), cnt(8, 0);
        for (int b = 0; b < nb; b++) {
            const int l = mpccbf::dev::xcd_block(b, nb);
            if (l < 0 || l >= nb || seen[l]++) { printf("nb %d b %d -> %d: not a bijection\n", nb, b, l); return 1; }
            const int x = b % 8;
            lo[x] = l < lo[x] ? l : lo[x];
            hi[x] = l > hi[x] ? l : hi[x];
            cnt[x]++;
        }
        for (int x = 0; x < 8; x++)
            if (cnt[x] && hi[x] - lo[x] + 1 != cnt[x]) { printf("nb %d xcd %d: range not contiguous\n", nb, x); return 1; }
    }
    printf("ok\n");
    return 0;
}
"""


def test_xcd_block_is_a_contiguous_bijection():
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "xcd.hip")
        exe = os.path.join(td, "xcd")
        with open(src, "w") as f:
            f.write(SRC)
        r = subprocess.run([hipcc, "-O1", "-std=c++17", "--offload-arch=gfx950", f"-I{KDIR}", src, "-o", exe],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-2000:]
        out = subprocess.run([exe], capture_output=True, text=True)
        assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
