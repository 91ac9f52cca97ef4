"""CPU: the C ABI library builds, loads and exports every symbol include/*.h declares; the
host-side operator precompute (condensing onto the equality null space, exact row removal)
reproduces the oracle's full-space QP. No GPU needed (no compute calls on the device)."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

import oracle_lib as O
from mpccbf import swarm

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(mpccbf_\w+)\s*\(", src):
            names.add(m.group(1))
    return sorted(names)


def test_library_exports_every_declared_symbol(mpclib):
    lib = ctypes.CDLL(mpclib.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 12
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(mpclib._lib.EXPORTED) <= set(names)


def test_abi_version_and_status_strings(mpclib):
    L = mpclib.load()
    assert L.mpccbf_abi_version() == 12
    assert [L.mpccbf_status_string(i).decode() for i in range(7)] == mpclib.STATUS_NAMES


def test_release_library_reads_no_solver_env_vars(mpclib):
    """Solver decisions come from mpccbf_options alone: the release library does not even name the
    diagnostics build's tuning variables (capi.hip, MPCCBF_DIAG_ENV); no getenv call site is
    compiled in (the GPU-side check: test_gpu_parity.py::test_solver_env_vars_have_no_effect)."""
    blob = open(mpclib.LIB_PATH, "rb").read()
    for name in (b"MPCCBF_DUAL_AS", b"MPCCBF_EARLY_IT", b"MPCCBF_FAST_START", b"MPCCBF_LEAN",
                 b"MPCCBF_DAS_WARM", b"MPCCBF_WARM_DELTA"):
        assert name not in blob, name


def test_param_validation_messages(mpclib):
    bad = swarm.config(15)
    bad["cbf_horizon"] = 20  # > k_hor  (parsing.hpp:192-197)
    with pytest.raises(mpclib.MpccbfError, match="CBF horizon"):
        mpclib._lib.host_operators(bad)
    bad = dict(swarm.BASE_CONFIG, k_hor=40)  # (k_hor-1) h > pieces * T  (parsing.hpp:199-213)
    with pytest.raises(mpclib.MpccbfError, match="sampling range"):
        mpclib._lib.host_operators(bad)
    with pytest.raises(ValueError):
        swarm.config(40)


@pytest.mark.parametrize("K", [10, 15])
def test_condensed_operators_reproduce_oracle_qp(mpclib, oracle, K):
    cfg = swarm.config(K)
    ops = mpclib._lib.host_operators(cfg)
    assert ops["nz"] == 6 and ops["n"] == 36
    p = O.make_params(cfg)
    rng = np.random.default_rng(K)
    for _ in range(5):
        s0 = np.concatenate([rng.uniform(-5, 5, 3), rng.uniform(-1.5, 1.5, 3)])
        t = rng.uniform(-5, 5, 3)
        y = rng.normal(size=ops["nz"]) * 3
        x = ops["Xs"] @ s0 + ops["Z"] @ y
        qp = oracle.assemble_qp(p, s0, np.tile(t, K), np.zeros((0, 6)))
        eq = qp["lo"] == qp["hi"]
        # every x = Xs s0 + Z y satisfies the equality rows (initial state + continuity)
        assert np.abs(qp["A"][eq] @ x - qp["lo"][eq]).max() < 1e-10
        obj_full = x @ qp["H"] @ x + qp["c"] @ x
        q = ops["Qs"] @ s0 + ops["Qt"] @ t
        obj_red = 0.5 * y @ ops["Pr"] @ y + q @ y + s0 @ ops["Ks"] @ s0 + t @ ops["Kt"] @ s0
        assert abs(obj_full - obj_red) <= 1e-12 * max(1.0, abs(obj_full))
        assert np.abs(qp["H"] - ops["H"]).max() <= 1e-14 * np.abs(qp["H"]).max()


@pytest.mark.parametrize("K", [10, 15])
def test_row_removal_is_exact(mpclib, oracle, K):
    """Every box row the host drops is implied by the kept rows (LP check per dropped row), and
    every 'constant' row is independent of the free variables."""
    from scipy.optimize import linprog
    cfg = swarm.config(K)
    full = mpclib._lib.host_operators(cfg, keep_redundant=True)
    red = mpclib._lib.host_operators(cfg)
    assert red["rows_removed"] > 0 and full["rows_removed"] == 0
    assert red["m"] + red["mc"] + red["rows_removed"] == red["rows_total"]
    rng = np.random.default_rng(1)
    for _ in range(3):
        s0 = np.concatenate([rng.uniform(-5, 5, 3), rng.uniform(-1.5, 1.5, 3)])
        # kept rows as A_ub y <= b_ub
        G, lo, hi = red["G"], red["lo"] - red["Gs"] @ s0, red["hi"] - red["Gs"] @ s0
        A_ub = np.vstack([G, -G])
        b_ub = np.concatenate([hi, -lo])
        Gf, lof, hif = full["G"], full["lo"] - full["Gs"] @ s0, full["hi"] - full["Gs"] @ s0
        for i in range(full["m"]):
            for sign, bound in ((1.0, hif[i]), (-1.0, -lof[i])):
                res = linprog(-sign * Gf[i], A_ub=A_ub, b_ub=b_ub, bounds=[(None, None)] * red["nz"],
                              method="highs")
                if res.status == 2:  # kept set infeasible for this s0: nothing to check
                    continue
                assert res.status == 0
                assert -res.fun <= bound + 1e-9 * max(1.0, abs(bound)), (i, sign, -res.fun, bound)
    # constant rows: the k = 0 velocity rows (pinned by the initial-velocity equality)
    assert red["mc"] == 3
    assert np.abs(red["Cs"][:, 3:] - np.eye(3)).max() < 1e-12


def test_ctypes_structs_match_the_c_header(tmp_path):
    """The ctypes mirrors in mpccbf/_lib.py have the sizes and field offsets of include/mpccbf.h
    (compiled here with gcc), so no field is shifted across the boundary."""
    import ctypes
    import subprocess
    from mpccbf import _lib
    structs = {"mpccbf_params": _lib.Params, "mpccbf_options": _lib.Options,
               "mpccbf_batch": _lib.Batch, "mpccbf_run": _lib.Run, "mpccbf_dense_qp": _lib.DenseQP,
               "mpccbf_host_ops": _lib.HostOps, "mpccbf_fov_control_params": _lib.FovControlParams,
               "mpccbf_fov_control_batch": _lib.FovControlBatch,
               "mpccbf_connectivity_control_params": _lib.ConnControlParams,
               "mpccbf_connectivity_control_batch": _lib.ConnControlBatch}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mpccbf.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "sizes.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "sizes"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", "-std=c11", "-I", inc, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for ln in out:
        if not ln:
            continue
        cname, f, v = ln.split()
        py = structs[cname]
        got = ctypes.sizeof(py) if f == "size" else getattr(py, f).offset
        assert got == int(v), (cname, f, got, v)
