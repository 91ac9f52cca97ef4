"""Writes fov_cbf_golden.json: FoV CBF rows (Ac, Bc) evaluated from an independent symbolic
derivation that follows FovCBF's construction step by step (cbf/src/detail/FovCBF.cpp:152-535):
barrier b(state, target) in the robot frame, grad, L_f b, grad of L_f b, L_f^2 b, L_f alpha(b),
Ac = L_g L_f b, Bc = L_f^2 b + L_f alpha(b) + alpha(L_f b + alpha(b)), alpha(x) = 0.1 x^5,
f = A x with A = [[0, I], [0, 0]], g = [0; I]. The reference holds no known-answer tests for
these rows, so this symbolic restatement is what pins the oracle's closed forms.

Run:  python tests/golden/make_fov_golden.py
"""
import json
import math
import os

import numpy as np
import sympy as sp

GAMMA = 0.1
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fov_cbf_golden.json")


def derive(fov, Ds, Rs):
    px, py, th, vx, vy, w, xt, yt = sp.symbols("px py th vx vy w xt yt", real=True)
    state = [px, py, th, vx, vy, w]
    f = [vx, vy, w, 0, 0, 0]
    d = sp.Matrix([xt - px, yt - py])
    R = sp.Matrix([[sp.cos(th), sp.sin(th)], [-sp.sin(th), sp.cos(th)]])
    rel = R * d
    norm2 = rel[0] ** 2 + rel[1] ** 2

    def alpha(x):
        return GAMMA * x ** 5

    def hocbf(b):
        if b is None:
            return None
        lfb = sum(sp.diff(b, s) * fi for s, fi in zip(state, f))
        lf2b = sum(sp.diff(lfb, s) * fi for s, fi in zip(state, f))
        ab = alpha(b)
        lfa = sum(sp.diff(ab, s) * fi for s, fi in zip(state, f))
        Ac = [sp.diff(lfb, s) for s in (vx, vy, w)]  # g = [0; I]
        Bc = lf2b + lfa + alpha(lfb + ab)
        return Ac, Bc

    b_safe = norm2 - Ds ** 2
    if fov < math.pi:
        b_lb = math.tan(fov / 2) * rel[0] + rel[1]
        b_rb = math.tan(fov / 2) * rel[0] - rel[1]
    elif fov == math.pi:
        b_lb = rel[0]
        b_rb = rel[0]
    elif abs(fov - 2 * math.pi) < 1e-9:
        b_lb = b_rb = None
    else:  # GiNaC's `py >= 0` / `py < 0` on a free symbol evaluate to false (FovCBF.cpp:214-231)
        t2 = math.tan((2 * math.pi - fov) / 2)
        b_lb = t2 * rel[0] - rel[1]
        b_rb = t2 * rel[0] + rel[1]
    b_range = -norm2 + Rs ** 2
    rows = [hocbf(b) for b in (b_safe, b_lb, b_rb, b_range)]
    syms = (px, py, th, vx, vy, w, xt, yt)
    fns = []
    for r in rows:
        if r is None:
            fns.append(None)
        else:
            fns.append(sp.lambdify(syms, [*r[0], r[1]], "mpmath"))
    return fns


def main():
    import mpmath
    mpmath.mp.dps = 40
    rng = np.random.default_rng(20251015)
    cases = []
    for fov_deg in (120.0, 180.0, 240.0, 360.0):
        fov = fov_deg * math.pi / 180.0
        Ds, Rs = 0.2, 6.0
        fns = derive(fov, Ds, Rs)
        for _ in range(6):
            st = [float(rng.uniform(-3, 3)), float(rng.uniform(-3, 3)), float(rng.uniform(-math.pi, math.pi)),
                  float(rng.uniform(-1.5, 1.5)), float(rng.uniform(-1.5, 1.5)), float(rng.uniform(-2, 2))]
            tg = [st[0] + float(rng.uniform(-4, 4)), st[1] + float(rng.uniform(-4, 4))]
            rows = []
            for fn in fns:
                if fn is None:
                    rows.append(None)
                else:
                    vals = fn(*[mpmath.mpf(v) for v in st], *[mpmath.mpf(v) for v in tg])
                    rows.append([float(v) for v in vals])
            cases.append({"fov": fov, "Ds": Ds, "Rs": Rs, "state": st, "target": tg, "rows": rows})
    json.dump({"source": "symbolic restatement of cbf/src/detail/FovCBF.cpp:152-535 (sympy, 40 digits)",
               "row_order": ["safety", "left_border", "right_border", "range"],
               "row_layout": "[Ac_x, Ac_y, Ac_w, Bc]; null = vacuous row (fov = 2 pi)",
               "cases": cases}, open(OUT, "w"), indent=1)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
