"""GPU: the FoV controller's per-neighbour rows as the IMPC kernel evaluates them
(mpccbf_fov_rows_eval: the same device functions voronoi_row / fov_cbf_row): the Voronoi rows
against the reference's own VoronoiTest known-answer tests (VoronoiTest.cpp:10-73) and the oracle
(box-shifted), the FoV HOCBF rows against the 40-digit symbolic derivation
(tests/golden/fov_cbf_golden.json) the oracle is pinned by."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from test_oracle_fov import voronoi_kat_checks

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _dev(a):
    import torch
    return torch.tensor(np.asarray(a, dtype=np.float64), device="cuda")


def _eval(mpclib, ego, nb, fov=2.0943951023931953, Ds=0.2, Rs=6.0, bbox=(0.0, 0.0, 0.0)):
    import torch
    vor, rows = mpclib._lib.fov_rows_eval(_dev(ego), _dev(nb), fov, Ds, Rs, bbox)
    torch.cuda.synchronize()
    return vor.cpu().numpy(), rows.cpu().numpy()


def test_device_voronoi_rows_pass_reference_kats(mpclib, oracle):
    k = json.load(open(os.path.join(GOLDEN, "reference_kats.json")))["voronoi"]
    for case in k["cases"]:
        def dev_vor(p1, p2):
            ego = np.zeros((1, 6))
            ego[0, :2] = p1
            vor, _ = _eval(mpclib, ego, np.array([p2]))
            return vor[0, :3], vor[0, 3]
        voronoi_kat_checks(dev_vor, case, k["tolerance"])
    # box-shifted rows on random pairs: device == oracle
    rng = np.random.default_rng(7)
    ego = rng.uniform(-5, 5, (64, 6))
    nb = rng.uniform(-5, 5, (64, 2))
    bbox = (0.2, 0.25, 0.1)
    vor, _ = _eval(mpclib, ego, nb, bbox=bbox)
    for i in range(64):
        n, off = O.voronoi(ego[i, :2], nb[i], bbox)
        np.testing.assert_allclose(vor[i, :3], n, rtol=0, atol=1e-15)
        assert abs(vor[i, 3] - off) <= 1e-13 * max(1.0, abs(off))


def test_device_fov_rows_match_symbolic_derivation(mpclib):
    g = json.load(open(os.path.join(GOLDEN, "fov_cbf_golden.json")))
    for case in g["cases"]:
        _, rows = _eval(mpclib, np.array([case["state"]]), np.array([case["target"]]), case["fov"],
                        case["Ds"], case["Rs"])
        for r, ref in enumerate(case["rows"]):
            if ref is None:
                assert rows[0, r, 3] == np.finfo(np.float64).max
                continue
            np.testing.assert_allclose(rows[0, r, :3], ref[:3], rtol=1e-12, atol=1e-12)
            assert abs(rows[0, r, 3] - ref[3]) <= 1e-11 * max(1.0, abs(ref[3])), (r, rows[0, r, 3], ref[3])
