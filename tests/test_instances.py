"""The reference's experiment files as inputs (mpccbf.instances): the 16 baseline instances
(tests/golden/reference_instances.json, transcribed from workspace/experiments/config/baseline by
make_reference_instances.py), the preprocess.py:21 overlay, the parsing.hpp keys and validation, and
the example's start state (zero velocity, MPCCBFFormationControl_example.cpp:105-115). CPU only."""
import copy

import numpy as np
import pytest

from mpccbf import instances as I
from mpccbf import swarm


def test_sixteen_baseline_instances():
    names = I.names()
    assert len(names) == 16
    assert "2r/line" in names and "8r/circle" in names  # the CI default and the crowded circle
    counts = {n: len(I.load_fixture()["instances"][n]["tasks"]["so"]) for n in names}
    assert counts["2r/line"] == 2 and counts["8r/circle"] == 8 and counts["3r/line3"] == 8


@pytest.mark.parametrize("name", ["2r/line", "8r/circle", "5r/expand"])
def test_overlay_gives_base_config_and_zero_velocity(name):
    cfg, states, targets, shape, kind, noise = I.instance(name)
    base = swarm.config(16)  # base_config.json: k_hor 16
    for k in ("h", "Ts", "k_hor", "w_pos_err", "w_u_eff", "spd_f", "v_min", "v_max", "a_min", "a_max",
              "d_min", "cbf_horizon", "impc_iter", "slack_mode", "num_pieces", "num_control_points",
              "piece_max_parameter", "continuity_upto_degree"):
        assert cfg[k] == base[k], k
    ins = I.load_fixture()["instances"][name]["tasks"]
    np.testing.assert_array_equal(states[:, :3], np.asarray(ins["so"], dtype=float))
    np.testing.assert_array_equal(states[:, 3:], 0.0)
    np.testing.assert_array_equal(targets, np.asarray(ins["sf"], dtype=float))
    assert kind == "box" and shape == [0.2, 0.2]  # aligned_box first, as collision_check.py:103-110
    assert noise == {"pos_std": 0.001, "vel_std": 0.01}


def test_instance_files_alone_do_not_parse():
    """Without the overlay an instance lacks cbf_horizon / impc_iter / the continuity degree (the
    reference's parser reads them unconditionally, parsing.hpp:25-26,126-127)."""
    with pytest.raises(ValueError, match="cbf_horizon"):
        I.instance("2r/line", preprocess=False)


def test_8r_circle_starts_inside_d_min():
    cfg, states, *_ = I.instance("8r/circle")
    d = np.sqrt(((states[:, None, :2] - states[None, :, :2]) ** 2).sum(-1))
    np.fill_diagonal(d, np.inf)
    assert d.min() < cfg["d_min"]  # 1.53 m against d_min = 2: the infeasible-start regime


def test_parse_config_validation_messages():
    js = copy.deepcopy(I.overlay(I.load_fixture()["base_config"], I.load_fixture()["instances"]["2r/line"]))
    bad = copy.deepcopy(js)
    bad["cbf_params"]["cbf_horizon"] = 20
    with pytest.raises(ValueError, match="CBF horizon must be <= MPC prediction horizon"):
        I.from_json(bad)
    bad = copy.deepcopy(js)
    bad["mpc_params"]["Ts"] = 0.2
    with pytest.raises(ValueError, match="Ts must be <= MPC timestep"):
        I.from_json(bad)
    bad = copy.deepcopy(js)
    bad["mpc_params"]["k_hor"] = 17  # (17 - 1) * 0.1 > 3 * 0.5
    with pytest.raises(ValueError, match="exceeds Bezier curve parameter range"):
        I.from_json(bad)
    bad = copy.deepcopy(js)
    del bad["tasks"]["sf"]
    with pytest.raises(ValueError, match="tasks.sf"):
        I.from_json(bad)
