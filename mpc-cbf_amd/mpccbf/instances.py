"""The reference's experiment configuration files: parsing, the base-config overlay, instances.

An experiment file is the JSON the example reads (MPCCBFFormationControl_example.cpp:62-117):
parameter sections (mpc_params, physical_limits, cbf_params, bezier_params, robot_params) and
tasks.so / tasks.sf, the robots' start and goal positions. Before a run the reference replaces every
section except "tasks" by experiments/config/base_config.json (experiments/python/preprocess.py:21),
so the effective parameters of every instance are the base config's; start velocities are zero
(example :108-111) and every other robot is a neighbour (:96-97, ConnectivityIMPCCBF.cpp:59-67).

parse_config() reads the sections like common/parsing.hpp:20-214 (same keys, same validation
messages) into the dict mpccbf.Context takes; overlay() is preprocess.py:21; instance() returns one
instance of mpccbf/data/reference_instances.json (the 16 baseline instances, transcribed as data
by tests/golden/make_reference_instances.py) ready for mpccbf.sim.Simulator.
"""
from __future__ import annotations

import json
import os

import numpy as np

from . import swarm

# the instances as data beside the package (written by tests/golden/make_reference_instances.py)
FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "reference_instances.json")


def _req(js: dict, *path):
    """js[path...] — a missing key is an error, as the reference's json lookups are."""
    v = js
    for k in path:
        if not isinstance(v, dict) or k not in v:
            raise ValueError("missing configuration key: " + ".".join(path))
        v = v[k]
    return v


def parse_config(js: dict) -> dict:
    """The parameter sections of an experiment JSON as a Context config (parsing.hpp:20-214:
    parsePiecewiseBezierParams, parseMPCParams, parseIMPCParams, parseConnectivityCBFParams,
    parseCollisionShape, validateCrossParameterRelationships). Raises ValueError with the
    reference's message on invalid values."""
    cfg = dict(swarm.BASE_CONFIG)
    cfg.update(
        h=float(_req(js, "mpc_params", "h")), Ts=float(_req(js, "mpc_params", "Ts")),
        k_hor=int(_req(js, "mpc_params", "k_hor")),
        w_pos_err=float(_req(js, "mpc_params", "mpc_tuning", "w_pos_err")),
        w_u_eff=float(_req(js, "mpc_params", "mpc_tuning", "w_u_eff")),
        spd_f=int(_req(js, "mpc_params", "mpc_tuning", "spd_f")),
        v_min=[float(v) for v in _req(js, "physical_limits", "v_min")[:3]],
        v_max=[float(v) for v in _req(js, "physical_limits", "v_max")[:3]],
        a_min=[float(v) for v in _req(js, "physical_limits", "a_min")[:3]],
        a_max=[float(v) for v in _req(js, "physical_limits", "a_max")[:3]],
        d_min=float(_req(js, "cbf_params", "d_min")),
        slack_mode=int(bool(_req(js, "cbf_params", "slack_mode"))),
        slack_cost=float(_req(js, "cbf_params", "slack_cost")),
        slack_decay_rate=float(_req(js, "cbf_params", "slack_decay_rate")),
        cbf_horizon=int(_req(js, "cbf_params", "cbf_horizon")),
        impc_iter=int(_req(js, "cbf_params", "impc_iter")),
        num_pieces=int(_req(js, "bezier_params", "num_pieces")),
        num_control_points=int(_req(js, "bezier_params", "num_control_points")),
        piece_max_parameter=float(_req(js, "bezier_params", "piece_max_parameter")),
        continuity_upto_degree=int(_req(js, "bezier_params", "bezier_continuity_upto_degree")),
    )
    box = js.get("robot_params", {}).get("collision_shape", {}).get("aligned_box")
    if box is not None:
        cfg["bbox"] = [float(v) for v in box[:3]]
    swarm.validate(cfg)
    return cfg


def collision_shape(js: dict):
    """(shape, type) the reference's collision_check.py scores with (:103-110): the aligned box's
    half extents (x, y) when present, else the radius."""
    sh = _req(js, "robot_params", "collision_shape")
    if "aligned_box" in sh:
        return [float(v) for v in sh["aligned_box"][:2]], "box"
    if "radius" in sh:
        return float(sh["radius"]), "circle"
    raise ValueError("Missing collision shape: must provide either 'aligned_box' or 'radius'")


def overlay(base: dict, task: dict) -> dict:
    """preprocess.py:21: the base configuration with the task file's "tasks" section."""
    return {**base, "tasks": task.get("tasks", {})}


def load_fixture(path: str = FIXTURE) -> dict:
    with open(path) as f:
        return json.load(f)


def names(path: str = FIXTURE) -> list:
    return sorted(load_fixture(path)["instances"].keys())


def from_json(js: dict):
    """(cfg, states, targets, shape, shape_type, noise) of an experiment JSON as the example loads
    it: states [px, py, yaw, 0, 0, 0] from tasks.so (zero start velocity, example :105-111),
    targets tasks.sf (:112-115), noise = physical_limits pos_std / vel_std."""
    cfg = parse_config(js)
    so = np.asarray(_req(js, "tasks", "so"), dtype=np.float64).reshape(-1, 3)
    sf = np.asarray(_req(js, "tasks", "sf"), dtype=np.float64).reshape(-1, 3)
    if so.shape != sf.shape:
        raise ValueError("tasks.so and tasks.sf differ in length")
    states = np.zeros((len(so), 6))
    states[:, :3] = so
    shape, kind = collision_shape(js)
    noise = dict(pos_std=float(_req(js, "physical_limits", "pos_std")),
                 vel_std=float(_req(js, "physical_limits", "vel_std")))
    return cfg, states, sf, shape, kind, noise


def own_params(base: dict, ins: dict) -> dict:
    """The instance file's own sections, with the keys it lacks (cbf_horizon, impc_iter,
    bezier_continuity_upto_degree) taken from the base config: what the file itself says."""
    def merge(b, o):
        if isinstance(b, dict) and isinstance(o, dict):
            return {k: merge(b.get(k), o[k]) if k in o else b[k] for k in set(b) | set(o)}
        return o if o is not None else b
    js = {k: merge(base.get(k), v) for k, v in ins["own_params"].items()}
    for k, v in base.items():
        js.setdefault(k, v)
    return {**js, "tasks": ins["tasks"]}


def instance(name: str, path: str = FIXTURE, preprocess="base"):
    """One baseline instance (e.g. "2r/line", the example's default). preprocess:
      "base" (or True) — the reference's run semantics: base_config.json overlaid (preprocess.py:21);
      "own"            — the instance file's own parameters (d_min 0.8 etc.), the keys it lacks from
                         the base config;
      False            — the file alone, which lacks cbf_horizon / impc_iter /
                         bezier_continuity_upto_degree and does not parse."""
    fx = load_fixture(path)
    ins = fx["instances"][name]
    if preprocess is True or preprocess == "base":
        js = overlay(fx["base_config"], ins)
    elif preprocess == "own":
        js = own_params(fx["base_config"], ins)
    else:
        js = {**ins["own_params"], "tasks": ins["tasks"]}
    return from_json(js)
