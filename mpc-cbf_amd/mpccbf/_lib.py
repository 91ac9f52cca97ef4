"""ctypes marshalling for libmpccbf.so. Mirrors include/mpccbf.h one to one."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # mpc-cbf_amd/
LIB_PATH = os.environ.get("MPCCBF_LIB") or os.path.join(PKG_DIR, "build", "libmpccbf.so")

OPTIMAL, FEASIBLE, UNBOUNDED, INFEASIBLE, ERROR, UNKNOWN, INFEASIBLEORUNBOUNDED = range(7)
STATUS_NAMES = ["OPTIMAL", "FEASIBLE", "UNBOUNDED", "INFEASIBLE", "ERROR", "UNKNOWN",
                "INFEASIBLEORUNBOUNDED"]

# every symbol include/mpccbf.h declares (checked by tests/test_capi_symbols.py)
EXPORTED = [
    "mpccbf_create", "mpccbf_destroy", "mpccbf_num_vars", "mpccbf_reduced_dim",
    "mpccbf_num_shared_rows", "mpccbf_impc_solve", "mpccbf_set_variant", "mpccbf_build_neighbors",
    "mpccbf_qp_solve_dense", "mpccbf_qp_solve_dense_batch", "mpccbf_last_error",
    "mpccbf_status_string", "mpccbf_abi_version", "mpccbf_run_steps", "mpccbf_comm_unique_id",
    "mpccbf_comm_create", "mpccbf_comm_destroy", "mpccbf_kernel_name", "mpccbf_fov_control_solve",
    "mpccbf_connectivity_control_solve", "mpccbf_host_operators", "mpccbf_host_last_error",
    "mpccbf_comm_create_local", "mpccbf_fov_rows_eval", "mpccbf_impc_launch_waves",
]


class MpccbfError(RuntimeError):
    pass


def kernel_clock_us(clock) -> np.ndarray:
    """Per-launch durations in microseconds from a (num_steps, W, 2) kernel_clock array (numpy
    int64 / uint64): the largest wave end minus the smallest wave start over the written pairs;
    NaN for a step with no pair."""
    c = np.asarray(clock).view(np.uint64).astype(np.float64)
    t0, t1 = c[..., 0], c[..., 1]
    on = t1 > 0
    start = np.where(on, t0, np.inf).min(axis=1)
    end = np.where(on, t1, -np.inf).max(axis=1)
    return np.where(np.isfinite(start), (end - start) * 1e-2, np.nan)


def status_name(s: int) -> str:
    return STATUS_NAMES[s] if 0 <= s < len(STATUS_NAMES) else str(s)


class Params(C.Structure):
    _fields_ = [
        ("h", C.c_double), ("Ts", C.c_double), ("k_hor", C.c_int32),
        ("w_pos_err", C.c_double), ("w_u_eff", C.c_double), ("spd_f", C.c_int32),
        ("v_min", C.c_double * 3), ("v_max", C.c_double * 3),
        ("a_min", C.c_double * 3), ("a_max", C.c_double * 3),
        ("d_min", C.c_double),
        ("cbf_horizon", C.c_int32), ("impc_iter", C.c_int32), ("slack_mode", C.c_int32),
        ("slack_cost", C.c_double), ("slack_decay_rate", C.c_double),
        ("num_pieces", C.c_int32), ("num_control_points", C.c_int32),
        ("piece_max_parameter", C.c_double), ("continuity_upto_degree", C.c_int32),
        ("cbf_mode", C.c_int32), ("fov_beta", C.c_double), ("fov_Ds", C.c_double),
        ("fov_Rs", C.c_double), ("bbox", C.c_double * 3),
    ]

    @classmethod
    def from_dict(cls, cfg: dict) -> "Params":
        p = cls()
        for k, v in cfg.items():
            if isinstance(v, (list, tuple)):
                arr = getattr(p, k)
                for i, x in enumerate(v):
                    arr[i] = x
            else:
                setattr(p, k, v)
        return p


class Options(C.Structure):
    _fields_ = [("device", C.c_int32), ("keep_redundant", C.c_int32),
                ("no_cbf_filter", C.c_int32), ("max_pdip_iters", C.c_int32),
                ("tolerance", C.c_double), ("warm_delta", C.c_double),
                ("dual_as_steps", C.c_int32), ("no_fast_start", C.c_int32), ("early_it", C.c_int32),
                ("das_warm_steps", C.c_int32), ("lean", C.c_int32)]


class Batch(C.Structure):
    _fields_ = [
        ("num_states", C.c_int32), ("states", C.c_void_p), ("agent_first", C.c_int32),
        ("num_agents", C.c_int32), ("targets", C.c_void_p), ("refs", C.c_void_p),
        ("nb_row_ptr", C.c_void_p), ("nb_col", C.c_void_p), ("x", C.c_void_p),
        ("status", C.c_void_p), ("obj", C.c_void_p), ("iters", C.c_void_p),
        ("next_states", C.c_void_p), ("knn_k", C.c_int32), ("knn_radius", C.c_double),
        ("stamps", C.c_void_p), ("traj_t", C.c_void_p), ("pos_std", C.c_double),
        ("vel_std", C.c_double), ("noise_seed", C.c_uint64), ("step_index", C.c_int64),
        ("cov", C.c_void_p), ("primal_res", C.c_void_p), ("dual_res", C.c_void_p),
        ("substeps", C.c_void_p), ("nb_out", C.c_void_p),
    ]


class Run(C.Structure):
    _fields_ = [("num_steps", C.c_int32), ("states_alt", C.c_void_p), ("status_log", C.c_void_p),
                ("iters_log", C.c_void_p), ("step_ms", C.c_void_p), ("solve_ms", C.c_void_p),
                ("comm", C.c_void_p), ("reserve_steps", C.c_int32), ("solve_stride", C.c_int32),
                ("final_table", C.c_int32), ("kernel_clock", C.c_void_p),
                ("kernel_clock_waves", C.c_int32), ("continue_tables", C.c_int32)]


class DenseQP(C.Structure):
    _fields_ = [("n", C.c_int32), ("m", C.c_int32), ("H", C.c_void_p), ("c", C.c_void_p),
                ("c0", C.c_double), ("A", C.c_void_p), ("lo", C.c_void_p), ("hi", C.c_void_p),
                ("vlo", C.c_void_p), ("vhi", C.c_void_p)]


def build_library(quiet: bool = True) -> str:
    """Compile libmpccbf.so for gfx950 with hipcc (works without a GPU)."""
    out = subprocess.run(["make", "-C", PKG_DIR, "-j8"], capture_output=True, text=True)
    if out.returncode != 0:
        raise MpccbfError("libmpccbf build failed:\n" + out.stdout[-4000:] + out.stderr[-4000:])
    return LIB_PATH


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MpccbfError(f"{LIB_PATH} not built: run `make -C mpc-cbf_amd` (no CPU fallback)")
    # torch ships its own libamdhip64 (soname libamdhip64.so.7, the one libmpccbf needs). Load
    # torch first so the dynamic loader binds libmpccbf to that same HIP runtime: one runtime per
    # process, so torch's device pointers, streams and events are valid handles for the library.
    # (Loading libmpccbf first would pull /opt/rocm's copy and leave torch with a second one.)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.mpccbf_create.argtypes = [C.POINTER(Params), C.POINTER(Options), C.POINTER(vp)]
    L.mpccbf_destroy.argtypes = [vp]
    L.mpccbf_destroy.restype = None
    for f in ("mpccbf_num_vars", "mpccbf_reduced_dim", "mpccbf_num_shared_rows"):
        getattr(L, f).argtypes = [vp]
    L.mpccbf_impc_solve.argtypes = [vp, C.POINTER(Batch), vp]
    L.mpccbf_set_variant.argtypes = [vp, C.c_int]
    L.mpccbf_build_neighbors.argtypes = [vp, vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                         C.c_double, vp, vp, vp]
    L.mpccbf_qp_solve_dense.argtypes = [C.POINTER(DenseQP), vp, vp, vp]
    L.mpccbf_qp_solve_dense_batch.argtypes = [C.c_int32, C.POINTER(DenseQP), vp, vp, vp]
    L.mpccbf_run_steps.argtypes = [vp, C.POINTER(Batch), C.POINTER(Run), vp]
    L.mpccbf_comm_unique_id.argtypes = [C.c_char_p]
    L.mpccbf_comm_create.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(vp)]
    L.mpccbf_comm_create_local.argtypes = [C.c_int32, C.c_int32, C.POINTER(vp)]
    L.mpccbf_comm_destroy.argtypes = [vp]
    L.mpccbf_comm_destroy.restype = None
    L.mpccbf_kernel_name.argtypes = [vp]
    L.mpccbf_kernel_name.restype = C.c_char_p
    L.mpccbf_impc_launch_waves.argtypes = [vp, C.c_int32]
    L.mpccbf_impc_launch_waves.restype = C.c_int32
    L.mpccbf_last_error.restype = C.c_char_p
    L.mpccbf_fov_rows_eval.argtypes = [C.c_int32, vp, vp, C.c_double, C.c_double, C.c_double, vp, vp, vp, vp]
    L.mpccbf_status_string.restype = C.c_char_p
    L.mpccbf_status_string.argtypes = [C.c_int32]
    _lib = L
    return L


def _check(rc: int):
    if rc != 0:
        msg = load().mpccbf_last_error().decode()
        raise MpccbfError(f"mpccbf error {rc}: {msg}")


def _ptr(t) -> int | None:
    if t is None:
        return None
    import torch  # noqa: F401  (device tensors only)
    if not t.is_cuda:
        raise MpccbfError("libmpccbf batch entry points take device tensors")
    if not t.is_contiguous():
        raise MpccbfError("tensor must be contiguous")
    return t.data_ptr()


def _stream(stream):
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


class PreparedRun:
    """One marshalled mpccbf_run_steps call (Context.prepare_run_steps): calling it runs the steps
    (the C call alone); it holds the tensors its pointers refer to."""

    def __init__(self, ctx, batch, run, stream, states, states_alt, num_steps, step_ms, solve_ms, keep):
        self._ctx, self._b, self._r, self._s = ctx, batch, run, stream
        self._fn = load().mpccbf_run_steps
        self._tables = (states, states_alt)
        self._n, self._step_ms, self._solve_ms, self._keep = num_steps, step_ms, solve_ms, keep

    def __call__(self):
        _check(self._fn(self._ctx._h, C.byref(self._b), C.byref(self._r), self._s))
        out = {"final": self._tables[0] if self._r.final_table == 0 else self._tables[1]}
        if self._solve_ms is not None:
            out["step_ms"] = None if self._step_ms is None else self._step_ms[:self._n]
            sm = self._solve_ms[:self._n]
            out["solve_ms"] = sm[sm >= 0]
        return out


class Context:
    """One controller configuration on one device (mpccbf_create / mpccbf_destroy)."""

    def __init__(self, cfg: dict, device: int = 0, keep_redundant: bool = False,
                 no_cbf_filter: bool = False, max_iters: int = 0, tol: float = 0.0,
                 warm_delta: float = 0.0, dual_as_steps: int = 0, no_fast_start: bool = False,
                 early_it: int = 0, das_warm_steps: int = 0, lean: bool = False):
        """warm_delta: IMPC iteration-1 warm start floor (0 = default 0.3, < 0 = cold start);
        dual_as_steps: active-set step limit (0 = default, < 0 = the PDIP alone); the other solver
        options as mpccbf_options (include/mpccbf.h), 0 = default."""
        L = load()
        self.cfg = dict(cfg)
        self.params = Params.from_dict(cfg)
        o = Options(device=device, keep_redundant=int(keep_redundant),
                    no_cbf_filter=int(no_cbf_filter), max_pdip_iters=max_iters, tolerance=tol,
                    warm_delta=warm_delta, dual_as_steps=int(dual_as_steps),
                    no_fast_start=int(no_fast_start), early_it=int(early_it),
                    das_warm_steps=int(das_warm_steps), lean=int(lean))
        h = C.c_void_p()
        _check(L.mpccbf_create(C.byref(self.params), C.byref(o), C.byref(h)))
        self._h = h
        self.n = L.mpccbf_num_vars(h)
        self.nz = L.mpccbf_reduced_dim(h)
        self.shared_rows = L.mpccbf_num_shared_rows(h)
        self.impc_iter = int(cfg["impc_iter"])
        self.k_hor = int(cfg["k_hor"])
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            load().mpccbf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_variant(self, v: int):
        _check(load().mpccbf_set_variant(self._h, v))

    @property
    def kernel_name(self) -> str:
        return load().mpccbf_kernel_name(self._h).decode()

    def build_neighbors(self, states, first, count, k, radius, row_ptr, col, stream=None):
        _check(load().mpccbf_build_neighbors(self._h, _ptr(states), states.shape[0], first, count,
                                             k, float(radius), _ptr(row_ptr), _ptr(col),
                                             _stream(stream)))

    def impc_solve(self, states, nb_row_ptr=None, nb_col=None, targets=None, refs=None,
                   agent_first=0, num_agents=None, x=None, status=None, obj=None, iters=None,
                   next_states=None, knn_k=0, knn_radius=0.0, stream=None, stamps=None,
                   traj_t=None, pos_std=0.0, vel_std=0.0, noise_seed=0, step_index=0, cov=None,
                   primal_res=None, dual_res=None, substeps=None, nb_out=None):
        """CSR neighbours (nb_row_ptr/nb_col) or, with both None, the knn_k nearest within
        knn_radius found on the device in the same launch sequence. traj_t (float64, one per
        agent, initialised to -1) turns on the closed-loop simulator semantics: x persists the
        last successful curve and the next state follows it (see mpccbf_batch)."""
        if num_agents is None:
            num_agents = states.shape[0] - agent_first
        b = Batch(num_states=states.shape[0], states=_ptr(states), agent_first=agent_first,
                  num_agents=num_agents, targets=_ptr(targets), refs=_ptr(refs),
                  nb_row_ptr=_ptr(nb_row_ptr), nb_col=_ptr(nb_col), x=_ptr(x),
                  status=_ptr(status), obj=_ptr(obj), iters=_ptr(iters),
                  next_states=_ptr(next_states), knn_k=int(knn_k), knn_radius=float(knn_radius),
                  stamps=_ptr(stamps), traj_t=_ptr(traj_t), pos_std=float(pos_std),
                  vel_std=float(vel_std), noise_seed=int(noise_seed), step_index=int(step_index),
                  cov=_ptr(cov), primal_res=_ptr(primal_res), dual_res=_ptr(dual_res),
                  substeps=_ptr(substeps), nb_out=_ptr(nb_out))
        _check(load().mpccbf_impc_solve(self._h, C.byref(b), _stream(stream)))

    def run_steps(self, *args, **kw):
        """Closed-loop control steps on the device (mpccbf_run_steps): prepare_run_steps(...)()
        in one call; see prepare_run_steps for the arguments and the returned dict."""
        return self.prepare_run_steps(*args, **kw)()

    def prepare_run_steps(self, states, states_alt, num_steps, targets=None, refs=None, agent_first=0,
                  num_agents=None, knn_k=0, knn_radius=0.0, nb_row_ptr=None, nb_col=None, x=None,
                  status=None, obj=None, iters=None, status_log=None, iters_log=None,
                  timing=False, comm=None, reserve_steps=0, solve_stride=1, step_timing=True,
                  stream=None, traj_t=None, pos_std=0.0, vel_std=0.0, noise_seed=0, step_index=0,
                  cov=None, kernel_clock=None, stamps=None, continue_tables=False):
        """The arguments of one mpccbf_run_steps call, marshalled once (checks, ctypes structures,
        the stream handle): returns a PreparedRun whose call () runs the steps — a caller that
        times the steps prepares them outside its timed region. The call returns a dict with the
        table holding the final states ('final', a tensor) and, with timing=True, per-step
        device times 'step_ms' and IMPC-kernel times 'solve_ms' (numpy, ms). kernel_clock: a
        (num_steps, W, 2) device tensor (torch.int64, W >= launch_waves(num_agents)) for every
        wave's start / end of every IMPC launch (s_memrealtime, 100 MHz ticks; zero: no wave);
        kernel_clock_us() turns it into per-launch durations. stamps: the diagnostics builds' phase
        stamps (as impc_solve; every step overwrites them)."""
        if num_agents is None:
            num_agents = states.shape[0] - agent_first
        if kernel_clock is not None:
            # the library writes num_steps x W x 2 uint64 words from the base pointer: a shorter,
            # narrower or strided tensor would be written out of bounds (W itself is checked
            # against the launch's waves by mpccbf_run_steps)
            if (kernel_clock.dim() != 3 or not kernel_clock.is_contiguous() or kernel_clock.element_size() != 8
                    or kernel_clock.shape[0] < num_steps or kernel_clock.shape[2] != 2):
                raise ValueError("kernel_clock must be a contiguous (>= num_steps, W, 2) tensor of 8-byte elements")
        b = Batch(num_states=states.shape[0], states=_ptr(states), agent_first=agent_first,
                  num_agents=num_agents, targets=_ptr(targets), refs=_ptr(refs),
                  nb_row_ptr=_ptr(nb_row_ptr), nb_col=_ptr(nb_col), x=_ptr(x),
                  status=_ptr(status), obj=_ptr(obj), iters=_ptr(iters), next_states=None,
                  knn_k=int(knn_k), knn_radius=float(knn_radius), stamps=_ptr(stamps),
                  traj_t=_ptr(traj_t), pos_std=float(pos_std), vel_std=float(vel_std),
                  noise_seed=int(noise_seed), step_index=int(step_index), cov=_ptr(cov))
        step_ms = np.zeros(max(num_steps, 1), dtype=np.float32) if timing and step_timing else None
        solve_ms = np.zeros(max(num_steps, 1), dtype=np.float32) if timing else None
        r = Run(num_steps=num_steps, states_alt=_ptr(states_alt), status_log=_ptr(status_log),
                iters_log=_ptr(iters_log),
                step_ms=None if step_ms is None else step_ms.ctypes.data,
                solve_ms=None if solve_ms is None else solve_ms.ctypes.data,
                comm=None if comm is None else comm.handle, reserve_steps=reserve_steps,
                solve_stride=solve_stride, kernel_clock=_ptr(kernel_clock),
                kernel_clock_waves=0 if kernel_clock is None else int(kernel_clock.shape[1]),
                continue_tables=int(bool(continue_tables)))
        return PreparedRun(self, b, r, _stream(stream), states, states_alt, num_steps, step_ms, solve_ms,
                           keep=(targets, refs, nb_row_ptr, nb_col, x, status, obj, iters, status_log,
                                 iters_log, traj_t, cov, kernel_clock, stamps))

    def launch_waves(self, num_agents: int) -> int:
        """Waves of the IMPC launch for num_agents that write the launch clock (0: no clock)."""
        return int(load().mpccbf_impc_launch_waves(self._h, int(num_agents)))

    def alloc_outputs(self, num_agents: int, device=None):
        import torch
        dev = device or torch.device("cuda", self.device)
        return dict(
            x=torch.empty((num_agents, self.n), dtype=torch.float64, device=dev),
            status=torch.empty((num_agents, self.impc_iter), dtype=torch.int32, device=dev),
            obj=torch.empty((num_agents, self.impc_iter), dtype=torch.float64, device=dev),
            iters=torch.empty((num_agents, self.impc_iter), dtype=torch.int32, device=dev),
            next_states=torch.empty((num_agents, 6), dtype=torch.float64, device=dev),
            primal_res=torch.empty((num_agents, self.impc_iter), dtype=torch.float64, device=dev),
            dual_res=torch.empty((num_agents, self.impc_iter), dtype=torch.float64, device=dev),
        )


class HostOps(C.Structure):
    _fields_ = [("n", C.c_int32), ("nz", C.c_int32), ("m", C.c_int32), ("mc", C.c_int32),
                ("rows_total", C.c_int32), ("rows_removed", C.c_int32),
                ("capacity_ok", C.c_int32)] + [
        (f, C.c_void_p) for f in ("H", "Z", "Xs", "Pr", "Qs", "Qt", "Ks", "Kt", "G", "Gs", "lo",
                                  "hi", "Cs", "clo", "chi", "UZ0", "US0")]


def host_operators(cfg: dict, keep_redundant: bool = False) -> dict:
    """Host-only condensed operators (mpccbf_host_operators); no GPU needed."""
    L = load()
    L.mpccbf_host_operators.argtypes = [C.POINTER(Params), C.c_int32, C.POINTER(HostOps)]
    L.mpccbf_host_last_error.restype = C.c_char_p
    p = Params.from_dict(cfg)
    o = HostOps(capacity_ok=0)
    rc = L.mpccbf_host_operators(C.byref(p), int(keep_redundant), C.byref(o))
    if rc != 0:
        raise MpccbfError(L.mpccbf_host_last_error().decode())
    n, nz, m, mc = o.n, o.nz, o.m, o.mc
    shapes = dict(H=(n, n), Z=(n, nz), Xs=(n, 6), Pr=(nz, nz), Qs=(nz, 6), Qt=(nz, 3),
                  Ks=(6, 6), Kt=(3, 6), G=(m, nz), Gs=(m, 6), lo=(m,), hi=(m,), Cs=(mc, 6),
                  clo=(mc,), chi=(mc,), UZ0=(3, nz), US0=(3, 6))
    arrs = {k: np.zeros(s) for k, s in shapes.items()}
    o.capacity_ok = 1
    for k, a in arrs.items():
        setattr(o, k, a.ctypes.data if a.size else None)
    rc = L.mpccbf_host_operators(C.byref(p), int(keep_redundant), C.byref(o))
    if rc != 0:
        raise MpccbfError(L.mpccbf_host_last_error().decode())
    arrs.update(n=n, nz=nz, m=m, mc=mc, rows_total=o.rows_total, rows_removed=o.rows_removed)
    return arrs


def dense_qp_solve(H, c, A, lo, hi, vlo=None, vhi=None, c0=0.0):
    """Generic dense QP (mpccbf_qp_solve_dense); host numpy arrays. Returns (status, x, obj)."""
    L = load()
    H = np.ascontiguousarray(H, dtype=np.float64)
    c = np.ascontiguousarray(c, dtype=np.float64)
    n = c.shape[0]
    A = np.ascontiguousarray(A, dtype=np.float64).reshape(-1, n)
    lo = np.ascontiguousarray(lo, dtype=np.float64)
    hi = np.ascontiguousarray(hi, dtype=np.float64)
    vlo_a = None if vlo is None else np.ascontiguousarray(vlo, dtype=np.float64)
    vhi_a = None if vhi is None else np.ascontiguousarray(vhi, dtype=np.float64)
    qp = DenseQP(n=n, m=A.shape[0], H=H.ctypes.data, c=c.ctypes.data, c0=c0, A=A.ctypes.data,
                 lo=lo.ctypes.data, hi=hi.ctypes.data,
                 vlo=None if vlo_a is None else vlo_a.ctypes.data,
                 vhi=None if vhi_a is None else vhi_a.ctypes.data)
    x = np.zeros(n)
    obj = np.zeros(1)
    st = np.zeros(1, dtype=np.int32)
    _check(L.mpccbf_qp_solve_dense(C.byref(qp), x.ctypes.data, obj.ctypes.data, st.ctypes.data))
    return int(st[0]), x, float(obj[0])


class DenseBatchCall:
    """A batch of generic dense QPs marshalled once into the C ABI's mpccbf_dense_qp array (what a
    C++ caller holds anyway: pointers to its own arrays); run() is one
    mpccbf_qp_solve_dense_batch call on them. qps: list of dicts with H, c, A, lo, hi and
    optional vlo, vhi, c0."""

    def __init__(self, qps):
        self.L = load()
        self.keep = []  # hold the arrays alive for the calls
        self.count = len(qps)
        self.arr = (DenseQP * max(self.count, 1))()
        self.xs = []
        for k, q in enumerate(qps):
            c = np.ascontiguousarray(q["c"], dtype=np.float64)
            n = c.shape[0]
            H = np.ascontiguousarray(q["H"], dtype=np.float64).reshape(n, n)
            A = np.ascontiguousarray(q.get("A", np.zeros((0, n))), dtype=np.float64).reshape(-1, n)
            lo = np.ascontiguousarray(q.get("lo", np.zeros(0)), dtype=np.float64)
            hi = np.ascontiguousarray(q.get("hi", np.zeros(0)), dtype=np.float64)
            vlo = q.get("vlo")
            vhi = q.get("vhi")
            vlo = None if vlo is None else np.ascontiguousarray(vlo, dtype=np.float64)
            vhi = None if vhi is None else np.ascontiguousarray(vhi, dtype=np.float64)
            self.keep += [c, H, A, lo, hi, vlo, vhi]
            self.arr[k] = DenseQP(n=n, m=A.shape[0], H=H.ctypes.data, c=c.ctypes.data, c0=q.get("c0", 0.0),
                                  A=A.ctypes.data if A.size else None, lo=lo.ctypes.data if lo.size else None,
                                  hi=hi.ctypes.data if hi.size else None,
                                  vlo=None if vlo is None else vlo.ctypes.data,
                                  vhi=None if vhi is None else vhi.ctypes.data)
            self.xs.append(np.full(n, np.nan))
        self.xptr = (C.c_void_p * max(self.count, 1))(*[x.ctypes.data for x in self.xs])
        self.obj = np.zeros(max(self.count, 1))
        self.st = np.zeros(max(self.count, 1), dtype=np.int32)

    def run(self):
        """Returns (status[count], list of x (None unless OPTIMAL), obj[count])."""
        for x in self.xs:
            x.fill(np.nan)
        _check(self.L.mpccbf_qp_solve_dense_batch(self.count, self.arr, C.cast(self.xptr, C.c_void_p),
                                                  self.obj.ctypes.data, self.st.ctypes.data))
        n = self.count
        return (self.st[:n].copy(), [self.xs[k].copy() if self.st[k] == 0 else None for k in range(n)],
                self.obj[:n].copy())

    def run_raw(self):
        """The C call alone (outputs stay in self.st / self.obj / self.xs)."""
        _check(self.L.mpccbf_qp_solve_dense_batch(self.count, self.arr, C.cast(self.xptr, C.c_void_p),
                                                  self.obj.ctypes.data, self.st.ctypes.data))


def dense_qp_solve_batch(qps):
    """Batched generic dense QPs (mpccbf_qp_solve_dense_batch): one launch for all of them.
    qps: list of dicts with H, c, A, lo, hi and optional vlo, vhi, c0. Returns
    (status[count], list of x (None unless OPTIMAL), obj[count])."""
    return DenseBatchCall(qps).run()


COMM_ID_BYTES = 128


class FovControlParams(C.Structure):
    _fields_ = [("fov", C.c_double), ("Ds", C.c_double), ("Rs", C.c_double),
                ("v_min", C.c_double * 3), ("v_max", C.c_double * 3),
                ("u_min", C.c_double * 3), ("u_max", C.c_double * 3),
                ("slack_mode", C.c_int32), ("slack_cost", C.c_double),
                ("slack_decay_rate", C.c_double), ("max_pdip_iters", C.c_int32),
                ("tolerance", C.c_double)]


class FovControlBatch(C.Structure):
    _fields_ = [("num_agents", C.c_int32), ("states", C.c_void_p), ("desired_u", C.c_void_p),
                ("nb_row_ptr", C.c_void_p), ("nb_xy", C.c_void_p), ("u", C.c_void_p),
                ("status", C.c_void_p), ("obj", C.c_void_p), ("iters", C.c_void_p),
                ("nb_cov", C.c_void_p)]


def fov_control_params(cfg: dict) -> FovControlParams:
    """FovControl parameters from a config dict: fov_beta / fov_Ds / fov_Rs, v_min / v_max and the
    control bounds u_min / u_max (default: the acceleration bounds a_min / a_max)."""
    p = FovControlParams()
    p.fov, p.Ds, p.Rs = cfg["fov_beta"], cfg["fov_Ds"], cfg["fov_Rs"]
    for d in range(3):
        p.v_min[d], p.v_max[d] = cfg["v_min"][d], cfg["v_max"][d]
        p.u_min[d] = cfg.get("u_min", cfg["a_min"])[d]
        p.u_max[d] = cfg.get("u_max", cfg["a_max"])[d]
    p.slack_mode = int(cfg.get("control_slack_mode", 0))
    p.slack_cost = cfg.get("slack_cost", 0.0)
    p.slack_decay_rate = cfg.get("slack_decay_rate", 1.0)
    return p


def fov_control_solve(cfg: dict, states, desired_u, nb_row_ptr, nb_xy, u, status=None, obj=None,
                      iters=None, device: int = 0, stream=None, nb_cov=None):
    """Batched FovControl::optimize (mpccbf_fov_control_solve): device tensors in, u out.
    Slack mode: cfg["control_slack_mode"] with slack_cost / slack_decay_rate; nb_cov (one
    (cxx, cxy, cyy) row per observed neighbour) orders the slack weights."""
    b = FovControlBatch(num_agents=states.shape[0], states=_ptr(states), desired_u=_ptr(desired_u),
                        nb_row_ptr=_ptr(nb_row_ptr), nb_xy=_ptr(nb_xy), u=_ptr(u),
                        status=_ptr(status), obj=_ptr(obj), iters=_ptr(iters), nb_cov=_ptr(nb_cov))
    p = fov_control_params(cfg)
    _check(load().mpccbf_fov_control_solve(C.byref(p), C.byref(b), device, _stream(stream)))


def fov_rows_eval(ego, nb_xy, fov: float, Ds: float, Rs: float, bbox=(0.0, 0.0, 0.0), stream=None):
    """The FoV controller's per-neighbour rows on the device (mpccbf_fov_rows_eval): ego (n x 6)
    and nb_xy (n x 2) device tensors -> (voronoi n x 4 = (nx, ny, 0, offset), fov rows n x 4 x 4 =
    (a0, a1, a2, b) per kind: safety, left, right, range)."""
    import torch
    n = ego.shape[0]
    vor = torch.empty((n, 4), dtype=torch.float64, device=ego.device)
    rows = torch.empty((n, 4, 4), dtype=torch.float64, device=ego.device)
    bb = (C.c_double * 3)(*bbox)
    _check(load().mpccbf_fov_rows_eval(n, _ptr(ego), _ptr(nb_xy), fov, Ds, Rs, C.cast(bb, C.c_void_p),
                                       _ptr(vor), _ptr(rows), _stream(stream)))
    return vor, rows


class ConnControlParams(C.Structure):
    _fields_ = [("d_min", C.c_double), ("d_max", C.c_double), ("v_min", C.c_double * 3),
                ("v_max", C.c_double * 3), ("slack_mode", C.c_int32), ("slack_cost", C.c_double),
                ("slack_decay_rate", C.c_double), ("max_pdip_iters", C.c_int32),
                ("tolerance", C.c_double)]


class ConnControlBatch(C.Structure):
    _fields_ = [("num_teams", C.c_int32), ("team_ptr", C.c_void_p), ("states", C.c_void_p),
                ("desired_u", C.c_void_p), ("u", C.c_void_p), ("status", C.c_void_p),
                ("obj", C.c_void_p), ("iters", C.c_void_p), ("lambda2", C.c_void_p)]


def connectivity_control_solve(cfg: dict, team_ptr, states, desired_u, u, status=None, obj=None,
                               iters=None, lambda2=None, device: int = 0, stream=None):
    """Batched ConnectivityControl::optimize (mpccbf_connectivity_control_solve) for teams of
    robots (team t = rows team_ptr[t] .. team_ptr[t+1]-1 of states / desired_u). cfg keys: d_min,
    d_max, v_min, v_max, control_slack_mode, slack_cost, slack_decay_rate."""
    p = ConnControlParams()
    p.d_min, p.d_max = cfg["d_min"], cfg["d_max"]
    for d in range(3):
        p.v_min[d], p.v_max[d] = cfg["v_min"][d], cfg["v_max"][d]
    p.slack_mode = int(cfg.get("control_slack_mode", 0))
    p.slack_cost = cfg.get("slack_cost", 0.0)
    p.slack_decay_rate = cfg.get("slack_decay_rate", 1.0)
    b = ConnControlBatch(num_teams=team_ptr.shape[0] - 1, team_ptr=_ptr(team_ptr),
                         states=_ptr(states), desired_u=_ptr(desired_u), u=_ptr(u),
                         status=_ptr(status), obj=_ptr(obj), iters=_ptr(iters),
                         lambda2=_ptr(lambda2))
    _check(load().mpccbf_connectivity_control_solve(C.byref(p), C.byref(b), device, _stream(stream)))


def comm_unique_id() -> bytes:
    """RCCL unique id (mpccbf_comm_unique_id), created on one rank and shared with the others."""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(load().mpccbf_comm_unique_id(buf))
    return buf.raw


class Comm:
    """RCCL communicator for the per-step all-gather of agent states (mpccbf_comm_create):
    collective — every rank constructs it with the same id."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int, _handle=None):
        if _handle is not None:
            self.handle, self.nranks, self.rank = _handle, nranks, rank
            return
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("communicator id must be 128 bytes")
        h = C.c_void_p()
        _check(load().mpccbf_comm_create(uid, nranks, rank, device, C.byref(h)))
        self.handle = h
        self.nranks, self.rank = nranks, rank

    @classmethod
    def local_group(cls, nranks: int, device: int = 0) -> list:
        """mpccbf_comm_create_local: nranks in-process communicators (one host thread per rank,
        one device), the multi-GPU data flow of mpccbf_run_steps on a single GPU."""
        hs = (C.c_void_p * nranks)()
        _check(load().mpccbf_comm_create_local(nranks, device, hs))
        return [cls(b"", nranks, r, device, _handle=C.c_void_p(hs[r])) for r in range(nranks)]

    def close(self):
        if getattr(self, "handle", None):
            load().mpccbf_comm_destroy(self.handle)
            self.handle = None
