"""Python host binding of the MI355X iLQR hot path (ctypes over the C ABI in
include/ilqg_amd.h, library lib/libilqg_amd.so built by this directory's
Makefile).

The reference's host side is C++ (inc/ilqr.h, inc/differentiator.h,
src/mjderivative.cpp); this module mirrors its operator surface for tests,
the bench and Python callers:

  Model.load(path)                      mj_loadXML            cmd/basic.cpp:123
  Model.step(...) / Model.forward(...)  mj_step / mj_forward  inc/ilqr.h:86,128
  Model.calc_derivatives(...)           calcMJDerivatives     inc/mjderivative.h:7
  ILQR(model, dmain, N, cost)           ILQR<nv,nu,N> ctor    inc/ilqr.h:69-97
  ILQR.set_dinit / forward_pass / backward_pass / iterate     inc/ilqr.h:110-186

There is no CPU fallback: a missing library or missing GPU raises.
"""
from __future__ import annotations

import ctypes
import sys
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ILQG_LIB") or os.path.join(_HERE, "lib", "libilqg_amd.so")

_c_double_p = ctypes.POINTER(ctypes.c_double)
_c_int_p = ctypes.POINTER(ctypes.c_int)


class IlqgError(RuntimeError):
    pass


class _Cost(ctypes.Structure):
    _fields_ = [(n, _c_double_p) for n in ("wq", "tq", "lq", "wv", "tv", "lv", "wu", "tu", "lu")]


class _Opts(ctypes.Structure):
    _fields_ = [
        ("horizon", ctypes.c_int),
        ("nseed", ctypes.c_int),
        ("nalpha", ctypes.c_int),
        ("alphas", _c_double_p),
        ("select_mode", ctypes.c_int),
        ("mu", ctypes.c_double),
        ("device", ctypes.c_int),
    ]


EXPORTS = [
    "ilqg_last_error", "ilqg_version", "ilqg_device_count",
    "ilqg_model_load_xml", "ilqg_model_load_xml_string", "ilqg_model_free", "ilqg_model_sizes",
    "ilqg_model_timestep", "ilqg_model_qpos0", "ilqg_model_blob",
    "ilqg_step_batch", "ilqg_forward_batch", "ilqg_fd_batch",
    "ilqg_solver_create", "ilqg_solver_free", "ilqg_solver_init", "ilqg_solver_set_dinit",
    "ilqg_solver_set_traj", "ilqg_solver_get_traj", "ilqg_solver_set_gains", "ilqg_solver_get_gains",
    "ilqg_model_static_key", "ilqg_model_static_id",
    "ilqg_solver_get_deriv", "ilqg_solver_set_deriv", "ilqg_solver_get_value", "ilqg_solver_get_costs",
    "ilqg_forward", "ilqg_fd_sweep", "ilqg_backward", "ilqg_iterate", "ilqg_synchronize",
    "ilqg_solver_stream", "ilqg_solver_device_costs", "ilqg_solver_set_stream", "ilqg_solver_set_timing",
    "ilqg_solver_get_timing",
    "ilqg_solver_debug_set_fault", "ilqg_solver_device_traj", "ilqg_solver_set_layout", "ilqg_solver_set_value", "ilqg_solver_debug_plan",
    "ilqg_solver_set_riccati", "ilqg_selftest_div", "ilqg_solver_set_fd_precision",
    "ilqg_solver_set_mu", "ilqg_solver_get_deriv_point", "ilqg_solver_debug_plant_schedule",
    "ilqg_fd_sweep_range", "ilqg_solver_device_deriv", "ilqg_solver_set_groups", "ilqg_solver_get_groups",
    "ilqg_solver_join_stream", "ilqg_source_sha", "ilqg_forward_sharded", "ilqg_point_owners",
    "ilqg_solver_point_owners",
]
KERNELS = ("rollout", "select", "fd_centre", "fd_cols", "backward", "fd_backward")

_lib = None


def source_sha() -> str:
    """sha256 (16 hex digits) of the device/host sources the library is built
    from (csrc/**, Makefile; srcsha.py): names the kernel code a measurement
    belongs to without git (the GPU box has no .git)"""
    from srcsha import source_sha as _sha
    return _sha(_HERE)


def library_sha(path: str = None) -> str:
    """the source digest compiled into a built library (ilqg_source_sha)"""
    L = ctypes.CDLL(path or LIB_PATH)
    try:
        f = L.ilqg_source_sha
    except AttributeError:
        return None
    f.restype = ctypes.c_char_p
    return f().decode()


def lib() -> ctypes.CDLL:
    """Load the HIP library (fails loudly if it was not built, or was built
    from other sources than the ones beside it)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise IlqgError(f"{LIB_PATH} missing: run `make -C ilqg-mujoco_amd` (hipcc, gfx950)")
        # torch bundles a HIP runtime of its own: when both share the process,
        # torch's must initialise first (the other order leaves torch with "No
        # HIP GPUs are available" on the GPU box), so a torch already imported
        # is initialised here
        t = sys.modules.get("torch")
        if t is not None:
            try:
                t.cuda.is_available()
            except Exception:
                pass
        # provenance: the digest compiled into the library must be the digest
        # of the sources beside it (a stale prebuilt .so is refused, not measured)
        built, here = library_sha(LIB_PATH), source_sha()
        if built != here:
            raise IlqgError(f"{LIB_PATH} was built from sources {built}, but the sources here are {here}: "
                            "rebuild with `make -C ilqg-mujoco_amd`")
        L = ctypes.CDLL(LIB_PATH)
        L.ilqg_last_error.restype = ctypes.c_char_p
        L.ilqg_solver_stream.restype = ctypes.c_void_p
        _lib = L
    return _lib


def _check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().ilqg_last_error().decode(errors="replace")
        raise IlqgError(f"{what} failed (code {rc}): {msg}")


def _ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_c_double_p)


def _f64(a, shape=None) -> Optional[np.ndarray]:
    if a is None:
        return None
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if shape is not None:
        a = a.reshape(shape)
    return a


def point_owners(npoint: int, chunk: int, world: int) -> np.ndarray:
    """owner rank of every trajectory point when one seed's FD sweep is sharded
    over `world` ranks behind a pipelined rollout of `chunk`-point chunks
    (ilqg_point_owners: host logic, no device)"""
    out = np.zeros(npoint, dtype=np.int32)
    _check(lib().ilqg_point_owners(int(npoint), int(chunk), int(world), out.ctypes.data_as(_c_int_p)),
           "point_owners")
    return out


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().ilqg_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def selftest_div(a, b):
    """a / b through the device's split fp64 division (ilqg_selftest_div):
    returns (every-lane form, one-lane form)."""
    a = _f64(a).ravel()
    b = _f64(b).ravel()
    assert a.shape == b.shape
    q = np.empty_like(a)
    q2 = np.empty_like(a)
    _check(lib().ilqg_selftest_div(_ptr(a), _ptr(b), _ptr(q), _ptr(q2), ctypes.c_int(a.size)), "ilqg_selftest_div")
    return q, q2


@dataclass
class Cost:
    """Diagonal-quadratic + linear step cost (ilqg_cost in include/ilqg_amd.h)."""
    wq: Sequence[float] = ()
    tq: Sequence[float] = ()
    lq: Sequence[float] = ()
    wv: Sequence[float] = ()
    tv: Sequence[float] = ()
    lv: Sequence[float] = ()
    wu: Sequence[float] = ()
    tu: Sequence[float] = ()
    lu: Sequence[float] = ()

    def packed(self, nq, nv, nu):
        def arr(x, n):
            a = np.zeros(n)
            x = np.asarray(x, dtype=np.float64).ravel()
            a[: len(x)] = x
            return a
        return {k: arr(getattr(self, k), n) for k, n in
                (("wq", nq), ("tq", nq), ("lq", nq), ("wv", nv), ("tv", nv), ("lv", nv),
                 ("wu", nu), ("tu", nu), ("lu", nu))}

    def struct(self, nq, nv, nu):
        p = self.packed(nq, nv, nu)
        c = _Cost(**{k: _ptr(v) for k, v in p.items()})
        c._keep = p
        return c


# inc/inverted_pendulum/cost.h:7-17
PENDULUM_COST = Cost(wq=[1.0, 10.0], wv=[1.0, 10.0], wu=[1.0])
# build-defined hopper cost (the reference has none):
# keep the torso up (rootz -> 1.25) and level, damp velocities, small effort
HOPPER_COST = Cost(wq=[0.0, 10.0, 1.0, 0.1, 0.1, 0.1], tq=[0.0, 1.25, 0.0, 0.0, 0.0, 0.0],
                   wv=[0.1] * 6, wu=[0.01] * 3)
# build-defined humanoid cost (nq=28, nv=27, nu=21): torso height -> 1.4, upright
# torso (quaternion w -> 1), damped velocities, small effort
HUMANOID_COST = Cost(wq=[0.0, 0.0, 10.0, 1.0] + [0.0] * 24, tq=[0.0, 0.0, 1.4, 1.0] + [0.0] * 24,
                     wv=[0.05] * 27, wu=[0.001] * 21)


class Model:
    """Compiled MJCF model (mjModel equivalent), host + lazily uploaded device copy."""

    def __init__(self, handle):
        self._h = handle
        s = (ctypes.c_int * 10)()
        _check(lib().ilqg_model_sizes(self._h, s), "ilqg_model_sizes")
        (self.nq, self.nv, self.nu, self.nbody, self.njnt, self.ngeom,
         self.maxcon, self.maxefc, self.nconmax, self.njmax) = list(s)
        dt = ctypes.c_double()
        _check(lib().ilqg_model_timestep(self._h, ctypes.byref(dt)))
        self.timestep = dt.value
        q0 = np.zeros(self.nq)
        _check(lib().ilqg_model_qpos0(self._h, _ptr(q0)))
        self.qpos0 = q0
        self.D = self.nv * (2 * self.nv + self.nu) + 2 * self.nv + self.nu

    @classmethod
    def load(cls, path: str) -> "Model":
        h = ctypes.c_void_p()
        _check(lib().ilqg_model_load_xml(path.encode(), ctypes.byref(h)), f"load {path}")
        return cls(h)

    @classmethod
    def from_string(cls, xml: str) -> "Model":
        h = ctypes.c_void_p()
        _check(lib().ilqg_model_load_xml_string(xml.encode(), ctypes.byref(h)), "load xml string")
        return cls(h)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ilqg_model_free(self._h)
            self._h = None

    def blob(self) -> bytes:
        n = ctypes.c_size_t()
        _check(lib().ilqg_model_blob(self._h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        _check(lib().ilqg_model_blob(self._h, buf, n.value, ctypes.byref(n)))
        return buf.raw

    def static_key(self) -> np.ndarray:
        """integer data compiled into model-specific kernels (ilqg_model_static_key)"""
        n = ctypes.c_int()
        _check(lib().ilqg_model_static_key(self._h, None, 0, ctypes.byref(n)))
        key = np.zeros(n.value, dtype=np.int32)
        _check(lib().ilqg_model_static_key(self._h, key.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), n.value,
                                           ctypes.byref(n)))
        return key

    def static_id(self) -> int:
        """compiled model-specific kernel set this model runs on (0 = generic)"""
        v = ctypes.c_int()
        _check(lib().ilqg_model_static_id(self._h, ctypes.byref(v)))
        return v.value

    def reset_state(self, n=1):
        """mj_resetData: qpos0, zero velocity/warmstart/ctrl/time."""
        return State(time=np.zeros(n), qpos=np.tile(self.qpos0, (n, 1)), qvel=np.zeros((n, self.nv)),
                     warm=np.zeros((n, self.nv)), ctrl=np.zeros((n, self.nu)))

    # ---- batched single-point physics on the GPU ----
    def step(self, st: "State", nstep: int = 1, qfrc_applied=None, xfrc_applied=None):
        n = st.qpos.shape[0]
        _check(lib().ilqg_step_batch(self._h, n, nstep, _ptr(st.time), _ptr(st.qpos), _ptr(st.qvel),
                                     _ptr(st.warm), _ptr(st.ctrl), _ptr(_f64(qfrc_applied)),
                                     _ptr(_f64(xfrc_applied))), "ilqg_step_batch")
        return st

    def forward(self, st: "State", qfrc_applied=None, xfrc_applied=None):
        n = st.qpos.shape[0]
        qacc = np.zeros((n, self.nv))
        _check(lib().ilqg_forward_batch(self._h, n, _ptr(st.qpos), _ptr(st.qvel), _ptr(st.warm),
                                        _ptr(st.ctrl), _ptr(_f64(qfrc_applied)), _ptr(_f64(xfrc_applied)),
                                        _ptr(qacc)), "ilqg_forward_batch")
        return qacc

    def calc_derivatives(self, st: "State", cost: Optional[Cost] = None, qfrc_applied=None, xfrc_applied=None):
        """calcMJDerivatives at every state of `st` -> (n, D) reference-layout records."""
        n = st.qpos.shape[0]
        deriv = np.zeros((n, self.D))
        cs = cost.struct(self.nq, self.nv, self.nu) if cost is not None else None
        _check(lib().ilqg_fd_batch(self._h, n, _ptr(st.qpos), _ptr(st.qvel), _ptr(st.warm), _ptr(st.ctrl),
                                   _ptr(_f64(qfrc_applied)), _ptr(_f64(xfrc_applied)),
                                   ctypes.byref(cs) if cs is not None else None, _ptr(deriv)), "ilqg_fd_batch")
        return deriv


@dataclass
class State:
    """Batch of mjData state records (cpMjData fields, src/util.cpp:4-14)."""
    time: np.ndarray
    qpos: np.ndarray
    qvel: np.ndarray
    warm: np.ndarray
    ctrl: np.ndarray

    def __post_init__(self):
        for k in ("time", "qpos", "qvel", "warm", "ctrl"):
            setattr(self, k, np.ascontiguousarray(np.asarray(getattr(self, k), dtype=np.float64)))
        n = self.qpos.shape[0]
        self.time = self.time.reshape(n)

    def copy(self):
        return State(self.time.copy(), self.qpos.copy(), self.qvel.copy(), self.warm.copy(), self.ctrl.copy())


def assemble_AB(deriv: np.ndarray, nv: int, nu: int, dt: float, layout: str = "reference"):
    """Differentiator::updateDerivatives (inc/differentiator.h:66-71,89-92).
    'reference' reproduces the column-major Map of the row-major record (quirk
    Q1); 'corrected' reads the record's true Jacobians (ilqg_solver_set_layout)."""
    nx = 2 * nv
    order = "F" if layout == "reference" else "C"
    A = np.zeros((nx, nx))
    A[:nv, :nv] = np.eye(nv)
    A[:nv, nv:] = np.eye(nv) * dt
    A[nv:, :nv] = deriv[: nv * nv].reshape(nv, nv, order=order) * dt
    A[nv:, nv:] = np.eye(nv) + deriv[nv * nv: 2 * nv * nv].reshape(nv, nv, order=order) * dt
    B = np.zeros((nx, nu))
    B[nv:, :] = deriv[2 * nv * nv: 2 * nv * nv + nv * nu].reshape(nv, nu, order=order) * dt
    return A, B


class ILQR:
    """ILQR<nv,nu,N> (inc/ilqr.h:14-188) over `nseed` independent seeds and
    `alphas` rollout candidates, all on one GPU.  alphas[0] == 1 with
    select='reference' reproduces the reference's forwardPass exactly."""

    def __init__(self, model: Model, dmain: State, horizon: int, cost: Cost, alphas=(1.0,),
                 select: str = "reference", mu: float = 1000.0, device: int = 0,
                 qfrc_applied=None, xfrc_applied=None):
        self.model = model
        self.N = horizon
        self.P = horizon + 1
        self.S = dmain.qpos.shape[0]
        self.alphas = np.ascontiguousarray(np.asarray(alphas, dtype=np.float64))
        self.A = len(self.alphas)
        self.nx = 2 * model.nv
        o = _Opts(horizon=horizon, nseed=self.S, nalpha=self.A, alphas=_ptr(self.alphas),
                  select_mode=0 if select == "reference" else 1, mu=mu, device=device)
        cs = cost.struct(model.nq, model.nv, model.nu)
        h = ctypes.c_void_p()
        _check(lib().ilqg_solver_create(model._h, ctypes.byref(o), ctypes.byref(cs), ctypes.byref(h)),
               "ilqg_solver_create")
        self._h = h
        self._cost = cs
        _check(lib().ilqg_solver_init(self._h, _ptr(dmain.time), _ptr(dmain.qpos), _ptr(dmain.qvel),
                                      _ptr(dmain.warm), _ptr(dmain.ctrl), _ptr(_f64(qfrc_applied)),
                                      _ptr(_f64(xfrc_applied))), "ilqg_solver_init")

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ilqg_solver_free(self._h)
            self._h = None

    def set_dinit(self, d: State):
        _check(lib().ilqg_solver_set_dinit(self._h, _ptr(d.time), _ptr(d.qpos), _ptr(d.qvel), _ptr(d.warm),
                                           _ptr(d.ctrl)), "set_dinit")

    def set_traj(self, t: State):
        _check(lib().ilqg_solver_set_traj(self._h, _ptr(t.time), _ptr(t.qpos), _ptr(t.qvel), _ptr(t.warm),
                                          _ptr(t.ctrl)), "set_traj")

    def traj(self) -> State:
        m, S, P = self.model, self.S, self.P
        t = State(np.zeros(S * P), np.zeros((S * P, m.nq)), np.zeros((S * P, m.nv)),
                  np.zeros((S * P, m.nv)), np.zeros((S * P, m.nu)))
        _check(lib().ilqg_solver_get_traj(self._h, _ptr(t.time), _ptr(t.qpos), _ptr(t.qvel), _ptr(t.warm),
                                          _ptr(t.ctrl)), "get_traj")
        return t

    def gains(self):
        m = self.model
        K = np.zeros((self.S, self.P, m.nu * self.nx))
        k = np.zeros((self.S, self.P, m.nu))
        _check(lib().ilqg_solver_get_gains(self._h, _ptr(K), _ptr(k)), "get_gains")
        return K, k

    def set_gains(self, K, k):
        K = _f64(K); k = _f64(k)
        _check(lib().ilqg_solver_set_gains(self._h, _ptr(K), _ptr(k)), "set_gains")

    def deriv(self):
        d = np.zeros((self.S, self.P, self.model.D))
        _check(lib().ilqg_solver_get_deriv(self._h, _ptr(d)), "get_deriv")
        return d

    def set_deriv(self, d):
        d = _f64(d)
        if d.size != self.S * self.P * self.model.D:
            raise IlqgError(f"deriv must hold {self.S}x{self.P}x{self.model.D} doubles")
        _check(lib().ilqg_solver_set_deriv(self._h, _ptr(d)), "set_deriv")

    def value(self):
        V = np.zeros((self.S, self.nx * self.nx))
        v = np.zeros((self.S, self.nx))
        _check(lib().ilqg_solver_get_value(self._h, _ptr(V), _ptr(v)), "get_value")
        return V, v

    def costs(self):
        c = np.zeros((self.S, self.A))
        sel = np.zeros(self.S, dtype=np.int32)
        _check(lib().ilqg_solver_get_costs(self._h, _ptr(c), sel.ctypes.data_as(_c_int_p)), "get_costs")
        return c, sel

    def forward_pass(self):
        _check(lib().ilqg_forward(self._h), "ilqg_forward")

    def fd_sweep(self):
        _check(lib().ilqg_fd_sweep(self._h), "ilqg_fd_sweep")

    def fd_sweep_range(self, p0: int, np_: int):
        """calcMJDerivatives at points p0 .. p0+np_-1 of every seed (a rank's
        share of a point-sharded sweep): ilqg_fd_sweep_range"""
        _check(lib().ilqg_fd_sweep_range(self._h, int(p0), int(np_)), "fd_sweep_range")

    def forward_sharded(self, rank: int, world: int):
        """one rank's share of a point-sharded, pipelined iteration
        (ilqg_forward_sharded): the whole rollout, the FD sweep of the points
        this rank owns behind each rollout chunk (point_owners), selection;
        the caller gathers the other records, then riccati_pass()"""
        _check(lib().ilqg_forward_sharded(self._h, int(rank), int(world)), "forward_sharded")

    def point_owners(self, world: int) -> np.ndarray:
        """owner rank of every point under forward_sharded (ilqg_solver_point_owners)"""
        out = np.zeros(self.P, dtype=np.int32)
        _check(lib().ilqg_solver_point_owners(self._h, int(world), out.ctypes.data_as(_c_int_p)), "point_owners")
        return out

    def device_deriv(self):
        """(device pointer, record stride in doubles) of the resident FD records [S][P][stride]"""
        p = ctypes.POINTER(ctypes.c_double)()
        st = ctypes.c_int(0)
        _check(lib().ilqg_solver_device_deriv(self._h, ctypes.byref(p), ctypes.byref(st)), "device_deriv")
        return ctypes.cast(p, ctypes.c_void_p).value, st.value

    def backward_pass(self):
        """initV + Riccati; the FD sweep it depends on is ilqg_fd_sweep."""
        _check(lib().ilqg_fd_sweep(self._h), "ilqg_fd_sweep")
        _check(lib().ilqg_backward(self._h), "ilqg_backward")

    def riccati_pass(self):
        """initV + the Riccati recursion over the resident FD records (ilqg_backward),
        without a sweep: the records are whatever set_deriv / the last sweep left"""
        _check(lib().ilqg_backward(self._h), "ilqg_backward")

    def iterate(self):
        _check(lib().ilqg_iterate(self._h), "ilqg_iterate")

    def synchronize(self):
        _check(lib().ilqg_synchronize(self._h), "ilqg_synchronize")

    @property
    def stream(self) -> int:
        return lib().ilqg_solver_stream(self._h)

    def set_stream(self, stream: Optional[int]):
        """enqueue on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream)"""
        _check(lib().ilqg_solver_set_stream(self._h, ctypes.c_void_p(stream) if stream else None), "set_stream")

    def set_layout(self, layout: str):
        """'reference' (default: the Differentiator's column-major read of the
        row-major FD blocks, quirk Q1) or 'corrected' (A lower = dt J, B lower =
        dt J_u): ilqg_solver_set_layout"""
        _check(lib().ilqg_solver_set_layout(self._h, {"reference": 0, "corrected": 1}[layout]), "set_layout")

    def set_value(self, V, v):
        """initV override (virtual ILQR::initV, inc/ilqr.h:100-107): the next
        backward pass starts from V (S x nx x nx, column-major) and v (S x nx)"""
        V = _f64(V); v = _f64(v)
        if V.size != self.S * self.nx * self.nx or v.size != self.S * self.nx:
            raise IlqgError(f"V / v must hold {self.S}x{self.nx}x{self.nx} / {self.S}x{self.nx} doubles")
        _check(lib().ilqg_solver_set_value(self._h, _ptr(V), _ptr(v)), "set_value")

    def set_mu(self, mu: float):
        """Levenberg-Marquardt constant (ILQR::mu, inc/ilqr.h:65,166) for the
        backward passes enqueued from now on: ilqg_solver_set_mu"""
        _check(lib().ilqg_solver_set_mu(self._h, ctypes.c_double(mu)), "set_mu")

    def set_groups(self, ngroups: int):
        """seed groups (ilqg_solver_set_groups): iterate() software-pipelines
        the seeds as ngroups contiguous ranges -- one group's fused sweep beside
        the next group's rollout, each on CU-masked streams; the same bits as
        the ungrouped iterate.  1 restores it."""
        _check(lib().ilqg_solver_set_groups(self._h, int(ngroups)), "set_groups")

    def join_stream(self):
        """the next iterate()'s seed groups wait for everything enqueued on the
        solver's stream so far -- call it after work of your own there (the
        RCCL cost all-gather) and before the next iterate()"""
        _check(lib().ilqg_solver_join_stream(self._h), "join_stream")

    @property
    def groups(self) -> int:
        g = ctypes.c_int(0)
        _check(lib().ilqg_solver_get_groups(self._h, ctypes.byref(g), None), "get_groups")
        return g.value

    @property
    def group_rollout_cus(self) -> int:
        """CUs in each group's rollout mask (0: unmasked streams or no groups)"""
        g, c = ctypes.c_int(0), ctypes.c_int(0)
        _check(lib().ilqg_solver_get_groups(self._h, ctypes.byref(g), ctypes.byref(c)), "get_groups")
        return c.value

    def set_riccati(self, mode: str):
        """'exact' (bit-identical to the oracle, default) or 'mfma' (matrix-core
        products, fp64; agrees to rounding): ilqg_solver_set_riccati"""
        _check(lib().ilqg_solver_set_riccati(self._h, {"exact": 0, "mfma": 1}[mode]), "set_riccati")

    def set_fd_precision(self, prec: str):
        """'f64' (the reference's arithmetic, eps 1e-6, bit-exact; default) or
        'f32' (BASELINE.json cfg 5: fp32 FD physics, eps 1e-3, fp64 records):
        ilqg_solver_set_fd_precision"""
        _check(lib().ilqg_solver_set_fd_precision(self._h, {"f64": 0, "f32": 1}[prec]), "set_fd_precision")

    def set_timing(self, enable: bool):
        _check(lib().ilqg_solver_set_timing(self._h, int(enable)), "set_timing")

    def timing(self):
        """{kernel: (total_ms, launches)} since the last call (HIP events on the launch stream)"""
        ms = (ctypes.c_double * len(KERNELS))()
        n = (ctypes.c_int * len(KERNELS))()
        _check(lib().ilqg_solver_get_timing(self._h, ms, n), "get_timing")
        return {k: (ms[i], n[i]) for i, k in enumerate(KERNELS)}

    def _debug_set_fault(self, value: int):
        """test hook: preset the hand-off fault report word (ilqg_solver_debug_set_fault)"""
        _check(lib().ilqg_solver_debug_set_fault(self._h, ctypes.c_uint(value)), "debug_set_fault")

    def _debug_plant_schedule(self, slot: int, item: int):
        """test hook: the next fused sweep's ticket map gets order[slot] = item
        before the device validates it (ilqg_solver_debug_plant_schedule)"""
        _check(lib().ilqg_solver_debug_plant_schedule(self._h, ctypes.c_uint(slot), ctypes.c_uint(item)),
               "debug_plant_schedule")

    def device_traj_ptr(self, field: str) -> int:
        """device pointer to the resident nominal trajectory field (seed-major [S][P][...])"""
        idx = ("time", "qpos", "qvel", "warm", "ctrl").index(field)
        p = ctypes.POINTER(ctypes.c_double)()
        _check(lib().ilqg_solver_device_traj(self._h, idx, ctypes.byref(p)), "device_traj")
        return ctypes.cast(p, ctypes.c_void_p).value

    def device_costs_ptr(self) -> int:
        p = ctypes.POINTER(ctypes.c_double)()
        _check(lib().ilqg_solver_device_costs(self._h, ctypes.byref(p)), "device_costs")
        return ctypes.cast(p, ctypes.c_void_p).value
