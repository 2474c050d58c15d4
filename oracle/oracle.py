"""ORACLE / TEST INFRASTRUCTURE ONLY -- the checker, never the product.

ctypes wrapper over
  oracle/liboracle.so          plain-C restatement (mjsub.c physics, ilqr_ora.c hot path)
  oracle/_ref/libilqg_ref.so   the reference's own src/{mjderivative,util,update}.cpp compiled
                               unmodified against oracle/include/mujoco/mujoco.h (+ restated physics)
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libilqg_ref.so")

_dp = ctypes.POINTER(ctypes.c_double)


def build(ref: bool = True):
    """make -C oracle (and the reference build when /root/reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    if ref and os.path.exists("/root/reference/src/mjderivative.cpp"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


class CostDesc(ctypes.Structure):
    _fields_ = [("nq", ctypes.c_int), ("nv", ctypes.c_int), ("nu", ctypes.c_int)] + [
        (n, ctypes.c_double * 64) for n in ("wq", "tq", "lq", "wv", "tv", "lv", "wu", "tu", "lu")]

    @classmethod
    def from_cost(cls, cost, nq, nv, nu):
        c = cls()
        c.nq, c.nv, c.nu = nq, nv, nu
        p = cost.packed(nq, nv, nu)
        for k, v in p.items():
            arr = getattr(c, k)
            for i, x in enumerate(v):
                arr[i] = float(x)
        return c


class Lib:
    def __init__(self, path):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing (make -C oracle{' ref' if '_ref' in path else ''})")
        self.L = ctypes.CDLL(path)
        L = self.L
        L.mj_loadBlob.restype = ctypes.c_void_p
        L.mj_loadBlob.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_int]
        L.mj_makeData.restype = ctypes.c_void_p
        L.mj_makeData.argtypes = [ctypes.c_void_p]
        for f in ("mj_deleteData", "mj_deleteModel"):
            getattr(L, f).argtypes = [ctypes.c_void_p]
        for f in ("mj_step", "mj_forward", "mj_resetData"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.mj_forwardSkip.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.ora_d_field.restype = _dp
        L.ora_d_field.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ora_d_int.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ora_model_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), _dp]
        L.ora_set_solver.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double]
        L.ora_get_solver.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), _dp]
        L.ora_cpMjData.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.ora_calcMJDerivatives.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _dp, ctypes.c_void_p]
        L.ora_calcMJDerivatives_tuned.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _dp, ctypes.c_void_p,
                                                  ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]
        L.ora_set_nthread.argtypes = [ctypes.c_int]
        L.ora_set_fd_eps.argtypes = [ctypes.c_double]
        L.ora_set_cost_desc.argtypes = [ctypes.POINTER(CostDesc)]
        L.ora_ilqr_create.restype = ctypes.c_void_p
        L.ora_ilqr_create.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]
        for f in ("ora_ilqr_free", "ora_ilqr_forwardPass", "ora_ilqr_backwardPass", "ora_ilqr_iterate"):
            getattr(L, f).argtypes = [ctypes.c_void_p]
        L.ora_ilqr_setDInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.ora_ilqr_fd_point.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ora_ilqr_get_traj.argtypes = [ctypes.c_void_p] + [_dp] * 5
        _ip = ctypes.POINTER(ctypes.c_int)
        for f in ("ora_ilqr_forward_candidates", "ora_ilqr_iterate_ls"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_int, _dp, ctypes.c_int, _dp, _ip]
        L.ora_ilqr_set_gains.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.ora_set_layout.argtypes = [ctypes.c_int]
        L.ora_ilqr_backwardPass_v0.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.ora_ilqr_iterate_v0.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.ora_riccati_step.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                       _dp, _dp, _dp, _dp, _dp, _dp, _dp]
        if hasattr(L, "ref_calcMJDerivatives"):
            L.ref_calcMJDerivatives.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _dp, ctypes.c_void_p]
            L.ref_cpMjData.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            L.ref_forwardStep.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            L.ref_forwardFrame.argtypes = [ctypes.c_void_p, ctypes.c_void_p]

    def fnptr(self, name):
        return ctypes.cast(getattr(self.L, name), ctypes.c_void_p)


_libs = {}


def oracle_lib() -> Lib:
    if "o" not in _libs:
        _libs["o"] = Lib(ORACLE_SO)
    return _libs["o"]


def ref_lib() -> Lib:
    if "r" not in _libs:
        _libs["r"] = Lib(REF_SO)
    return _libs["r"]


class OModel:
    def __init__(self, blob: bytes, lib: Lib = None):
        self.lib = lib or oracle_lib()
        err = ctypes.create_string_buffer(512)
        self.m = self.lib.L.mj_loadBlob(blob, len(blob), err, 512)
        if not self.m:
            raise RuntimeError("oracle mj_loadBlob: " + err.value.decode())
        info = (ctypes.c_int * 10)()
        dt = ctypes.c_double()
        self.lib.L.ora_model_info(self.m, info, ctypes.byref(dt))
        (self.nq, self.nv, self.nu, self.nbody, self.njnt, self.ngeom, self.nconmax, self.njmax,
         self.nstack, self.nbuffer) = list(info)
        self.timestep = dt.value
        self.D = self.nv * (2 * self.nv + self.nu) + 2 * self.nv + self.nu

    def __del__(self):
        if getattr(self, "m", None):
            self.lib.L.mj_deleteModel(self.m)
            self.m = None

    def make_data(self) -> "OData":
        return OData(self)

    def set_solver(self, iterations, tolerance):
        self.lib.L.ora_set_solver(self.m, iterations, tolerance)


_FIELDS = {"qpos": (0, "nq"), "qvel": (1, "nv"), "ctrl": (2, "nu"), "qacc": (3, "nv"),
           "warm": (4, "nv"), "qfrc_applied": (5, "nv"), "qfrc_bias": (8, "nv"), "qacc_smooth": (10, "nv")}


class OData:
    def __init__(self, model: OModel, handle=None):
        self.model = model
        self.lib = model.lib
        self.d = handle if handle is not None else self.lib.L.mj_makeData(model.m)
        self._owned = handle is None

    def __del__(self):
        if getattr(self, "_owned", False) and self.d:
            self.lib.L.mj_deleteData(self.d)
            self.d = None

    def arr(self, name):
        idx, sz = _FIELDS[name]
        n = getattr(self.model, sz)
        p = self.lib.L.ora_d_field(self.d, idx)
        return np.ctypeslib.as_array(p, shape=(n,))

    def xfrc(self):
        p = self.lib.L.ora_d_field(self.d, 6)
        return np.ctypeslib.as_array(p, shape=(6 * self.model.nbody,))

    @property
    def time(self):
        return self.lib.L.ora_d_field(self.d, 7)[0]

    @time.setter
    def time(self, v):
        self.lib.L.ora_d_field(self.d, 7)[0] = v

    def ncon(self):
        return self.lib.L.ora_d_int(self.d, 0)

    def nefc(self):
        return self.lib.L.ora_d_int(self.d, 1)

    def solver_iter(self):
        return self.lib.L.ora_d_int(self.d, 2)

    def step(self, n=1):
        for _ in range(n):
            self.lib.L.mj_step(self.model.m, self.d)

    def forward(self):
        self.lib.L.mj_forward(self.model.m, self.d)

    def state(self):
        return dict(time=self.time, qpos=self.arr("qpos").copy(), qvel=self.arr("qvel").copy(),
                    warm=self.arr("warm").copy(), ctrl=self.arr("ctrl").copy())

    def set_state(self, time=None, qpos=None, qvel=None, warm=None, ctrl=None):
        if time is not None:
            self.time = float(time)
        for k, v in (("qpos", qpos), ("qvel", qvel), ("warm", warm), ("ctrl", ctrl)):
            if v is not None:
                self.arr(k)[:] = v


class layout:
    """with oracle.layout("corrected"): ... -- the Differentiator's A/B
    assembly in the corrected layout for the block;
    "reference" (quirk Q1) is the default."""

    def __init__(self, name: str, lib: "Lib" = None):
        self.value = {"reference": 0, "corrected": 1}[name]
        self.lib = lib or oracle_lib()

    def __enter__(self):
        self.lib.L.ora_set_layout(self.value)
        return self

    def __exit__(self, *exc):
        self.lib.L.ora_set_layout(0)


def calc_derivatives(model: OModel, d: OData, cost_fn: str = "ora_cost_pendulum", use_ref=False, nthread=0):
    """calcMJDerivatives at d: the oracle restatement, or (use_ref) the reference's own
    compiled mjderivative.cpp.  cost_fn names a C function in the library."""
    deriv = np.zeros(model.D)
    lib = model.lib
    lib.L.ora_set_nthread(nthread)
    fp = lib.fnptr(cost_fn)
    if use_ref:
        lib.L.ref_calcMJDerivatives(model.m, d.d, deriv.ctypes.data_as(_dp), fp)
    else:
        lib.L.ora_calcMJDerivatives(model.m, d.d, deriv.ctypes.data_as(_dp), fp)
    return deriv


class OILQR:
    """ora_ilqr: restatement of ILQR<nv,nu,N> (inc/ilqr.h)."""

    def __init__(self, model: OModel, dmain: OData, N: int, cost_fn="ora_cost_pendulum", use_ref_fd=False):
        self.model = model
        self.lib = model.lib
        calc = self.lib.fnptr("ref_calcMJDerivatives") if use_ref_fd else None
        self.s = self.lib.L.ora_ilqr_create(model.m, dmain.d, N, self.lib.fnptr(cost_fn), calc)
        self.N = N

    def __del__(self):
        if getattr(self, "s", None):
            self.lib.L.ora_ilqr_free(self.s)
            self.s = None

    def set_dinit(self, d: OData):
        self.lib.L.ora_ilqr_setDInit(self.s, d.d)

    def forward_pass(self):
        self.lib.L.ora_ilqr_forwardPass(self.s)

    def backward_pass(self):
        self.lib.L.ora_ilqr_backwardPass(self.s)

    def iterate(self):
        self.lib.L.ora_ilqr_iterate(self.s)

    def backward_pass_v0(self, V0, v0):
        """backwardPass with an overridden initV (inc/ilqr.h:100,142): the
        recursion starts from V0 (nx x nx, column-major) and v0."""
        V0 = np.ascontiguousarray(V0, dtype=np.float64).ravel()
        v0 = np.ascontiguousarray(v0, dtype=np.float64).ravel()
        self.lib.L.ora_ilqr_backwardPass_v0(self.s, V0.ctypes.data_as(_dp), v0.ctypes.data_as(_dp))

    def iterate_v0(self, V0, v0):
        """iterate() of an ILQR subclass whose initV override sets V0, v0"""
        V0 = np.ascontiguousarray(V0, dtype=np.float64).ravel()
        v0 = np.ascontiguousarray(v0, dtype=np.float64).ravel()
        self.lib.L.ora_ilqr_iterate_v0(self.s, V0.ctypes.data_as(_dp), v0.ctypes.data_as(_dp))

    def iterate_ls(self, alphas, select="min_cost"):
        """iterate() with the line-search extension (every candidate rolled out,
        selection, setDInit, backwardPass); returns (costs[A], selected)."""
        return self._candidates(alphas, select, "ora_ilqr_iterate_ls")

    def forward_candidates(self, alphas, select="min_cost"):
        return self._candidates(alphas, select, "ora_ilqr_forward_candidates")

    def _candidates(self, alphas, select, fn):
        a = np.ascontiguousarray(alphas, dtype=np.float64)
        costs = np.zeros(len(a))
        sel = ctypes.c_int(-1)
        mode = {"reference": 0, "min_cost": 1}[select]
        getattr(self.lib.L, fn)(self.s, len(a), a.ctypes.data_as(_dp), mode, costs.ctypes.data_as(_dp),
                                ctypes.byref(sel))
        return costs, sel.value

    def set_gains(self, K, k):
        K = np.ascontiguousarray(K, dtype=np.float64)
        k = np.ascontiguousarray(k, dtype=np.float64)
        self.lib.L.ora_ilqr_set_gains(self.s, K.ctypes.data_as(_dp), k.ctypes.data_as(_dp))

    def traj(self):
        m, P = self.model, self.N + 1
        t = np.zeros(P); q = np.zeros((P, m.nq)); v = np.zeros((P, m.nv)); w = np.zeros((P, m.nv))
        u = np.zeros((P, m.nu))
        self.lib.L.ora_ilqr_get_traj(self.s, *(a.ctypes.data_as(_dp) for a in (t, q, v, w, u)))
        return dict(time=t, qpos=q, qvel=v, warm=w, ctrl=u)

    def _view(self, off_name):
        raise NotImplementedError

    def set_mu(self, mu: float):
        """the Levenberg-Marquardt constant (ILQR::mu, inc/ilqr.h:65; 1000 at
        creation), written into the oracle's ora_ilqr struct (ilqr_ora.h)"""
        class S(ctypes.Structure):
            _fields_ = [("m", ctypes.c_void_p), ("N", ctypes.c_int), ("nv", ctypes.c_int), ("nu", ctypes.c_int),
                        ("nx", ctypes.c_int), ("D", ctypes.c_int), ("d", ctypes.c_void_p),
                        ("dArray", ctypes.c_void_p), ("deriv", _dp), ("V", _dp), ("v", _dp), ("K", _dp),
                        ("k", _dp), ("mu", ctypes.c_double)]
        ctypes.cast(self.s, ctypes.POINTER(S)).contents.mu = float(mu)

    def point(self, n: int) -> "OData":
        """dArray[n] (the oracle's own mjData, not a copy: writes change the trajectory)"""
        class S(ctypes.Structure):
            _fields_ = [("m", ctypes.c_void_p), ("N", ctypes.c_int), ("nv", ctypes.c_int), ("nu", ctypes.c_int),
                        ("nx", ctypes.c_int), ("D", ctypes.c_int), ("d", ctypes.c_void_p),
                        ("dArray", ctypes.POINTER(ctypes.c_void_p))]
        st = ctypes.cast(self.s, ctypes.POINTER(S)).contents
        return OData(self.model, handle=st.dArray[n])

    def backward_from_records(self, deriv):
        """backwardPass (initV + the recursion, inc/ilqr.h:100-107,133-176) over
        the given FD records (P x D) instead of the oracle's own sweep"""
        class S(ctypes.Structure):
            _fields_ = [("m", ctypes.c_void_p), ("N", ctypes.c_int), ("nv", ctypes.c_int), ("nu", ctypes.c_int),
                        ("nx", ctypes.c_int), ("D", ctypes.c_int), ("d", ctypes.c_void_p),
                        ("dArray", ctypes.c_void_p), ("deriv", _dp), ("V", _dp), ("v", _dp), ("K", _dp),
                        ("k", _dp), ("mu", ctypes.c_double), ("cost", ctypes.c_void_p),
                        ("calc", ctypes.c_void_p), ("cout_lines", ctypes.c_long)]
        st = ctypes.cast(self.s, ctypes.POINTER(S)).contents
        P = self.N + 1
        rec = np.ascontiguousarray(deriv, dtype=np.float64).reshape(P, st.D)
        np.ctypeslib.as_array(st.deriv, shape=(P, st.D))[:] = rec
        calc = st.calc
        st.calc = self.lib.fnptr("ora_calc_none").value
        try:
            self.lib.L.ora_ilqr_backwardPass(self.s)
        finally:
            st.calc = calc

    def arrays(self):
        """K (P, nu*nx), k (P, nu), deriv (P, D), V (nx*nx), v (nx) copied out of the C struct."""
        m, P = self.model, self.N + 1
        nx = 2 * m.nv

        class S(ctypes.Structure):
            _fields_ = [("m", ctypes.c_void_p), ("N", ctypes.c_int), ("nv", ctypes.c_int), ("nu", ctypes.c_int),
                        ("nx", ctypes.c_int), ("D", ctypes.c_int), ("d", ctypes.c_void_p),
                        ("dArray", ctypes.c_void_p), ("deriv", _dp), ("V", _dp), ("v", _dp), ("K", _dp),
                        ("k", _dp), ("mu", ctypes.c_double), ("cost", ctypes.c_void_p),
                        ("calc", ctypes.c_void_p), ("cout_lines", ctypes.c_long)]
        st = ctypes.cast(self.s, ctypes.POINTER(S)).contents
        K = np.ctypeslib.as_array(st.K, shape=(P, m.nu * nx)).copy()
        k = np.ctypeslib.as_array(st.k, shape=(P, m.nu)).copy()
        deriv = np.ctypeslib.as_array(st.deriv, shape=(P, m.D)).copy()
        V = np.ctypeslib.as_array(st.V, shape=(nx * nx,)).copy()
        v = np.ctypeslib.as_array(st.v, shape=(nx,)).copy()
        return dict(K=K, k=k, deriv=deriv, V=V, v=v, cout_lines=st.cout_lines)
