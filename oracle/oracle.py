"""ctypes front-end of the CPU oracle (``oracle/liboracle.so``).

TEST INFRASTRUCTURE ONLY: tests/, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg may import this module, as the checker or the timed CPU
baseline. The product package (``civiwave-fem_amd/cwf``) never imports it.

Each wrapper restates a reference entry point (see cwf_oracle.c for the
file:line of every fold):
  apply_keff            -> src/gpu/pcg.cpp:505-694
  block_jacobi          -> src/gpu/pcg.cpp:270-408, 479-503
  dot                   -> src/gpu/pcg.cpp:170-207
  solve_pcg             -> src/gpu/pcg.cpp:696-918
  Stepper.step          -> src/gpu/newmark_stepper.cpp:1094-1379 (CPU branch)
  preprocess_tets       -> src/mesh/preprocess.cpp:268-405 + src/mesh/pack.cpp:41-200
  dense_newmark_step    -> src/physics/solver.cpp:159-378
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < max(
            os.path.getmtime(os.path.join(_HERE, f)) for f in ("cwf_oracle.c", "hex8_oracle.c", "cwf_oracle.h")
        ):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        u64, f64, i32 = C.c_uint64, C.c_double, C.c_int
        L.orc_last_message.restype = C.c_char_p
        L.orc_last_context.restype = C.c_char_p
        L.orc_make_stiffness.argtypes = [f64, f64, P]
        L.orc_rayleigh.argtypes = [f64, f64, f64, P, P]
        L.orc_newmark_coefficients.argtypes = [f64, f64, f64, P, P]
        L.orc_preprocess_tets.argtypes = [u64, u64] + [P] * 12
        L.orc_preprocess_tets.restype = i32
        L.orc_evaluate_curve.argtypes = [P, P, u64, f64]
        L.orc_evaluate_curve.restype = f64
        L.orc_gravity_loads.argtypes = [u64, P, P, P]
        L.orc_point_loads.argtypes = [u64, P, P, f64, P]
        L.orc_apply_keff.argtypes = [P, P, P]
        L.orc_apply_keff.restype = i32
        L.orc_block_jacobi.argtypes = [P, P]
        L.orc_block_jacobi.restype = i32
        L.orc_dot.argtypes = [P, P, P, P]
        L.orc_dot.restype = f64
        L.orc_solve_pcg.argtypes = [P, P, u64, f64, i32, P, P, P, P, P, P, P, P]
        L.orc_solve_pcg.restype = i32
        L.orc_stepper_step.argtypes = [P, f64, i32, P]
        L.orc_stepper_step.restype = i32
        L.orc_dense_assemble.argtypes = [u64, u64, P, P, P, P, P, P]
        L.orc_dense_assemble.restype = i32
        L.orc_dense_newmark_step.argtypes = [u64, P, P, P, P, P, f64, f64, P, P, P, P, f64, u64, P, P, P, P]
        L.orc_dense_newmark_step.restype = i32
        L.orc_derived_fields.argtypes = [P, P, P, P]
        L.orc_derived_fields.restype = i32
        L.orc_hex8_preprocess.argtypes = [u64, u64, P, P, P, P, u64, P, P, P]
        L.orc_hex8_preprocess.restype = i32
        L.orc_hex8_apply.argtypes = [u64, u64, P, P, P, P, f64, f64, P, P, P, P, P]
        L.orc_hex8_apply.restype = i32
        L.orc_hex8_apply64.argtypes = [u64, u64, P, P, P, P, f64, f64, P, P, P, P]
        L.orc_hex8_apply64.restype = i32
        L.orc_hex8_diag_blocks.argtypes = [u64, u64, P, P, P, P, f64, P]
        L.orc_hex8_diag_blocks.restype = i32
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class OracleError(RuntimeError):
    def __init__(self, code: int):
        L = lib()
        self.code = code
        self.message = L.orc_last_message().decode()
        ctx = L.orc_last_context().decode()
        self.context = [ctx] if ctx else []
        super().__init__(f"{self.message} {self.context}")


class _System(C.Structure):
    _fields_ = [
        ("node_count", C.c_uint64),
        ("element_count", C.c_uint64),
        ("dof_count", C.c_uint64),
        ("connectivity", C.c_void_p),
        ("gradients", C.c_void_p),
        ("volume", C.c_void_p),
        ("material_index", C.c_void_p),
        ("stiffness", C.c_void_p),
        ("material_count", C.c_uint64),
        ("lumped_mass", C.c_void_p),
        ("bc_mask", C.c_void_p),
        ("stiffness_scale", C.c_double),
        ("mass_factor", C.c_double),
        ("reduction_block", C.c_uint64),
        ("reduction_partials", C.c_uint64),
    ]


class Telemetry(C.Structure):
    _fields_ = [
        ("iterations", C.c_uint64),
        ("residual_norm", C.c_double),
        ("rhs_norm", C.c_double),
        ("alpha_last", C.c_double),
        ("beta_last", C.c_double),
        ("converged", C.c_int32),
        ("pad", C.c_int32),
    ]


class StepTelemetry(C.Structure):
    _fields_ = [
        ("simulation_time", C.c_double),
        ("time_step", C.c_double),
        ("applied_tolerance", C.c_double),
        ("paused_mode", C.c_int32),
        ("dt_increased", C.c_int32),
        ("dt_decreased", C.c_int32),
        ("dt_clamped_min", C.c_int32),
        ("dt_clamped_max", C.c_int32),
        ("pad", C.c_int32),
        ("pcg", Telemetry),
    ]


class _Stepper(C.Structure):
    _fields_ = [
        ("system", C.c_void_p),
        ("rayleigh_alpha", C.c_double),
        ("rayleigh_beta", C.c_double),
        ("runtime_tolerance", C.c_double),
        ("pause_tolerance", C.c_double),
        ("max_iterations", C.c_uint64),
        ("adaptive", C.c_int32),
        ("warm_start", C.c_int32),
        ("min_dt", C.c_double),
        ("max_dt", C.c_double),
        ("low_iteration_ratio", C.c_double),
        ("increase_factor", C.c_double),
        ("decrease_factor", C.c_double),
        ("dt", C.c_double),
        ("beta", C.c_double),
        ("gamma", C.c_double),
        ("accumulated_time", C.c_double),
        ("frame_index", C.c_uint64),
    ] + [(n, C.c_void_p) for n in (
        "u", "v", "a", "external_force", "bc_value", "u_pred", "v_pred", "rhs", "damping_rhs",
        "damping_out", "x", "r", "p", "z", "Ap", "partials")]


def make_stiffness(E: float, nu: float) -> np.ndarray:
    D = np.zeros(36, np.float64)
    lib().orc_make_stiffness(E, nu, _p(D))
    return D


def rayleigh(xi: float, w1: float, w2: float):
    a, b = C.c_double(), C.c_double()
    lib().orc_rayleigh(xi, w1, w2, C.byref(a), C.byref(b))
    return a.value, b.value


def newmark_coefficients(dt: float, beta: float = 0.25, gamma: float = 0.5):
    a = np.zeros(6)
    u = np.zeros(2)
    lib().orc_newmark_coefficients(dt, beta, gamma, _p(a), _p(u))
    return a, u


@dataclass
class Packed:
    """Reference PackingResult subset (include/cwf/mesh/pack.hpp:95-140), dof = 3n+k."""

    node_count: int
    element_count: int
    connectivity: np.ndarray  # u32 [E*8]
    gradients: np.ndarray  # f32 [E*24]
    volume: np.ndarray  # f32 [E]
    material_index: np.ndarray  # u32 [E]
    mass64: np.ndarray  # f64 [N]
    lumped_mass: np.ndarray  # f32 [N]
    offsets: np.ndarray
    adj_elem: np.ndarray
    adj_local: np.ndarray


def preprocess_tets(coords: np.ndarray, tets: np.ndarray, material_index: np.ndarray, density) -> Packed:
    coords = np.ascontiguousarray(coords, np.float64).reshape(-1)
    tets = np.ascontiguousarray(tets, np.uint32).reshape(-1)
    N = coords.size // 3
    E = tets.size // 4
    mi = np.ascontiguousarray(material_index, np.uint32)
    dens = np.ascontiguousarray(np.atleast_1d(density), np.float64)
    grads = np.zeros(E * 24, np.float32)
    vol = np.zeros(E, np.float32)
    m64 = np.zeros(N, np.float64)
    m32 = np.zeros(N, np.float32)
    off = np.zeros(N + 1, np.uint32)
    ae = np.zeros(E * 4, np.uint32)
    al = np.zeros(E * 4, np.uint8)
    conn = np.zeros(E * 8, np.uint32)
    st = lib().orc_preprocess_tets(N, E, _p(coords), _p(tets), _p(mi), _p(dens), _p(grads), _p(vol), _p(m64),
                                   _p(m32), _p(off), _p(ae), _p(al), _p(conn))
    if st:
        raise OracleError(st)
    return Packed(N, E, conn, grads, vol, mi, m64, m32, off, ae, al)


class System:
    """Oracle view of cwf::gpu::pcg::MatrixFreeSystem (pcg.hpp:67-86)."""

    def __init__(self, packed: Packed, stiffness: np.ndarray, bc_mask: np.ndarray, stiffness_scale: float,
                 mass_factor: float, reduction_block: int = 256):
        self.packed = packed
        self.stiffness = np.ascontiguousarray(stiffness, np.float64).reshape(-1)
        self.bc_mask = np.ascontiguousarray(bc_mask, np.uint32)
        N = packed.node_count
        D = 3 * N
        self.dof_count = D
        self.reduction_block = reduction_block
        self.reduction_partials = max(1, (D + reduction_block - 1) // reduction_block)
        self._s = _System(N, packed.element_count, D, _p(packed.connectivity), _p(packed.gradients),
                          _p(packed.volume), _p(packed.material_index), _p(self.stiffness),
                          self.stiffness.size // 36, _p(packed.lumped_mass), _p(self.bc_mask), stiffness_scale,
                          mass_factor, reduction_block, self.reduction_partials)

    def set_scalars(self, stiffness_scale: float, mass_factor: float):
        self._s.stiffness_scale = stiffness_scale
        self._s.mass_factor = mass_factor

    @property
    def ptr(self):
        return C.byref(self._s)

    def apply_keff(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(self.dof_count, np.float32)
        st = lib().orc_apply_keff(self.ptr, _p(x), _p(y))
        if st:
            raise OracleError(st)
        return y

    def derived_fields(self, u: np.ndarray):
        """derived_fields.cpp:139-211 -> (f32 [E,13], f32 [N,13]) {strain[6], stress[6], von_mises}."""
        u = np.ascontiguousarray(u, np.float32)
        el = np.zeros((self.packed.element_count, 13), np.float32)
        nd = np.zeros((self.packed.node_count, 13), np.float32)
        st = lib().orc_derived_fields(self.ptr, _p(u), _p(el), _p(nd))
        if st:
            raise OracleError(st)
        return el, nd

    def block_jacobi(self) -> np.ndarray:
        inv = np.zeros(self.packed.node_count * 9, np.float32)
        st = lib().orc_block_jacobi(self.ptr, _p(inv))
        if st:
            raise OracleError(st)
        return inv

    def dot(self, a: np.ndarray, b: np.ndarray):
        a = np.ascontiguousarray(a, np.float32)
        b = np.ascontiguousarray(b, np.float32)
        part = np.zeros(self.reduction_partials, np.float64)
        return lib().orc_dot(self.ptr, _p(a), _p(b), _p(part)), part

    def solve_pcg(self, rhs: np.ndarray, max_iterations: int = 128, relative_tolerance: float = 3e-4,
                  warm_start: bool = False, x: np.ndarray | None = None, history: bool = False):
        D = self.dof_count
        rhs = np.ascontiguousarray(rhs, np.float32)
        x = np.zeros(D, np.float32) if x is None else np.ascontiguousarray(x, np.float32).copy()
        r, p, z, Ap = (np.zeros(D, np.float32) for _ in range(4))
        part = np.zeros(self.reduction_partials, np.float64)
        tel = Telemetry()
        hist = np.zeros(max_iterations + 1, np.float64) if history else None
        st = lib().orc_solve_pcg(self.ptr, _p(rhs), max_iterations, relative_tolerance, int(warm_start), _p(x),
                                 _p(r), _p(p), _p(z), _p(Ap), _p(part), C.byref(tel),
                                 _p(hist) if hist is not None else None)
        if st:
            raise OracleError(st)
        out = dict(x=x, r=r, p=p, z=z, Ap=Ap, telemetry=tel)
        if hist is not None:
            out["history"] = hist[: tel.iterations + 1].copy()
        return out


class Stepper:
    """Oracle of cwf::gpu::newmark::Stepper's CPU branch (newmark_stepper.cpp:1005-1379)."""

    def __init__(self, system: System, external_force: np.ndarray, bc_value: np.ndarray, rayleigh_ab,
                 runtime_tolerance: float, pause_tolerance: float, max_iterations: int, initial_dt: float,
                 adaptive: bool = False, min_dt: float = 0.0, max_dt: float = 0.0, low_iteration_ratio: float = 0.3,
                 increase_factor: float = 1.1, decrease_factor: float = 0.5, warm_start: bool = True):
        self.system = system
        D = system.dof_count
        self.u, self.v, self.a = (np.zeros(D, np.float32) for _ in range(3))
        self.external_force = np.ascontiguousarray(external_force, np.float32).copy()
        self.bc_value = np.ascontiguousarray(bc_value, np.float32).copy()
        self._scratch = [np.zeros(D, np.float32) for _ in range(10)]
        self.partials = np.zeros(system.reduction_partials, np.float64)
        (self.u_pred, self.v_pred, self.rhs, self.damping_rhs, self.damping_out, self.x, self.r, self.p, self.z,
         self.Ap) = self._scratch
        s = _Stepper()
        s.system = C.cast(C.pointer(system._s), C.c_void_p)
        s.rayleigh_alpha, s.rayleigh_beta = rayleigh_ab
        s.runtime_tolerance, s.pause_tolerance = runtime_tolerance, pause_tolerance
        s.max_iterations = max_iterations
        s.adaptive, s.warm_start = int(adaptive), int(warm_start)
        s.min_dt, s.max_dt = min_dt, max_dt
        s.low_iteration_ratio, s.increase_factor, s.decrease_factor = (low_iteration_ratio, increase_factor,
                                                                       decrease_factor)
        s.dt = initial_dt if initial_dt > 0.0 else 1.0e-3
        s.beta, s.gamma = 0.25, 0.5
        for name in ("u", "v", "a", "external_force", "bc_value", "u_pred", "v_pred", "rhs", "damping_rhs",
                     "damping_out", "x", "r", "p", "z", "Ap", "partials"):
            setattr(s, name, _p(getattr(self, name)).value)
        self._s = s

    def set_warm_start(self, enabled: bool):
        self._s.warm_start = int(enabled)

    def set_external_force(self, f: np.ndarray):
        self.external_force[:] = np.asarray(f, np.float32)

    @property
    def time_step(self):
        return self._s.dt

    @property
    def current_time(self):
        return self._s.accumulated_time

    def step(self, sim_time: float, paused: bool = False) -> StepTelemetry:
        tel = StepTelemetry()
        st = lib().orc_stepper_step(C.byref(self._s), sim_time, int(paused), C.byref(tel))
        if st:
            raise OracleError(st)
        return tel


def evaluate_curve(points, time: float) -> float:
    t = np.ascontiguousarray([p[0] for p in points], np.float64)
    v = np.ascontiguousarray([p[1] for p in points], np.float64)
    return lib().orc_evaluate_curve(_p(t), _p(v), len(points), time)


def assemble_loads(mass64: np.ndarray, gravity, point_groups=()) -> np.ndarray:
    """loads.cpp:87-174 for gravity + point loads (tractions: see tests)."""
    N = mass64.size
    loads = np.zeros(3 * N, np.float64)
    g = np.ascontiguousarray(gravity, np.float64)
    lib().orc_gravity_loads(N, _p(np.ascontiguousarray(mass64)), _p(g), _p(loads))
    for nodes, value, scale in point_groups:
        nodes = np.ascontiguousarray(nodes, np.uint32)
        val = np.ascontiguousarray(value, np.float64)
        lib().orc_point_loads(nodes.size, _p(nodes), _p(val), float(scale), _p(loads))
    return loads


def dense_assemble(packed: Packed, tets: np.ndarray, grads64: np.ndarray, volume64: np.ndarray,
                   stiffness: np.ndarray) -> np.ndarray:
    n = 3 * packed.node_count
    K = np.zeros(n * n, np.float64)
    st = lib().orc_dense_assemble(packed.node_count, packed.element_count,
                                  _p(np.ascontiguousarray(tets, np.uint32)),
                                  _p(np.ascontiguousarray(grads64, np.float64)),
                                  _p(np.ascontiguousarray(volume64, np.float64)), _p(packed.material_index),
                                  _p(np.ascontiguousarray(stiffness, np.float64)), _p(K))
    if st:
        raise OracleError(st)
    return K


def dense_newmark_step(K, mass_diag, load, mask, targets, rayleigh_ab, dt, u0, v0, a0, tolerance, max_iterations,
                       beta=0.25, gamma=0.5):
    n = mass_diag.size
    a, _ = newmark_coefficients(dt, beta, gamma)
    coef = np.concatenate([[beta, gamma, dt], a]).astype(np.float64)
    u1, v1, a1 = (np.zeros(n) for _ in range(3))
    stats = (C.c_uint64 * 4)()
    st = lib().orc_dense_newmark_step(n, _p(K), _p(np.ascontiguousarray(mass_diag, np.float64)),
                                      _p(np.ascontiguousarray(load, np.float64)),
                                      _p(np.ascontiguousarray(mask, np.uint8)),
                                      _p(np.ascontiguousarray(targets, np.float64)), rayleigh_ab[0], rayleigh_ab[1],
                                      _p(coef), _p(np.ascontiguousarray(u0, np.float64)),
                                      _p(np.ascontiguousarray(v0, np.float64)),
                                      _p(np.ascontiguousarray(a0, np.float64)), tolerance, max_iterations, _p(u1),
                                      _p(v1), _p(a1), stats)
    if st:
        raise OracleError(st)
    raw = bytes(stats)
    iters = int.from_bytes(raw[0:8], "little")
    res = np.frombuffer(raw[8:16], np.float64)[0]
    conv = int.from_bytes(raw[16:20], "little", signed=True)
    return dict(u=u1, v=v1, a=a1, iterations=iters, residual_norm=float(res), converged=bool(conv))


def fnv1a64_words(x: np.ndarray) -> str:
    """64-bit FNV-1a over the f32 words (as the survey's reference driver hashed s.x)."""
    h = 1469598103934665603
    for w in np.ascontiguousarray(x, np.float32).view(np.uint32).tolist():
        h = ((h ^ w) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


# ---- native hex8 (hex8_oracle.c): PARITY UNPINNED -- the reference rejects hex8 elements
# (src/mesh/preprocess.cpp:326-330); this is the textbook fp64 isoparametric element the GPU
# hex8 kernels are checked against, plus physics checks in the tests.
def hex8_preprocess(coords: np.ndarray, hexes: np.ndarray, material_index: np.ndarray, density):
    """-> (volume f64 [E], lumped mass f64 [N], centroid gradients f32 [E*24])"""
    coords = np.ascontiguousarray(coords, np.float64)
    hexes = np.ascontiguousarray(hexes, np.uint32).reshape(-1, 8)
    mat = np.ascontiguousarray(material_index, np.uint32)
    dens = np.ascontiguousarray(np.atleast_1d(density), np.float64)
    N, E = coords.shape[0], hexes.shape[0]
    vol, mass, grads = np.zeros(E), np.zeros(N), np.zeros(E * 24, np.float32)
    st = lib().orc_hex8_preprocess(N, E, _p(coords), _p(hexes), _p(mat), _p(dens), dens.size, _p(vol), _p(mass),
                                   _p(grads))
    if st:
        raise OracleError(st)
    return vol, mass, grads


def hex8_apply(coords, hexes, material_index, D36s, sK, sM, mass, mask, x) -> np.ndarray:
    """y = K_eff x (fp64 accumulation, f32 out) with apply_keff's Dirichlet semantics."""
    coords = np.ascontiguousarray(coords, np.float64)
    hexes = np.ascontiguousarray(hexes, np.uint32).reshape(-1, 8)
    mat = np.ascontiguousarray(material_index, np.uint32)
    D = np.ascontiguousarray(D36s, np.float64)
    mass = np.ascontiguousarray(mass, np.float32)
    mask = np.ascontiguousarray(mask, np.uint32)
    x = np.ascontiguousarray(x, np.float32)
    N, E = coords.shape[0], hexes.shape[0]
    y, acc = np.zeros(3 * N, np.float32), np.zeros(3 * N)
    st = lib().orc_hex8_apply(N, E, _p(coords), _p(hexes), _p(mat), _p(D), sK, sM, _p(mass), _p(mask), _p(x), _p(y),
                              _p(acc))
    if st:
        raise OracleError(st)
    return y


def hex8_diag_blocks(coords, hexes, material_index, D36s, sK) -> np.ndarray:
    """node diagonal 3x3 blocks of the assembled stiffness (x sK), f64 [N, 3, 3]"""
    coords = np.ascontiguousarray(coords, np.float64)
    hexes = np.ascontiguousarray(hexes, np.uint32).reshape(-1, 8)
    mat = np.ascontiguousarray(material_index, np.uint32)
    D = np.ascontiguousarray(D36s, np.float64)
    N, E = coords.shape[0], hexes.shape[0]
    out = np.zeros(9 * N)
    st = lib().orc_hex8_diag_blocks(N, E, _p(coords), _p(hexes), _p(mat), _p(D), sK, _p(out))
    if st:
        raise OracleError(st)
    return out.reshape(N, 3, 3)


def hex8_solve64(coords, hexes, material_index, D36s, sK, sM, mass, mask, rhs, tol=1e-11, max_iterations=20000):
    """fp64 block-Jacobi PCG on the fp64 hex8 operator (the reference solution for the GPU tests)."""
    coords = np.ascontiguousarray(coords, np.float64)
    hexes = np.ascontiguousarray(hexes, np.uint32).reshape(-1, 8)
    mat = np.ascontiguousarray(material_index, np.uint32)
    D = np.ascontiguousarray(D36s, np.float64)
    mass = np.ascontiguousarray(mass, np.float32)
    mask = np.ascontiguousarray(mask, np.uint32)
    N, E = coords.shape[0], hexes.shape[0]
    L = lib()

    def A(v):
        v = np.ascontiguousarray(v, np.float64)
        out = np.zeros(3 * N)
        L.orc_hex8_apply64(N, E, _p(coords), _p(hexes), _p(mat), _p(D), sK, sM, _p(mass), _p(mask), _p(v), _p(out))
        return out

    blk = hex8_diag_blocks(coords, hexes, mat, D, sK) + (mass.astype(np.float64) * sM)[:, None, None] * np.eye(3)
    fixed = np.repeat(mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), N)
    for k in range(3):
        c = (mask & (1 << k)) != 0
        blk[c, k, :] = 0.0
        blk[c, :, k] = 0.0
        blk[c, k, k] = 1.0
    inv = np.linalg.inv(blk)
    b = np.asarray(rhs, np.float64).copy()
    x = np.where(fixed != 0, b, 0.0)
    r = b - A(x)
    z = np.einsum("nij,nj->ni", inv, r.reshape(-1, 3)).reshape(-1)
    p = z.copy()
    rz = r @ z
    nb = np.linalg.norm(b)
    for _ in range(max_iterations):
        Ap = A(p)
        al = rz / (p @ Ap)
        x += al * p
        r -= al * Ap
        if np.linalg.norm(r) <= tol * nb:
            break
        z = np.einsum("nij,nj->ni", inv, r.reshape(-1, 3)).reshape(-1)
        rz, rz0 = r @ z, rz
        p = z + (rz / rz0) * p
    return x
