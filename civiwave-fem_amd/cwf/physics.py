"""Host scalars of the hot path: materials (include/cwf/physics/materials.hpp:116-155),
Newmark coefficients (src/physics/newmark.cpp:34-81) and the config records they read
(include/cwf/config/config.hpp:64-237). Plain float64 Python arithmetic in the reference's
operand order, so every scalar is bit-identical to the C++ values."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional


# ---- config records (config.hpp) -------------------------------------------------------
@dataclass
class Material:
    name: str
    youngs_modulus: float
    poisson_ratio: float
    density: float


@dataclass
class Assignment:
    group: str
    material: str


@dataclass
class Damping:
    xi: float
    w1: float
    w2: float


@dataclass
class TimeSettings:
    initial_dt: float
    adaptive: bool = False
    min_dt: float = 0.0
    max_dt: float = 0.0


@dataclass
class SolverSettings:
    type: str = "pcg"
    preconditioner: str = "block_jacobi"
    runtime_tolerance: float = 3.0e-4
    pause_tolerance: float = 1.0e-5
    max_iterations: int = 128


@dataclass
class PrecisionSettings:
    vector_precision: str = "fp32"
    reduction_precision: str = "fp64"


@dataclass
class Curve:
    points: list = field(default_factory=list)  # [(time, value)]


@dataclass
class SurfaceTraction:
    group: str
    value: tuple
    scale_curve: str = ""


@dataclass
class PointLoad:
    group: str
    value: tuple
    scale_curve: str = ""


@dataclass
class Loads:
    gravity: tuple = (0.0, 0.0, 0.0)
    tractions: list = field(default_factory=list)
    points: list = field(default_factory=list)


@dataclass
class DirichletFix:
    group: str
    constrain_axis: tuple = (True, True, True)
    value: tuple = (None, None, None)  # optional per-axis targets


@dataclass
class OutputSettings:
    vtu_stride: int = 10
    probes: list = field(default_factory=list)


@dataclass
class Config:
    mesh_path: str = ""
    materials: list = field(default_factory=list)
    assignments: list = field(default_factory=list)
    damping: Damping = field(default_factory=lambda: Damping(0.0, 1.0, 1.0))
    time: TimeSettings = field(default_factory=lambda: TimeSettings(0.01))
    solver: SolverSettings = field(default_factory=SolverSettings)
    precision: PrecisionSettings = field(default_factory=PrecisionSettings)
    loads: Loads = field(default_factory=Loads)
    curves: dict = field(default_factory=dict)
    dirichlet: list = field(default_factory=list)
    output: OutputSettings = field(default_factory=OutputSettings)


# ---- materials.hpp -----------------------------------------------------------------------
@dataclass
class LamePair:
    lambda_: float
    mu: float


@dataclass
class ElasticProperties:
    youngs_modulus: float
    poisson_ratio: float
    bulk_modulus: float
    shear_modulus: float
    lame: LamePair
    stiffness: list  # 36 floats, Voigt (xx, yy, zz, xy, yz, xz), row-major


@dataclass
class RayleighCoefficients:
    alpha: float
    beta: float


def compute_lame(E: float, nu: float) -> LamePair:
    denom = (1.0 + nu) * (1.0 - 2.0 * nu)
    lam = (nu * E) / denom
    mu = E / (2.0 * (1.0 + nu))
    return LamePair(lam, mu)


def make_stiffness_matrix(E: float, nu: float) -> list:
    l = compute_lame(E, nu)
    c = l.lambda_ + 2.0 * l.mu
    lam, mu = l.lambda_, l.mu
    return [c, lam, lam, 0.0, 0.0, 0.0,
            lam, c, lam, 0.0, 0.0, 0.0,
            lam, lam, c, 0.0, 0.0, 0.0,
            0.0, 0.0, 0.0, mu, 0.0, 0.0,
            0.0, 0.0, 0.0, 0.0, mu, 0.0,
            0.0, 0.0, 0.0, 0.0, 0.0, mu]


def make_properties(material: Material) -> ElasticProperties:
    l = compute_lame(material.youngs_modulus, material.poisson_ratio)
    bulk = l.lambda_ + (2.0 / 3.0) * l.mu
    return ElasticProperties(material.youngs_modulus, material.poisson_ratio, bulk, l.mu, l,
                             make_stiffness_matrix(material.youngs_modulus, material.poisson_ratio))


def compute_rayleigh(damping: Damping) -> RayleighCoefficients:
    denom = damping.w1 + damping.w2
    alpha = 2.0 * damping.xi * damping.w1 * damping.w2 / denom
    beta = 2.0 * damping.xi / denom
    return RayleighCoefficients(alpha, beta)


# ---- newmark.cpp ---------------------------------------------------------------------------
@dataclass
class Coefficients:
    beta: float
    gamma: float
    dt: float
    a0: float
    a1: float
    a2: float
    a3: float
    a4: float
    a5: float


@dataclass
class UpdateScalars:
    inv_beta_dt2: float
    gamma_over_beta_dt: float


def make_coefficients(dt: float, beta: float = 0.25, gamma: float = 0.5) -> Coefficients:
    return Coefficients(beta, gamma, dt,
                        1.0 / (beta * dt * dt),
                        gamma / (beta * dt),
                        1.0 / (beta * dt),
                        (1.0 / (2.0 * beta)) - 1.0,
                        (gamma / beta) - 1.0,
                        dt * ((gamma / (2.0 * beta)) - 1.0))


def compute_update_scalars(c: Coefficients) -> UpdateScalars:
    beta_dt = c.beta * c.dt
    return UpdateScalars(1.0 / (c.beta * c.dt * c.dt), c.gamma / beta_dt)


def evaluate_curve(curve: Curve, time: float) -> float:
    """loads.cpp:63-85 (std::lerp as in libstdc++)."""
    pts = curve.points
    if not pts:
        return 1.0
    if time <= pts[0][0]:
        return pts[0][1]
    for i in range(1, len(pts)):
        t0, v0 = pts[i - 1]
        t1, v1 = pts[i]
        if time <= t1:
            span = t1 - t0
            w = (time - t0) / span if span > 0.0 else 0.0
            return _lerp(v0, v1, w)
    return pts[-1][1]


def _lerp(a: float, b: float, t: float) -> float:
    if (a <= 0 and b >= 0) or (a >= 0 and b <= 0):
        return t * b + (1 - t) * a
    if t == 1:
        return b
    x = a + t * (b - a)
    return (x if b < x else b) if ((t > 1) == (b > a)) else (x if b > x else b)


def effective_scalars(c: Coefficients, r: RayleighCoefficients) -> tuple[float, float]:
    """(stiffness_scale, mass_factor) of newmark_stepper.cpp:1322-1326 / newmark.cpp:83-100."""
    return 1.0 + c.a1 * r.beta, c.a0 + c.a1 * r.alpha
