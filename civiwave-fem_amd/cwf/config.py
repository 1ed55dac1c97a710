"""``cwf::config`` mirror (include/cwf/config/config.hpp:272-298) over the native parser.

``load_config_from_file`` / ``load_config_from_string`` run the library's YAML-subset parser and
parse_config_node validation (src/config/config.cpp:148-605, csrc/config.cpp): the same messages and
breadcrumbs come back as a ``ConfigError`` inside an ``Expected``; a valid document becomes the
``physics.Config`` records the rest of the host path consumes.
"""
from __future__ import annotations

import ctypes as C
import json
import os
from dataclasses import dataclass, field

from . import _lib
from .pcg import Expected
from .physics import (Assignment, Config, Curve, Damping, DirichletFix, Loads, Material, OutputSettings, PointLoad,
                      PrecisionSettings, SolverSettings, SurfaceTraction, TimeSettings)


@dataclass
class ConfigError:
    message: str
    context: list = field(default_factory=list)


def _f3(v):
    return tuple(float(x) for x in v)


def _from_json(d: dict) -> Config:
    f = float
    return Config(
        mesh_path=d["mesh_path"],
        materials=[Material(m["name"], f(m["E"]), f(m["nu"]), f(m["rho"])) for m in d["materials"]],
        assignments=[Assignment(a["group"], a["material"]) for a in d["assignments"]],
        damping=Damping(f(d["damping"]["xi"]), f(d["damping"]["w1"]), f(d["damping"]["w2"])),
        time=TimeSettings(f(d["time"]["initial_dt"]), bool(d["time"]["adaptive"]), f(d["time"]["min_dt"]),
                          f(d["time"]["max_dt"])),
        solver=SolverSettings(d["solver"]["type"], d["solver"]["preconditioner"], f(d["solver"]["runtime_tolerance"]),
                              f(d["solver"]["pause_tolerance"]), int(d["solver"]["max_iterations"])),
        precision=PrecisionSettings(**d["precision"]),
        loads=Loads(_f3(d["loads"]["gravity"]),
                    [SurfaceTraction(t["group"], _f3(t["value"]), t["scale_curve"]) for t in d["loads"]["tractions"]],
                    [PointLoad(p["group"], _f3(p["value"]), p["scale_curve"]) for p in d["loads"]["points"]]),
        curves={k: Curve([(f(p[0]), f(p[1])) for p in v]) for k, v in d["curves"].items()},
        dirichlet=[DirichletFix(x["group"], tuple(x["constrain_axis"]),
                                tuple(None if v is None else f(v) for v in x["value"])) for x in d["dirichlet"]],
        output=OutputSettings(d["output"]["vtu_stride"], list(d["output"]["probes"])),
    )


def _finish(rc: int, h: C.c_void_p) -> Expected:
    L = _lib.load()
    if rc:
        msg, ctx = _lib.last_error(None)
        return Expected(error=ConfigError(msg, ctx))
    try:
        return Expected(_from_json(json.loads(L.cwf_config_json(h).decode())))
    finally:
        L.cwf_config_destroy(h)


def load_config_from_string(yaml_text: str) -> Expected:
    h = C.c_void_p()
    return _finish(_lib.load().cwf_config_load_string(yaml_text.encode(), C.byref(h)), h)


def load_config_from_file(path) -> Expected:
    h = C.c_void_p()
    return _finish(_lib.load().cwf_config_load_file(os.fsencode(str(path)), C.byref(h)), h)
