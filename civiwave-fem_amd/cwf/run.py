"""Scenario driver: YAML scenario -> Gmsh mesh -> preprocess/pack -> device Newmark steps -> VTU/probes.

    python -m cwf.run scenario.yaml [--steps N] [--out DIR] [--mode parity|fast] [--paused]
                                    [--time-varying-loads] [--device K]

The reference has no such executable (its only binary is the viewer demo);
this wires its pieces in the order the viewer backend does (src/ui/viewer.cpp:200-277):
load_config_from_file -> load_gmsh_file -> pre::run + pack::build_packed_buffers -> Stepper, then per
frame ``step(simulation_time)``, ``simulation_time = telemetry.simulation_time + telemetry.time_step``
and OutputManager::handle_frame. The external force is evaluated once at pack time (t = 0), as in the
reference (newmark_stepper.cpp:1369-1379); ``--time-varying-loads`` re-evaluates the load curves at
every step's start time instead (the viewer's custom-load path, viewer.cpp:262-266).

Mesh paths are resolved like the reference (relative to the working directory) and, failing that,
relative to the YAML file's directory. One JSON line per step is printed; the last line is a summary.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

from . import _lib, config, mesh, pack, post
from .physics import compute_rayleigh, make_properties
from .stepper import Stepper


class ScenarioError(RuntimeError):
    pass


def resolve_mesh_path(cfg_path: str, mesh_path: str) -> str:
    if os.path.isabs(mesh_path) or os.path.exists(mesh_path):
        return mesh_path
    here = os.path.dirname(os.path.abspath(cfg_path))
    for cand in (os.path.join(here, mesh_path), os.path.join(here, os.path.basename(mesh_path))):
        if os.path.exists(cand):
            return cand
    return mesh_path


def load_scenario(cfg_path: str, allow_hex8: bool = False):
    """-> (config, tet mesh, packing, materials). Raises ScenarioError with the reference's texts.
    allow_hex8: an all-hex8 Gmsh mesh runs as native hex8 (FAST mode only)."""
    rc = config.load_config_from_file(cfg_path)
    if not rc.has_value():
        raise ScenarioError(f"config: {rc.error().message} {rc.error().context}")
    cfg = rc.value()
    rm = mesh.load_gmsh_file(resolve_mesh_path(cfg_path, cfg.mesh_path))
    if not rm.has_value():
        raise ScenarioError(f"mesh: {rm.error().message} {rm.error().context}")
    try:
        m = rm.value().to_tet_mesh(allow_hex8)
        P = pack.build_packed_buffers(m, cfg)
    except pack.PackError as e:
        raise ScenarioError(f"preprocess: {e.message} {e.context}") from None
    return cfg, m, P, [make_properties(x) for x in cfg.materials]


def run_scenario(cfg_path: str, steps: int, out_dir: str | None, mode: int = _lib.MODE_PARITY, device: int = 0,
                 paused: bool = False, time_varying_loads: bool = False, log=print) -> dict:
    cfg, m, P, materials = load_scenario(cfg_path, allow_hex8=mode == _lib.MODE_FAST)
    st = Stepper(P, materials, compute_rayleigh(cfg.damping), cfg.solver, cfg.time, mode=mode, device=device)
    om = post.OutputManager(out_dir, m, P, materials, cfg.output, stepper=st) if out_dir else None
    t_sim, total_iters, wall0 = 0.0, 0, time.perf_counter()
    last = None
    try:
        for frame in range(steps):
            if time_varying_loads:
                f = pack._safe_f32(pack.assemble_load_vector(m, cfg, P.lumped_mass64, t_sim))
                st.set_external_force(f)
            r = st.step(t_sim, paused)
            if not r.has_value():
                raise ScenarioError(f"step {frame}: {r.error().message} {r.error().context}")
            tel = r.value()
            t_sim = tel.simulation_time + tel.time_step
            total_iters += tel.pcg.iterations
            if om is not None:
                o = om.handle_frame(t_sim, frame)
                if not o.has_value():
                    raise ScenarioError(f"output frame {frame}: {o.error().message} {o.error().context}")
            last = dict(frame=frame, time=t_sim, dt=tel.time_step, iterations=tel.pcg.iterations,
                        residual=tel.pcg.residual_norm, converged=tel.pcg.converged,
                        dt_increased=tel.dt_increased, dt_decreased=tel.dt_decreased)
            log(json.dumps(last))
        wall = time.perf_counter() - wall0
        return dict(scenario=cfg_path, nodes=P.node_count, tets=P.element_count, dofs=P.dof_count, steps=steps,
                    pcg_iterations=total_iters, wall_s=wall, final_time=t_sim, last=last,
                    mode="fast" if mode == _lib.MODE_FAST else "parity")
    finally:
        if om is not None:
            om.close()
        st.close()
        st.system.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m cwf.run", description=__doc__.split("\n\n")[0])
    ap.add_argument("scenario")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--out", default=None, help="output root (vtu/, probes/); omitted: no files")
    ap.add_argument("--mode", choices=["parity", "fast"], default="parity")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--paused", action="store_true")
    ap.add_argument("--time-varying-loads", action="store_true")
    a = ap.parse_args(argv)
    try:
        s = run_scenario(a.scenario, a.steps, a.out, _lib.MODE_FAST if a.mode == "fast" else _lib.MODE_PARITY,
                         a.device, a.paused, a.time_varying_loads)
    except ScenarioError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    print(json.dumps(dict(summary=s)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
