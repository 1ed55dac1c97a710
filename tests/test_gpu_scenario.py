"""End-to-end scenario driver on the GPU: YAML + Gmsh files -> device Newmark steps -> VTU / probes,
bit-exact (PARITY) with the oracle's Stepper CPU branch on the same packing."""
import json
import os

import numpy as np
import pytest

import oracle as O
from cwf import _lib, run
from cwf.stepper import Stepper
from helpers import assert_bitwise, oracle_system
from scenario_files import write_block_scenario
from test_post import reference_vtu_bytes

pytestmark = pytest.mark.gpu


def test_run_scenario_parity_matches_oracle_stepper(tmp_path):
    y = write_block_scenario(str(tmp_path), 6, 3, 3, xi=0.05, w=(10.0, 100.0), tol=1e-6, stride=2)
    out = tmp_path / "out"
    lines = []
    s = run.run_scenario(y, 3, str(out), _lib.MODE_PARITY, log=lines.append)
    assert s["steps"] == 3 and len(lines) == 3
    cfg, m, P, mats = run.load_scenario(y)
    from cwf.physics import compute_rayleigh, effective_scalars, make_coefficients
    r = compute_rayleigh(cfg.damping)
    sK, sM = effective_scalars(make_coefficients(cfg.time.initial_dt), r)
    o = oracle_system(P, mats, sK, sM)
    ost = O.Stepper(o, P.external_force, P.bc_value, (r.alpha, r.beta), cfg.solver.runtime_tolerance,
                    cfg.solver.pause_tolerance, cfg.solver.max_iterations, cfg.time.initial_dt)
    t = 0.0
    for k in range(3):
        rt = ost.step(t)
        assert json.loads(lines[k])["iterations"] == rt.pcg.iterations
        t = rt.simulation_time + rt.time_step
    # the driver's last VTU frame (frame 2) is the reference format of the oracle's final state
    P.displacement, P.velocity, P.acceleration = ost.u.copy(), ost.v.copy(), ost.a.copy()
    el, nd = oracle_system(P, mats, 1.0, 0.0).derived_fields(ost.u)
    assert (out / "vtu" / "frame_00002.vtu").read_bytes() == reference_vtu_bytes(P, el, nd, t, 2)
    assert not (out / "vtu" / "frame_00001.vtu").exists()
    rows = (out / "probes" / "probes.csv").read_text().splitlines()
    assert len(rows) == 1 + 3 * 2 and rows[-1].startswith(f"2,{t:.9f},5,")


def test_run_scenario_fast_mode_and_cli(tmp_path, capsys):
    y = write_block_scenario(str(tmp_path), 6, 3, 3, tol=1e-5)
    rc = run.main([y, "--steps", "2", "--mode", "fast", "--out", str(tmp_path / "o")])
    assert rc == 0
    out = capsys.readouterr().out.strip().splitlines()
    summary = json.loads(out[-1])["summary"]
    assert summary["steps"] == 2 and summary["mode"] == "fast" and summary["pcg_iterations"] > 0
    assert (tmp_path / "o" / "vtu" / "frame_00000.vtu").exists()
