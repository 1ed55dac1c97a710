"""Derived fields on the GPU (post.hip) bit for bit against the oracle, and the output manager
cadence of the reference's export_writer_test.cpp:146-183 driven from a device-resident Stepper."""
import os

import numpy as np
import pytest

from cwf import _lib, pcg, post, scenarios
from cwf.stepper import Stepper
from helpers import assert_bitwise, oracle_system
from test_post import reference_vtu_bytes, single_tet_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["single_tet", "kuhn_rayleigh", "jitter"])
def test_derived_fields_bitwise(name):
    if name == "single_tet":
        mesh, cfg, P = single_tet_case()
        from cwf import physics
        mats = [physics.make_properties(m) for m in cfg.materials]
    else:
        case = (scenarios.block_case(5, 4, 3, h=0.1, xi=0.05, w=(10.0, 100.0)) if name == "kuhn_rayleigh"
                else scenarios.block_case(6, 5, 4, h=0.1, jitter=True))
        P, mats = case.packing, case.materials
    rng = np.random.Generator(np.random.PCG64(21))
    u = rng.uniform(-1e-3, 1e-3, P.dof_count).astype(np.float32)
    P.displacement = u
    for mode in (_lib.MODE_PARITY, _lib.MODE_FAST):
        s = pcg.MatrixFreeSystem.from_packing(P, mats, 1.0, 0.0, mode=mode)
        d = post.compute_derived_fields(P, mats, system=s)
        el, nd = oracle_system(P, mats, 1.0, 0.0).derived_fields(u)
        assert_bitwise(d.elements, el, f"{name} element fields")
        assert_bitwise(d.nodes, nd, f"{name} node fields")
        s.close()


def test_derived_fields_from_device_displacement():
    import torch

    case = scenarios.block_case(4, 3, 3, h=0.1)
    P = case.packing
    rng = np.random.Generator(np.random.PCG64(4))
    u = rng.uniform(-1e-3, 1e-3, P.dof_count).astype(np.float32)
    P.displacement = u
    d_host = post.compute_derived_fields(P, case.materials)
    d_dev = post.compute_derived_fields(P, case.materials, displacement=torch.from_numpy(u).cuda())
    assert_bitwise(d_dev.elements, d_host.elements)
    assert_bitwise(d_dev.nodes, d_host.nodes)


def test_output_manager_stride_probes_and_stepper_state(tmp_path):
    # export_writer_test.cpp:146-183 (stride 2, probe node 0), driven by two device Newmark steps
    case = scenarios.block_case(4, 3, 3, h=0.1)
    P = case.packing
    st = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time)
    settings = type(case.cfg.output)(vtu_stride=2, probes=[0, 7])
    om = post.OutputManager(tmp_path, case.mesh, P, case.materials, settings, stepper=st)
    t = 0.0
    for frame in range(3):
        assert st.step(t).has_value()
        t += case.cfg.time.initial_dt
        assert om.handle_frame(t, frame).has_value()
    assert (tmp_path / "vtu" / "frame_00000.vtu").exists()
    assert not (tmp_path / "vtu" / "frame_00001.vtu").exists()
    assert (tmp_path / "vtu" / "frame_00002.vtu").exists()
    lines = (tmp_path / "probes" / "probes.csv").read_text().splitlines()
    assert len(lines) == 1 + 3 * 2
    # the last frame's file is the reference format over the stepper's device state
    u = st.get_state(Stepper.DISPLACEMENT)
    assert np.array_equal(u.view(np.uint32), P.displacement.view(np.uint32))
    el, nd = oracle_system(P, case.materials, 1.0, 0.0).derived_fields(u)
    got = (tmp_path / "vtu" / "frame_00002.vtu").read_bytes()
    assert got == reference_vtu_bytes(P, el, nd, t, 2)
    om.close()
