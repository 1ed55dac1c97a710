"""FAST handles renumber their nodes internally (Morton order of node_coords, cwf_hip.h
CWF_DESC_KEEP_NODE_ORDER): every vector crossing the ABI is in the caller's order. Checked on the
permuted C4-style mesh against a keep-order handle and the oracle."""
import numpy as np
import pytest

from cwf import _lib, pcg, scenarios
from cwf.stepper import Stepper
from helpers import oracle_system

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def case():
    return scenarios.block_case(9, 7, 6, h=0.1, jitter=True, tol=1e-6, max_iterations=800)


def _fast(case, keep):
    P = case.packing
    return pcg.MatrixFreeSystem(P.connectivity, P.gradients, P.volume, P.material_index, case.materials,
                                P.lumped_mass, P.bc_mask, P.node_count, P.element_count, P.dof_count,
                                *case.scalars(), 256, None, None, _lib.MODE_FAST, 0, P.position64,
                                keep_node_order=keep)


def test_renumbered_handle_matches_keep_order_and_oracle(case):
    P = case.packing
    a, b = _fast(case, False), _fast(case, True)
    o = oracle_system(P, case.materials, *case.scalars())
    x = np.random.Generator(np.random.PCG64(4)).uniform(-1, 1, P.dof_count).astype(np.float32)
    ya, yb = np.zeros_like(x), np.zeros_like(x)
    pcg.apply_keff(a, x, ya).value()
    pcg.apply_keff(b, x, yb).value()
    ref = o.apply_keff(x).astype(np.float64)
    for y in (ya, yb):
        assert np.max(np.abs(y - ref)) <= 2e-5 * np.max(np.abs(ref))
    ia, ib = np.zeros(9 * P.node_count, np.float32), np.zeros(9 * P.node_count, np.float32)
    pcg.build_block_jacobi_inverse(a, None, ia).value()
    pcg.build_block_jacobi_inverse(b, None, ib).value()
    assert np.array_equal(ia, ib)  # node-local fp64 setup: the renumbering only moves rows
    rhs = case.static_rhs()
    xa, xb = np.zeros_like(rhs), np.zeros_like(rhs)
    ra = np.zeros_like(rhs)
    ta = pcg.solve_pcg(a, rhs, pcg.PcgSettings(800, 1e-6), pcg.PcgVectors(xa, ra)).value()
    tb = pcg.solve_pcg(b, rhs, pcg.PcgSettings(800, 1e-6), pcg.PcgVectors(xb, np.zeros_like(rhs))).value()
    assert ta.converged and tb.converged and abs(ta.iterations - tb.iterations) <= 3
    assert np.linalg.norm(xa - xb) <= 1e-4 * np.linalg.norm(xb)
    # the residual comes back in the caller's order: zero on the caller's Dirichlet rows (pcg.cpp:458-475),
    # its norm the telemetry's (fp32 vector vs the fp64 device fold)
    mask = np.repeat(P.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), P.node_count)
    assert np.all(ra[mask != 0] == 0.0) and np.any(ra[mask == 0] != 0.0)
    assert abs(np.linalg.norm(ra.astype(np.float64)) - ta.residual_norm) <= 1e-4 * ta.residual_norm


def test_renumbered_stepper_state_in_caller_order(case):
    P = case.packing
    st = {}
    for keep in (False, True):
        s = _fast(case, keep)
        t = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=_lib.MODE_FAST,
                    system=s)
        for i in range(2):
            t.step(0.01 * i).value()
        st[keep] = t.get_state(Stepper.DISPLACEMENT)
        t.close()
    assert np.linalg.norm(st[False] - st[True]) <= 1e-4 * np.linalg.norm(st[True])


def test_renumbered_handle_rejects_parity_switch_and_attach(case):
    s = _fast(case, False)
    h = s.handle()
    L = _lib.load()
    assert L.cwf_hip_system_set_mode(h, _lib.MODE_PARITY) == -13
    assert "cannot switch to CWF_MODE_PARITY" in _lib.last_error(h)[0]
