"""The fused lattice iteration's algorithm (lattice_fused.inc) on the CPU, before any kernel: one global reduction
per iteration (alpha from the direct rho_j = r_j.z_j and p_j.Ap_j; beta's numerator r_(j+1).z_(j+1) expanded through
r_(j+1) = r_j - alpha_j Ap_j from the same launch's z_j.Ap_j and Ap_j.M^-1 Ap_j, re-based on the direct dots every
iteration) against the reference loop (pcg.cpp:840-901), both emulated in FAST arithmetic (fp32 vectors, fp64 dot
accumulation) on the oracle's operator by tools/cg_variants.py. The fused form must converge in the reference loop's
iteration count (to a few iterations) to the same solution; the device kernels are checked against the two-kernel
loop in tests/test_gpu_lattice.py."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import cg_variants as cg  # noqa: E402


@pytest.mark.parametrize("shape,tol,static", [((20, 5, 10), 2e-4, True), ((20, 5, 10), 2e-4, False),
                                              ((17, 7, 5), 1e-6, True)])
def test_fused_recurrence_matches_reference_loop(shape, tol, static):
    o, inv, rhs, mask = cg.setup(*shape, tol, static)
    its, xs = cg.standard(o, inv, rhs, mask, tol, 4000)
    itf, xf, rel = cg.fused(o, inv, rhs, mask, tol, 4000)
    assert its < 4000 and itf < 4000
    assert abs(itf - its) <= max(3, its // 25), (itf, its)
    # the stop is decided on the direct |r| of the formed r_j, as the device kernel decides it
    assert rel <= tol, rel
    dx = np.linalg.norm(xf.astype(np.float64) - xs) / np.linalg.norm(xs)
    assert dx <= 50 * tol, dx
