"""FAST mode's 16-B block-Jacobi record (csrc/blockinv_pack.hpp), on the CPU through the library's host
entry point cwf_pack_block_inverse (the code the device's k_sym_inverse runs).

The reference stores the per-node 3x3 inverse in f32 with constrained rows = identity
(pcg.cpp:270-408). FAST applies the symmetrised free-free block, packed as an fp32 scale,
fp16 row scales t_k = sqrt(B_kk/S) and fp16 correlations C_ij; blocks that do not fit that form fall
back to fp32. Tolerances below: each applied entry within 2^-10 of its own scale sqrt(B_ii B_jj)."""
import numpy as np
import pytest

from cwf import pcg, scenarios
from helpers import oracle_system

UP = [(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]


def upper(b):
    return np.array([b[i, j] for i, j in UP], np.float32)


def decode(w):
    """numpy restatement of unpack_block_inverse (the update pass's decode)."""
    S = w[:1].view(np.float32)[0]
    h = np.array([w[1] & 0xFFFF, w[1] >> 16, w[2] & 0xFFFF, w[2] >> 16, w[3] & 0xFFFF, w[3] >> 16],
                 np.uint16).view(np.float16).astype(np.float32)
    t0, t1, t2, c01, c02, c12 = h
    f = np.float32
    return np.array([S * f(t0 * t0), S * f(f(t0 * t1) * c01), S * f(f(t0 * t2) * c02), S * f(t1 * t1),
                     S * f(f(t1 * t2) * c12), S * f(t2 * t2)], np.float32)


def check_close(v, d, mk):
    diag = {0: v[0], 1: v[3], 2: v[5]}
    for (i, j), vi, di in zip(UP, v, d):
        if (mk >> i) & 1 or (mk >> j) & 1:
            assert di == 0.0
        else:
            scale = np.sqrt(float(diag[i]) * float(diag[j]))
            assert abs(float(di) - float(vi)) <= 2.0 ** -10 * scale, (i, j, vi, di)


def test_partial_mask_keeps_free_entries_at_physical_scale():
    # free entries ~1e-10 (1/K at E = 30 GPa) next to a constrained axis whose reference row is identity
    b = np.array([[1.0, 0.0, 0.0], [0.0, 3.1e-10, -4.0e-11], [0.0, -4.0e-11, 2.2e-10]])
    for mk in (1, 0b011, 0b101):
        ok, w, d = pcg.pack_block_inverse(upper(b), mk)
        assert ok
        check_close(upper(b), d, mk)
        assert np.array_equal(decode(w).view(np.uint32), d.view(np.uint32))
    # the old single-scale fp16 packing (scale = block max = the identity's 1.0) flushed these to zero
    assert np.float16(3.1e-10) == 0


def test_diagonal_spread_and_fully_masked():
    rng = np.random.Generator(np.random.PCG64(5))
    for _ in range(200):
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        ev = 10.0 ** rng.uniform(-11, -8, 3)  # eigenvalues 3 decades apart
        b = (q * ev) @ q.T
        ok, w, d = pcg.pack_block_inverse(upper(b), 0)
        v = upper(b)
        if ok:
            check_close(v, d, 0)
            assert np.array_equal(decode(w).view(np.uint32), d.view(np.uint32))
            m = np.array([[d[0], d[1], d[2]], [d[1], d[3], d[4]], [d[2], d[4], d[5]]], np.float64)
            assert np.all(np.linalg.eigvalsh(m) > 0)  # the applied preconditioner stays SPD
        else:
            assert w[0] == np.float32(-1.0).view(np.uint32) and np.array_equal(d, v)
    ok, w, d = pcg.pack_block_inverse(upper(np.eye(3)), 7)
    assert ok and not d.any() and w[0] == 0


@pytest.mark.parametrize("b", [
    np.array([[1e-10, 0.9999e-10, 0], [0.9999e-10, 1e-10, 0], [0, 0, 1e-10]]),  # near-singular correlation
    np.array([[-1e-10, 0, 0], [0, 1e-10, 0], [0, 0, 1e-10]]),  # not positive
    np.array([[np.inf, 0, 0], [0, 1e-10, 0], [0, 0, 1e-10]]),
    np.array([[1.0, 0, 0], [0, 1e-10, 0], [0, 0, 1e-10]]),  # diagonal spread 1e10 > 2^28
])
def test_fallback_blocks_apply_fp32(b):
    ok, w, d = pcg.pack_block_inverse(upper(b), 0)
    assert not ok
    assert w[0] == np.float32(-1.0).view(np.uint32)
    assert np.array_equal(d.view(np.uint32), upper(b).view(np.uint32))


@pytest.mark.parametrize("element", ["tet4"])
def test_reference_blocks_of_a_roller_case_pack_without_fallback(element):
    """Every block of the reference inverse (oracle) on a mesh with partial masks packs within tolerance."""
    case = scenarios.roller_case(6, 4, 3, element=element)
    P = case.packing
    inv = oracle_system(P, case.materials, *case.scalars()).block_jacobi().reshape(-1, 3, 3)
    fallbacks = 0
    for n in range(P.node_count):
        b = inv[n].astype(np.float64)
        sym = np.triu(b) + np.triu(b, 1).T  # upper triangle wins
        ok, w, d = pcg.pack_block_inverse(upper(sym), int(P.bc_mask[n]))
        fallbacks += not ok
        if ok:
            check_close(upper(sym), d, int(P.bc_mask[n]))
    assert fallbacks == 0
