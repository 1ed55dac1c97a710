#!/usr/bin/env python3
"""Numerics of PCG iteration forms in FAST arithmetic (fp32 vectors, fp64 dot accumulation), emulated in numpy on the
oracle's operator (CPU only; a design check, not a test of the device code).

  standard : the reference loop (pcg.cpp:840-901): alpha = rho / p.Ap; r -= alpha Ap; z = M^-1 r; rho' = r.z (a
             second global reduction); beta = rho' / rho; p = z + beta p.   Two reductions per iteration.
  fused    : one reduction per iteration (the device's lattice_fused.inc; the convergence test on the direct |r|). Kernel i+1 forms r_{i+1}, z_{i+1}, p_{i+1} and Ap_{i+1} itself, so the
             dots it has at its start are those kernel i reduced: the direct rho_i = r_i.z_i and |r_i|^2 of the
             vectors kernel i formed, and p_i.Ap_i, z_i.Ap_i, Ap_i.M^-1 Ap_i, r_i.Ap_i, Ap_i.Ap_i. Then
               alpha_i = rho_i / p_i.Ap_i                                   (the reference's alpha, direct rho)
               rho_{i+1} ~ rho_i - 2 alpha_i z_i.Ap_i + alpha_i^2 Ap_i.M^-1 Ap_i   (one step of recurrence, re-based
               |r_{i+1}|^2 ~ |r_i|^2 - 2 alpha_i r_i.Ap_i + alpha_i^2 Ap_i.Ap_i     on the direct dots every iteration)
             and beta_{i+1} = rho_{i+1} / rho_i, the convergence test on |r_{i+1}|.

usage: python tools/cg_variants.py [nx ny nz] [tol]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "civiwave-fem_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

from cwf import scenarios  # noqa: E402
from helpers import oracle_system  # noqa: E402


def setup(nx, ny, nz, tol, static=True):
    case = scenarios.block_case(nx, ny, nz, h=0.1, tol=tol)
    P = case.packing
    sK, sM = case.scalars()
    if static:
        sM = 0.0
    o = oracle_system(P, case.materials, sK, sM)
    inv = o.block_jacobi().reshape(-1, 3, 3).astype(np.float32)
    rhs = case.static_rhs().astype(np.float32)
    mask = (np.repeat(P.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), P.node_count)) != 0
    return o, inv, rhs, mask


def prec(inv, r):
    return np.einsum("nij,nj->ni", inv, r.reshape(-1, 3)).astype(np.float32).reshape(-1)


def d64(a, b):
    return float(np.dot(a.astype(np.float64), b.astype(np.float64)))


def standard(o, inv, rhs, mask, tol, maxit):
    x = np.zeros_like(rhs)
    r = rhs.copy()
    r[mask] = 0.0
    z = prec(inv, r)
    z[mask] = 0.0
    p = z.copy()
    rho = d64(r, z)
    nb = np.sqrt(d64(rhs, rhs))
    for it in range(1, maxit + 1):
        Ap = o.apply_keff(p).astype(np.float32)
        alpha = rho / d64(p, Ap)
        x = (x + np.float32(alpha) * p).astype(np.float32)
        r = (r - np.float32(alpha) * Ap).astype(np.float32)
        r[mask] = 0.0
        if np.sqrt(d64(r, r)) <= tol * nb:
            return it, x
        z = prec(inv, r)
        z[mask] = 0.0
        rn = d64(r, z)
        p = (z + np.float32(rn / rho) * p).astype(np.float32)
        rho = rn
    return maxit, x


def fused(o, inv, rhs, mask, tol, maxit, direct=True):
    """direct (the device kernel, lattice_fused.inc): the convergence test on the direct |r_j| of the formed r (launch
    j + 1 tests launch j's r_j.r_j share); else on the recurrence |r_(j+1)|^2 ~ |r_j|^2 - 2 alpha r.Ap + alpha^2 Ap.Ap"""
    x = np.zeros_like(rhs)
    r = rhs.copy()
    r[mask] = 0.0
    z = prec(inv, r)
    z[mask] = 0.0
    p = z.copy()
    nb = np.sqrt(d64(rhs, rhs))
    Ap = o.apply_keff(p).astype(np.float32)
    # kernel 0's reductions (the prologue)
    rho, rr = d64(r, z), d64(r, r)
    for it in range(1, maxit + 1):
        MAp = prec(inv, Ap)
        MAp[mask] = 0.0
        pAp, zAp, AMA, rAp, AA = d64(p, Ap), d64(z, Ap), d64(Ap, MAp), d64(r, Ap), d64(Ap, Ap)
        alpha = rho / pAp
        rho_n = rho - 2 * alpha * zAp + alpha * alpha * AMA
        rr_n = rr - 2 * alpha * rAp + alpha * alpha * AA
        # kernel it: r, x, z, the convergence test on the extrapolated |r|, p, Ap, and the direct dots
        x = (x + np.float32(alpha) * p).astype(np.float32)
        r = (r - np.float32(alpha) * Ap).astype(np.float32)
        r[mask] = 0.0
        if np.sqrt(max(d64(r, r) if direct else rr_n, 0.0)) <= tol * nb:
            return it, x, np.sqrt(d64(r, r)) / nb
        z = prec(inv, r)
        z[mask] = 0.0
        p = (z + np.float32(rho_n / rho) * p).astype(np.float32)
        Ap = o.apply_keff(p).astype(np.float32)
        rho, rr = d64(r, z), d64(r, r)
    return maxit, x, np.sqrt(d64(r, r)) / nb


def main():
    a = sys.argv[1:]
    nx, ny, nz = (int(v) for v in a[:3]) if len(a) >= 3 else (33, 9, 5)
    tol = float(a[3]) if len(a) > 3 else 1e-6
    for static in (True, False):
        o, inv, rhs, mask = setup(nx, ny, nz, tol, static)
        its, xs = standard(o, inv, rhs, mask, tol, 5000)
        itf, xf, rel = fused(o, inv, rhs, mask, tol, 5000)
        dx = np.linalg.norm(xf.astype(np.float64) - xs) / np.linalg.norm(xs)
        print(f"{nx}x{ny}x{nz} tol {tol:g} {'static' if static else 'newmark'}: standard {its} it, fused {itf} it "
              f"(true |r|/|b| at stop {rel:.3g}), |x_f - x_s| / |x_s| {dx:.2e}")


if __name__ == "__main__":
    main()
