#!/usr/bin/env python3
"""PCG iteration counts of one static solve (33x9x5 block, tol 1e-6) per K_eff path, hex8 and Kuhn tets, and the
apply error on the solution vector (a smooth field) against the fp64 oracle operator: a diagnostic for paths whose
counts part from each other (tests/test_gpu_lattice.py test_fused_iteration_matches_two_kernel_loop[hex])."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "civiwave-fem_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402
from cwf import _lib, pcg, scenarios  # noqa: E402
from helpers import oracle_system  # noqa: E402

VARIANTS = {"fused": {"CWF_FUSED": "1"}, "two-kernel": {"CWF_FUSED": "0"},
            "two-kernel-zr": {"CWF_FUSED": "0", "CWF_LAT_ZR": "1"},
            "tiles": {"CWF_LATTICE": "0"}, "tiles256": {"CWF_LATTICE": "0", "CWF_HEX_NT": "256"}}


def main():
    D = O.make_stiffness(30.0e9, 0.2)
    for element in ("hex8",):
        case = scenarios.block_case(33, 9, 5, h=0.1, element=element, tol=1e-6, max_iterations=2000)
        P = case.packing
        sK, sM = case.scalars()
        rhs = case.static_rhs()
        if element == "hex8":
            ref_apply = lambda x: O.hex8_apply(case.mesh.coords, case.mesh.tets, P.material_index, D, sK, sM,
                                               P.lumped_mass, P.bc_mask, x).astype(np.float64)
        else:
            ref_apply = oracle_system(P, case.materials, sK, sM).apply_keff
        A = lambda x: ref_apply(x.astype(np.float32)).astype(np.float64)
        N = P.node_count
        mask = np.repeat(P.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), N)
        if element == "hex8":
            blk = O.hex8_diag_blocks(case.mesh.coords, case.mesh.tets, P.material_index, D, sK)
            B = blk + sM * P.lumped_mass.astype(np.float64)[:, None, None] * np.eye(3)
            for n in range(N):
                for k in range(3):
                    if mask[3 * n + k]:
                        B[n][k, :] = 0
                        B[n][:, k] = 0
                        B[n][k, k] = 1
            Binv = np.linalg.inv(B)
        else:
            Binv = None
        b64 = rhs.astype(np.float64)

        def cpu_pcg(prec):
            x = np.zeros_like(b64)
            r = b64.copy()
            z = prec(r)
            p = z.copy()
            rz = r @ z
            for it in range(1, 3000):
                Ap = A(p)
                a = rz / (p @ Ap)
                x += a * p
                r -= a * Ap
                if np.linalg.norm(r) <= 1e-6 * np.linalg.norm(b64):
                    return it
                z = prec(r)
                rz2 = r @ z
                p = z + rz2 / rz * p
                rz = rz2
            return None

        xref = O.hex8_solve64(case.mesh.coords, case.mesh.tets, P.material_index, D, sK, sM, P.lumped_mass,
                              P.bc_mask, rhs)
        if Binv is not None:
            print(f"{element}: fp64 its with the oracle's block inverse {cpu_pcg(lambda r: np.einsum('nij,nj->ni', Binv, r.reshape(-1, 3)).reshape(-1))}")
        for name, env in VARIANTS.items():
            if element == "tet4" and "256" in name:
                continue
            for k in ("CWF_FUSED", "CWF_LAT_ZR", "CWF_LATTICE", "CWF_HEX_NT"):
                os.environ.pop(k, None)
            os.environ.update(env)
            s = pcg.MatrixFreeSystem.from_packing(P, case.materials, sK, sM, mode=_lib.MODE_FAST)
            kern = (_lib.load().cwf_hip_system_keff_kernel(s.handle()) or b"").decode()
            x = np.zeros_like(rhs)
            t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(2000, 1e-6), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
            y = np.zeros_like(x)
            pcg.apply_keff(s, x, y).value()
            ref = ref_apply(x)
            err = np.linalg.norm(y - ref) / np.linalg.norm(ref)
            rng = np.random.Generator(np.random.PCG64(3))
            a, b = rng.uniform(-1, 1, (2, x.size)).astype(np.float32)
            ya, yb = np.zeros_like(a), np.zeros_like(b)
            pcg.apply_keff(s, a, ya).value()
            pcg.apply_keff(s, b, yb).value()
            asym = abs(float(b.astype(np.float64) @ ya) - float(a.astype(np.float64) @ yb)) / abs(
                float(a.astype(np.float64) @ ya))
            tr = np.linalg.norm(b64 - A(x)) / np.linalg.norm(b64)
            xe = np.linalg.norm(x - xref) / np.linalg.norm(xref)
            print(f"   oracle-operator residual of x {tr:.2e}, |x - x64| / |x64| {xe:.2e}")
            inv = np.zeros(9 * P.node_count, np.float32)
            pcg.fast_block_inverse(s, inv).value()
            inv = inv.reshape(-1, 3, 3).astype(np.float64)
            ierr = np.abs(inv - Binv).max() / np.abs(Binv).max()
            worst = int(np.abs(inv - Binv).reshape(len(inv), -1).max(1).argmax())
            cpu_its = cpu_pcg(lambda r: np.einsum("nij,nj->ni", inv, r.reshape(-1, 3)).reshape(-1))
            print(f"   inverse err {ierr:.2e} (worst node {worst}, mask {P.bc_mask[worst]}) fp64 its with it {cpu_its}")
            print(f"{element:5s} {name:14s} its {t.iterations:5d} conv {t.converged} res {t.residual_norm:.3e} "
                  f"apply-err(x) {err:.2e} asym {asym:.2e}  {kern}", flush=True)


if __name__ == "__main__":
    main()
