#!/usr/bin/env python3
"""GPU diagnostic: the sharded fused iteration against the one-handle fused iteration after 1, 2, 3, ... iterations
(LOCAL communicator, slab sub-meshes). Prints the relative x difference per iteration count."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "civiwave-fem_amd"), os.path.join(ROOT, "tests")]
from cwf import _lib, pcg, scenarios, shard  # noqa: E402


def run(nranks, its, shape=(11, 7, 3), fused="1"):
    os.environ["CWF_FUSED"] = fused
    glob = scenarios.block_case(shape[0], shape[1], shape[2] * nranks, h=0.1, tol=1e-6, max_iterations=800)
    P = glob.packing
    sK, sM = glob.scalars()
    single = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_FAST)
    rhs = glob.static_rhs()
    x1 = np.zeros_like(rhs)
    t1 = pcg.solve_pcg(single, rhs, pcg.PcgSettings(its, 1e-12), pcg.PcgVectors(x1, None))
    comm = shard.Comm.local(nranks)
    systems, shards, rl, xs = [], [], [], []
    for r in range(nranks):
        case, node_global, begin = scenarios.slab_case_shape(shape, nranks, r, tol=1e-6)
        src = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=_lib.MODE_FAST)
        sh = shard.build_shard(src, begin, r, node_global)
        s = sh.system(glob.materials, sK, sM)
        comm.attach(s, sh)
        systems.append(s)
        shards.append(sh)
        rl.append(sh.local_dofs(case.static_rhs()))
        xs.append(np.zeros(3 * sh.local_nodes, np.float32))
    kern = (_lib.load().cwf_hip_system_keff_kernel(systems[0].handle()) or b"").decode()
    tel = shard.solve_pcg_group(systems, rl, pcg.PcgSettings(its, 1e-12), xs)
    xg = np.zeros((P.node_count, 3), np.float32)
    for sh, xl in zip(shards, xs):
        xg[sh.node_global[: sh.owned_nodes].astype(np.int64)] = xl.reshape(-1, 3)[: sh.owned_nodes]
    comm.close()
    d = np.linalg.norm(xg.reshape(-1) - x1) / max(np.linalg.norm(x1), 1e-30)
    ts = tel.value() if tel.has_value() else tel.error()
    print(f"nranks {nranks} fused {fused} its {its}: |x_shard - x_single| / |x_single| = {d:.3e}  {kern}  "
          f"single res {t1.value().residual_norm if t1.has_value() else t1.error()}  shard {ts}", flush=True)


for its in (1, 2, 3, 5, 20):
    run(2, its)
run(2, 20, fused="0")
