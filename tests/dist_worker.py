"""Rank body of the world-size-2 gloo tests (test_shard_dist.py): the sharded PCG schedule of
csrc/comm.cpp restated on the CPU -- every rank builds its slab sub-mesh and shard exactly as bench.py
does, applies the oracle's K_eff to its local system, refreshes ghost rows through the halo plan
(gloo isend/irecv) and all-gathers per-rank scalars that every rank folds in rank order."""
import os

import numpy as np


def _halo(dist, torch, sh, v):
    """ghost rows of the node-interleaved local vector v <- the owners' values (in place)."""
    reqs, bufs = [], []
    for k, q in enumerate(sh.neighbor_ranks):
        idx = sh.send_nodes[int(sh.send_offsets[k]):int(sh.send_offsets[k + 1])].astype(np.int64)
        out = torch.from_numpy(np.ascontiguousarray(v.reshape(-1, 3)[idx].reshape(-1)))
        reqs.append(dist.isend(out, int(q), tag=0))
        n = int(sh.recv_offsets[k + 1] - sh.recv_offsets[k])
        buf = torch.empty(3 * n, dtype=out.dtype)
        reqs.append(dist.irecv(buf, int(q), tag=0))
        bufs.append((k, buf))
    for r in reqs:
        r.wait()
    for k, buf in bufs:
        a = 3 * (sh.owned_nodes + int(sh.recv_offsets[k]))
        v[a:a + buf.numel()] = buf.numpy()


def _allsum(dist, torch, world, vals):
    """all-gather the per-rank fp64 values, fold in rank order (identical on every rank)."""
    t = torch.tensor(np.asarray(vals, np.float64))
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    acc = np.zeros(len(vals), np.float64)
    for o in out:
        acc = acc + o.numpy()
    return acc


def run_rank(rank, world, port, out_dir, shape=(5, 4, 4), rel_tol=1e-6, max_iterations=400):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from cwf import pcg, scenarios, shard
    from helpers import shard_oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case, node_global, begin = scenarios.slab_case_shape(shape, world, rank)
        sK, sM = case.scalars()
        sysm = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=1)
        sh = shard.build_shard(sysm, begin, rank, node_global)
        # (1) the halo plans agree across processes: ghosts receive their owners' global ids
        gid = sh.node_global.astype(np.float64).repeat(3)
        probe = gid.copy()
        probe[3 * sh.owned_nodes:] = -1.0
        _halo(dist, torch, sh, probe)
        assert np.array_equal(probe, gid), "halo plan mismatch"
        # (2) distributed PCG (fp32 vectors, fp64 scalars, owned-row reductions, rank-order folds)
        loc = shard_oracle(sh, case, sK, sM)
        no = sh.owned_nodes
        Do = 3 * no
        mask = (np.repeat(sh.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), sh.local_nodes)) != 0
        rhs = sh.local_dofs(case.static_rhs())
        inv = loc.block_jacobi().reshape(-1, 3, 3)

        def precond(r):
            z = np.einsum("nij,nj->ni", inv.astype(np.float64), r.reshape(-1, 3).astype(np.float64))
            z = z.reshape(-1).astype(np.float32)
            z[mask] = 0.0
            return z

        x = np.zeros(3 * sh.local_nodes, np.float32)
        r = (rhs - loc.apply_keff(x)).astype(np.float32)
        r[mask] = 0.0
        rhs_sq, rr = _allsum(dist, torch, world, [np.dot(rhs[:Do].astype(np.float64), rhs[:Do]),
                                                   np.dot(r[:Do].astype(np.float64), r[:Do])])
        rn = np.sqrt(rhs_sq)
        tol = rel_tol * (rn if rn >= 1e-12 else 1.0)  # pcg.cpp:779-790
        z = precond(r)
        _halo(dist, torch, sh, z)
        p = z.copy()
        (rho,) = _allsum(dist, torch, world, [np.dot(r[:Do].astype(np.float64), z[:Do])])
        it = 0
        res = np.sqrt(rr)
        while it < max_iterations and res > tol:
            Ap = loc.apply_keff(p)
            (pap,) = _allsum(dist, torch, world, [np.dot(p[:Do].astype(np.float64), Ap[:Do])])
            alpha = rho / pap
            x[:Do] = (x[:Do] + alpha * p[:Do].astype(np.float64)).astype(np.float32)
            r[:Do] = (r[:Do] - alpha * Ap[:Do].astype(np.float64)).astype(np.float32)
            r[mask] = 0.0
            it += 1
            z = precond(r)
            _halo(dist, torch, sh, z)
            rr, rz = _allsum(dist, torch, world, [np.dot(r[:Do].astype(np.float64), r[:Do]),
                                                  np.dot(r[:Do].astype(np.float64), z[:Do])])
            res = np.sqrt(rr)
            beta = rz / rho
            rho = rz
            p = (z + beta * p.astype(np.float64)).astype(np.float32)  # ghost rows from the exchanged z
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), x=x[:Do], gid=sh.node_global[:no], iterations=it,
                 res=res, tol=tol)
    finally:
        dist.destroy_process_group()
