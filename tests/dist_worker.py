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


def _gather_fold(dist, torch, world, parts):
    """all-gather every rank's chunk partials (zero-padded to a common stride), fold them rank after rank,
    chunk after chunk, sequentially from +0.0 (pcg.cpp:170-207 over the global chunk order)."""
    stride = torch.tensor([len(parts)], dtype=torch.int64)
    counts = [torch.empty_like(stride) for _ in range(world)]
    dist.all_gather(counts, stride)
    S = int(max(int(c) for c in counts))
    t = torch.zeros(S, dtype=torch.float64)
    t[: len(parts)] = torch.from_numpy(np.asarray(parts, np.float64))
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    acc = 0.0
    for o in out:
        for v in o.tolist():
            acc += v
    return acc


def run_rank_parity(rank, world, port, out_dir, shape=(15, 15, 2), rel_tol=1e-6, max_iterations=400):
    """The sharded PARITY schedule of csrc/comm.cpp (sharded_parity_*) restated in numpy on the oracle: owned
    ranges aligned to 256 nodes (a 15 x 15 cross-section is 256 nodes per plane), owned K_eff / block-Jacobi
    rows from the rank's local oracle system, 256-DOF chunk partials of the owned rows all-gathered and folded
    in global chunk order, p refreshed on the ghosts after every p update. Every scalar rounds as pcg.cpp does,
    so x and the residual history must equal the single-process oracle solve bit for bit."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from cwf import pcg, scenarios, shard
    from helpers import shard_oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case, node_global, begin = scenarios.slab_case_shape(shape, world, rank)
        assert all(int(b) % 256 == 0 for b in begin[:-1])
        sK, sM = case.scalars()
        sysm = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=0)
        sh = shard.build_shard(sysm, begin, rank, node_global)
        loc = shard_oracle(sh, case, sK, sM)
        Do = 3 * sh.owned_nodes
        nchunks = (Do + 255) // 256
        mask = (np.repeat(sh.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), sh.local_nodes)) != 0
        rhs = sh.local_dofs(case.static_rhs())
        inv = loc.block_jacobi().reshape(-1, 3, 3).astype(np.float64)

        def dot(a, b):
            a = a.copy()
            a[Do:] = 0.0
            _, parts = loc.dot(a, b)
            return _gather_fold(dist, torch, world, parts[:nchunks])

        def precond(r):
            r64 = r.reshape(-1, 3).astype(np.float64)
            z = np.zeros_like(r64)
            for k in range(3):
                s = 0.0 + inv[:, k, 0] * r64[:, 0]
                s = s + inv[:, k, 1] * r64[:, 1]
                s = s + inv[:, k, 2] * r64[:, 2]
                z[:, k] = s
            z = z.reshape(-1).astype(np.float32)
            z[mask] = 0.0
            return z

        def enforce(x, r):
            x[mask] = rhs[mask]
            r[mask] = 0.0

        x = np.zeros(3 * sh.local_nodes, np.float32)
        r = (rhs - loc.apply_keff(x)).astype(np.float32)
        enforce(x, r)
        rhs_sq = dot(rhs, rhs)
        rhs_norm = np.sqrt(rhs_sq)
        rhs_norm = 1.0 if rhs_norm < 1e-12 else rhs_norm
        res = float(np.sqrt(dot(r, r)))
        hist = [res]
        tol = rel_tol * rhs_norm
        z = precond(r)
        rho = dot(r, z)
        p = z.copy()
        p[mask] = 0.0
        _halo(dist, torch, sh, p)
        it = 0
        while it < max_iterations and res > tol:
            Ap = loc.apply_keff(p)
            alpha = rho / dot(p, Ap)
            x = (x + (alpha * p.astype(np.float64)).astype(np.float32)).astype(np.float32)
            r = (r - (alpha * Ap.astype(np.float64)).astype(np.float32)).astype(np.float32)
            enforce(x, r)
            res = float(np.sqrt(dot(r, r)))
            hist.append(res)
            it += 1
            if res <= tol:
                break
            z = precond(r)
            rho_new = dot(r, z)
            beta = rho_new / rho
            rho = rho_new
            p = (z.astype(np.float64) + beta * p.astype(np.float64)).astype(np.float32)
            p[mask] = 0.0
            _halo(dist, torch, sh, p)  # ghost p <- owners (ghost z rows are not meaningful)
        np.savez(os.path.join(out_dir, f"parity_rank{rank}.npz"), x=x[:Do], r=r[:Do], gid=sh.node_global[: sh.owned_nodes],
                 iterations=it, hist=np.asarray(hist, np.float64))
    finally:
        dist.destroy_process_group()
