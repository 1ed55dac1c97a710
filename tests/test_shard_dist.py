"""World-size-2 gloo run of the sharded PCG schedule (dist_worker.py) on the CPU: the halo plans
built independently by each process agree, and the distributed solve (owned-row reductions folded
in rank order, z halo per iteration) converges to the single-process oracle solution."""
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import dist_worker
from helpers import oracle_system
from cwf import scenarios


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_pcg_matches_oracle(tmp_path, world):
    shape = (5, 4, 4)
    mp.spawn(dist_worker.run_rank, args=(world, _port(), str(tmp_path), shape), nprocs=world, join=True)
    glob = scenarios.block_case(shape[0], shape[1], shape[2] * world, h=0.1)
    sK, sM = glob.scalars()
    ref = oracle_system(glob.packing, glob.materials, sK, sM).solve_pcg(glob.static_rhs(), 400, 1e-6)
    x_ref = ref["x"].reshape(-1, 3)
    x = np.zeros_like(x_ref)
    its = set()
    for r in range(world):
        d = np.load(tmp_path / f"rank{r}.npz")
        x[d["gid"].astype(np.int64)] = d["x"].reshape(-1, 3)
        its.add(int(d["iterations"]))
        assert float(d["res"]) <= float(d["tol"])
    assert len(its) == 1  # identical control flow on every rank
    assert abs(its.pop() - int(ref["telemetry"].iterations)) <= 3
    err = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
    assert err < 1e-4, err


def test_gloo_sharded_parity_schedule_is_bitwise_the_single_solve(tmp_path):
    """The PARITY gate of SURVEY.md 8e on two processes: chunk partials of 256-node-aligned owned ranges,
    all-gathered and folded in global chunk order, give x, r and the fp64 residual history of the one-process
    oracle solve bit for bit (dist_worker.run_rank_parity restates csrc/comm.cpp sharded_parity_*)."""
    world, shape = 2, (15, 15, 2)
    mp.spawn(dist_worker.run_rank_parity, args=(world, _port(), str(tmp_path), shape), nprocs=world, join=True)
    glob = scenarios.block_case(shape[0], shape[1], shape[2] * world, h=0.1)
    sK, sM = glob.scalars()
    ref = oracle_system(glob.packing, glob.materials, sK, sM).solve_pcg(glob.static_rhs(), 400, 1e-6, history=True)
    x = np.zeros_like(ref["x"]).reshape(-1, 3)
    r = np.zeros_like(x)
    for k in range(world):
        d = np.load(tmp_path / f"parity_rank{k}.npz")
        g = d["gid"].astype(np.int64)
        x[g] = d["x"].reshape(-1, 3)
        r[g] = d["r"].reshape(-1, 3)
        assert int(d["iterations"]) == int(ref["telemetry"].iterations)
        assert np.array_equal(d["hist"], ref["history"])
    assert x.reshape(-1).tobytes() == ref["x"].tobytes()
    assert r.reshape(-1).tobytes() == ref["r"].tobytes()
