"""Node-range shards (cwf_shard_build) on the CPU: partition invariants, halo
plan symmetry, sub-mesh input, and that the oracle's parity K_eff on every shard reproduces the
global K_eff on the owned rows bit for bit (the complete-rows property the sharded solver relies on)."""
import numpy as np
import pytest

import oracle as O
from cwf import pcg, scenarios, shard
from cwf import _lib

from helpers import assert_bitwise, shard_oracle as _local_oracle


def _global_case():
    return scenarios.block_case(5, 4, 7, h=0.1)


def _system(case, mode=_lib.MODE_FAST):
    sK, sM = case.scalars()
    return pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=mode)


@pytest.mark.parametrize("nranks", [2, 3, 5])
def test_partition_invariants(nranks):
    case = _global_case()
    P = case.packing
    sysm = _system(case)
    begin = shard.slab_ranges(P.node_count, nranks)
    shards = [shard.build_shard(sysm, begin, r) for r in range(nranks)]
    conn = P.connectivity.reshape(-1, 8)[:, :4].astype(np.int64)
    owned_all = np.concatenate([s.node_global[: s.owned_nodes] for s in shards])
    assert np.array_equal(np.sort(owned_all), np.arange(P.node_count))
    for s in shards:
        lo, hi = int(begin[s.rank]), int(begin[s.rank + 1])
        own = s.node_global[: s.owned_nodes].astype(np.int64)
        assert np.array_equal(own, np.arange(lo, hi))  # owned first, ascending global id
        touches = np.any((conn >= lo) & (conn < hi), axis=1)
        assert np.array_equal(s.element_source, np.nonzero(touches)[0])  # ascending global element order
        ghosts = s.node_global[s.owned_nodes:].astype(np.int64)
        want = np.setdiff1d(np.unique(conn[touches]), own)
        assert np.array_equal(np.sort(ghosts), want)
        owners = np.searchsorted(begin.astype(np.int64), ghosts, side="right") - 1
        assert np.all(np.diff(owners) >= 0)  # grouped by owner rank
        for k, q in enumerate(s.neighbor_ranks):
            a, b = int(s.recv_offsets[k]), int(s.recv_offsets[k + 1])
            assert np.all(owners[a:b] == q)
        # local connectivity maps back to the global one
        lc = s.connectivity.reshape(-1, 8)
        assert np.all(lc[:, 4:] == 0xFFFFFFFF)
        assert np.array_equal(s.node_global[lc[:, :4].astype(np.int64)].astype(np.int64), conn[touches])
    # halo symmetry: r's send list to q == q's ghosts from r (same order)
    for s in shards:
        for k, q in enumerate(s.neighbor_ranks):
            t = shards[q]
            j = list(t.neighbor_ranks).index(s.rank)
            sent = s.node_global[s.send_nodes[int(s.send_offsets[k]):int(s.send_offsets[k + 1])].astype(np.int64)]
            recv = t.node_global[t.owned_nodes + int(t.recv_offsets[j]): t.owned_nodes + int(t.recv_offsets[j + 1])]
            assert np.array_equal(sent, recv)


def test_submesh_input_matches_global():
    """The bench feeds every rank its own slab sub-mesh (scenarios.slab_case); the shard must equal the
    one cut from the global mesh."""
    nranks = 3
    glob = scenarios.block_case(4, 3, 3 * nranks, h=0.1)
    gsys = _system(glob)
    for r in range(nranks):
        sub, node_global, begin = scenarios.slab_case_shape((4, 3, 3), nranks, r)
        a = shard.build_shard(gsys, begin, r)
        b = shard.build_shard(_system(sub), begin, r, node_global)
        assert a.owned_nodes == b.owned_nodes and a.local_nodes == b.local_nodes
        assert np.array_equal(a.node_global, b.node_global)
        assert np.array_equal(a.connectivity, b.connectivity)
        assert np.array_equal(a.neighbor_ranks, b.neighbor_ranks)
        assert np.array_equal(a.send_nodes, b.send_nodes)
        assert_bitwise(a.gradients, b.gradients, "gradients")
        assert_bitwise(a.volume, b.volume, "volume")
        assert_bitwise(a.lumped_mass[: a.owned_nodes], b.lumped_mass[: b.owned_nodes], "owned masses")
        assert np.array_equal(a.bc_mask, b.bc_mask)


@pytest.mark.parametrize("nranks", [2, 4])
def test_shard_rows_bitwise(nranks):
    case = _global_case()
    P = case.packing
    sK, sM = case.scalars()
    sysm = _system(case)
    ref = O.System(O.Packed(P.node_count, P.element_count, P.connectivity, P.gradients, P.volume, P.material_index,
                            P.lumped_mass64, P.lumped_mass, P.offsets, P.element_indices, P.local_indices),
                   np.concatenate([np.asarray(m.stiffness, np.float64).reshape(-1) for m in case.materials]),
                   P.bc_mask, sK, sM, 256)
    x = ((np.arange(P.dof_count, dtype=np.uint64) * 2654435761) % 1000).astype(np.float32) / np.float32(1000.0)
    y = ref.apply_keff(x)
    begin = shard.slab_ranges(P.node_count, nranks)
    for r in range(nranks):
        s = shard.build_shard(sysm, begin, r)
        loc = _local_oracle(s, case, sK, sM)
        yl = loc.apply_keff(s.local_dofs(x))
        own = s.node_global[: s.owned_nodes].astype(np.int64)
        assert_bitwise(yl[: 3 * s.owned_nodes], y.reshape(-1, 3)[own].reshape(-1), f"rank {r} owned rows")


def test_shard_errors():
    case = _global_case()
    sysm = _system(case)
    with pytest.raises(RuntimeError, match="outside every rank"):
        shard.build_shard(sysm, np.array([0, 10], np.uint64), 0)
    with pytest.raises(RuntimeError, match="rank out of range"):
        shard.build_shard(sysm, shard.slab_ranges(case.packing.node_count, 2), 2)


@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_strong_slab_submeshes_match_global(nranks):
    """bench.py --scaling strong: the config's block itself split into `nranks` slabs; every rank's slab
    sub-mesh gives the shard cut from the global mesh, and the owned ranges cover it once."""
    shape = (4, 3, 7)
    glob = scenarios.block_case(*shape, h=0.1)
    gsys = _system(glob)
    owned = []
    for r in range(nranks):
        sub, node_global, begin = scenarios.slab_case_shape(shape, nranks, r, stack=False)
        assert int(begin[-1]) == glob.packing.node_count
        a = shard.build_shard(gsys, begin, r)
        b = shard.build_shard(_system(sub), begin, r, node_global)
        assert np.array_equal(a.node_global, b.node_global) and np.array_equal(a.connectivity, b.connectivity)
        assert np.array_equal(a.send_nodes, b.send_nodes)
        owned.append(a.node_global[: a.owned_nodes])
    assert np.array_equal(np.sort(np.concatenate(owned)), np.arange(glob.packing.node_count))


@pytest.mark.parametrize("nranks", [3, 8])
def test_rcb_partition_of_permuted_mesh(nranks):
    """C4's decomposition (scenarios.rcb_case): an RCB node partition of the jittered + permuted mesh,
    renumbered part after part. Parts are balanced, every node is owned once, the halo plans are symmetric,
    owned K_eff rows are bitwise the global rows, and halos stay small (a contiguous range of the random
    numbering would make nearly every node a ghost)."""
    case = scenarios.block_case(12, 10, 9, h=0.1, jitter=True)
    P = case.packing
    sK, sM = case.scalars()
    gid, begin = shard.rcb_node_ranges(case.mesh.coords, nranks)
    assert np.array_equal(np.sort(gid), np.arange(P.node_count, dtype=np.uint64))
    sizes = np.diff(begin.astype(np.int64))
    assert sizes.max() - sizes.min() <= 1
    sysm = _system(case)
    shards = [shard.build_shard(sysm, begin, r, gid) for r in range(nranks)]
    ref = O.System(O.Packed(P.node_count, P.element_count, P.connectivity, P.gradients, P.volume, P.material_index,
                            P.lumped_mass64, P.lumped_mass, P.offsets, P.element_indices, P.local_indices),
                   np.concatenate([np.asarray(m.stiffness, np.float64).reshape(-1) for m in case.materials]),
                   P.bc_mask, sK, sM, 256)
    x = ((np.arange(P.dof_count, dtype=np.uint64) * 2654435761) % 1000).astype(np.float32) / np.float32(1000.0)
    y = ref.apply_keff(x).reshape(-1, 3)
    ghosts = 0
    for s in shards:
        src = s.node_source[: s.owned_nodes].astype(np.int64)
        assert np.array_equal(gid[src], np.arange(int(begin[s.rank]), int(begin[s.rank + 1]), dtype=np.uint64))
        yl = _local_oracle(s, case, sK, sM).apply_keff(s.local_dofs(x))
        assert_bitwise(yl[: 3 * s.owned_nodes], y[src].reshape(-1), f"rank {s.rank} owned rows")
        ghosts += s.local_nodes - s.owned_nodes
        for k, q in enumerate(s.neighbor_ranks):
            t = shards[q]
            j = list(t.neighbor_ranks).index(s.rank)
            sent = s.node_global[s.send_nodes[int(s.send_offsets[k]):int(s.send_offsets[k + 1])].astype(np.int64)]
            recv = t.node_global[t.owned_nodes + int(t.recv_offsets[j]): t.owned_nodes + int(t.recv_offsets[j + 1])]
            assert np.array_equal(sent, recv)
    assert ghosts < 0.8 * P.node_count


@pytest.mark.parametrize("nranks", [2, 3])
def test_hex8_shards_rows_and_submeshes(nranks):
    """Native hex8 shards: 8-corner elements touching the owned nodes, owned rows of the fp64
    hex8 operator (oracle/hex8_oracle.c, ascending element scatter) bitwise the global rows, and every rank's
    hex slab sub-mesh gives the shard cut from the global mesh."""
    shape = (4, 3, 2 * nranks)
    glob = scenarios.block_case(*shape, h=0.1, element="hex8")
    P = glob.packing
    sK, sM = glob.scalars()
    D = np.concatenate([np.asarray(m.stiffness, np.float64).reshape(-1) for m in glob.materials])
    x = ((np.arange(P.dof_count, dtype=np.uint64) * 2654435761) % 1000).astype(np.float32) / np.float32(1000.0)
    y = O.hex8_apply(glob.mesh.coords, glob.mesh.tets, P.material_index, D, sK, sM, P.lumped_mass, P.bc_mask,
                     x).reshape(-1, 3)
    gsys = _system(glob)
    for r in range(nranks):
        sub, node_global, begin = scenarios.slab_case_shape(shape, nranks, r, stack=False, element="hex8")
        a = shard.build_shard(gsys, begin, r)
        b = shard.build_shard(_system(sub), begin, r, node_global)
        assert np.array_equal(a.node_global, b.node_global) and np.array_equal(a.connectivity, b.connectivity)
        assert np.array_equal(a.send_nodes, b.send_nodes)
        lc = a.connectivity.reshape(-1, 8)
        assert np.all(lc != 0xFFFFFFFF)
        yl = O.hex8_apply(a.node_coords.reshape(-1, 3), lc, a.material_index, D, sK, sM, a.lumped_mass, a.bc_mask,
                          a.local_dofs(x))
        own = a.node_global[: a.owned_nodes].astype(np.int64)
        assert_bitwise(yl[: 3 * a.owned_nodes], y[own].reshape(-1), f"hex rank {r} owned rows")
