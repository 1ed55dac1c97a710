"""Synthetic tet meshes for the benchmark configurations.

Structured hex blocks with lexicographic node numbering (i fastest) where every hex is
split into 6 conforming Kuhn tetrahedra (local cube corners {0,1,3,7},{0,1,5,7},
{0,2,3,7},{0,2,6,7},{0,4,5,7},{0,4,6,7}, corner bit pattern (i,j,k)). The reference
solver accepts tet4 only (src/mesh/preprocess.cpp:326-330), so a "hex8 block" config
is carried by this expansion. Coordinates are computed as ``h * i`` in float64, the
same expression the survey's reference drivers used.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

KUHN = np.array([[0, 1, 3, 7], [0, 1, 5, 7], [0, 2, 3, 7], [0, 2, 6, 7], [0, 4, 5, 7], [0, 4, 6, 7]], np.int64)


@dataclass
class TetMesh:
    coords: np.ndarray  # f64 [N,3]
    tets: np.ndarray  # u32 [E,4]
    node_groups: dict = field(default_factory=dict)  # name -> u32 node indices
    shape: tuple | None = None  # (nx, ny, nz) hexes for structured blocks

    @property
    def node_count(self) -> int:
        return self.coords.shape[0]

    @property
    def element_count(self) -> int:
        return self.tets.shape[0]


def kuhn_block(nx: int, ny: int, nz: int, h: float = 1.0) -> TetMesh:
    """nx*ny*nz hexes -> 6*nx*ny*nz tets; groups FIXED (x=0 face) and TIP (x=max face)."""
    A, B, Cn = nx + 1, ny + 1, nz + 1
    k, j, i = np.meshgrid(np.arange(Cn), np.arange(B), np.arange(A), indexing="ij")
    if h == 1.0:
        coords = np.stack([i, j, k], -1).reshape(-1, 3).astype(np.float64)
    else:
        coords = np.stack([h * i.astype(np.float64), h * j.astype(np.float64), h * k.astype(np.float64)],
                          -1).reshape(-1, 3)
    hk, hj, hi = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    hk, hj, hi = hk.reshape(-1), hj.reshape(-1), hi.reshape(-1)
    corners = np.empty((hk.size, 8), np.int64)
    for b in range(8):
        corners[:, b] = ((hk + ((b >> 2) & 1)) * B + (hj + ((b >> 1) & 1))) * A + (hi + (b & 1))
    tets = corners[:, KUHN].reshape(-1, 4).astype(np.uint32)
    kk, jj = np.meshgrid(np.arange(Cn), np.arange(B), indexing="ij")
    fixed = ((kk * B + jj) * A).reshape(-1).astype(np.uint32)
    tip = ((kk * B + jj) * A + nx).reshape(-1).astype(np.uint32)
    return TetMesh(coords, tets, {"FIXED": fixed, "TIP": tip,
                                  "CORNER": np.array([(nz * B + ny) * A + nx], np.uint32)}, (nx, ny, nz))


# hex corner bit pattern (i, j, k) -> Gmsh/VTK hexahedron order 0(-,-,-) 1(+,-,-) 2(+,+,-) 3(-,+,-) 4..7 (z+)
HEX_GMSH = np.array([0, 1, 3, 2, 4, 5, 7, 6], np.int64)


def hex_block(nx: int, ny: int, nz: int, h: float = 1.0) -> TetMesh:
    """The same structured block as native hex8 elements: nx*ny*nz hexes, [E, 8]
    connectivity in Gmsh/VTK corner order, the node numbering and groups of kuhn_block."""
    A, B, Cn = nx + 1, ny + 1, nz + 1
    k, j, i = np.meshgrid(np.arange(Cn), np.arange(B), np.arange(A), indexing="ij")
    if h == 1.0:
        coords = np.stack([i, j, k], -1).reshape(-1, 3).astype(np.float64)
    else:
        coords = np.stack([h * i.astype(np.float64), h * j.astype(np.float64), h * k.astype(np.float64)],
                          -1).reshape(-1, 3)
    hk, hj, hi = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    hk, hj, hi = hk.reshape(-1), hj.reshape(-1), hi.reshape(-1)
    corners = np.empty((hk.size, 8), np.int64)
    for b in range(8):
        corners[:, b] = ((hk + ((b >> 2) & 1)) * B + (hj + ((b >> 1) & 1))) * A + (hi + (b & 1))
    hexes = corners[:, HEX_GMSH].astype(np.uint32)
    kk, jj = np.meshgrid(np.arange(Cn), np.arange(B), indexing="ij")
    fixed = ((kk * B + jj) * A).reshape(-1).astype(np.uint32)
    tip = ((kk * B + jj) * A + nx).reshape(-1).astype(np.uint32)
    return TetMesh(coords, hexes, {"FIXED": fixed, "TIP": tip,
                                   "CORNER": np.array([(nz * B + ny) * A + nx], np.uint32)}, (nx, ny, nz))


def kuhn_slab(nx: int, ny: int, nz: int, kc0: int, kc1: int, h: float = 1.0, element: str = "tet4"):
    """Cells k in [kc0, kc1) of the nx*ny*nz Kuhn block (element="hex8": the native hex block), nodes on
    planes kc0..kc1, numbered compactly but in the global order -> (TetMesh, global node id per sub-mesh
    node). Elements keep the global (k-slowest) order, so a rank's sub-mesh feeds cwf_shard_build directly."""
    A, B = nx + 1, ny + 1
    sub = (hex_block if element == "hex8" else kuhn_block)(nx, ny, kc1 - kc0, h)
    kk = np.arange(kc0, kc1 + 1, dtype=np.float64).repeat(A * B)
    sub.coords[:, 2] = kk if h == 1.0 else h * kk  # the same expression kuhn_block uses
    node_global = np.arange(sub.node_count, dtype=np.uint64) + np.uint64(kc0 * A * B)
    groups = {k: v for k, v in sub.node_groups.items() if k != "CORNER"}
    if kc1 == nz:
        groups["CORNER"] = np.array([((kc1 - kc0) * B + ny) * A + nx], np.uint32)
    return TetMesh(sub.coords, sub.tets, groups, (nx, ny, kc1 - kc0)), node_global


def jitter_and_permute(mesh: TetMesh, h: float, jitter: float = 0.15, seed_jitter: int = 12345,
                       seed_perm: int = 42) -> TetMesh:
    """C4: jitter interior nodes by +-jitter*h and randomly permute node/element order.

    Boundary nodes (on the block faces) are kept on their face so the group definitions
    stay meaningful. A deterministic numpy PCG64 stream is used.
    """
    rng = np.random.Generator(np.random.PCG64(seed_jitter))
    c = mesh.coords.copy()
    lo, hi = c.min(0), c.max(0)
    interior = np.all((c > lo + 1e-9) & (c < hi - 1e-9), axis=1)
    c[interior] += rng.uniform(-jitter * h, jitter * h, size=(int(interior.sum()), 3))
    prng = np.random.Generator(np.random.PCG64(seed_perm))
    node_perm = prng.permutation(mesh.node_count)  # new index -> old index
    old_to_new = np.empty_like(node_perm)
    old_to_new[node_perm] = np.arange(node_perm.size)
    elem_perm = prng.permutation(mesh.element_count)
    tets = old_to_new[mesh.tets.astype(np.int64)][elem_perm].astype(np.uint32)
    groups = {k: np.sort(old_to_new[v.astype(np.int64)]).astype(np.uint32) for k, v in mesh.node_groups.items()}
    return TetMesh(c[node_perm], tets, groups, None)


def morton_renumber(mesh: TetMesh) -> TetMesh:
    """Nodes renumbered along a Morton curve of their coordinates (elements keep their order); groups
    remapped. A diagnostic for how much node-order locality is worth to the FAST kernels."""
    c = mesh.coords
    lo, hi = c.min(0), c.max(0)
    q = np.floor((c - lo) / max(float((hi - lo).max()), 1e-300) * ((1 << 20) - 1)).astype(np.uint64)

    def spread(v):
        v = v & np.uint64(0x1FFFFF)
        v = (v | v << np.uint64(32)) & np.uint64(0x1F00000000FFFF)
        v = (v | v << np.uint64(16)) & np.uint64(0x1F0000FF0000FF)
        v = (v | v << np.uint64(8)) & np.uint64(0x100F00F00F00F00F)
        v = (v | v << np.uint64(4)) & np.uint64(0x10C30C30C30C30C3)
        v = (v | v << np.uint64(2)) & np.uint64(0x1249249249249249)
        return v

    key = spread(q[:, 0]) | spread(q[:, 1]) << np.uint64(1) | spread(q[:, 2]) << np.uint64(2)
    order = np.argsort(key, kind="stable")  # new -> old
    old_to_new = np.empty_like(order)
    old_to_new[order] = np.arange(order.size)
    tets = old_to_new[mesh.tets.astype(np.int64)].astype(np.uint32)
    groups = {k: np.sort(old_to_new[v.astype(np.int64)]).astype(np.uint32) for k, v in mesh.node_groups.items()}
    return TetMesh(c[order], tets, groups, None)


def single_tet() -> TetMesh:
    """The reference test fixture (tests/pcg_test.cpp:35-74): unit tet, base face fixed."""
    coords = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float64)
    tets = np.array([[0, 1, 2, 3]], np.uint32)
    return TetMesh(coords, tets, {"FIXED": np.array([0, 1, 2], np.uint32), "POINT": np.array([3], np.uint32)})


# BASELINE.json configs
CONFIGS = {
    "c1": dict(name="cantilever 20x5x10 hex (Kuhn tets)", shape=(20, 5, 10), h=0.1, xi=0.02, w=(5.0, 50.0),
               tol=2e-4),
    "c2": dict(name="cube 69^3 hex (Kuhn tets), 1.03M DOF", shape=(69, 69, 69), h=0.1, xi=0.02, w=(5.0, 50.0),
               tol=3e-4),
    "c3": dict(name="cube 149^3 hex (Kuhn tets), 10.1M DOF, Rayleigh", shape=(149, 149, 149), h=0.1, xi=0.05,
               w=(10.0, 100.0), tol=3e-4),
    "c4": dict(name="jittered/permuted 118^3 hex (Kuhn tets), 5.06M DOF, harmonic tip load", shape=(118, 118, 118),
               h=0.1, xi=0.02, w=(5.0, 50.0), tol=3e-4, jitter=True, harmonic=5.0),
    "c5": dict(name="slab 800x400x50 hex (Kuhn tets), 49.1M DOF", shape=(800, 400, 50), h=0.1, xi=0.02,
               w=(5.0, 50.0), tol=3e-4),
}


# hex8 faces (Gmsh corner order), each counter-clockwise seen from outside
HEX_FACES = [[0, 3, 2, 1], [4, 5, 6, 7], [0, 1, 5, 4], [1, 2, 6, 5], [2, 3, 7, 6], [3, 0, 4, 7]]


def boundary_faces(tets: np.ndarray, nodes) -> np.ndarray:
    """Boundary faces (faces of exactly one element) whose nodes all lie in `nodes`: triangles u32 [F,3]
    of a tet4 mesh, quads u32 [F,4] of a hex8 mesh."""
    t = np.asarray(tets, np.int64)
    if t.shape[1] == 8:
        faces = np.concatenate([t[:, f] for f in HEX_FACES])
    else:
        faces = np.concatenate([t[:, [0, 1, 2]], t[:, [0, 1, 3]], t[:, [0, 2, 3]], t[:, [1, 2, 3]]])
    key = np.sort(faces, 1)
    _, inv, cnt = np.unique(key, axis=0, return_inverse=True, return_counts=True)
    inv = inv.reshape(-1)
    member = np.zeros(int(t.max()) + 1, bool)
    member[np.asarray(nodes, np.int64)] = True
    keep = (cnt[inv] == 1) & member[faces].all(1)
    return faces[keep].astype(np.uint32)


def write_gmsh(tm: TetMesh, path: str, solid: str = "SOLID", surface_groups=("FIXED", "TIP"),
               node_groups=None) -> None:
    """Gmsh MSH 4.1 ASCII of a TetMesh that cwf.mesh.load_gmsh_file reads back in the same node and
    element order: physical volume `solid` (id 1) holds the tets; every name in `surface_groups` becomes
    a physical surface of its boundary triangles; every name in `node_groups` (default: all of
    tm.node_groups) tags its nodes through $Entities (Mesh::node_groups). Node blocks follow the node
    order (one block per run of nodes of the same entity), so node i of the mesh is node i of the file."""
    names = list(tm.node_groups) if node_groups is None else list(node_groups)
    phys = {solid: (3, 1)}
    for i, n in enumerate(names):
        phys[n] = (2, i + 2)
    N = tm.node_count
    owner = np.zeros(N, np.int64)  # entity per node: 0 = volume entity, k = surface entity of names[k-1]
    for k, n in enumerate(names, start=1):
        sel = np.asarray(tm.node_groups[n], np.int64)
        free = sel[owner[sel] == 0]
        owner[free] = k
    lines = ["$MeshFormat", "4.1 0 8", "$EndMeshFormat", "$PhysicalNames", str(len(phys))]
    lines += [f'{d} {i} "{n}"' for n, (d, i) in phys.items()]
    lines += ["$EndPhysicalNames", "$Entities", f"0 0 {len(names)} 1"]
    lines += [f"{k} 0 0 0 1 1 1 1 {phys[n][1]} 0" for k, n in enumerate(names, start=1)]
    lines += [f"1 0 0 0 1 1 1 1 {phys[solid][1]} 0", "$EndEntities"]
    # node blocks: runs of equal owner
    runs = []
    start = 0
    for i in range(1, N + 1):
        if i == N or owner[i] != owner[start]:
            runs.append((start, i))
            start = i
    lines += ["$Nodes", f"{len(runs)} {N} 1 {N}"]
    for a, b in runs:
        dim, tag = (3, 1) if owner[a] == 0 else (2, int(owner[a]))
        lines.append(f"{dim} {tag} 0 {b - a}")
        lines += [str(i + 1) for i in range(a, b)]
        lines += [f"{x!r} {y!r} {z!r}" for x, y, z in tm.coords[a:b].tolist()]
    lines.append("$EndNodes")
    surf = [(k, boundary_faces(tm.tets, tm.node_groups[n])) for k, n in enumerate(names, start=1)
            if n in surface_groups]
    surf = [(k, f) for k, f in surf if len(f)]
    E = tm.element_count
    total = E + sum(len(f) for _, f in surf)
    lines += ["$Elements", f"{1 + len(surf)} {total} 1 {total}"]
    tag = 1
    hexes = tm.tets.shape[1] == 8  # Gmsh type 5 volumes with type 3 (quad) faces, else type 4 / type 2
    for k, f in surf:
        lines.append(f"2 {k} {3 if hexes else 2} {len(f)}")
        for face in f.tolist():
            lines.append(f"{tag} " + " ".join(str(v + 1) for v in face))
            tag += 1
    lines.append(f"3 1 {5 if hexes else 4} {E}")
    for t in tm.tets.tolist():
        lines.append(f"{tag} " + " ".join(str(v + 1) for v in t))
        tag += 1
    lines.append("$EndElements")
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
