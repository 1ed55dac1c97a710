"""``cwf::mesh::load_gmsh_file`` / ``load_gmsh_from_string`` mirror (include/cwf/mesh/mesh.hpp:148-160)
over the native MSH 4.1 loader (csrc/gmsh.cpp).

``GmshMesh`` keeps the reference Mesh fields (nodes, elements with geometry and physical group,
surfaces, physical groups, node groups); ``to_tet_mesh()`` hands the volume part to the packer and
rejects non-tet elements with preprocess.cpp:326-330's error, as ``mesh::pre::run`` does.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib, pack
from .pcg import Expected


@dataclass
class MeshError:
    message: str
    context: list = field(default_factory=list)


@dataclass
class PhysicalGroup:
    dimension: int
    id: int
    name: str


@dataclass
class GmshMesh:
    coords: np.ndarray  # f64 [N,3]
    node_ids: np.ndarray  # u32 [N] original (Gmsh) ids
    elements: np.ndarray  # u32 [E,8], UINT32_MAX padded
    geometry: np.ndarray  # u8 [E] 4 = tet4, 8 = hex8
    element_group: np.ndarray  # u32 [E]
    element_ids: np.ndarray  # u32 [E]
    surfaces: np.ndarray  # u32 [S,4]
    surface_geometry: np.ndarray  # u8 [S] 3 / 4
    surface_group: np.ndarray  # u32 [S]
    physical_groups: list  # [PhysicalGroup], ascending id
    node_groups: dict  # physical id -> u32 node indices

    @property
    def group_lookup(self) -> dict:
        return {g.id: i for i, g in enumerate(self.physical_groups)}

    @property
    def surface_groups(self) -> dict:
        out: dict = {}
        for i, g in enumerate(self.surface_group.tolist()):
            out.setdefault(g, []).append(i)
        return out

    def to_tet_mesh(self, allow_hex8: bool = False) -> pack.Mesh:
        """The reference's preprocess input (tet4 only, preprocess.cpp:326-330). allow_hex8: an all-hex8
        mesh is passed on as native hex8 elements (FAST mode only)."""
        if len(self.coords) == 0:
            raise pack.PackError("mesh has zero nodes", ["mesh"])
        if len(self.geometry) == 0:
            raise pack.PackError("mesh has zero elements", ["mesh"])
        K = 8 if allow_hex8 and np.all(self.geometry == 8) else 4
        bad = np.nonzero(self.geometry != K)[0]
        if bad.size:
            raise pack.PackError("only tetrahedron elements supported in Phase 3", ["elements", f"[{int(bad[0])}]"])
        names = {}
        for g in self.physical_groups:
            names.setdefault(g.name, g.id)
        surf = [(int(g), tuple(int(n) for n in s[: int(k)]))
                for g, s, k in zip(self.surface_group, self.surfaces, self.surface_geometry)]
        return pack.Mesh(np.ascontiguousarray(self.coords), np.ascontiguousarray(self.elements[:, :K]),
                         np.ascontiguousarray(self.element_group), names, dict(self.node_groups), surf)


def _finish(rc: int, h: C.c_void_p) -> Expected:
    L = _lib.load()
    if rc:
        msg, ctx = _lib.last_error(None)
        return Expected(error=MeshError(msg, ctx))
    try:
        info = _lib.MeshInfoC()
        L.cwf_mesh_get_info(h, C.byref(info))
        N, E, S, G = info.node_count, info.element_count, info.surface_count, info.group_count
        coords = np.zeros((N, 3), np.float64)
        nid = np.zeros(N, np.uint32)
        L.cwf_mesh_nodes(h, _lib.ptr(coords), _lib.ptr(nid))
        el = np.zeros((E, 8), np.uint32)
        geo = np.zeros(E, np.uint8)
        grp = np.zeros(E, np.uint32)
        eid = np.zeros(E, np.uint32)
        L.cwf_mesh_elements(h, _lib.ptr(el), _lib.ptr(geo), _lib.ptr(grp), _lib.ptr(eid))
        sn = np.zeros((S, 4), np.uint32)
        sg = np.zeros(S, np.uint8)
        sgr = np.zeros(S, np.uint32)
        L.cwf_mesh_surfaces(h, _lib.ptr(sn), _lib.ptr(sg), _lib.ptr(sgr))
        groups, node_groups = [], {}
        for i in range(G):
            dim, gid, name = C.c_uint32(), C.c_uint32(), C.c_char_p()
            L.cwf_mesh_group(h, i, C.byref(dim), C.byref(gid), C.byref(name))
            groups.append(PhysicalGroup(dim.value, gid.value, name.value.decode()))
            ptr, cnt = C.POINTER(C.c_uint32)(), C.c_uint64()
            L.cwf_mesh_node_group(h, gid.value, C.byref(ptr), C.byref(cnt))
            if cnt.value:
                node_groups[gid.value] = np.ctypeslib.as_array(ptr, (cnt.value,)).copy()
        return Expected(GmshMesh(coords, nid, el, geo, grp, eid, sn, sg, sgr, groups, node_groups))
    finally:
        L.cwf_mesh_destroy(h)


def load_gmsh_from_string(text: str) -> Expected:
    h = C.c_void_p()
    return _finish(_lib.load().cwf_mesh_load_string(text.encode(), C.byref(h)), h)


def load_gmsh_file(path) -> Expected:
    h = C.c_void_p()
    return _finish(_lib.load().cwf_mesh_load_file(os.fsencode(str(path)), C.byref(h)), h)
