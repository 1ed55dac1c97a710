"""Post stack on the CPU: the oracle's derived fields pinned to the reference's own test
(tests/derived_fields_test.cpp:90-140), and the host writers (no GPU needed) checked byte for byte
against an independent restatement of the reference formats (src/post/vtu_writer.cpp:171-297,
src/post/probe_logger.cpp:21-124)."""
import os
import struct

import numpy as np
import pytest

import oracle as O
from cwf import meshgen, pack, physics, post, scenarios
from helpers import oracle_system


def single_tet_case():
    tm = meshgen.single_tet()
    mesh = pack.from_tetmesh(tm)
    cfg = scenarios.make_config(gravity=(0.0, 0.0, 0.0), point=(0.0, 0.0, 0.0))
    cfg.dirichlet = []
    cfg.loads.point_loads = []
    return mesh, cfg, pack.build_packed_buffers(mesh, cfg)


def test_oracle_derived_fields_uniform_x_strain_like_reference_test():
    # derived_fields_test.cpp:90-140: u_x = 0.01 x on the unit tet, E = 30 GPa, nu = 0.2
    mesh, cfg, P = single_tet_case()
    mats = [physics.make_properties(m) for m in cfg.materials]
    o = oracle_system(P, mats, 1.0, 0.0)
    u = np.zeros(P.dof_count, np.float32)
    u[0::3] = (0.01 * mesh.coords[:, 0]).astype(np.float32)
    el, nd = o.derived_fields(u)
    E, nu = 30.0e9, 0.2
    lam = nu * E / ((1 + nu) * (1 - 2 * nu))
    mu = E / (2 * (1 + nu))
    assert abs(el[0, 0] - 0.01) <= 1e-5 and abs(el[0, 1]) <= 1e-5 and abs(el[0, 2]) <= 1e-5 and abs(el[0, 3]) <= 1e-5
    assert abs(el[0, 6] - (lam + 2 * mu) * 0.01) <= 5e3
    assert abs(el[0, 7] - lam * 0.01) <= 5e3 and abs(el[0, 8] - lam * 0.01) <= 5e3
    for n in range(P.node_count):
        assert abs(nd[n, 0] - 0.01) <= 1e-4 and abs(nd[n, 6] - (lam + 2 * mu) * 0.01) <= 5e3
    # von Mises of a uniaxial-strain state, fp64 restated
    s = el[0, 6:12].astype(np.float64)
    vm = np.sqrt(0.5 * ((s[0] - s[1]) ** 2 + (s[1] - s[2]) ** 2 + (s[2] - s[0]) ** 2) + 3 * (s[3:] ** 2).sum())
    assert abs(el[0, 12] - vm) <= 1e-6 * vm


def test_oracle_node_fields_are_volume_weighted_element_averages():
    case = scenarios.block_case(3, 2, 2, h=0.1, jitter=True)
    P = case.packing
    o = oracle_system(P, case.materials, 1.0, 0.0)
    rng = np.random.Generator(np.random.PCG64(11))
    u = rng.uniform(-1e-3, 1e-3, P.dof_count).astype(np.float32)
    el, nd = o.derived_fields(u)
    tets = P.connectivity.reshape(-1, 8)[:, :4].astype(np.int64)
    vol = P.volume.astype(np.float64)
    for n in (0, 7, P.node_count - 1):
        es = np.nonzero((tets == n).any(1))[0]
        w = vol[es]
        # element f32 outputs are rounded fp64 tensors: the node average agrees to f32 rounding
        avg = (el[es, 0:12].astype(np.float64) * w[:, None]).sum(0) / w.sum()
        np.testing.assert_allclose(nd[n, 0:12], avg, rtol=1e-5, atol=1e-9 * np.abs(avg).max())


# ---- VTU: independent restatement of vtu_writer.cpp:171-297 -------------------------------------

def reference_vtu_bytes(P, el, nd, time, frame):
    N, E = P.node_count, P.element_count
    blob = bytearray()

    def block(arr):
        off = len(blob)
        b = np.ascontiguousarray(arr).tobytes()
        blob.extend(struct.pack("<I", len(b)))
        blob.extend(b)
        return off

    f32 = lambda a: np.asarray(a, np.float32)  # noqa: E731
    po = [block(f32(P.displacement)), block(f32(P.velocity)), block(f32(P.acceleration)),
          block(f32(nd[:, 0:6])), block(f32(nd[:, 6:12])), block(f32(nd[:, 12]))]
    co = [block(f32(el[:, 0:6])), block(f32(el[:, 6:12])), block(f32(el[:, 12]))]
    pts = (np.asarray(P.position0, np.float32).reshape(-1) + f32(P.displacement)).astype(np.float32)
    conn8 = P.connectivity.reshape(E, 8)
    conn, offs, types, run = [], [], [], 0
    for e in range(E):
        lc = 4 if (conn8[e] != 0xFFFFFFFF).sum() == 4 else 8
        conn.extend(int(c) for c in conn8[e, :lc])
        run += lc
        offs.append(run)
        types.append(10 if lc == 4 else 12)
    pts_o = block(pts)
    conn_o = block(np.asarray(conn, np.int32))
    offs_o = block(np.asarray(offs, np.int32))
    types_o = block(np.asarray(types, np.uint8))
    head = ['<?xml version="1.0"?>',
            '<VTKFile type="UnstructuredGrid" version="1.0" byte_order="LittleEndian" header_type="UInt32">',
            '  <UnstructuredGrid>', '    <FieldData>',
            f'      <DataArray type="Float64" Name="time" NumberOfTuples="1">{time:g}</DataArray>',
            f'      <DataArray type="UInt32" Name="frame" NumberOfTuples="1">{frame}</DataArray>',
            '    </FieldData>', f'    <Piece NumberOfPoints="{N}" NumberOfCells="{E}">',
            '      <PointData Scalars="von_mises_node">']
    for name, comp, off in zip(["displacement", "velocity", "acceleration", "strain_node", "stress_node",
                                "von_mises_node"], [3, 3, 3, 6, 6, 1], po):
        head.append(f'        <DataArray type="Float32" Name="{name}" NumberOfComponents="{comp}" '
                    f'format="appended" offset="{off}"/>')
    head += ['      </PointData>', '      <CellData Scalars="von_mises_elem">']
    for name, comp, off in zip(["strain_elem", "stress_elem", "von_mises_elem"], [6, 6, 1], co):
        head.append(f'        <DataArray type="Float32" Name="{name}" NumberOfComponents="{comp}" '
                    f'format="appended" offset="{off}"/>')
    head += ['      </CellData>', '      <Points>',
             f'        <DataArray type="Float32" NumberOfComponents="3" format="appended" offset="{pts_o}"/>',
             '      </Points>', '      <Cells>',
             f'        <DataArray type="Int32" Name="connectivity" format="appended" offset="{conn_o}"/>',
             f'        <DataArray type="Int32" Name="offsets" format="appended" offset="{offs_o}"/>',
             f'        <DataArray type="UInt8" Name="types" format="appended" offset="{types_o}"/>',
             '      </Cells>', '    </Piece>', '  </UnstructuredGrid>', '  <AppendedData encoding="raw">']
    return ("\n".join(head) + "\n_").encode() + bytes(blob) + b"\n  </AppendedData>\n</VTKFile>\n"


def frame_case(seed=5):
    case = scenarios.block_case(3, 2, 2, h=0.1, jitter=True)
    P = case.packing
    rng = np.random.Generator(np.random.PCG64(seed))
    P.displacement = rng.uniform(-1e-3, 1e-3, P.dof_count).astype(np.float32)
    P.velocity = rng.uniform(-1, 1, P.dof_count).astype(np.float32)
    P.acceleration = rng.uniform(-10, 10, P.dof_count).astype(np.float32)
    o = oracle_system(P, case.materials, 1.0, 0.0)
    el, nd = o.derived_fields(P.displacement)
    return case, P, post.DerivedFieldSet(el, nd)


@pytest.mark.parametrize("time,frame", [(0.0, 0), (0.01, 7), (1.25e-5, 123)])
def test_vtu_bytes_match_reference_format(tmp_path, time, frame):
    case, P, d = frame_case()
    path = tmp_path / "sub" / "frame.vtu"
    assert post.write_vtu(path, P, d, time, frame).has_value()
    got = path.read_bytes()
    assert got == reference_vtu_bytes(P, d.elements, d.nodes, time, frame)
    assert b"VTKFile" in got[:128]  # export_writer_test.cpp:102-108


def test_vtu_single_tet_and_open_failure(tmp_path):
    mesh, cfg, P = single_tet_case()
    o = oracle_system(P, [physics.make_properties(m) for m in cfg.materials], 1.0, 0.0)
    el, nd = o.derived_fields(P.displacement)
    d = post.DerivedFieldSet(el, nd)
    path = tmp_path / "frame_0.vtu"
    assert post.write_vtu(path, P, d, 0.0, 0).has_value()
    assert path.read_bytes() == reference_vtu_bytes(P, el, nd, 0.0, 0)
    (tmp_path / "blocker").write_text("x")  # a file where the parent directory should be
    r = post.write_vtu(tmp_path / "blocker" / "f.vtu", P, d, 0.0, 0)
    assert not r.has_value()


def test_probe_csv_rows_and_errors(tmp_path):
    case, P, d = frame_case(7)
    path = tmp_path / "probes" / "probes.csv"
    lg = post.ProbeLogger(path, [0, 5])
    assert lg.log_frame(0.02, 3, P, d).has_value()
    assert lg.log_frame(0.03, 4, P, d).has_value()
    lines = path.read_text().splitlines()
    assert lines[0] == ("frame,time,node,ux,uy,uz,vx,vy,vz,ax,ay,az,strain_xx,strain_yy,strain_zz,strain_xy,"
                        "strain_yz,strain_xz,stress_xx,stress_yy,stress_zz,stress_xy,stress_yz,stress_xz,"
                        "von_mises")
    assert len(lines) == 5

    def row(frame, t, n):
        vals = [P.displacement[3 * n:3 * n + 3], P.velocity[3 * n:3 * n + 3], P.acceleration[3 * n:3 * n + 3],
                d.nodes[n]]
        return f"{frame},{t:.9f},{n}," + ",".join(f"{float(v):.9f}" for a in vals for v in a)

    assert lines[1] == row(3, 0.02, 0) and lines[2] == row(3, 0.02, 5) and lines[4] == row(4, 0.03, 5)
    # a fresh logger truncates and rewrites the header (probe_logger.cpp:64-89)
    assert post.ProbeLogger(path, [1]).log_frame(0.0, 0, P, d).has_value()
    assert len(path.read_text().splitlines()) == 2
    bad = post.ProbeLogger(tmp_path / "b.csv", [P.node_count])
    r = bad.log_frame(0.0, 0, P, d)
    assert not r.has_value()
    assert r.error().message == "probe index out of range" and r.error().context == [str(P.node_count)]
    # no probes: nothing is written (probe_logger.cpp:99-103)
    assert post.ProbeLogger(tmp_path / "none.csv", []).log_frame(0.0, 0, P, d).has_value()
    assert not (tmp_path / "none.csv").exists()
