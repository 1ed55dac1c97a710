"""CPU-side checks of the product library: it loads, exports every symbol include/cwf_hip.h
declares, and its host preprocessing / load / Dirichlet builders equal the oracle's bit for bit.
No compute call touches a GPU here."""
import numpy as np
import pytest

import oracle as O
from cwf import _lib, meshgen, pack, physics, scenarios


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    declared = _lib.declared_symbols()
    assert "cwf_hip_solve_pcg" in declared and "cwf_preprocess_tets" in declared
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert L.cwf_hip_abi_version() == 1


@pytest.mark.parametrize("jitter", [False, True])
def test_native_preprocess_bitwise_equals_oracle(jitter):
    case = scenarios.block_case(7, 5, 4, h=0.1, jitter=jitter)
    P = case.packing
    pk = O.preprocess_tets(case.mesh.coords, case.mesh.tets, P.material_index, [2500.0])
    pairs = {"gradients": (P.gradients, pk.gradients), "volume": (P.volume, pk.volume),
             "mass32": (P.lumped_mass, pk.lumped_mass), "mass64": (P.lumped_mass64, pk.mass64),
             "offsets": (P.offsets, pk.offsets), "adj_elem": (P.element_indices, pk.adj_elem),
             "adj_local": (P.local_indices, pk.adj_local), "conn8": (P.connectivity, pk.connectivity)}
    for k, (a, b) in pairs.items():
        assert a.tobytes() == b.tobytes(), k


def test_loads_equal_oracle_gravity_and_point_loads():
    case = scenarios.block_case(5, 3, 3, h=0.1)
    P = case.packing
    tip = case.mesh.node_groups[case.mesh.group_names["TIP"]]
    ref = O.assemble_loads(P.lumped_mass64, (0.0, 0.0, -9.81), [(tip, (0.0, 0.0, -500.0), 1.0)])
    got = pack.assemble_load_vector(case.mesh, case.cfg, P.lumped_mass64)
    assert got.tobytes() == ref.tobytes()
    assert P.external_force.tobytes() == ref.astype(np.float32).tobytes()


def test_dirichlet_mask_locks_fixed_face_only():
    # tests/physics_test.cpp:407-428 semantics: every fixed-group dof masked with target 0
    case = scenarios.block_case(3, 2, 2, h=0.1)
    P = case.packing
    fixed = case.mesh.node_groups[case.mesh.group_names["FIXED"]]
    assert np.all(P.bc_mask[fixed] == 7)
    others = np.setdiff1d(np.arange(P.node_count), fixed)
    assert np.all(P.bc_mask[others] == 0)
    assert np.all(P.bc_value == 0)


def test_preprocess_rejects_degenerate_tet():
    tm = meshgen.single_tet()
    tm.coords[3] = [0.5, 0.5, 0.0]  # flat
    mesh = pack.from_tetmesh(tm)
    cfg = scenarios.make_config(point_group="POINT")
    with pytest.raises(pack.PackError) as e:
        pack.build_packed_buffers(mesh, cfg)
    assert e.value.message == "tetrahedron volume non-positive"


def test_preprocess_reports_missing_assignment():
    tm = meshgen.single_tet()
    mesh = pack.from_tetmesh(tm)
    cfg = scenarios.make_config(point_group="POINT")
    cfg.assignments = [physics.Assignment("NOPE", "steel")]
    with pytest.raises(pack.PackError) as e:
        pack.build_packed_buffers(mesh, cfg)
    assert e.value.message == "assignment references missing physical group 'NOPE'"


def test_kuhn_block_counts_match_survey_table():
    for key, (N, E) in {"c1": (1386, 6000), "c2": (343000, 1971054)}.items():
        sx, sy, sz = meshgen.CONFIGS[key]["shape"]
        assert (sx + 1) * (sy + 1) * (sz + 1) == N and 6 * sx * sy * sz == E


def _build_cpp_test(tmp_path):
    import subprocess
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    libdir = os.path.join(root, "civiwave-fem_amd", "lib")
    exe = str(tmp_path / "pcg_api_test")
    subprocess.run(["g++", "-std=c++20", "-O1", "-Wall", "-I/opt/rocm/include",
                    os.path.join(root, "tests", "cpp", "pcg_api_test.cpp"), "-o", exe, f"-L{libdir}", "-lcwf_hip",
                    f"-Wl,-rpath,{libdir}"], check=True)
    return exe


def test_cpp_mirror_header_compiles_and_links(tmp_path):
    """include/cwf_hip.hpp (C++ mirror of cwf::gpu::pcg / Stepper) builds with the image's g++."""
    assert _build_cpp_test(tmp_path)
