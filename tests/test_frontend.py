"""Scenario front-end on the CPU (no GPU): the native YAML-subset config parser against the
reference's config tests (tests/config_validation_test.cpp:46-296, with the YAML text its
tests/support/config_builder.hpp generates restated below as test-data generation), the native Gmsh
MSH 4.1 loader against tests/mesh_loader_test.cpp:48-118, and a PyYAML cross-check of the parser on
the reference's fixture (tests/golden/data/cantilever.* are copies of the reference's test data)."""
import copy
import os

import pytest

from cwf import config, mesh, pack

DATA = os.path.join(os.path.dirname(__file__), "golden", "data")
NONE3 = (None, None, None)

DEFAULTS = dict(
    include_mesh=True, mesh_path="tests/data/cantilever.msh",
    include_materials=True, materials=[("concrete", 3.0e10, 0.2, 2500.0)],
    include_assignments=True, assignments=[("SOLID", "concrete")],
    include_damping=True, damping_xi=0.02, damping_w1=10.0, damping_w2=100.0,
    include_time=True, time_dt=0.01111, time_adaptive=True, include_time_min_dt=True, time_min_dt=0.005,
    include_time_max_dt=True, time_max_dt=0.02,
    include_solver=True, solver_type="pcg", solver_preconditioner="block_jacobi", solver_runtime_tol=2.0e-4,
    solver_pause_tol=1.0e-5, solver_max_iters=120,
    include_precision=True, vector_precision="fp32", reduction_precision="fp64",
    include_curves=True, curves=[("load_curve1", [(0.0, 0.0), (0.5, 0.75), (1.0, 1.0)])],
    include_loads=True, gravity=(0.0, 0.0, -9.81), tractions=[("LOAD_FACE", (0.0, 0.0, -1.0e5), "load_curve1")],
    include_point_loads=True, point_loads=[],
    include_dirichlet=True, dirichlet_fixes=[("FIXED_BASE", (True, True, True), NONE3)],
    include_output=True, output_stride=10, output_probes=[1, 2],
)


def g12(v):  # std::ostream << double with setprecision(12)
    return format(v, ".12g")


def make_config_yaml(**over):
    """YAML text of config_builder.hpp make_config_yaml(options) (test-data generation)."""
    o = copy.deepcopy(DEFAULTS)
    o.update(over)
    out = []
    if o["include_mesh"]:
        out += ["mesh:", f"  path: {o['mesh_path']}"]
    if o["include_materials"]:
        out.append("materials:")
        if not o["materials"]:
            out.append("  []")
        for n, E, nu, rho in o["materials"]:
            out += [f"  - name: {n}", f"    E: {g12(E)}", f"    nu: {g12(nu)}", f"    rho: {g12(rho)}"]
    if o["include_assignments"]:
        out.append("assignments:")
        if not o["assignments"]:
            out.append("  []")
        for g, m in o["assignments"]:
            out += [f"  - group: {g}", f"    material: {m}"]
    if o["include_damping"]:
        out += ["damping:", f"  xi: {g12(o['damping_xi'])}", f"  w1: {g12(o['damping_w1'])}",
                f"  w2: {g12(o['damping_w2'])}"]
    if o["include_time"]:
        out += ["time:", f"  dt: {g12(o['time_dt'])}", f"  adaptive: {str(o['time_adaptive']).lower()}"]
        if o["include_time_min_dt"]:
            out.append(f"  min_dt: {g12(o['time_min_dt'])}")
        if o["include_time_max_dt"]:
            out.append(f"  max_dt: {g12(o['time_max_dt'])}")
    if o["include_solver"]:
        out += ["solver:", f"  type: {o['solver_type']}", f"  preconditioner: {o['solver_preconditioner']}",
                f"  tol_runtime: {g12(o['solver_runtime_tol'])}", f"  tol_pause: {g12(o['solver_pause_tol'])}",
                f"  max_iters: {o['solver_max_iters']}"]
    if o["include_precision"]:
        out += ["precision:", f"  vectors: {o['vector_precision']}", f"  reductions: {o['reduction_precision']}"]
    if o["include_curves"] and o["curves"]:
        out.append("curves:")
        for name, pts in o["curves"]:
            out.append(f"  {name}:")
            out += [f"    - [{g12(t)}, {g12(v)}]" for t, v in pts]
    if o["include_loads"]:
        out += ["loads:", f"  gravity: [{', '.join(g12(v) for v in o['gravity'])}]"]
        if o["tractions"]:
            out.append("  tractions:")
            for g, val, curve in o["tractions"]:
                out += [f"    - group: {g}", f"      value: [{', '.join(g12(v) for v in val)}]"]
                if curve:
                    out.append(f"      scale_curve: {curve}")
        if o["include_point_loads"] and o["point_loads"]:
            out.append("  points:")
            for g, val, curve in o["point_loads"]:
                out += [f"    - group: {g}", f"      value: [{', '.join(g12(v) for v in val)}]"]
                if curve:
                    out.append(f"      scale_curve: {curve}")
    if o["include_dirichlet"] and o["dirichlet_fixes"]:
        out += ["dirichlet:", "  fixes:"]
        for g, mask, vals in o["dirichlet_fixes"]:
            dof = ", ".join(a for a, m in zip("xyz", mask) if m)
            out += [f"    - group: {g}", f"      dof: [{dof}]"]
            if any(v is not None for v in vals):
                out.append("      value: [" + ", ".join("null" if v is None else g12(v) for v in vals) + "]")
    if o["include_output"]:
        out += ["output:", f"  vtu_stride: {o['output_stride']}"]
        if o["output_probes"]:
            out.append(f"  probes: [{', '.join(str(p) for p in o['output_probes'])}]")
    return "\n".join(out) + "\n"


def test_parses_golden_config_from_builder():
    r = config.load_config_from_string(make_config_yaml())
    assert r.has_value(), r.error()
    c = r.value()
    assert c.mesh_path == "tests/data/cantilever.msh"
    assert len(c.materials) == 1 and c.materials[0].name == "concrete" and c.materials[0].youngs_modulus == 3.0e10
    assert c.assignments[0].group == "SOLID" and c.damping.xi == 0.02 and c.time.initial_dt == 0.01111
    assert c.time.adaptive and c.solver.type == "pcg" and c.precision.vector_precision == "fp32"
    assert list(c.curves) == ["load_curve1"] and c.loads.gravity == (0.0, 0.0, -9.81) and not c.loads.points
    assert len(c.dirichlet) == 1 and c.dirichlet[0].constrain_axis[0] and c.output.vtu_stride == 10


def test_loads_config_fixture_on_disk():
    r = config.load_config_from_file(os.path.join(DATA, "cantilever.yaml"))
    assert r.has_value(), r.error()
    assert r.value().mesh_path == "tests/data/cantilever.msh"


def test_parses_point_loads_with_optional_curve():
    y = make_config_yaml(point_loads=[("FIXED_BASE", (0.0, 0.0, -1234.5), "load_curve1"),
                                      ("LOAD_FACE", (10.0, 0.0, 0.0), "")])
    r = config.load_config_from_string(y)
    assert r.has_value(), r.error()
    p = r.value().loads.points
    assert len(p) == 2 and p[0].group == "FIXED_BASE" and p[0].value[2] == -1234.5
    assert p[0].scale_curve == "load_curve1" and p[1].scale_curve == ""


def _replace(token, new):
    return lambda y: y.replace(token, new, 1)


INVALID = [
    ("MissingMeshSection", dict(include_mesh=False), "missing 'mesh' section", ["mesh"], None),
    ("NegativeYoungsModulus", dict(materials=[("concrete", -1.0, 0.2, 2500.0)]), "material.E must be > 0",
     ["materials", "[0]", "E"], None),
    ("PoissonRatioTooLarge", dict(materials=[("concrete", 3.0e10, 0.75, 2500.0)]),
     "material.nu must be (-0.999, 0.5)", ["materials", "[0]", "nu"], None),
    ("DuplicateMaterialNames", dict(materials=[("duplicate", 3.0e10, 0.2, 2500.0), ("duplicate", 1.0e11, 0.3, 7800.0)]),
     "material names must be unique", ["materials", "[1]", "name"], None),
    ("AssignmentUnknownMaterial", dict(assignments=[("SOLID", "missing")]), "assignment references unknown material",
     ["assignments", "[0]", "material"], None),
    ("DampingXiOutOfRange", dict(damping_xi=1.2), "damping.xi must be (0,1)", ["damping", "xi"], None),
    ("DampingW2TooSmall", dict(damping_w1=10.0, damping_w2=5.0), "damping.w2 must be > damping.w1",
     ["damping", "w2"], None),
    ("NegativeTimeStep", dict(time_dt=-0.01), "time.dt must be > 0", ["time", "dt"], None),
    ("NegativeMinDt", dict(time_min_dt=-0.01), "time.min_dt must be >= 0", ["time", "min_dt"], None),
    ("MaxDtBelowInitial", dict(time_max_dt=0.001), "time.max_dt must be >= time.dt", ["time", "max_dt"], None),
    ("ZeroSolverIterations", dict(solver_max_iters=0), "solver.max_iters must be >= 1", ["solver", "max_iters"], None),
    ("NegativeSolverTolerance", dict(solver_runtime_tol=-1.0), "solver tolerances must be > 0", ["solver"], None),
    ("MissingPrecisionSection", dict(include_precision=False), "missing precision map", ["precision"], None),
    ("CurveTimesNotMonotonic", dict(curves=[("load_curve1", [(0.0, 0.0), (0.6, 1.0), (0.5, 1.1)])]),
     "curve times must be non-decreasing", ["curves", "load_curve1", "[2]"], None),
    ("TractionUnknownCurve", dict(include_curves=False, tractions=[("LOAD_FACE", (0.0, 0.0, -1.0e5), "load_curve1")]),
     "traction references unknown curve", ["loads", "tractions", "[0]", "scale_curve"], None),
    ("EmptyDirichletDof", dict(dirichlet_fixes=[("FIXED_BASE", (False, False, False), NONE3)]),
     "dirichlet.dof must not be empty", ["dirichlet", "fixes", "[0]", "dof"], None),
    ("ZeroOutputStride", dict(output_stride=0), "output.vtu_stride must be >= 1", ["output", "vtu_stride"], None),
    ("MissingOutputSection", dict(include_output=False), "missing output map", ["output"], None),
    ("DirichletInvalidAxis", dict(), "dirichlet.dof must be subset of {x,y,z}", ["dirichlet", "fixes", "[0]", "dof"],
     _replace("dof: [x, y, z]", "dof: [x, q]")),
    # beyond the reference's table: the remaining validation branches of config.cpp
    ("EmptyMaterials", dict(materials=[]), "materials must be a non-empty sequence", ["materials"], None),
    ("PointLoadUnknownCurve", dict(point_loads=[("TIP", (0.0, 0.0, 1.0), "nope")]),
     "point load references unknown curve", ["loads", "points", "[0]", "scale_curve"], None),
    ("GravityNotVec3", dict(gravity=(0.0, -9.81)), "expected sequence[3] for vector", ["loads", "gravity"], None),
    ("CurvePointNotPair", dict(), "curve point must be sequence[2]", ["curves", "load_curve1", "[1]"],
     _replace("    - [0.5, 0.75]", "    - [0.5, 0.75, 1]")),
    ("DampingW1NonPositive", dict(damping_w1=0.0), "damping.w1 must be > 0", ["damping", "w1"], None),
    ("MaterialBadNumber", dict(), "bad conversion", ["materials", "[0]"], _replace("E: 30000000000", "E: lots")),
    ("MissingRootMap", dict(), "config root must be a mapping", [], lambda y: "- just\n- a list\n"),
]


@pytest.mark.parametrize("name,opts,msg,ctx,mutate", INVALID, ids=[c[0] for c in INVALID])
def test_reports_detailed_validation_errors(name, opts, msg, ctx, mutate):
    y = make_config_yaml(**opts)
    if mutate:
        y = mutate(y)
    r = config.load_config_from_string(y)
    assert not r.has_value(), name
    assert msg in r.error().message, (name, r.error())
    if ctx:
        assert r.error().context == ctx, (name, r.error())


def test_yaml_syntax_and_io_errors():
    r = config.load_config_from_string("mesh:\n  path: [a, b\n")
    assert not r.has_value() and r.error().message.startswith("YAML parse error: ")
    r = config.load_config_from_file(os.path.join(DATA, "definitely_missing.yaml"))
    assert not r.has_value() and "unable to open config file" in r.error().message


def test_parser_agrees_with_pyyaml_on_fixtures():
    yaml = pytest.importorskip("yaml")
    for text in (open(os.path.join(DATA, "cantilever.yaml")).read(),
                 make_config_yaml(point_loads=[("TIP", (1.5, -2.0, 3.25e-3), "")],
                                  dirichlet_fixes=[("FIXED_BASE", (True, False, True), (0.0, None, -1e-3))])):
        d = yaml.safe_load(text)
        c = config.load_config_from_string(text).value()
        assert c.mesh_path == d["mesh"]["path"]
        assert [(m.name, m.youngs_modulus, m.poisson_ratio, m.density) for m in c.materials] == \
            [(m["name"], float(m["E"]), float(m["nu"]), float(m["rho"])) for m in d["materials"]]
        # PyYAML is YAML 1.1 ("1e-05" stays a string there); yaml-cpp's as<double> reads it as a number
        assert (c.time.initial_dt, c.time.adaptive, c.time.min_dt, c.time.max_dt) == \
            (float(d["time"]["dt"]), d["time"]["adaptive"], float(d["time"]["min_dt"]), float(d["time"]["max_dt"]))
        assert (c.solver.runtime_tolerance, c.solver.pause_tolerance, c.solver.max_iterations) == \
            (float(d["solver"]["tol_runtime"]), float(d["solver"]["tol_pause"]), d["solver"]["max_iters"])
        assert {k: [tuple(p) for p in v.points] for k, v in c.curves.items()} == \
            {k: [tuple(float(x) for x in p) for p in v] for k, v in d["curves"].items()}
        assert list(c.loads.gravity) == [float(x) for x in d["loads"]["gravity"]]
        assert [list(t.value) for t in c.loads.tractions] == \
            [[float(x) for x in t["value"]] for t in d["loads"].get("tractions", [])]
        assert [list(p.value) for p in c.loads.points] == \
            [[float(x) for x in p["value"]] for p in d["loads"].get("points", [])]
        for f, fd in zip(c.dirichlet, d["dirichlet"]["fixes"]):
            assert f.constrain_axis == tuple(a in fd["dof"] for a in "xyz")
            assert list(f.value) == [None if v is None else float(v) for v in fd.get("value", [None] * 3)]
        assert (c.output.vtu_stride, c.output.probes) == (d["output"]["vtu_stride"], d["output"]["probes"])


# ---- Gmsh loader: tests/mesh_loader_test.cpp -------------------------------------------------

HEADER = ("$MeshFormat\n4.1 0 8\n$EndMeshFormat\n$Nodes\n1 4 1 4\n3 3 0 4\n1\n2\n3\n4\n"
          "0 0 0\n1 0 0\n0 1 0\n0 0 1\n$EndNodes\n")


def tet_block(nodes, etype=4):
    return "$Elements\n1 1 1 1\n" + f"3 3 {etype} 1\n1 " + " ".join(str(n) for n in nodes) + "\n$EndElements\n"


def test_loads_cantilever_fixture_and_physical_lookup():
    r = mesh.load_gmsh_file(os.path.join(DATA, "cantilever.msh"))
    assert r.has_value(), r.error()
    m = r.value()
    assert m.coords.shape == (4, 3) and list(m.coords[0]) == [0, 0, 0] and list(m.coords[1]) == [1, 0, 0]
    assert len(m.elements) == 1 and m.geometry[0] == 4 and list(m.elements[0, :4]) == [0, 1, 2, 3]
    assert len(m.surfaces) == 2 and set(m.surface_groups) >= {1, 2}
    assert len(m.surface_groups[1]) == 1 and len(m.surface_groups[2]) == 1
    assert m.physical_groups and m.physical_groups[m.group_lookup[3]].name == "SOLID"


def test_mesh_io_and_section_errors():
    r = mesh.load_gmsh_file(os.path.join(DATA, "definitely_missing.msh"))
    assert not r.has_value() and "failed to open mesh file" in r.error().message
    r = mesh.load_gmsh_from_string(HEADER)
    assert not r.has_value() and "missing $Elements section" in r.error().message
    r = mesh.load_gmsh_from_string(HEADER + tet_block([1, 2, 3, 99]))
    assert not r.has_value() and "element references unknown node" in r.error().message
    assert r.error().context == ["Elements", "elementTag=1"]
    r = mesh.load_gmsh_from_string(HEADER + tet_block([1, 2, 3, 4], 6))
    assert not r.has_value() and "unsupported Gmsh element type" in r.error().message
    r = mesh.load_gmsh_from_string(HEADER.replace("1 4 1 4\n", "1 5 1 4\n") + tet_block([1, 2, 3, 4]))
    assert not r.has_value() and r.error().message == "node count mismatch"


def test_entities_tag_node_groups_and_hex_is_rejected_by_preprocess():
    text = ("$MeshFormat\n4.1 0 8\n$EndMeshFormat\n$PhysicalNames\n2\n2 7 \"TIP\"\n3 9 \"SOLID\"\n"
            "$EndPhysicalNames\n$Entities\n0 0 1 1\n5 0 0 0 1 1 1 1 7 0\n4 0 0 0 1 1 1 1 9 0\n$EndEntities\n"
            "$Nodes\n2 8 1 8\n2 5 0 2\n1\n2\n0 0 0\n1 0 0\n3 4 0 6\n3\n4\n5\n6\n7\n8\n"
            "1 1 0\n0 1 0\n0 0 1\n1 0 1\n1 1 1\n0 1 1\n$EndNodes\n"
            "$Elements\n1 1 1 1\n3 4 5 1\n1 1 2 3 4 5 6 7 8\n$EndElements\n")
    r = mesh.load_gmsh_from_string(text)
    assert r.has_value(), r.error()
    m = r.value()
    assert list(m.node_groups[7]) == [0, 1] and m.element_group[0] == 9 and m.geometry[0] == 8
    assert [(g.id, g.dimension, g.name) for g in m.physical_groups] == [(7, 2, "TIP"), (9, 3, "SOLID")]
    with pytest.raises(pack.PackError) as e:
        m.to_tet_mesh()
    assert e.value.message == "only tetrahedron elements supported in Phase 3" and e.value.context == ["elements", "[0]"]


# ---- scenario files -> packing (cwf.run.load_scenario) ------------------------------------

def test_scenario_files_pack_like_the_direct_builder(tmp_path):
    from cwf import run, scenarios
    from helpers import assert_bitwise
    from scenario_files import write_block_scenario

    y = write_block_scenario(str(tmp_path), 5, 3, 2, xi=0.05, w=(10.0, 100.0))
    cfg, m, P, mats = run.load_scenario(y)  # mesh path resolved relative to the YAML
    ref = scenarios.block_case(5, 3, 2, h=0.1, xi=0.05, w=(10.0, 100.0)).packing
    for name in ("connectivity", "gradients", "volume", "material_index", "lumped_mass", "lumped_mass64", "bc_mask",
                 "bc_value", "external_force", "offsets", "element_indices", "local_indices", "position0"):
        assert_bitwise(getattr(P, name), getattr(ref, name), name)
    assert cfg.damping.xi == 0.05 and cfg.output.vtu_stride == 2


def test_scenario_errors_carry_reference_texts(tmp_path):
    from cwf import run
    from scenario_files import write_block_scenario

    y = write_block_scenario(str(tmp_path), 2, 2, 2)
    os.remove(os.path.join(str(tmp_path), "block.msh"))
    with pytest.raises(run.ScenarioError, match="failed to open mesh file"):
        run.load_scenario(y)
    bad = tmp_path / "bad.yaml"
    bad.write_text(open(y).read().replace("E: 3.0e10", "E: -3.0"))
    with pytest.raises(run.ScenarioError, match=r"material.E must be > 0"):
        run.load_scenario(str(bad))


def test_cpp_mirror_frontend_and_writers(tmp_path):
    """tests/cpp/frontend_api_test.cpp through include/cwf_hip.hpp (config, mesh, VTU, probes; no GPU)."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    libdir = os.path.join(root, "civiwave-fem_amd", "lib")
    exe = str(tmp_path / "frontend_api_test")
    subprocess.run(["g++", "-std=c++20", "-O1", "-Wall", "-I/opt/rocm/include",
                    os.path.join(root, "tests", "cpp", "frontend_api_test.cpp"), "-o", exe, f"-L{libdir}",
                    "-lcwf_hip", f"-Wl,-rpath,{libdir}"], check=True)
    out = subprocess.run([exe, DATA, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
