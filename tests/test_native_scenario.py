"""Native C++ scenario driver (cwf_scenario_*, apps/cwf_run) against the Python driver (cwf.run).

CPU: with CWF_SCENARIO_PACK_ONLY the native driver stops after pack::build_packed_buffers, and every
packed buffer must equal the Python packing byte for byte (tet4 block, hex8 block, tractions on quad and
triangle faces with load curves, Dirichlet values); the load vector re-evaluated at later times must
equal pack.assemble_load_vector; errors carry the Python driver's texts; the cwf_run binary reports
them with exit status 1. GPU: cwf_run's VTU frames and probe CSV equal `python -m cwf.run`'s bytes.
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

from cwf import _lib, pack, run
from scenario_files import write_block_scenario

RUNNER = os.path.join(os.path.dirname(_lib.LIB_PATH), "cwf_run")
BUFFERS = {"position0": np.float32, "external_force": np.float32, "bc_mask": np.uint32, "bc_value": np.float32,
           "lumped_mass": np.float32, "lumped_mass64": np.float64, "connectivity": np.uint32,
           "gradients": np.float32, "volume": np.float32, "material_index": np.uint32, "offsets": np.uint32,
           "element_indices": np.uint32, "local_indices": np.uint8}
PY_FIELD = {"position0": "position0", "lumped_mass": "lumped_mass", "lumped_mass64": "lumped_mass64"}

TRACTION_YAML = """curves:
  ramp:
    - [0.0, 0.0]
    - [0.005, 0.6]
    - [0.02, 1.0]
  pulse:
    - [0.0, 1.0]
    - [0.01, -0.5]
"""


class NativeScenario:
    def __init__(self, path, mode=_lib.MODE_PARITY, flags=_lib.SCENARIO_PACK_ONLY):
        self.L = _lib.load()
        self.h = C.c_void_p()
        rc = self.L.cwf_scenario_create(os.fsencode(path), mode, 0, flags, C.byref(self.h))
        if rc:
            self.h = None
            raise run.ScenarioError(_error_text())

    def packed(self, name):
        data, nbytes = C.c_void_p(), C.c_uint64()
        assert self.L.cwf_scenario_packed(self.h, name.encode(), C.byref(data), C.byref(nbytes)) == 0
        dt = np.dtype(BUFFERS[name])
        if nbytes.value == 0:
            return np.zeros(0, dt)
        return np.frombuffer(C.string_at(data, nbytes.value), dt).copy()

    def external_force(self, t, n):
        out = np.zeros(n, np.float32)
        assert self.L.cwf_scenario_external_force(self.h, t, _lib.ptr(out), n) == 0
        return out

    def close(self):
        if self.h:
            self.L.cwf_scenario_destroy(self.h)
            self.h = None


def _error_text():
    return _lib.last_error(None)


def _python_error(path):
    with pytest.raises(run.ScenarioError) as ei:
        run.load_scenario(path)
    return str(ei.value)


def _edit(path, fn):
    text = open(path).read()
    with open(path, "w") as f:
        f.write(fn(text))


def _add_tractions(yaml_path):
    """Traction on the TIP faces under a ramp curve, a second one on FIXED under a pulse, a prescribed
    Dirichlet value, and the point load under the pulse curve."""
    text = open(yaml_path).read()
    text = text.replace("loads:\n  gravity: [0.0, 0.0, -9.81]\n",
                        TRACTION_YAML + "loads:\n  gravity: [0.0, 0.0, -9.81]\n  tractions:\n"
                        "    - group: TIP\n      value: [1.0e4, -2.5e3, -7.0e4]\n      scale_curve: ramp\n"
                        "    - group: FIXED\n      value: [0.0, 3.0e2, 0.0]\n      scale_curve: pulse\n")
    text = text.replace("      value: [0.0, 0.0, -500.0]\n", "      value: [0.0, 0.0, -500.0]\n      scale_curve: pulse\n")
    text = text.replace("      dof: [x, y, z]\n", "      dof: [x, y, z]\n      value: [null, 1.0e-3, null]\n")
    open(yaml_path, "w").write(text)
    return yaml_path


def _compare_packing(path, mode=_lib.MODE_PARITY):
    cfg, m, P, _ = run.load_scenario(path, allow_hex8=mode == _lib.MODE_FAST)
    ns = NativeScenario(path, mode)
    try:
        for name in BUFFERS:
            want = getattr(P, PY_FIELD.get(name, name))
            got = ns.packed(name)
            want = np.ascontiguousarray(want).reshape(-1).astype(BUFFERS[name], copy=False)
            assert got.tobytes() == want.tobytes(), name
        for t in (0.0, 0.003, 0.01, 0.5):
            want = pack._safe_f32(pack.assemble_load_vector(m, cfg, P.lumped_mass64, t))
            assert ns.external_force(t, P.dof_count).tobytes() == want.tobytes(), t
    finally:
        ns.close()
    return P


def test_native_packing_tet4_block_matches_python(tmp_path):
    P = _compare_packing(write_block_scenario(str(tmp_path), 5, 3, 2))
    assert P.element_count == 5 * 3 * 2 * 6


def test_native_packing_with_tractions_curves_and_values(tmp_path):
    y = _add_tractions(write_block_scenario(str(tmp_path), 4, 3, 3, h=0.07))
    cfg, m, P, _ = run.load_scenario(y)
    assert len(cfg.loads.tractions) == 2 and len(m.surfaces) > 0
    assert np.any(P.bc_value != 0.0)
    _compare_packing(y)


def test_native_packing_hex8_fast_matches_python(tmp_path):
    y = _add_tractions(write_block_scenario(str(tmp_path), 4, 3, 2, element="hex8"))
    P = _compare_packing(y, _lib.MODE_FAST)
    assert P.element_count == 24 and int(P.connectivity[4]) != 0xFFFFFFFF


def test_native_mesh_path_next_to_yaml(tmp_path, monkeypatch):
    y = write_block_scenario(str(tmp_path), 2, 2, 2)
    monkeypatch.chdir("/")
    NativeScenario(y).close()  # resolved relative to the YAML file


@pytest.mark.parametrize("edit, element, prefix", [
    (lambda t: t.replace("material: steel", "material: granite"), "tet4",
     "config: assignment references unknown material"),
    (lambda t: t.replace("  - group: SOLID\n", "  - group: ROCK\n"), "tet4",
     "preprocess: assignment references missing physical group 'ROCK'"),
    (lambda t: t.replace("    E: 3.0e10", "    E: -1.0"), "tet4", "config: material.E must be > 0"),
    (lambda t: t.replace("block.msh", "nowhere.msh"), "tet4", "mesh: "),
    (lambda t: t, "hex8", "preprocess: only tetrahedron elements supported"),  # hex8 in PARITY mode
])
def test_native_errors_match_python_driver(tmp_path, edit, element, prefix):
    y = write_block_scenario(str(tmp_path), 2, 2, 2, element=element)
    _edit(y, edit)
    py = _python_error(y)
    with pytest.raises(run.ScenarioError) as ei:
        NativeScenario(y)
    msg, ctx = ei.value.args[0]
    assert py == f"{msg} {ctx}" and py.startswith(prefix)


def test_pack_only_handle_refuses_steps(tmp_path):
    ns = NativeScenario(write_block_scenario(str(tmp_path), 2, 2, 2))
    tel = (C.c_char * 256)()
    assert ns.L.cwf_scenario_step(ns.h, 0, tel) == -11  # CWF_ERR_ARGUMENT
    assert "PACK_ONLY" in _lib.last_error(None)[0]
    ns.close()


def test_cwf_run_cli_errors(tmp_path):
    assert os.path.exists(RUNNER), "cwf_run not built (make -C civiwave-fem_amd/csrc)"
    r = subprocess.run([RUNNER], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr
    y = write_block_scenario(str(tmp_path), 2, 2, 2)
    _edit(y, lambda t: t.replace("material: steel", "material: granite"))
    r = subprocess.run([RUNNER, y, "--steps", "1"], capture_output=True, text=True)
    assert r.returncode == 1
    assert r.stderr.startswith("error: config: assignment references unknown material assignments [0] material")


# ---- GPU: byte equality of the two drivers' outputs ----------------------------------------------
def _run_both(tmp_path, y, mode, steps, extra=()):
    out_py, out_cc = tmp_path / "py", tmp_path / "cc"
    lines = []
    run.run_scenario(y, steps, str(out_py), _lib.MODE_FAST if mode == "fast" else _lib.MODE_PARITY,
                     time_varying_loads="--time-varying-loads" in extra, log=lines.append)
    r = subprocess.run([RUNNER, y, "--steps", str(steps), "--out", str(out_cc), "--mode", mode, *extra],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    native = r.stdout.strip().splitlines()
    assert len(native) == steps + 1
    for a, b in zip(lines, native[:-1]):
        pa, pb = json.loads(a), json.loads(b)
        assert pa == pb, (pa, pb)
    files = sorted(p.relative_to(out_py) for p in out_py.rglob("*") if p.is_file())
    assert files == sorted(p.relative_to(out_cc) for p in out_cc.rglob("*") if p.is_file())
    for f in files:
        assert (out_py / f).read_bytes() == (out_cc / f).read_bytes(), str(f)
    return files


@pytest.mark.gpu
def test_cwf_run_parity_outputs_byte_identical(tmp_path):
    y = _add_tractions(write_block_scenario(str(tmp_path), 6, 3, 3, xi=0.05, w=(10.0, 100.0), tol=1e-6, stride=2))
    files = _run_both(tmp_path, y, "parity", 3)
    assert len(files) == 3  # frames 0 and 2 + probes.csv


@pytest.mark.gpu
def test_cwf_run_time_varying_loads_byte_identical(tmp_path):
    y = _add_tractions(write_block_scenario(str(tmp_path), 5, 3, 3, tol=1e-6, stride=1))
    _run_both(tmp_path, y, "parity", 3, ("--time-varying-loads",))


@pytest.mark.gpu
def test_cwf_run_hex8_fast_byte_identical(tmp_path):
    y = write_block_scenario(str(tmp_path), 6, 3, 3, tol=1e-6, stride=1, element="hex8")
    _run_both(tmp_path, y, "fast", 2)
