"""ctypes binding of libcwf_hip.so (include/cwf_hip.h).

The library is built in-tree (``civiwave-fem_amd/lib/libcwf_hip.so``) by
``__graft_entry__.build()`` / ``make -C civiwave-fem_amd/csrc``. There is no CPU
fallback: if the shared object is missing, importing the compute API raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(PKG_ROOT, "lib", "libcwf_hip.so")
LIB_PATH = os.environ.get("CWF_LIB_PATH") or DEFAULT_LIB  # env: A/B builds
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "cwf_hip.h")

PTR_HOST, PTR_DEVICE = 0, 1
MODE_PARITY, MODE_FAST = 0, 1
DESC_KEEP_NODE_ORDER = 1  # cwf_system_desc.reserved flag (cwf_hip.h)
SCENARIO_TIME_VARYING_LOADS, SCENARIO_PACK_ONLY = 1, 2  # cwf_scenario_create flags
PEER_MAILBOX_DEVICE, PEER_MAILBOX_FINEGRAINED, PEER_MAILBOX_UNCACHED = 0, 1, 2  # cwf_hip_comm_peer_mailbox_kind

STATUS = {
    0: "CWF_OK", -1: "CWF_ERR_SIZE", -2: "CWF_ERR_NODE_RANGE", -3: "CWF_ERR_MATERIAL_RANGE",
    -4: "CWF_ERR_MATERIALS", -5: "CWF_ERR_REDUCTION", -6: "CWF_ERR_MAX_ITERATIONS", -7: "CWF_ERR_RHO_ZERO",
    -8: "CWF_ERR_DENOM_ZERO", -9: "CWF_ERR_ALLOC", -10: "CWF_ERR_HIP", -11: "CWF_ERR_ARGUMENT",
    -12: "CWF_ERR_COMM", -13: "CWF_ERR_UNSUPPORTED", -14: "CWF_ERR_IO", -15: "CWF_ERR_INDEX",
    -16: "CWF_ERR_PARSE",
}


class SystemDesc(C.Structure):
    _fields_ = [
        ("node_count", C.c_uint64), ("element_count", C.c_uint64), ("dof_count", C.c_uint64),
        ("element_connectivity", C.c_void_p), ("element_gradients", C.c_void_p), ("element_volume", C.c_void_p),
        ("element_material_index", C.c_void_p), ("material_stiffness", C.c_void_p), ("material_count", C.c_uint64),
        ("lumped_mass", C.c_void_p), ("bc_mask", C.c_void_p), ("adjacency_offsets", C.c_void_p),
        ("adjacency_elements", C.c_void_p), ("adjacency_local", C.c_void_p), ("stiffness_scale", C.c_double),
        ("mass_factor", C.c_double), ("reduction_block", C.c_uint64), ("reduction_partials", C.c_uint64),
        ("mode", C.c_int32), ("reserved", C.c_int32), ("node_coords", C.c_void_p),
    ]


class PcgSettingsC(C.Structure):
    _fields_ = [("max_iterations", C.c_uint64), ("relative_tolerance", C.c_double), ("warm_start", C.c_int32),
                ("check_interval", C.c_int32)]


class PcgTelemetryC(C.Structure):
    _fields_ = [("iterations", C.c_uint64), ("residual_norm", C.c_double), ("rhs_norm", C.c_double),
                ("alpha_last", C.c_double), ("beta_last", C.c_double), ("converged", C.c_int32),
                ("reserved", C.c_int32)]


class StepperDescC(C.Structure):
    _fields_ = [
        ("rayleigh_alpha", C.c_double), ("rayleigh_beta", C.c_double), ("runtime_tolerance", C.c_double),
        ("pause_tolerance", C.c_double), ("max_iterations", C.c_uint64), ("initial_dt", C.c_double),
        ("adaptive", C.c_int32), ("warm_start", C.c_int32), ("min_dt", C.c_double), ("max_dt", C.c_double),
        ("low_iteration_ratio", C.c_double), ("increase_factor", C.c_double), ("decrease_factor", C.c_double),
        ("external_force", C.c_void_p), ("bc_value", C.c_void_p),
    ]


class StepTelemetryC(C.Structure):
    _fields_ = [
        ("simulation_time", C.c_double), ("time_step", C.c_double), ("applied_tolerance", C.c_double),
        ("paused_mode", C.c_int32), ("dt_increased", C.c_int32), ("dt_decreased", C.c_int32),
        ("dt_clamped_min", C.c_int32), ("dt_clamped_max", C.c_int32), ("reserved", C.c_int32),
        ("pcg", PcgTelemetryC),
    ]


class ShardInfoC(C.Structure):
    _fields_ = [
        ("owned_nodes", C.c_uint64), ("local_nodes", C.c_uint64), ("local_elements", C.c_uint64),
        ("neighbor_count", C.c_uint32), ("reserved", C.c_uint32), ("neighbor_ranks", C.c_void_p),
        ("send_offsets", C.c_void_p), ("send_nodes", C.c_void_p), ("recv_offsets", C.c_void_p),
        ("node_global", C.c_void_p), ("element_source", C.c_void_p), ("node_source", C.c_void_p),
    ]


class MeshInfoC(C.Structure):
    _fields_ = [("node_count", C.c_uint64), ("element_count", C.c_uint64), ("surface_count", C.c_uint64),
                ("group_count", C.c_uint64)]


class FrameViewC(C.Structure):
    _fields_ = [
        ("node_count", C.c_uint64), ("element_count", C.c_uint64), ("position0", C.c_void_p),
        ("displacement", C.c_void_p), ("velocity", C.c_void_p), ("acceleration", C.c_void_p),
        ("element_fields", C.c_void_p), ("node_fields", C.c_void_p), ("connectivity", C.c_void_p),
    ]


COMM_ID_BYTES = 128
IPC_HANDLE_BYTES = 64  # CWF_IPC_HANDLE_BYTES

_lib = None


def declared_symbols() -> list[str]:
    """Function names declared in include/cwf_hip.h."""
    import re

    text = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(cwf_(?:hip_)?[a-z0-9_]+)\s*\(", text)))


def load() -> C.CDLL:
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libcwf_hip.so not built ({LIB_PATH}); run __graft_entry__.build() or "
                           f"make -C civiwave-fem_amd/csrc -- there is no CPU fallback")
    try:  # torch first, when present: device tensors and the library then share one HIP runtime
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P, u64, f64, i32 = C.c_void_p, C.c_uint64, C.c_double, C.c_int
    sig = {
        "cwf_hip_abi_version": ([], i32),
        "cwf_hip_device_count": ([P], i32),
        "cwf_hip_last_error": ([P], C.c_char_p),
        "cwf_hip_last_context": ([P], C.c_char_p),
        "cwf_hip_system_create": ([P, i32, P], i32),
        "cwf_hip_system_destroy": ([P], None),
        "cwf_hip_system_set_scalars": ([P, f64, f64], i32),
        "cwf_hip_system_set_mode": ([P, i32], i32),
        "cwf_hip_system_memory": ([P, P], i32),
        "cwf_hip_bandwidth_probe": ([i32, u64, i32, P], i32),
        "cwf_hip_system_keff_traffic": ([P, P, P], i32),
        "cwf_hip_system_keff_kernel": ([P], C.c_char_p),
        "cwf_hip_system_exchange_schedule": ([P], i32),
        "cwf_hip_system_keff_source_hash": ([P], C.c_char_p),
        "cwf_lattice_describe": ([P, i32, P, P, P], i32),
        "cwf_hip_system_set_timing": ([P, i32], i32),
        "cwf_hip_system_timing": ([P, P, P], i32),
        "cwf_hip_keff_timed": ([P, P, P, i32, P], i32),
        "cwf_hip_apply_keff": ([P, P, P, u64, i32], i32),
        "cwf_hip_build_block_jacobi_inverse": ([P, P, u64, i32], i32),
        "cwf_hip_fast_block_inverse": ([P, P, u64, i32, P, P], i32),
        "cwf_pack_block_inverse": ([P, C.c_uint32, P, P], i32),
        "cwf_hip_dot": ([P, P, P, u64, i32, P, P], i32),
        "cwf_hip_solve_pcg": ([P, P, P, P, P, u64, i32, P], i32),
        "cwf_hip_residual_history": ([P, P, u64, P], i32),
        "cwf_hip_stepper_create": ([P, P, P], i32),
        "cwf_hip_stepper_destroy": ([P], None),
        "cwf_hip_stepper_step": ([P, f64, i32, P], i32),
        "cwf_hip_stepper_get_state": ([P, i32, P, u64, i32], i32),
        "cwf_hip_stepper_set_state": ([P, i32, P, u64, i32], i32),
        "cwf_hip_stepper_set_external_force": ([P, P, u64, i32], i32),
        "cwf_hip_stepper_set_warm_start": ([P, i32], i32),
        "cwf_hip_stepper_set_load_pattern": ([P, P, P, u64], i32),
        "cwf_hip_stepper_set_load_scale": ([P, C.c_double], i32),
        "cwf_hip_stepper_time": ([P, P, P], i32),
        "cwf_shard_build": ([P, P, P, i32, i32, P], i32),
        "cwf_shard_get": ([P, P, P], i32),
        "cwf_shard_destroy": ([P], None),
        "cwf_hip_comm_unique_id": ([P], i32),
        "cwf_hip_comm_create_rccl": ([i32, i32, P, i32, P], i32),
        "cwf_hip_comm_create_local": ([i32, i32, P], i32),
        "cwf_hip_comm_destroy": ([P], None),
        "cwf_hip_comm_create_peer": ([i32, i32, i32, P], i32),
        "cwf_hip_comm_peer_handle": ([P, P], i32),
        "cwf_hip_comm_peer_connect": ([P, P], i32),
        "cwf_hip_comm_time_exchange": ([P, i32, P], i32),
        "cwf_hip_comm_peer_mailbox_kind": ([P, P], i32),
        "cwf_hip_system_attach": ([P, P, i32, P], i32),
        "cwf_hip_solve_pcg_group": ([P, i32, P, P, P, P, i32, P], i32),
        "cwf_preprocess_tets": ([u64, u64, P, P, P, P, u64, P, P, P, P, P, P, P, P], i32),
        "cwf_preprocess_hex8": ([u64, u64, P, P, P, P, u64, P, P, P, P, P, P, P, P], i32),
        "cwf_hip_derived_fields": ([P, P, u64, i32, P, P, i32], i32),
        "cwf_write_vtu": ([C.c_char_p, P, f64, C.c_uint32], i32),
        "cwf_probe_log_frame": ([C.c_char_p, P, P, u64, P, f64, C.c_uint32], i32),
        "cwf_config_load_file": ([C.c_char_p, P], i32),
        "cwf_config_load_string": ([C.c_char_p, P], i32),
        "cwf_config_json": ([P], C.c_char_p),
        "cwf_config_destroy": ([P], None),
        "cwf_mesh_load_file": ([C.c_char_p, P], i32),
        "cwf_mesh_load_string": ([C.c_char_p, P], i32),
        "cwf_mesh_destroy": ([P], None),
        "cwf_mesh_get_info": ([P, P], i32),
        "cwf_mesh_nodes": ([P, P, P], i32),
        "cwf_mesh_elements": ([P, P, P, P, P], i32),
        "cwf_mesh_surfaces": ([P, P, P, P], i32),
        "cwf_mesh_group": ([P, u64, P, P, P], i32),
        "cwf_mesh_node_group": ([P, C.c_uint32, P, P], i32),
        "cwf_scenario_create": ([C.c_char_p, i32, i32, i32, P], i32),
        "cwf_scenario_info": ([P, P, P, P], i32),
        "cwf_scenario_step": ([P, i32, P], i32),
        "cwf_scenario_output_frame": ([P, C.c_char_p], i32),
        "cwf_scenario_state": ([P, P, P, P, P, P], i32),
        "cwf_scenario_packed": ([P, C.c_char_p, P, P], i32),
        "cwf_scenario_external_force": ([P, f64, P, u64], i32),
        "cwf_scenario_destroy": ([P], None),
    }
    for name, (args, res) in sig.items():
        if LIB_PATH != DEFAULT_LIB and not hasattr(L, name):
            continue  # an older build under same-box A/B (CWF_LIB_PATH) may lack newer entry points
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def ptr(a) -> C.c_void_p:
    """Host numpy array or device tensor (anything with data_ptr()) -> void*."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(C.c_void_p)
    return C.c_void_p(a.data_ptr())


def last_error(handle=None) -> tuple[str, list[str]]:
    L = load()
    msg = L.cwf_hip_last_error(handle).decode()
    ctx = L.cwf_hip_last_context(handle).decode()
    return msg, (ctx.split("\n") if ctx else [])  # breadcrumb vectors are joined with '\n' 
