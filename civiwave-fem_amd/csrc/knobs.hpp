// knobs.hpp -- every environment switch libcwf_hip.so reads, in one place. None is needed for a solve: the
// defaults are the measured-best configuration (DESIGN.md sections 3 and 6); each switch exists for a test or a
// same-box A/B (tools/gpu_run.sh ab). knob() refuses (returns NULL for) a name that is not listed here.
#pragma once

#include <cstdlib>
#include <cstring>

namespace cwf
{
struct Knob
{
    const char *name;
    const char *doc;
};

inline constexpr Knob kKnobs[] = {
    // node order and tiling of a FAST handle (abi.cpp, groups.cpp, tiles.cpp)
    {"CWF_RENUMBER", "0: keep the caller's node order (no Morton / owner-tile renumbering)"},
    {"CWF_GEO", "0: the 48-B gradient records instead of recomputing geometry from tile-node coordinates"},
    {"CWF_GROUPS", "0: per-tet tiles (k_keff_tiles_pipe) instead of the fan groups"},
    {"CWF_GROUP_NT", "128: 128-lane fan-group tiles (default 256; tests/test_gpu_parity.py)"},
    {"CWF_TILE_ORDER", "morton|rcb: per-tet / hex8 tile order"},
    {"CWF_TILE_PIPE", "0: the one-tile-per-workgroup per-tet kernel (k_keff_tiles)"},
    {"CWF_HEX_NT", "128|256: lanes of the hex8 tiles (tests/test_hex8.py)"},
    {"CWF_LATTICE", "0: no structured-block stencil (lattice.cpp); structured Kuhn (hex8) blocks then run the fan groups (hex tiles)"},
    {"CWF_LAT_ZR", "0|1: the lattice update pass stores z / the K_eff pass forms z from r and the node class "
                   "(default: the latter from 2M nodes)"},
    {"CWF_LAT_L", "n: planes per lattice brick (default: about 1024 bricks of 256 threads, at least 4 planes)"},
    {"CWF_PARITY_TILES", "strip: PARITY node tiles of 256 consecutive nodes also on a single handle (default there: "
                         "compact breadth-first tiles and a separate p.Ap partials pass; shards always use strips)"},
    {"CWF_PARITY_STREAM", "0: the PARITY loop folds alpha / beta in their own kernels (k_pcg_alpha / k_pcg_beta) instead "
                          "of in workgroup 0 of the pass producing the chunk partials (kernels_parity.hip fold_stream)"},
    // PCG schedule (spmv_tiles.hip, resident.hip)
    {"CWF_RESIDENT", "0: a structured block that fits on chip runs the launch-per-iteration schedules instead of the "
                     "resident one-launch solve (resident.hip; also off whenever CWF_FUSED is set)"},
    {"CWF_FUSED", "0: structured blocks run the two-kernel iteration (k_keff_lattice + k_pcg_update_tiles) instead of "
                  "the fused one-launch iteration (lattice_fused.inc); 2: fused also where the grid walks the work items "
                  "persistently (default: fused only where one round of workgroups covers them)"},
    {"CWF_PEER_FUSED", "0: a PEER shard's fused iteration exchanges through a k_peer_step launch after each fused launch "
                       "instead of inside the launch (lattice_fused.inc fused_peer_wait / fused_peer_publish)"},
    {"CWF_FUSED_TRACE", "path (ablation build only): per-workgroup phase stamps of one fused launch per solve, appended"},
    {"CWF_RESIDENT_TRACE", "path: per-workgroup phase stamps of one phase (CWF_FUSED_TRACE_IT) of every resident solve, "
                           "appended (tools/resident_trace.py)"},
    {"CWF_FUSED_TRACE_IT", "n: the iteration whose launch CWF_FUSED_TRACE records (default 50)"},
    {"CWF_FUSED_MAXWG", "n: cap on the fused launch's grid (default 1024 workgroups; a grid below the work items walks them persistently)"},
    {"CWF_XLAG", "1..4: iterations per lazy x update (tests/test_gpu_parity.py compares 4 with 1)"},
    // multi-GPU (comm.cpp)
    {"CWF_RCCL_LIB", "path: load this NCCL-API library instead of librccl (tests/transport: the host-staged "
                     "test transport that runs several ranks on one GPU, where RCCL refuses duplicate devices)"},
    // diagnostics
    {"CWF_TIMED_PCG", "bits: cwf_hip_keff_timed times the PCG-mode tiles kernel dry (tools/ablate.py)"},
    {"CWF_VERBOSE", "1: print the tiling statistics at create"},
};

inline const char *knob(const char *name)
{
    for (const Knob &k : kKnobs)
        if (std::strcmp(k.name, name) == 0)
            return std::getenv(name);
    return nullptr;
}
}  // namespace cwf
