/*
 * cwf_hip.h -- C-ABI of the MI355X (gfx950) matrix-free Newmark/PCG hot path.
 *
 * Drop-in boundary for CiviWave-FEM's L4 solver core. Every entry point below replaces a
 * reference C++ interface (cited as /root/reference file:line); plain pointers and sizes
 * only, no torch or C++ types, no exceptions. Return value: 0 on success, a negative
 * cwf_status on failure; cwf_hip_last_error()/cwf_hip_last_context() then hold the
 * reference's message text and breadcrumb (e.g. "CG denominator approached zero",
 * "iteration=12").
 *
 * Threading: one handle = one device + one HIP stream, externally synchronised
 * (the reference Stepper is single-threaded, newmark_stepper.hpp:92). Distinct handles may
 * run concurrently on distinct threads.
 *
 * Pointer kinds: every vector argument is host memory when `ptr_kind == CWF_PTR_HOST`
 * (copied in/out, call is synchronous) or device memory (HBM) when CWF_PTR_DEVICE
 * (used in place, the call still returns after the work completes on the handle's stream).
 */
#ifndef CWF_HIP_H
#define CWF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CWF_HIP_ABI_VERSION 1

typedef enum cwf_status
{
    CWF_OK = 0,
    CWF_ERR_SIZE = -1,           /* pcg.cpp:82-125 "... size mismatch" */
    CWF_ERR_NODE_RANGE = -2,     /* pcg.cpp:609-613 "element connectivity references node out of range" */
    CWF_ERR_MATERIAL_RANGE = -3, /* pcg.cpp:566-570 "element references material out of range" */
    CWF_ERR_MATERIALS = -4,      /* pcg.cpp:126-129 "materials table is empty" */
    CWF_ERR_REDUCTION = -5,      /* pcg.cpp:130-137 reduction_block / reduction_partials == 0 */
    CWF_ERR_MAX_ITERATIONS = -6, /* pcg.cpp:739-742 "max_iterations must be >= 1" */
    CWF_ERR_RHO_ZERO = -7,       /* pcg.cpp:810-813, 889-892 */
    CWF_ERR_DENOM_ZERO = -8,     /* pcg.cpp:846-849 "CG denominator approached zero" */
    CWF_ERR_ALLOC = -9,          /* pcg.cpp:65-68 workspace allocation failure */
    CWF_ERR_HIP = -10,           /* HIP runtime error (message holds hipGetErrorString) */
    CWF_ERR_ARGUMENT = -11,      /* NULL handle / pointer */
    CWF_ERR_COMM = -12,          /* RCCL / communicator failure */
    CWF_ERR_UNSUPPORTED = -13,
    CWF_ERR_IO = -14,            /* vtu_writer.cpp / probe_logger.cpp / config / mesh file errors */
    CWF_ERR_INDEX = -15,         /* probe_logger.cpp:116-119 "probe index out of range" */
    CWF_ERR_PARSE = -16          /* config.cpp / mesh.cpp parse and validation errors */
} cwf_status;

typedef enum cwf_ptr_kind
{
    CWF_PTR_HOST = 0,
    CWF_PTR_DEVICE = 1
} cwf_ptr_kind;

/* Arithmetic mode. PARITY reproduces the reference fold order bit for bit (fp64 element math,
 * 256-DOF chunked sequential fp64 dots). FAST: fp32 element math, fp64 tree reductions,
 * tolerance-checked against the oracle. Both consume the same inputs. */
typedef enum cwf_mode
{
    CWF_MODE_PARITY = 0,
    CWF_MODE_FAST = 1
} cwf_mode;

/* Mirrors cwf::gpu::pcg::MatrixFreeSystem (include/cwf/gpu/pcg.hpp:67-86) plus the packed
 * adjacency of cwf::mesh::pack::AdjacencyBuffers (include/cwf/mesh/pack.hpp:120-125).
 * All pointers are host memory; the handle copies them to HBM at create time. */
/* cwf_system_desc.reserved flags. A CWF_MODE_FAST handle renumbers its nodes internally along a Morton
 * curve of node_coords (locality of the tile gathers and partial stores; 1.8x on a permuted mesh), and
 * converts every vector at the boundary, so callers always see their own node order. KEEP_NODE_ORDER
 * disables that: required for handles that are attached as shards (local numbering = the halo plan). */
#define CWF_DESC_KEEP_NODE_ORDER 1

typedef struct cwf_system_desc
{
    uint64_t node_count;
    uint64_t element_count;
    uint64_t dof_count;                 /* must equal 3 * node_count */
    const uint32_t *element_connectivity; /* [element_count * 8], tets use slots 0..3 */
    const float *element_gradients;     /* [element_count * 24], grad N_a xyz, a = 0..7 */
    const float *element_volume;        /* [element_count] */
    const uint32_t *element_material_index; /* [element_count] */
    const double *material_stiffness;   /* [material_count * 36], ElasticProperties::stiffness */
    uint64_t material_count;
    const float *lumped_mass;           /* [node_count] */
    const uint32_t *bc_mask;            /* [node_count], bit0/1/2 = x/y/z constrained */
    const uint32_t *adjacency_offsets;  /* [node_count + 1] or NULL (built from connectivity) */
    const uint32_t *adjacency_elements; /* [offsets[N]] ascending element index per node, or NULL */
    const uint8_t *adjacency_local;     /* [offsets[N]] local slot 0..3, or NULL */
    double stiffness_scale;             /* 1 + a1 * beta_R */
    double mass_factor;                 /* a0 + a1 * alpha_R */
    uint64_t reduction_block;           /* 256 in the reference (pack.hpp:183) */
    uint64_t reduction_partials;        /* >= ceil(dof_count / reduction_block) */
    int32_t mode;                       /* cwf_mode */
    int32_t reserved;                   /* flags: CWF_DESC_KEEP_NODE_ORDER */
    const double *node_coords;          /* [node_count * 3] or NULL: only used to order FAST-mode tiles */
} cwf_system_desc;

/* PcgSettings (pcg.hpp:115-120) */
typedef struct cwf_pcg_settings
{
    uint64_t max_iterations;
    double relative_tolerance;
    int32_t warm_start;
    int32_t check_interval; /* iterations enqueued between host convergence checks; 0 = auto */
} cwf_pcg_settings;

/* PcgTelemetry (pcg.hpp:125-133) */
typedef struct cwf_pcg_telemetry
{
    uint64_t iterations;
    double residual_norm;
    double rhs_norm;
    double alpha_last;
    double beta_last;
    int32_t converged;
    int32_t reserved;
} cwf_pcg_telemetry;

typedef struct cwf_hip_system cwf_hip_system;

/* Library / device info. */
int cwf_hip_abi_version(void);
int cwf_hip_device_count(int *count);
const char *cwf_hip_last_error(const cwf_hip_system *h);   /* h may be NULL: last create error */
const char *cwf_hip_last_context(const cwf_hip_system *h);

/* Create / destroy: replaces building a MatrixFreeSystem over packed buffers
 * (newmark_stepper.cpp:1034-1049) and DeviceBufferArena::create (device_buffers.cpp:132). */
int cwf_hip_system_create(const cwf_system_desc *desc, int device, cwf_hip_system **out);
void cwf_hip_system_destroy(cwf_hip_system *h);
/* update stiffness_scale / mass_factor (newmark_stepper.cpp:1322-1326) */
int cwf_hip_system_set_scalars(cwf_hip_system *h, double stiffness_scale, double mass_factor);
int cwf_hip_system_set_mode(cwf_hip_system *h, int mode);
/* bytes of HBM held by the handle */
int cwf_hip_system_memory(const cwf_hip_system *h, uint64_t *bytes);
/* STREAM-like device copy (16-B lanes, grid-stride) on `device`: *gbs = (read + write bytes) / time. The
 * measured HBM ceiling bench.py reports beside the 8 TB/s spec. No reference counterpart. */
int cwf_hip_bandwidth_probe(int device, uint64_t bytes, int reps, double *gbs);
/* Algorithmic (compulsory) HBM bytes of one PCG-loop K_eff launch (measurement support, not a
 * reference interface): `layout_bytes` = every array the handle's own K_eff kernel touches, counted
 * once (the headline roofline uses the build's own layout when it reads less);
 * `reference_layout_bytes` = 32 N + 72 E, the same SpMV over the reference's packed layout. */
int cwf_hip_system_keff_traffic(const cwf_hip_system *h, uint64_t *layout_bytes, uint64_t *reference_layout_bytes);
/* Name of the kernel the handle's K_eff launches in its current mode ("k_keff_lattice", "k_keff_groups_pipe",
 * "k_keff_tiles_pipe", "k_keff_tiles", "k_keff_hex_tiles" or "k_keff_parity"); NULL for a NULL handle. */
const char *cwf_hip_system_keff_kernel(const cwf_hip_system *h);
/* Diagnostic: the PCG schedule a sharded handle's FAST solves run, decided collectively at its first solve:
 * -1 not decided yet (or not sharded), 0 the two-kernel iteration (two exchange steps per iteration), 1 the fused
 * lattice iteration with one exchange step per iteration, 2 the fused iteration exchanging inside its launches
 * (PEER: the Ap send rows, rank totals and epoch flags pushed by the launch itself, no exchange launch), 3 the
 * resident solve (PEER slab shards: every iteration in one launch per solve, its surface records and rank totals
 * stored into the peers' mailboxes by the kernel). */
int cwf_hip_system_exchange_schedule(const cwf_hip_system *h);
/* 16 hex digits: a hash of the source files and build flags of the translation unit that holds that kernel
 * (csrc/Makefile FAST_SRC / PARITY_SRC), so a committed PMC profile can be matched to the code that ran */
const char *cwf_hip_system_keff_source_hash(const cwf_hip_system *h);
/* Structured-block introspection (host only, no device; not a reference interface): whether a FAST handle
 * created from the tet4 `desc` runs the structured Kuhn-block stencil (lattice.cpp; native hex8 blocks run their
 * own 27-point stencil and are not described here). Returns 1 and fills dims (nodes per
 * axis; bit 31 of dims[0]: the stencil pairs S_(-d) = S_d), coef (CWF_LATTICE_COEFS floats, row-major 3x3 blocks
 * unscaled by stiffness_scale: the 15 interior stencil blocks, then the 46 cell-pair blocks) and plane ([dims[2]] storage index of node (0, 0, k); NULL: not wanted) when it does, 0 when it
 * does not, a negative cwf_status code on bad arguments. `renumber` != 0 allows the lexicographic renumbering a handle
 * without CWF_DESC_KEEP_NODE_ORDER may apply. */
#define CWF_LATTICE_COEFS 549
int cwf_lattice_describe(const cwf_system_desc *desc, int renumber, uint32_t dims[3], float *coef, uint32_t *plane);

/* Live kernel timing (measurement support, not a reference interface): when enabled, every
 * K_eff launch inside solve_pcg / stepper_step is bracketed by hipEvents on the handle's stream;
 * cwf_hip_system_timing returns the summed device time (ms) and launch count of the launches that
 * did work, and resets the accumulators. `enabled` > 1 samples every enabled-th launch (iteration
 * index multiple of it), so the event markers do not sit between every pair of kernels. */
int cwf_hip_system_set_timing(cwf_hip_system *h, int enabled);
int cwf_hip_system_timing(cwf_hip_system *h, double *keff_ms, uint64_t *keff_launches);
/* Standalone timed K_eff: `reps` launches of the PCG-loop SpMV (no sanitize) on device x -> y,
 * bracketed by one hipEvent pair; *avg_ms = elapsed / reps. */
int cwf_hip_keff_timed(cwf_hip_system *h, const float *x_dev, float *y_dev, int reps, double *avg_ms);

/* cwf::gpu::pcg::apply_keff (pcg.hpp:161-163, pcg.cpp:505-694): y = K_eff x with
 * Dirichlet identity rows. n = dof_count. */
int cwf_hip_apply_keff(cwf_hip_system *h, const float *x, float *y, uint64_t n, int ptr_kind);

/* cwf::gpu::pcg::build_block_jacobi_inverse (pcg.hpp:226-227, pcg.cpp:479-503):
 * inv_out[node*9 + 3*i + j], row-major f32. n = node_count * 9. This is the reference's inverse in
 * every mode (constrained rows = identity). A FAST solve applies a symmetrised, 16-B-packed form of
 * it instead; cwf_hip_fast_block_inverse exports that operator. */
int cwf_hip_build_block_jacobi_inverse(cwf_hip_system *h, float *inv_out, uint64_t n, int ptr_kind);

/* The preconditioner a FAST solve actually applies (no reference counterpart): the block inverse
 * above, symmetrised (upper triangle), restricted to the free axes (constrained rows and columns 0:
 * z and r are 0 there) and dequantised from the update pass's 16-B record (blockinv_pack.hpp).
 * inv_out as above (n = node_count * 9); packed_out (nullable, host) receives the 16-B records,
 * [node_count * 4] u32; *fallback_nodes (nullable) counts the nodes whose block is applied in fp32. */
int cwf_hip_fast_block_inverse(cwf_hip_system *h, float *inv_out, uint64_t n, int ptr_kind, uint32_t *packed_out,
                               uint64_t *fallback_nodes);

/* Host restatement of that packing for one node (the same code the device runs): v = the block's
 * upper triangle {a00 a01 a02 a11 a12 a22}, mask bit k = axis k constrained. Writes the 16-B record
 * (w[4]) and the applied upper triangle (d[6]); returns 1 for a packed block, 0 for an fp32 fallback. */
int cwf_pack_block_inverse(const float *v, uint32_t mask, uint32_t *w, float *d);

/* dot_accumulate (pcg.cpp:170-207): chunked fp64 dot of two f32 DOF vectors. partials may be
 * NULL; otherwise [reduction_partials] chunk partials are written (host or device by ptr_kind). */
int cwf_hip_dot(cwf_hip_system *h, const float *a, const float *b, uint64_t n, int ptr_kind, double *out,
                double *partials);

/* cwf::gpu::pcg::solve_pcg (pcg.hpp:210-212, pcg.cpp:696-918). x_inout is the warm start
 * (settings->warm_start) and receives the solution; residual_out (nullable) receives r. */
int cwf_hip_solve_pcg(cwf_hip_system *h, const float *rhs, const cwf_pcg_settings *settings, float *x_inout,
                      float *residual_out, uint64_t n, int ptr_kind, cwf_pcg_telemetry *telemetry);

/* Residual history of the last solve_pcg (|r| after each iteration, entry 0 = initial),
 * up to `capacity` entries. Returns the number written via *count. */
int cwf_hip_residual_history(cwf_hip_system *h, double *out, uint64_t capacity, uint64_t *count);

/* ---------------------------------------------------------------------------------------
 * Newmark stepper: cwf::gpu::newmark::Stepper (newmark_stepper.hpp:92-190). Device-resident
 * node state (u, v, a, predictor, external force, bc values); one step = predictor -> RHS
 * (+ beta_R * K * d when beta_R != 0) -> Dirichlet clamp -> PCG -> corrector -> adaptive dt.
 * ------------------------------------------------------------------------------------- */

/* AdaptivePolicy (newmark_stepper.hpp:58-63) + config::SolverSettings / TimeSettings */
typedef struct cwf_stepper_desc
{
    double rayleigh_alpha, rayleigh_beta; /* RayleighCoefficients */
    double runtime_tolerance, pause_tolerance;
    uint64_t max_iterations;
    double initial_dt;
    int32_t adaptive;
    int32_t warm_start; /* Stepper::warm_start_enabled_ default true */
    double min_dt, max_dt;
    double low_iteration_ratio, increase_factor, decrease_factor; /* 0.3, 1.1, 0.5 */
    const float *external_force; /* [3N] interleaved dof = 3n+k (NodeBuffers::external_force) */
    const float *bc_value;       /* [3N] (NodeBuffers::bc_value) */
} cwf_stepper_desc;

/* StepTelemetry (newmark_stepper.hpp:68-79) */
typedef struct cwf_step_telemetry
{
    double simulation_time, time_step, applied_tolerance;
    int32_t paused_mode, dt_increased, dt_decreased, dt_clamped_min, dt_clamped_max, reserved;
    cwf_pcg_telemetry pcg;
} cwf_step_telemetry;

typedef struct cwf_hip_stepper cwf_hip_stepper;

int cwf_hip_stepper_create(cwf_hip_system *system, const cwf_stepper_desc *desc, cwf_hip_stepper **out);
void cwf_hip_stepper_destroy(cwf_hip_stepper *st);
/* Stepper::step(simulation_time_seconds, paused_mode) */
int cwf_hip_stepper_step(cwf_hip_stepper *st, double simulation_time, int paused, cwf_step_telemetry *tel);
/* which: 0 = displacement, 1 = velocity, 2 = acceleration, 3 = the last PCG solution x, 4 = external force
 * (get only); out [3N] */
int cwf_hip_stepper_get_state(cwf_hip_stepper *st, int which, float *out, uint64_t n, int ptr_kind);
int cwf_hip_stepper_set_state(cwf_hip_stepper *st, int which, const float *in, uint64_t n, int ptr_kind);
/* rewrite nodes.external_force between steps (viewer.cpp:262-266) */
int cwf_hip_stepper_set_external_force(cwf_hip_stepper *st, const float *f, uint64_t n, int ptr_kind);
/* Time-varying loads on the device (loads.cpp:87-174 evaluated for one curve-scaled pattern, cast as
 * pack.cpp:41-57): set_load_pattern uploads base = the loads no curve scales (gravity, unscaled tractions and
 * point loads) and pattern = the point-load values one curve scales, f64 [3N] host arrays in the caller's node
 * order; each set_load_scale(c) then writes external_force = safe_cast(base + c * pattern) on the handle's
 * stream, where c = evaluate_curve(curve, t) (loads.cpp:63-85). For point loads (at most one scaled group per
 * node) that is bitwise the external_force assemble_load_vector at t packs (loads.cpp:163-172 adds
 * scale * value[axis] after gravity); a scaled traction rounds as (area * scale / n) * value there and is not
 * covered. This is the viewer's per-step rewrite of nodes.external_force (viewer.cpp:262-266) without the
 * host round trip. */
int cwf_hip_stepper_set_load_pattern(cwf_hip_stepper *st, const double *base, const double *pattern, uint64_t n);
int cwf_hip_stepper_set_load_scale(cwf_hip_stepper *st, double scale);
int cwf_hip_stepper_set_warm_start(cwf_hip_stepper *st, int enabled);
int cwf_hip_stepper_time(const cwf_hip_stepper *st, double *current_time, double *time_step);

/* ---------------------------------------------------------------------------------------
 * Multi-GPU: node-range shards with a ghost element layer (the north
 * star's "mesh shards ... RCCL all-reduce for the PCG dot products and halo-DOF exchange").
 * The reference itself is single-device; its src/gpu/sharding.cpp:38-144 (plan_shards) only
 * splits packed buffers under Vulkan's 2 GiB cap, which HBM handles do not need.
 * ------------------------------------------------------------------------------------- */

/* Host-only (no GPU needed). Rank `rank` of `nranks` owns global nodes
 * [rank_node_begin[rank], rank_node_begin[rank+1]). `desc` is the global mesh or any sub-mesh
 * holding every element that touches an owned node (in ascending global element order);
 * node_global_ids maps desc node -> global id (NULL = identity). The shard's local system has
 * the owned nodes first (ascending global id), then the ghosts grouped by owner rank. */
typedef struct cwf_shard cwf_shard;
typedef struct cwf_shard_info
{
    uint64_t owned_nodes;          /* local ids [0, owned_nodes) */
    uint64_t local_nodes;          /* owned + ghost */
    uint64_t local_elements;
    uint32_t neighbor_count;
    uint32_t reserved;
    const int32_t *neighbor_ranks; /* [neighbor_count], ascending */
    const uint64_t *send_offsets;  /* [neighbor_count + 1] into send_nodes */
    const uint32_t *send_nodes;    /* owned local ids each neighbour needs, ascending global id */
    const uint64_t *recv_offsets;  /* [neighbor_count + 1]: ghosts of neighbour k are local ids
                                      owned_nodes + [recv_offsets[k], recv_offsets[k+1]) */
    const uint64_t *node_global;   /* [local_nodes] global node id */
    const uint64_t *element_source; /* [local_elements] element index in the input desc */
    const uint64_t *node_source;    /* [local_nodes] node index in the input desc */
} cwf_shard_info;

int cwf_shard_build(const cwf_system_desc *desc, const uint64_t *node_global_ids, const uint64_t *rank_node_begin,
                    int32_t nranks, int32_t rank, cwf_shard **out);
/* local_desc: the shard's local system (arrays owned by the shard; adjacency NULL) */
int cwf_shard_get(const cwf_shard *shard, cwf_system_desc *local_desc, cwf_shard_info *info);
void cwf_shard_destroy(cwf_shard *shard);

/* Communicators. RCCL: one process per GPU (ncclCommInitRank; the 128-byte unique id is made by
 * rank 0 and broadcast by the caller, e.g. over torch.distributed). LOCAL: every rank's handle
 * lives in this process on one device (exchanges are device copies on one shared stream); it runs
 * the identical sharded kernels and exists to test the decomposition on a single GPU. */
#define CWF_COMM_ID_BYTES 128
typedef struct cwf_hip_comm cwf_hip_comm;
int cwf_hip_comm_unique_id(uint8_t *id);
int cwf_hip_comm_create_rccl(int32_t nranks, int32_t rank, const uint8_t *id, int device, cwf_hip_comm **out);
int cwf_hip_comm_create_local(int32_t nranks, int device, cwf_hip_comm **out);
void cwf_hip_comm_destroy(cwf_hip_comm *comm); /* after every attached handle is destroyed */

/* PEER: one process per rank, as RCCL, but the FAST exchange steps (the per-rank scalar all-gathers and the
 * halos) are device-initiated stores into the peers' IPC-mapped mailboxes plus a flag per step (peer.hip; the
 * "one-shot P2P" of SURVEY.md section 7 (iv)); PARITY's chunk-partial all-gathers are refused
 * (CWF_ERR_UNSUPPORTED: use RCCL). Setup: create, cwf_hip_system_attach (allocates this rank's mailbox),
 * cwf_hip_comm_peer_handle, exchange the handles between the processes (e.g. torch.distributed
 * all_gather_object), cwf_hip_comm_peer_connect with every rank's handle in rank order. Replaces the RCCL
 * group calls comm.cpp issues where pcg.cpp:170-207's dots would cross ranks. <= 16 ranks. */
#define CWF_IPC_HANDLE_BYTES 64
int cwf_hip_comm_create_peer(int32_t nranks, int32_t rank, int device, cwf_hip_comm **out);
int cwf_hip_comm_peer_handle(cwf_hip_comm *comm, uint8_t *handle /* [CWF_IPC_HANDLE_BYTES] */);
int cwf_hip_comm_peer_connect(cwf_hip_comm *comm, const uint8_t *handles /* [nranks * CWF_IPC_HANDLE_BYTES] */);
/* `steps` exchange steps shaped like the FAST PCG iteration's second one (the {r.r, r.z} all-gather and the z
 * halo) on the attached handle's stream, hipEvent-timed: microseconds per step (collective: every rank calls);
 * any communicator kind. An untimed first step carries a known pattern in z (owned rows = f(global id), the
 * plan's node_global) and every ghost row must arrive as its owner's value, else CWF_ERR_COMM "halo check failed"
 * {ghost, global}; z is clobbered (the next solve recomputes it). */
int cwf_hip_comm_time_exchange(cwf_hip_system *h, int32_t steps, double *us_per_step);
/* the memory this rank's PEER mailbox was allocated in (after attach): uncached device memory
 * (hipDeviceMallocUncached: another device's xGMI stores are visible without trusting the receiver's L2), else
 * fine-grained, else plain device memory when neither allocation can be IPC-exported. A PEER step whose wait times
 * out marks the communicator dead (a sticky device word): every later step returns CWF_ERR_COMM at once, and
 * cwf_hip_comm_time_exchange reports such a trial as CWF_ERR_COMM. */
#define CWF_PEER_MAILBOX_DEVICE 0
#define CWF_PEER_MAILBOX_FINEGRAINED 1
#define CWF_PEER_MAILBOX_UNCACHED 2
int cwf_hip_comm_peer_mailbox_kind(const cwf_hip_comm *comm, int *kind);

/* Make `h` (created from a shard's local desc with CWF_DESC_KEEP_NODE_ORDER) rank `rank` of `comm` with the
 * shard's halo plan. Afterwards solve_pcg / stepper_step are collective: scalars are all-gathered and folded
 * in rank order on every rank (identical control flow everywhere), ghost DOFs are refreshed by the halo
 * exchange, and vectors are local [3 * local_nodes] with only the owned rows meaningful on output (x is
 * halo-consistent). Both modes: FAST all-gathers one fp64 per rank per scalar (p.Ap; r.r and r.z with the z
 * halo in one RCCL group). PARITY all-gathers every rank's 256-DOF chunk partials and folds them in global
 * chunk order (pcg.cpp:170-207), so x, r and the residual history equal one handle's PARITY solve bit for
 * bit; it requires owned ranges that are contiguous, ascending by rank from node 0, and (all but the last)
 * whole reduction blocks: 3 * owned_nodes % reduction_block == 0 (cwf/shard.py slab_ranges(align=256)),
 * else CWF_ERR_UNSUPPORTED at the first solve. */
int cwf_hip_system_attach(cwf_hip_system *h, cwf_hip_comm *comm, int32_t rank, const cwf_shard_info *plan);
/* solve_pcg over all ranks of a LOCAL communicator (members in rank order); for RCCL call
 * cwf_hip_solve_pcg on each rank's handle. Telemetry is identical on every rank. residual_out (nullable, or
 * NULL entries) receives each member's local r (owned rows meaningful). */
int cwf_hip_solve_pcg_group(cwf_hip_system *const *members, int32_t count, const float *const *rhs,
                            const cwf_pcg_settings *settings, float *const *x_inout, float *const *residual_out,
                            int ptr_kind, cwf_pcg_telemetry *telemetry);

/* ---------------------------------------------------------------------------------------
 * Host-side preprocessing (no GPU needed): tet gradients/volume/lumped mass/CSR exactly as
 * mesh::pre::run + pack::build_packed_buffers (preprocess.cpp:268-405, pack.cpp:41-200).
 * Outputs are caller-allocated: grads[E*24], volume[E], mass[N] (f64) and mass32[N],
 * offsets[N+1], adj_elem[4E], adj_local[4E], conn8[8E].
 * ------------------------------------------------------------------------------------- */
int cwf_preprocess_tets(uint64_t node_count, uint64_t element_count, const double *coords, const uint32_t *tets,
                        const uint32_t *material_index, const double *density, uint64_t material_count,
                        float *grads24, float *volume, double *mass64, float *mass32, uint32_t *offsets,
                        uint32_t *adj_elem, uint8_t *adj_local, uint32_t *conn8);

/* Native hex8 (no reference counterpart: the reference rejects hex8 in
 * preprocess.cpp:326-330, so parity is unpinned). Trilinear isoparametric element, Gmsh/VTK corner
 * order, 2x2x2 Gauss: volume = sum_gp det J, lumped mass rho V / 8 per corner, grads24 = dN_a/dx at
 * the element centre; CSR with 8E incidences (adj_local 0..7); conn8 = hexes. A system_desc whose
 * connectivity fills all 8 slots is a hex8 system: CWF_MODE_FAST only, node_coords required.
 * Errors: "hexahedron Jacobian non-positive (inverted or degenerate)" {"elements [e]"} (CWF_ERR_SIZE). */
int cwf_preprocess_hex8(uint64_t node_count, uint64_t element_count, const double *coords, const uint32_t *hexes,
                        const uint32_t *material_index, const double *density, uint64_t material_count,
                        float *grads24, float *volume, double *mass64, float *mass32, uint32_t *offsets,
                        uint32_t *adj_elem, uint8_t *adj_local, uint32_t *conn8);

/* ---- post stack ---------------------------------------------------------- */

/* cwf::post::compute_derived_fields (src/post/derived_fields.cpp:139-211), on the device and bit-exact:
 * u = displacement f32 [3N] node-interleaved (n = dof_count); outputs are 13 floats per element /
 * node {strain[6] (Voigt, engineering shear), stress[6], von_mises} -- the memory layout of
 * cwf::post::ElementField / NodeField (derived_fields.hpp:37-55). `elements` [13E] or `nodes` [13N] may
 * be NULL. */
int cwf_hip_derived_fields(cwf_hip_system *h, const float *u, uint64_t n, int u_kind, float *elements,
                           float *nodes, int out_kind);

/* One output frame, host memory (the PackingResult node buffers + DerivedFieldSet the reference
 * writers read). Vectors are node-interleaved f32 [3N]; connectivity is the packed u32 [8E] with
 * UINT32_MAX padding (4 valid slots = tet4 / VTK 10, otherwise hex8 / VTK 12). */
typedef struct cwf_frame_view
{
    uint64_t node_count;
    uint64_t element_count;
    const float *position0;      /* pack.hpp:96 Float3SoA position0 (f32) */
    const float *displacement;
    const float *velocity;
    const float *acceleration;
    const float *element_fields; /* [13E] */
    const float *node_fields;    /* [13N] */
    const uint32_t *connectivity;
} cwf_frame_view;

/* cwf::post::write_vtu (vtu_writer.cpp:171-297): binary-appended UnstructuredGrid, byte-identical to
 * the reference writer; parent directories are created. Errors: CWF_ERR_IO "failed to open VTU file"
 * {path}. cwf_hip_last_error(NULL) holds the message. */
int cwf_write_vtu(const char *path, const cwf_frame_view *frame, double simulation_time, uint32_t frame_index);

/* cwf::post::ProbeLogger::log_frame (probe_logger.cpp:91-124): appends one CSV row per probe node;
 * *header_written is the logger's header_written_ flag (0 -> truncate + header first, then set to 1).
 * Errors: "probe index out of range" {index} (CWF_ERR_INDEX), "failed to open probe CSV" (CWF_ERR_IO). */
int cwf_probe_log_frame(const char *path, int *header_written, const uint32_t *probes, uint64_t probe_count,
                        const cwf_frame_view *frame, double simulation_time, uint32_t frame_index);

/* ---- scenario front-end ------------------------------------------------------- */
/* Error contexts of these calls are the reference's breadcrumb vectors joined with '\n'. */

/* cwf::config::load_config_from_file / load_config_from_string (src/config/config.cpp:118-146) with
 * parse_config_node's validation (:148-605): same messages and breadcrumbs, e.g. "material.E must be
 * > 0" {"materials", "[0]", "E"} (CWF_ERR_PARSE). The YAML subset is parsed natively (no yaml-cpp). */
typedef struct cwf_config cwf_config;
int cwf_config_load_file(const char *path, cwf_config **out);
int cwf_config_load_string(const char *yaml_text, cwf_config **out);
/* the validated Config as canonical JSON (field names of config.hpp:41-237, doubles %.17g) */
const char *cwf_config_json(const cwf_config *cfg);
void cwf_config_destroy(cwf_config *cfg);

/* cwf::mesh::load_gmsh_file / load_gmsh_from_string (src/mesh/mesh.cpp:459-566): Gmsh MSH 4.1 ASCII. */
typedef struct cwf_mesh cwf_mesh;
typedef struct cwf_mesh_info
{
    uint64_t node_count;
    uint64_t element_count; /* volume elements (tet4 / hex8) */
    uint64_t surface_count; /* tri3 / quad4 boundary faces */
    uint64_t group_count;   /* physical groups */
} cwf_mesh_info;
int cwf_mesh_load_file(const char *path, cwf_mesh **out);
int cwf_mesh_load_string(const char *text, cwf_mesh **out);
void cwf_mesh_destroy(cwf_mesh *mesh);
int cwf_mesh_get_info(const cwf_mesh *mesh, cwf_mesh_info *info);
/* coords f64 [3N] (xyz per node, file order), original_ids u32 [N]; either may be NULL */
int cwf_mesh_nodes(const cwf_mesh *mesh, double *coords, uint32_t *original_ids);
/* nodes8 u32 [8E] (UINT32_MAX padded), geometry u8 [E] (4 = tet4, 8 = hex8), physical_group u32 [E] */
int cwf_mesh_elements(const cwf_mesh *mesh, uint32_t *nodes8, uint8_t *geometry, uint32_t *physical_group,
                      uint32_t *original_ids);
/* nodes4 u32 [4S] (UINT32_MAX padded), geometry u8 [S] (3 = tri3, 4 = quad4), physical_group u32 [S] */
int cwf_mesh_surfaces(const cwf_mesh *mesh, uint32_t *nodes4, uint8_t *geometry, uint32_t *physical_group);
/* physical group `index` (0 .. group_count-1, ascending id); *name stays valid until destroy */
int cwf_mesh_group(const cwf_mesh *mesh, uint64_t index, uint32_t *dimension, uint32_t *id, const char **name);
/* node indices tagged with physical group `group_id` through $Entities (Mesh::node_groups) */
int cwf_mesh_node_group(const cwf_mesh *mesh, uint32_t group_id, const uint32_t **nodes, uint64_t *count);

/* ---- native scenario driver ----------------------------------------------------
 * The viewer backend's sequence (src/ui/viewer.cpp:200-277) in C++: load_config_from_file ->
 * load_gmsh_file -> pre::run + pack::build_packed_buffers (loads at t = 0) -> Stepper; per frame
 * step(simulation_time) with simulation_time = telemetry.simulation_time + time_step, then
 * OutputManager::handle_frame (output_manager.cpp:49-87). The mesh path is taken as given, else
 * next to the YAML file. An all-hex8 mesh runs as native hex8 in CWF_MODE_FAST. Errors carry the
 * reference's texts prefixed "config: ", "mesh: " or "preprocess: "; every call leaves its message in
 * cwf_hip_last_error(NULL) / cwf_hip_last_context(NULL). */
typedef struct cwf_scenario cwf_scenario;
#define CWF_SCENARIO_TIME_VARYING_LOADS 1 /* re-evaluate load curves at each step's start time */
#define CWF_SCENARIO_PACK_ONLY 2          /* build the packed buffers only, no device handle (host tests) */
int cwf_scenario_create(const char *yaml_path, int mode, int device, int flags, cwf_scenario **out);
int cwf_scenario_info(const cwf_scenario *sc, uint64_t *nodes, uint64_t *elements, uint64_t *dofs);
/* one Newmark frame (Stepper::step errors, e.g. "CG denominator approached zero") */
int cwf_scenario_step(cwf_scenario *sc, int paused, cwf_step_telemetry *telemetry);
/* derived fields of the last stepped frame -> <out_root>/vtu/frame_%05u.vtu every vtu_stride frames
 * and one probe row per probe to <out_root>/probes/probes.csv */
int cwf_scenario_output_frame(cwf_scenario *sc, const char *out_root);
/* the Stepper's state after the last step (newmark_stepper.hpp:92-190: the pack's displacement / velocity /
 * acceleration node buffers, f32 [3N] each) and the derived fields OutputManager::handle_frame computes from it
 * (output_manager.cpp:49-87 -> derived_fields.cpp:139-211: element f32 [13E], node f32 [13N], the layout of
 * cwf_hip_derived_fields); any pointer may be NULL */
int cwf_scenario_state(cwf_scenario *sc, float *u, float *v, float *a, float *element_fields, float *node_fields);
/* read-only view of one packed host buffer (pack.hpp:93-183 names): position0, external_force, bc_mask,
 * bc_value, lumped_mass, lumped_mass64, connectivity, gradients, volume, material_index, offsets,
 * element_indices, local_indices. Unknown name: CWF_ERR_ARGUMENT. */
int cwf_scenario_packed(const cwf_scenario *sc, const char *name, const void **data, uint64_t *bytes);
/* loads.cpp:87-174 assemble_load_vector at `time`, cast like pack.cpp:41-57 -> out f32 [3N] */
int cwf_scenario_external_force(const cwf_scenario *sc, double time, float *out, uint64_t n);
void cwf_scenario_destroy(cwf_scenario *sc);

#ifdef __cplusplus
}
#endif
#endif /* CWF_HIP_H */
