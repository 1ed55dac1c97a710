// cwf_internal.hpp -- device data layout and host handle of the MI355X hot path.
//
// HBM layout (one handle):
//   erec     uint4[E*4]  64-B element record: {conn0..3} {gx0 gy0 gz0 gx1} {gy1 gz1 gx2 gy2} {gz2 gx3 gy3 gz3}
//                        (f32 gradient bits; one 64-B line per tet, read with 4 x dwordx4)
//   vol      f32[E], mat u32[E]
//   mass     f32[N], mask u32[N] (bit k = axis k constrained)
//   off      u32[N+1], inc u32[4E] = (element << 2) | local_slot, ascending element per node
//   dmat     f64[M*36] (+ isotropic flag: only the 12 structurally nonzero entries are used)
//   vectors  f32[3N] node-interleaved (dof = 3n + k), the reference's DOF order
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <initializer_list>
#include <string>
#include <vector>

#include "../../include/cwf_hip.h"
#include "knobs.hpp"

namespace cwf
{

// FAST-mode element tiles (tiles.cpp): element-centric K_eff with deterministic LDS folds
constexpr int kTileElems = 512;      // elements per tile (= per 256-thread workgroup)
constexpr int kMaxTileNodes = 512;  // distinct nodes per tile (LDS bound; two node slots per thread)
// hex8 tiles: <= NT hexes and <= 2 NT nodes per NT-lane workgroup, NT = hex_tile_lanes(E) (abi.cpp)
uint32_t hex_tile_lanes(uint64_t hexes);
// fan-group tiles of NT = 256 lanes (group_lanes(), abi.cpp; 128 on request): <= NT groups (one per lane), <= 2 NT nodes
// (two per lane; 9-bit local ids), <= kGroupSlotsPerLane NT pushed-force slots (padded runs, LDS) and <= 16
// pushes per tile node (4-bit ranks in the record)
#ifndef CWF_GROUP_SLOTS
#define CWF_GROUP_SLOTS 12
#endif
#ifndef CWF_GROUP_WAVES
#define CWF_GROUP_WAVES 1
#endif
constexpr uint32_t kGroupSlotsPerLane = CWF_GROUP_SLOTS;
constexpr int kGroupWavesPerSimd = CWF_GROUP_WAVES;  // k_keff_groups_pipe's minimum waves per SIMD (VGPR cap)
constexpr uint32_t kGroupMaxRun = 16;

struct DevTiles
{
    uint32_t ntiles = 0;
    uint32_t max_tile_nodes = 0;
    uint32_t total_tile_nodes = 0;
    uint32_t E = 0;
    int geo = 0;  // 1: geometry recomputed from tile-node coordinates (eid + tcoord), 0: 48-B planes
    int pipe = 0; // 1: persistent software-pipelined tiles kernel (GEO records, push fold)
    uint32_t pipe_grid = 0;  // its resident grid (occupancy x CUs, whole XCD groups)
    int pipe_nt = 256;       // its workgroup size; tiles hold <= 2 pipe_nt elements and <= pipe_nt nodes
    int push = 0;            // 1: elements store forces at their local-CSR positions; nodes fold contiguous runs
    // [3][E] 48-B records: {idx01, idx23, g0x, g0y} {g0z, g1x, g1y, g1z} {g2x, g2y, g2z, vol};
    // g3 = -(g0 + g1 + g2) (partition of unity of the linear tet)
    const uint4 *planes = nullptr;
    const uint2 *eid = nullptr;      // [E] {idx01, idx23} local corner ids (GEO)
    const float *tcoord = nullptr;   // [3][total] tile-relative node coordinates, tile-major (GEO)
    const uint32_t *mat = nullptr;            // [E] material per element (tile order), NULL when M == 1
    const uint4 *hdr = nullptr;               // [ntiles] {first element, #elements, first tile node, #nodes}
    const uint2 *tnode = nullptr;             // [total] {local node | owner bit 31, csr begin | csr end << 16}
                                              // (csr range relative to the tile's first entry 4*e0)
    const uint16_t *csr_ent = nullptr;        // [4E] element_local*4 + corner
    const uint2 *epos = nullptr;              // [E] (PUSH) each corner's position in the tile's local CSR
    // tet fan groups (groups.cpp): k_keff_groups_pipe, one group per lane, pushes per group node
    int grp = 0;
    uint32_t ngroups = 0;
    // [G] 9-bit local node ids of slots 0..7 (a b r0 .. r5), 3 per word in words 0-2 (bits 0-26), tet
    //     count f in word 0 bits 27-29, material in word 1 bits 27-31; word 3: 8 x 4-bit ranks in the runs
    const uint4 *grec = nullptr;
    // native hex8: k_keff_hex_tiles, 128-thread persistent grid (pipe_grid), push fold
    int hex = 0;
    int hex_all_affine = 0;        // every hex tile is a parallelepiped tile (affine-only kernel variant)
    int hex_nt = 128;              // lanes per hex tile / workgroup (128 or 256)
    const uint4 *eid8 = nullptr;   // [E] 8 u16 local corner ids (Gmsh corner order)
    const uint4 *epos8 = nullptr;  // [E] 8 u16 local-CSR positions
    const uint32_t *node_part_off = nullptr;  // [N+1] node -> range of its tile slots (ascending tile); with
                                              // off_mask, bits 29-31 of entry n carry bc_mask[n]
    int off_mask = 0;
    const uint32_t *part_slot = nullptr;      // [total] partial index of each of those slots
    // pipelined kernel: partials stored node-major (tile node q -> part[3 tslot[q]]), so a node's partials
    // are the contiguous run part[3 node_part_off[n] .. 3 node_part_off[n+1]) and part_slot is not read
    const uint32_t *tslot = nullptr;
    int node_major = 0;
    // fan groups: partials stored write-through (sc1), so their lines leave L2 during the kernel instead of in
    // the end-of-kernel write-back the update pass waits for; only pays while the working set stays in the
    // MALL (abi.cpp: < 4M tets)
    int wt_part = 0;
    float *part = nullptr;                    // [3*total] tile-node partial sums, node-major (scratch)
    // structured Kuhn block (lattice.cpp, lattice.inc): k_keff_lattice; part is one row value per node
    // (node_part_off[n] = n), ntiles = lnwork
    int lat = 0;
    uint32_t lnx = 0, lny = 0, lnz = 0;  // lattice nodes per axis (a shard: its local planes)
    uint32_t lk0 = 0, lk1 = 0;           // planes holding the rows this handle computes (a shard: its owned planes)
    // work items (lattice_plan): lnsb shell workgroups (a multiple of 8: one thread per surface node of the
    // computed planes, lnshell of them), then lnbx * lnby * ceil((lkI1 - lkI0) / lL) interior bricks (32 x 8
    // columns of the strict interior i, j in [1, n - 1) times lL planes of [lkI0, lkI1)); lnwork = all of them
    uint32_t lnbx = 0, lnby = 0, lL = 0, lnwork = 0, lnwm = 0, lnsb = 0, lnshell = 0, lkI0 = 0, lkI1 = 0;
    int lmu = 0;                         // every strict-interior node's lumped mass is lmass (the bricks read none)
    int lshl = 0;                        // shell workgroups after the bricks (grids of one resident round); 2: each
                                         // k-chunk's perimeter workgroups right after its bricks (lnsc per chunk),
                                         // the full end planes last
    uint32_t lnsc = 0;                   // lshl 2: perimeter workgroups per k-chunk
    int lzr = 0;                         // with lmu and the class table on an unattached handle: the update pass
                                         // stores no z, the K_eff pass forms it from r and the node's class
    float lmass = 0.f;
    const uint32_t *lplane = nullptr;    // [lnz] storage index of node (0, 0, k)
    uint32_t lpstride = 0;               // plane[k] == k lpstride for every k (the kernels then skip the plane[] load
                                         // in front of every plane's first gather); 0: read plane[]
    const float *lcoef = nullptr;        // [kLatCoef] stencil, cell-pair and face blocks (unscaled by s_K)
    int lsym = 0;                        // S_(-d) == S_d: the paired-direction instantiation
    int lhex = 0;                        // native hex8 cells: the 27-point instantiation
    // the update pass's preconditioner by node class (when the lumped mass is uniform per boundary class): class =
    // (27 boundary types) << 3 | Dirichlet mask per node, one representative node per class, its packed block
    // inverse and 9-float operator (rebuilt with the per-node inverse)
    const uint8_t *lcls = nullptr;  // [N]
    const uint32_t *lrep = nullptr;  // [kLatClasses], 0xFFFFFFFF: no node of the class
    uint4 *lcinv6 = nullptr;         // [kLatClasses]
    float *lcinv9 = nullptr;         // [9 kLatClasses]
    float4 *lcz = nullptr;           // [2 kLatClasses] the same inverse unpacked, {a00 a01 a02 a11} {a12 a22 0 0}:
                                     // loaded unconditionally in the K_eff prologue (lattice.inc, ZR)
};
// lattice work items for planes [lk0, lk1) (lattice.cpp): sets lnbx, lnby, lL, lnwork, ntiles
void lattice_plan(DevTiles &t);

struct HostTiles
{
    uint32_t ntiles = 0, max_tile_nodes = 0;
    std::vector<uint4> planes[3];
    std::vector<uint32_t> mat;
    std::vector<uint32_t> tile_elem_off, tile_node_off, tile_nodes, csr_off, node_part_off, node_part_slot,
        tile_slot;
    std::vector<uint16_t> csr_ent;
    std::vector<uint2> eid;        // [E] local corner ids
    std::vector<uint2> epos;       // [E] tile-relative local-CSR positions of the 4 (element, corner) pairs
    std::vector<uint4> eid8, epos8;  // hex8: [E] the 8 corners' local ids / local-CSR positions (u16 pairs)
    std::vector<uint8_t> tile_affine;  // hex8: 1 when every hex of the tile is a parallelepiped (constant J)
    std::vector<float> tcoord[3];  // [total] tile-relative coordinates (when node_coords are given)
};

// max_nodes: distinct nodes per tile (kMaxTileNodes; the pipelined kernel keeps one node per lane: 256)
// corners: 4 (tet4) or 8 (hex8: eid8/epos8 records, local-CSR entries element_local * 8 + corner)
int build_tiles(const cwf_system_desc *d, HostTiles &out, uint32_t max_nodes = kMaxTileNodes,
                uint32_t max_elems = kTileElems, int corners = 4);
// true when the supplied gradients / volumes are those of the supplied node coordinates (so FAST may
// recompute them on the fly instead of streaming them)
bool geometry_matches(const cwf_system_desc *d);
uint64_t spread21(uint64_t v);  // 21-bit Morton spread (one axis of a 63-bit key)
// recursive coordinate bisection of order's items (centroids c[3 id], mean extents ext) into leaves of at most
// max_elems, cut between layers (tiles.cpp); leaf_end receives each leaf's end in `order`
void rcb_partition(const std::vector<double> &c, const double ext[3], std::vector<uint32_t> &order,
                   uint64_t max_elems, std::vector<uint64_t> &leaf_end, int tdiv = 16, int wdiv = 16);

// FAST tet "fan groups" (groups.cpp): tets grouped around a shared edge (a, b) -- a closed or open fan of
// up to 6 tets {a, b, r_i, r_{(i+1) mod 6}} -- so one lane computes a group with its <= 8 nodes in
// registers and pushes one force per node instead of one per (tet, corner). A Kuhn-split hex is one
// closed 6-tet fan around its diagonal.
struct GroupTiles
{
    uint32_t ntiles = 0, ngroups = 0, max_tile_nodes = 0, max_tile_slots = 0;
    double tets_per_group = 0.0;
    // [G] 9-bit local ids of slots a b r0 .. r5 (3 per word, words 0-2), f << 27 in word 0, material << 27
    // in word 1 (groups are single-material), word 3: the 4-bit rank of each used slot in its node's run
    // (push position = run start + rank)
    std::vector<uint4> grec;
    std::vector<uint4> hdr;                // [ntiles] {first group, #groups, first tile node, #nodes}
    std::vector<uint32_t> tile_nodes;      // [T] global node | owner bit 31
    std::vector<uint32_t> run;             // [T] padded run begin | end << 16
    std::vector<float> tcoord[3];          // [T] tile-relative coordinates
    std::vector<uint32_t> node_part_off, tile_slot;  // [N+1] node -> slot range; [T] node-major slot
    std::vector<uint32_t> tet_group;       // [E] group of each tet (validation)
};
// nt: lanes per workgroup (one group per lane); max_nodes <= 512 (9-bit local ids); slot_budget: LDS push slots
// order_lanes: bank-aware lane order within each tile (groups.cpp); off where only the tiles' node sets matter
int build_group_tiles(const cwf_system_desc *d, GroupTiles &out, uint32_t nt, uint32_t max_nodes,
                      uint32_t slot_budget, bool order_lanes = true);

// Structured Kuhn blocks (lattice.cpp, lattice.inc): the 15 node-pair offsets of a Kuhn node's row (the node,
// +-x, +-y, +-z, +-(1,1,0), +-(1,0,1), +-(0,1,1), +-(1,1,1)) and the 46 corner pairs (c, c') of one cell that share
// a tet, with the offset index of c' - c
constexpr int kLatOffsets = 15, kLatPairs = 46;
constexpr int kLatOff[kLatOffsets][3] = {{0, 0, 0},  {1, 0, 0},  {-1, 0, 0},  {0, 1, 0},   {0, -1, 0},
                                         {0, 0, 1},  {0, 0, -1}, {1, 1, 0},   {-1, -1, 0}, {1, 0, 1},
                                         {-1, 0, -1}, {0, 1, 1}, {0, -1, -1}, {1, 1, 1},   {-1, -1, -1}};
constexpr int kLatPair[kLatPairs][2] = {
    {0, 0}, {0, 1}, {0, 2}, {0, 3}, {0, 4}, {0, 5}, {0, 6}, {0, 7},  // corner 0: every corner
    {1, 0}, {1, 1}, {1, 3}, {1, 5}, {1, 7},                          //
    {2, 0}, {2, 2}, {2, 3}, {2, 6}, {2, 7},                          //
    {3, 0}, {3, 1}, {3, 2}, {3, 3}, {3, 7},                          //
    {4, 0}, {4, 4}, {4, 5}, {4, 6}, {4, 7},                          //
    {5, 0}, {5, 1}, {5, 4}, {5, 5}, {5, 7},                          //
    {6, 0}, {6, 2}, {6, 4}, {6, 6}, {6, 7},                          //
    {7, 0}, {7, 1}, {7, 2}, {7, 3}, {7, 4}, {7, 5}, {7, 6}, {7, 7}};  // corner 7: every corner
constexpr int kLatPairOff[kLatPairs] = {0,  1,  3,  7,  5,  9,  11, 13,  // 0 -> 0..7
                                        2,  0,  3,  5,  11,              // 1 -> 0 1 3 5 7
                                        4,  0,  1,  5,  9,               // 2 -> 0 2 3 6 7
                                        8,  4,  2,  0,  5,               // 3 -> 0 1 2 3 7
                                        6,  0,  1,  3,  7,               // 4 -> 0 4 5 6 7
                                        10, 6,  2,  0,  3,               // 5 -> 0 1 4 5 7
                                        12, 6,  4,  0,  1,               // 6 -> 0 2 4 6 7
                                        14, 12, 10, 6,  8,  4,  2,  0};  // 7 -> 0..7
// Structured native hex8 blocks (one trilinear hex per cell): all 26 neighbours and the node, the offsets as
// (+d, -d) pairs after the node itself, and all 64 corner pairs (c, c') of a cell in (c, c') order
constexpr int kLatHexOffsets = 27, kLatHexPairs = 64;
constexpr int kLatHexOff[kLatHexOffsets][3] = {
    {0, 0, 0},   {1, 0, 0},  {-1, 0, 0},  {-1, 1, 0}, {1, -1, 0},  {0, 1, 0},   {0, -1, 0},  {1, 1, 0},  {-1, -1, 0},
    {-1, -1, 1}, {1, 1, -1}, {0, -1, 1},  {0, 1, -1}, {1, -1, 1},  {-1, 1, -1}, {-1, 0, 1},  {1, 0, -1}, {0, 0, 1},
    {0, 0, -1},  {1, 0, 1},  {-1, 0, -1}, {-1, 1, 1}, {1, -1, -1}, {0, 1, 1},   {0, -1, -1}, {1, 1, 1},  {-1, -1, -1}};
constexpr int kLatHexPairOff[kLatHexPairs] = {0,  1,  5,  7,  17, 19, 23, 25, 2,  0,  3,  5,  15, 17, 21, 23,
                                              6,  4,  0,  1,  11, 13, 17, 19, 8,  6,  2,  0,  9,  11, 15, 17,
                                              18, 16, 12, 10, 0,  1,  5,  7,  20, 18, 14, 12, 2,  0,  3,  5,
                                              24, 22, 18, 16, 6,  4,  0,  1,  26, 24, 20, 18, 8,  6,  2,  0};
// f32 coefficient table: [15][3][3] stencil blocks, then [46][3][3] cell blocks (hex8: [27] and [64])
constexpr int kLatCoefPairs = 9 * kLatOffsets;
constexpr int kLatCoef = kLatCoefPairs + 9 * kLatPairs;
constexpr int kLatHexCoef = 9 * (kLatHexOffsets + kLatHexPairs);
// k_keff_lattice bricks: kLatBrickX x kLatBrickY columns of the strict interior, one thread per column
constexpr int kLatBrickX = 32, kLatBrickY = 8, kLatThreads = kLatBrickX * kLatBrickY;
constexpr uint32_t kLatClasses = 27 * 8;  // (boundary type along x, y, z: lo / inside / hi) x Dirichlet mask

struct Lattice
{
    uint32_t nx = 0, ny = 0, nz = 0;  // nodes per axis
    std::vector<uint32_t> plane;      // [nz] storage index of node (0, 0, k)
    std::vector<uint32_t> perm;       // when renumbered: internal (lexicographic) index -> caller's node
    float coef[kLatHexCoef] = {};  // Kuhn: the first kLatCoef
    bool sym = false;  // S_(-d) == S_d for every direction (k_keff_lattice's paired form)
    bool hex = false;  // native hex8 cells (27-point stencil)
};
// true when the desc is a Kuhn-split box lattice with one gradient / volume set per Kuhn type (lattice.cpp);
// allow_perm: the handle may renumber (otherwise the nodes must already be lexicographic within planes)
bool detect_lattice(const cwf_system_desc *d, bool allow_perm, Lattice &L, std::string *why = nullptr);

constexpr uint32_t kPartOffBits = 0x1fffffffu;  // node_part_off value bits (the rest: bc_mask, off_mask)
// cap of the first batch of PCG iterations enqueued before the first control-block read-back (abi.cpp: sized from
// the handle's last two solves when they agree)
constexpr uint64_t kMaxFirstBatch = 2048;
// FAST PCG applies x += alpha_j p_j every kXLag iterations, from the last kXLag search directions (one p
// buffer each, rotating), instead of re-reading x and p every iteration
constexpr unsigned kXLag = 4;

struct DevSys
{
    uint32_t N = 0;  // nodes
    uint32_t E = 0;  // tets
    uint32_t D = 0;  // dofs
    uint32_t M = 0;  // materials
    uint32_t Nown = 0;  // owned nodes [0, Nown) (== N unless the handle is a shard; ghosts follow)
    const uint4 *erec = nullptr;
    const float *vol = nullptr;
    const uint32_t *mat = nullptr;
    const double *dmat = nullptr;
    const float *mass = nullptr;
    const uint32_t *mask = nullptr;
    const uint32_t *off = nullptr;
    const uint32_t *inc = nullptr;
    // node-tile PARITY K_eff (kernels_parity.hip k_keff_parity_tile; built at the first PARITY use): tile b = nodes
    // [256 b, 256 b + 256); ptile_tets[ptile_off[b] ..] its incident tets, ascending; pinc[j] = (the tile-local index
    // of incidence j's tet) << 2 | corner, for every incidence j of the node -> incidence CSR (off / inc order)
    const uint32_t *ptile_off = nullptr;
    const uint32_t *ptile_tets = nullptr;
    const uint32_t *pinc = nullptr;
    // compact tiles (unsharded handles): tile b = the nodes ptile_nodes[256 b ..] (0xFFFFFFFF pads), grown by
    // breadth-first search over the mesh so a tile is a blob, not a strip of the caller's order; pntile tiles. The
    // PCG loop's p.Ap chunk partials are then a separate pass (the tiles are not runs of consecutive DOFs)
    const uint32_t *ptile_nodes = nullptr;
    uint32_t pntile = 0;
    double sK = 1.0;  // stiffness_scale
    double sM = 0.0;  // mass_factor
    int iso = 0;      // every material has the isotropic Voigt zero pattern
    float d1[36] = {};  // M == 1: the material's D in f32, in the FAST kernels' table order (kernel
                        // arguments, so the element math reads it from SGPRs)
    int hex = 0;      // elements are hex8 (FAST only): hconn / hcoord feed the hex block-Jacobi setup
    const uint32_t *hconn = nullptr;  // [8E] hex corner nodes (Gmsh order)
    const double *hcoord = nullptr;   // [3N] node coordinates
    const float *hgrad = nullptr;     // [24E] element-centre dN_a/dx (the post stack's centroid strain)
    DevTiles t{};     // FAST-mode tiles (empty in a PARITY-only handle)
};

// Device-resident PCG control block: scalars of pcg.cpp:696-918 live here so that the
// iteration loop never waits on the host (the host polls `active` every few iterations).
struct Ctl
{
    double rho, alpha, beta, tol, res, rhs_norm, rhs_norm_raw, alpha_last, beta_last, denom, rr, rz;
    unsigned long long iterations;  // completed iterations
    int active;                     // 1 while the loop should keep running
    int converged;
    int error;       // cwf_status (0 = none)
    int error_iter;  // iteration index for the error context
    double rho2[2];  // FAST: rho by iteration parity (written by one kernel, read by the next)
    double alpha_h[kXLag];  // FAST: alpha of iteration j at [j % kXLag] (the lazy x update, spmv_tiles.hip)
};

// the resident solve of a structured block (resident.hip, resident.cpp): one persistent launch per PCG solve, one
// workgroup per box of the lattice, the vectors on chip. state: 0 not planned yet, 1 planned, -1 not eligible
struct ResidentPlan
{
    int state = 0;
    unsigned G = 0, npt = 0, nph = 0;  // workgroups; own / halo entries per thread (the instantiation)
    unsigned own_stride = 0, halo_stride = 0, npub = 0;
    size_t lds = 0;                     // dynamic LDS: the largest box image
    unsigned dims[3] = {0, 0, 0};       // boxes along x, y, z
    unsigned max_own = 0, max_halo = 0;
    uint64_t halo_total = 0;            // halo entries over every box (records read per phase)
    const uint4 *hdr = nullptr, *own = nullptr, *halo = nullptr;
    const float4 *tcoef = nullptr;  // [G][12][nOff][3] each box's boundary types' stencils
    float *pub = nullptr;
    double *sh = nullptr;
    uint32_t tag = 1;  // the next solve's granule tag base (resident.hip: phase j publishes tag + j + 1)
    bool shard = false;         // a PEER slab shard: ghost records in the mailbox, rank totals across ranks
    uint64_t remote_sends = 0;  // a shard: Ap granules stored into the neighbours' mailboxes per phase
    uint64_t ghost_total = 0;   // a shard: ghost halo entries over every box (one Ap granule read each per phase)
};

struct DevBuf
{
    void *p = nullptr;
    size_t bytes = 0;
};

}  // namespace cwf

struct cwf_hip_system
{
    int device = 0;
    hipStream_t stream = nullptr;
    int mode = CWF_MODE_PARITY;
    cwf::DevSys ds{};
    uint64_t reduction_block = 256;
    uint64_t reduction_partials = 1;
    // owned HBM
    std::vector<void *> owned;
    uint64_t bytes = 0;
    // solver scratch (f32 dofs) and partials
    // Ap is scratch (apply_keff staging, PARITY's K p, the prologues' K x); FAST PCG never reads it
    float *x = nullptr, *r = nullptr, *p = nullptr, *z = nullptr, *Ap = nullptr, *rhs = nullptr, *tmp = nullptr;
    float *p2 = nullptr, *p3 = nullptr, *p4 = nullptr;  // FAST: p_j lives in {p, p2, p3, p4}[(j + 1) % 4]
    // the fused lattice iteration (lattice_fused.inc): r and Ap by launch parity (r_j in {r2, r}[j & 1], Ap_j in
    // {Ap, ap2}[j & 1]) and the launches' five shares per workgroup, [2][5][lnwork]
    float *r2 = nullptr, *ap2 = nullptr;
    double *fsh = nullptr;
    double *g_fsh = nullptr;  // a shard's all-gathered rank totals of the fused shares, [nranks][8] (one rank: [8])
    bool cls_global = false;  // a shard's ghost class bytes hold their owners' (global) classes
    // a failed attach after the handle's plan was rewritten for its owned rows (comm.cpp cwf_hip_comm_attach): every
    // later call but destroy refuses the handle instead of computing a partial plan's rows
    bool unusable = false;
    int fused_agreed = -1;    // a shard: every rank runs the fused iteration (1) or none (0); -1: not asked yet
    int px_agreed = 0;        // ... and exchanges inside its launches (PEER, every rank eligible)
    int res_agreed = 0;       // ... and every rank runs the resident solve (PEER slab shards, every rank eligible)
    int32_t px_send_k[2] = {-1, -1};  // the lattice plane of each neighbour slot's send segment
    uint32_t px_ebase = 0;            // the communicator's epoch before the solve's launch 0
    unsigned fused_grid = 0, fused_items = 0;  // the fused launch's grid and the work items it was sized for
    bool fused_on = false;                     // CWF_FUSED as it was when the handle first asked
    cwf::ResidentPlan res;                     // the resident solve (resident.cpp), planned at the first FAST solve
    float *inv = nullptr;   // block Jacobi [9N]; FAST: the symmetrised operator the solve applies
    float *inv6 = nullptr;  // FAST: the same block packed to 16 B per node (blockinv_pack.hpp)
    // inv / inv6 hold the FAST operator for (inv_sK, inv_sM): the block inverse depends only on the handle's
    // immutable element data and mask and on the two scalars, so a FAST solve with unchanged scalars (every
    // fixed-step Newmark step) reuses it instead of rebuilding it (pcg.cpp:749 rebuilds per solve; same values)
    bool inv_fast = false;
    double inv_sK = 0.0, inv_sM = 0.0;
    double *part0 = nullptr, *part1 = nullptr, *part2 = nullptr;  // chunk / block partials
    // PARITY streamed scalar folds (kernels_parity.hip, single handle, 256-DOF chunks): tagged 16-B chunk-partial
    // granules [2 chunks] (null: the separate fold kernels) and the tag of the last streamed launch
    double *fgran = nullptr;
    uint32_t fgran_tag = 0;
    uint64_t part_cap = 0;
    // FAST-mode internal node renumbering (Morton order of the coordinates): perm[i] = caller's node of
    // internal node i; every vector crossing the ABI is gathered / scattered through it (pbuf: 13N staging)
    uint32_t *perm = nullptr;
    float *pbuf = nullptr;
    cwf::Ctl *ctl = nullptr;       // device
    cwf::Ctl *ctl_host = nullptr;  // pinned
    double *scal = nullptr;        // device scalar scratch
    double *hist = nullptr;        // device residual history
    uint64_t hist_cap = 0;
    uint64_t hist_count = 0;
    std::vector<uint32_t> lat_plane;  // structured block: host copy of ds.t.lplane (attach derives the owned planes)
    uint64_t last_iters = 0, prev_iters = 0;  // iterations of the last two solves on this handle (first batch size)
    std::string err, ctx;
    // live K_eff timing (cwf_hip_system_set_timing)
    int timing = 0;
    std::vector<hipEvent_t> ev;  // 2 per enqueued iteration of one batch
    double keff_ms = 0.0;
    uint64_t keff_count = 0;
    // shard of a multi-rank system (cwf_hip_system_attach); nranks == 1 otherwise
    cwf_hip_comm *comm = nullptr;
    int rank = 0, nranks = 1;
    hipStream_t own_stream = nullptr;  // the handle's stream while a LOCAL comm's stream is borrowed
    std::vector<int32_t> nbr;
    std::vector<uint64_t> send_off, recv_off;
    uint32_t *send_idx = nullptr;  // [nsend] owned local node ids, per neighbour
    float *sendbuf = nullptr;      // [kMaxHaloVecs][3 nsend]
    uint64_t nsend = 0;
    // all-gathered per-rank scalars, slot of rank r at [r * count]
    double *g_pap = nullptr;   // [nranks]      p.Ap
    double *g_rrz = nullptr;   // [2 nranks]    {r.r, r.z}
    double *g_init = nullptr;  // [2 nranks]    {rhs.rhs, r0.r0}
    double *g_rz0 = nullptr;   // [nranks]      r0.z0
    // sharded PARITY: every rank's 256-DOF chunk partials all-gathered into slot [r * pstride, (r+1) * pstride)
    // (zero-padded past the rank's own chunk count) and folded in that order on every rank = the global chunk
    // order of pcg.cpp:170-207, since the owned node ranges are ascending by rank and aligned to whole chunks
    double *gp0 = nullptr, *gp1 = nullptr;
    size_t gp_bytes = 0;  // the slot block gp0 starts (gp1 = gp0 + nranks * pstride)
    uint32_t pstride = 0;
    uint64_t gbegin = 0;            // global id of the first owned node (cwf_hip_system_attach)
    std::vector<uint64_t> node_gid;  // the plan's global id of every local node (when given): the halo check
    bool owned_contiguous = false;  // owned local i = global gbegin + i
    bool sharded() const { return nranks > 1 || comm != nullptr; }
};

struct cwf_hip_comm
{
    int kind = 0;  // 0 = LOCAL (one process, one device, shared stream), 1 = RCCL, 2 = PEER (peer.hip)
    int nranks = 1;
    int rank = 0;  // RCCL / PEER: this process's rank
    int device = 0;
    void *nccl = nullptr;
    hipStream_t stream = nullptr;                // LOCAL: the stream every member enqueues on
    std::vector<cwf_hip_system *> members;       // LOCAL: by rank
    // PEER: this rank's IPC-exported mailbox, the peers' mapped ones, their ghost counts and where my ghosts go
    // in them, the exchange-step epoch and the push kernel's ticket
    cwf_hip_system *peer_member = nullptr;
    void *mbox = nullptr;
    size_t mbox_bytes = 0;
    int mbox_kind = 0;  // CWF_PEER_MAILBOX_*
    uint32_t *ticket = nullptr;  // [0]: the exchange step's ticket; [32]: the sticky device error word
    std::vector<void *> peer_mbox;
    std::vector<uint64_t> peer_nghost, peer_recv_off;
    std::vector<int> peer_same_device;  // peer p's mailbox is on this rank's device (PCI bus id)
    uint32_t epoch = 0;
};

namespace cwf
{
// set the handle's (or global) error and return the code
int set_error(cwf_hip_system *h, int code, const std::string &msg, const std::string &ctx = "");
int hip_fail(cwf_hip_system *h, hipError_t e, const char *what);

// ---- kernels_parity.hip ----
uint32_t parity_chunk_count(const cwf_hip_system *h);
void parity_keff(const cwf_hip_system *h, const float *x, float *y, bool sanitize, const Ctl *ctl, hipStream_t st);
void parity_keff_ds(const DevSys &s, const float *x, float *y, bool sanitize, const Ctl *ctl, hipStream_t st);
void parity_block_jacobi(const cwf_hip_system *h, float *inv, hipStream_t st);
void hex_block_jacobi(const cwf_hip_system *h, float *inv, hipStream_t st);  // hex8 diagonal blocks -> inverse
void parity_dot_partials(const cwf_hip_system *h, const float *a, const float *b, const float *c, double *pab,
                         double *pac, const Ctl *ctl, hipStream_t st);
void parity_dot_partials_n(uint32_t D, uint32_t B, const float *a, const float *b, const float *c, double *pab,
                           double *pac, const Ctl *ctl, hipStream_t st);
void parity_fold(const double *part, uint32_t count, double *out, hipStream_t st);
void parity_init_scalars(cwf_hip_system *h, const double *p_rhs, const double *p_rr, uint32_t count, double rel_tol,
                         hipStream_t st);
void parity_init_rho(cwf_hip_system *h, const double *p_rz, uint32_t count, hipStream_t st);
void parity_alpha(cwf_hip_system *h, const double *p_pap, uint32_t count, hipStream_t st);
void parity_update(cwf_hip_system *h, const float *rhs, double *prr, double *prz, hipStream_t st);
// the PCG loop's K_eff p and the chunk partials of p . Ap over the owned nodes (fused for 256-DOF chunks); and
// parity_update's r . r / r . z partials likewise
void parity_keff_dot(const cwf_hip_system *h, const float *p, float *Ap, const Ctl *ctl, double *pdot, hipStream_t st);
void parity_beta(cwf_hip_system *h, const double *p_rr, const double *p_rz, uint32_t count, hipStream_t st);
void parity_p_update(cwf_hip_system *h, hipStream_t st);
void parity_pcg_init(cwf_hip_system *h, const float *rhs, double rel_tol, hipStream_t st);
void parity_pcg_iteration(cwf_hip_system *h, const float *rhs, hipStream_t st, hipEvent_t e0 = nullptr,
                          hipEvent_t e1 = nullptr);
void launch_init_residual(const cwf_hip_system *h, const float *rhs, hipStream_t st);
void launch_precond(const cwf_hip_system *h, const Ctl *ctl, hipStream_t st);
void launch_p_init(const cwf_hip_system *h, hipStream_t st);

// ---- kernels_fast.hip ----
// dst[w i + k] = src[w perm[i] + k] (gather = caller order -> internal) / dst[w perm[i] + k] = src[w i + k]
void copy16(const void *a, void *b, uint64_t bytes, hipStream_t st);  // bandwidth probe copy
void perm_gather(const uint32_t *perm, const float *src, float *dst, uint32_t N, int w, hipStream_t st);
void perm_scatter(const uint32_t *perm, const float *src, float *dst, uint32_t N, int w, hipStream_t st);
uint32_t fast_block_count(const cwf_hip_system *h);
uint32_t fast_dot_blocks(uint32_t D);
void fast_keff(const cwf_hip_system *h, const float *x, float *y, bool sanitize, const Ctl *ctl, double *part,
               hipStream_t st);
void fast_keff_ds(const DevSys &s, const float *x, float *y, bool sanitize, const Ctl *ctl, double *part,
                  hipStream_t st);
void fast_dot(const float *a, const float *b, const float *c, uint32_t D, double *pab, double *pac, hipStream_t st);
void fast_fold(const double *part, uint32_t count, double *out, hipStream_t st);
void fast_pcg_init(cwf_hip_system *h, const float *rhs, double rel_tol, hipStream_t st);
void fast_tiles_pcg(cwf_hip_system *h, unsigned it, hipStream_t st, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
void fast_update_pcg(cwf_hip_system *h, const float *rhs, unsigned it, hipStream_t st);
void fast_check_pcg(cwf_hip_system *h, unsigned it, hipStream_t st);
void fast_flush_x(cwf_hip_system *h, const float *rhs, hipStream_t st);  // the lazy x terms still pending
void fast_tiles_pcg_dry(cwf_hip_system *h, unsigned abl, int reps, hipStream_t st);
// the fused lattice iteration (lattice_fused.inc): one launch per PCG iteration on an unsharded structured block
bool fast_fused(const cwf_hip_system *h);
void fast_fused_init(cwf_hip_system *h, const float *rhs, double rel_tol, hipStream_t st, bool launch0 = true);
void fast_fused_iteration(cwf_hip_system *h, unsigned it, hipStream_t st, hipEvent_t e0 = nullptr,
                          hipEvent_t e1 = nullptr);
void fast_fused_check(cwf_hip_system *h, unsigned it, hipStream_t st);
void fast_fused_finish(cwf_hip_system *h, hipStream_t st);
void fast_fused_launch0(cwf_hip_system *h, hipStream_t st);
float *fast_fused_ap(cwf_hip_system *h, unsigned j);
void fast_fused_rank_totals(cwf_hip_system *h, unsigned j, hipStream_t st);
const double *fast_fused_shares(const cwf_hip_system *h, unsigned j, unsigned *stride, unsigned *count);
void fast_fused_cls_out(cwf_hip_system *h, hipStream_t st);  // owned class bytes -> tmp (x components)
void fast_fused_cls_in(cwf_hip_system *h, hipStream_t st);   // ghost class bytes <- tmp
constexpr size_t kFusedSlotHost = 8;  // doubles per rank of the gathered fused totals (lattice_fused.inc kFusedSlot)
// comm.cpp: the sharded fused iteration (one launch + one exchange: the rank totals and the Ap halo)
int sharded_fused_init(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs, double rel_tol);
int sharded_fused_iteration(const std::vector<cwf_hip_system *> &g, unsigned it, hipEvent_t e0, hipEvent_t e1);
int group_fused(const std::vector<cwf_hip_system *> &g);  // 1 fused, 0 two-kernel, < 0 error
// the resident solve (resident.cpp / resident.hip): whether this handle runs it (plans it at the first call; CWF_RESIDENT
// = 0 turns it off), the launch (fast_fused_init has run; one launch runs every iteration) and its residency query
bool resident_ready(cwf_hip_system *h);
void launch_pcg_resident(cwf_hip_system *h, uint32_t max_it, hipStream_t st, hipEvent_t e0, hipEvent_t e1);
int resident_blocks_per_cu(const DevSys &s, unsigned npt, unsigned nph, size_t lds, bool shard);
size_t resident_static_lds(const DevSys &s, bool small, bool shard);  // the instantiation's static LDS bytes
uint64_t resident_offchip_bytes(const cwf_hip_system *h);  // per phase: halo records read, surface records and shares
// a PEER slab shard's resident solve: planned on the rank's own at the schedule vote (group_fused), run only when every
// rank planned one (res_agreed); the init is the fused one's without its launch 0 and exchange step (comm.cpp)
bool resident_shard_ready(cwf_hip_system *h);
bool resident_on(const cwf_hip_system *h);  // the handle's FAST solves run the resident solve (planned and agreed)
int sharded_resident_init(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs, double rel_tol);
int sharded_fused_end(const std::vector<cwf_hip_system *> &g);  // after the last launch (PEER in-kernel epochs)

unsigned fast_tile_blocks(const DevSys &s);
unsigned fast_pipe_grid(const DevSys &s);
unsigned fast_update_blocks(const DevSys &s, bool flush);
unsigned fast_rrz_shares(const DevSys &s, unsigned it);  // the {r.r, r.z} shares iteration it's update pass writes  // grid of update pass (lazy-x iteration or not)
// sharded FAST PCG (comm.cpp orchestrates, spmv_tiles.hip / kernels_fast.hip launch)
// post.hip: derived fields (derived_fields.cpp:139-211) -> f32 [13 E] / [13 N] (either may be NULL)
void derived_fields(cwf_hip_system *h, const float *u, float *elem_out, float *node_out, hipStream_t st);
bool fast_direct_fold(const cwf_hip_system *h);  // unsharded: consumers fold per-workgroup shares
void fast_fold_pap(cwf_hip_system *h, hipStream_t st);  // local p.Ap shares -> g_pap[rank]
void fast_fold_rrz(cwf_hip_system *h, unsigned it, hipStream_t st);  // local r.r / r.z shares -> g_rrz[2 rank]
void halo_pack(cwf_hip_system *h, const float *v, hipStream_t st, float *dst = nullptr);  // dst: sendbuf
void fast_block_inverse(cwf_hip_system *h, hipStream_t st);  // parity BJ, symmetrised + packed to inv6
void fold_pair(const double *a, const double *b, uint32_t n, double *out, hipStream_t st);
void fast_init_scalars_strided(cwf_hip_system *h, const double *p_rhs, const double *p_rr, uint32_t count,
                               uint32_t stride, double rel_tol, hipStream_t st);
void fast_rho_from(cwf_hip_system *h, const double *p_rz, uint32_t count, hipStream_t st);
// comm.cpp
struct Gather
{
    double *cwf_hip_system::*buf;
    size_t count;
};
int comm_exchange(const std::vector<cwf_hip_system *> &g, std::initializer_list<Gather> gathers,
                  float *cwf_hip_system::*vec);
constexpr size_t kMaxHaloVecs = 3;  // halo vectors of one exchange step
constexpr int kMaxPeers = 16;       // ranks of a PEER communicator
// peer.hip: the PEER communicator's mailbox (at attach), its exchange step, and its teardown
int peer_attach(cwf_hip_system *h);
// fold (optional): the rank's own slot of gather 0 is computed in the step from this rank's per-workgroup shares
// (k_fold_pair's order), in place of a fold launch before it
struct PeerFold
{
    const double *a, *b;  // shares of slot 0 and (b) slot 1
    uint32_t n;
    uint32_t k5_stride = 0;  // > 0: the fused iteration's five share arrays a[q k5_stride + i] into slots 0..4, in
                             // k_fused_rank_totals' order (fold_k, 256 threads)
};
int peer_exchange(cwf_hip_system *h, std::initializer_list<Gather> gathers, const std::vector<float *> &vecs,
                  const PeerFold *fold = nullptr);
void peer_release(cwf_hip_comm *cm);
// The fused lattice iteration's exchange inside its own launch (PEER only; lattice_fused.inc): launch j of a solve
// pushes its Ap send rows (whole owned planes) straight into the neighbours' receive areas and, from its last
// workgroup, the rank totals into every rank's gather area and epoch ebase + j + 1 into every peer's flag; launch
// j + 1 waits for every peer's epoch ebase + j in its prologue. Launch arguments (this launch's parities):
struct FusedPeerArgs
{
    float *dst[2];          // send entry e: the neighbour's receive area at my segment's first float
    uint32_t dst_bytes[2];  // the descriptor range of dst[e] (0: no entry)
    int32_t send_k[2];      // the lattice plane entry e sends (-1: none); row (i, j) -> float 3 (j nx + i)
    double *gdst[kMaxPeers];    // per rank p: p's gather area, my slot (this rank's too)
    uint32_t *flag[kMaxPeers];  // per rank p != rank: p's flag line for my rank
    const uint32_t *flags;      // my flag lines (peer p's first word at flags[16 p])
    uint32_t *ticket, *sticky, *done;
    const float *arecv;  // my receive area of the previous launch's epoch (the ghost Ap rows), launch j > 0
    uint32_t epoch, nranks, rank;
};
// this rank's half of the collective decision (a host check of the halo plan: every send segment one whole owned
// plane in plane order, <= 2 of them; ranks on one device only while all their grids are resident together)
bool peer_fused_eligible(cwf_hip_system *h);
void peer_fused_args(const cwf_hip_system *h, unsigned j, FusedPeerArgs &pe, const double **gath_prev);
int peer_fused_begin(cwf_hip_system *h);  // before launch 0: the epoch base; the launch ticket cleared
int peer_fused_end(cwf_hip_system *h);    // after the solve: the communicator's epoch = the last launch that pushed
unsigned pcg_lattice_resident_count(const DevSys &s);  // resident workgroups of the fused launch
// the resident solve of a PEER slab shard (resident.hip): where its cross-rank granules go and come from. Each mailbox
// has a resident area by phase parity: the rank totals ([nranks][5] 16-B granules) and the ghosts' Ap granules
// ([nghost] 16 B, the ghosts' local order). Per neighbour slot e (the halo plan's k): the neighbour's granule area at
// my send segment; per rank p: p's rank-total area (my slot included)
struct ResPeerArgs
{
    uint32_t nranks = 1, rank = 0;
    float *rdst[2][2] = {};          // [e][parity] neighbour e's ghost granules of my segment
    uint32_t rdst_bytes[2] = {};     // 16 x my segment for e
    const float *grecv[2] = {};      // [parity] my ghosts' granules (written by the neighbours)
    uint32_t grecv_bytes = 0;
    uint32_t *tot[kMaxPeers][2] = {};  // [p][parity] rank p's rank-total area (granule (r, q) at 16 (5 r + q))
    const uint32_t *tot_mine[2] = {};  // [parity] my rank-total area
};
size_t peer_resident_bytes(int nranks, uint64_t nghost);  // the resident area, both parities (peer_attach adds it)
void peer_resident_args(const cwf_hip_system *h, ResPeerArgs &pa);
int peer_resident_clear(cwf_hip_system *h);  // tags 0 in this rank's resident area (before any resident solve)
int comm_exchange_vecs(const std::vector<cwf_hip_system *> &g, std::initializer_list<Gather> gathers,
                       const std::vector<std::vector<float *>> &vecs);
int comm_allgather(const std::vector<cwf_hip_system *> &g, double *cwf_hip_system::*buf, size_t count);
int comm_halo(const std::vector<cwf_hip_system *> &g, float *cwf_hip_system::*vec);
int sharded_pcg_init(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs, double rel_tol);
int sharded_parity_init(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs, double rel_tol);
int sharded_parity_iteration(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs,
                             hipEvent_t e0, hipEvent_t e1);
int fast_pcg_iteration_group(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs,
                             unsigned it, hipEvent_t e0, hipEvent_t e1);

// ---- stepper.hip ----
void stepper_predictor(uint32_t D, const float *u, const float *v, const float *a, float *up, float *vp, double dt,
                       double beta, double gamma, hipStream_t st);
void stepper_assemble_rhs(uint32_t N, const float *mass, const float *u, const float *v, const float *a,
                          const float *f, float *rhs, float *damp, const double *c6, double ralpha, hipStream_t st);
void stepper_rhs_damping(uint32_t D, float *rhs, const float *kd, float bf, hipStream_t st);
void stepper_clamp(uint32_t N, const uint32_t *mask, const float *bcv, const float *u, float *rhs, hipStream_t st);
void stepper_update(uint32_t D, const float *x, const float *up, const float *vp, float *u, float *v, float *a,
                    float ib, float gob, hipStream_t st);
void stepper_scaled_load(uint32_t D, const double *base, const double *pattern, double scale, float *f,
                         hipStream_t st);

}  // namespace cwf
