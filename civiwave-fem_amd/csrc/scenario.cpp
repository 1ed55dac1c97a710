// scenario.cpp -- native scenario driver: YAML config + Gmsh mesh -> packed buffers ->
// device Newmark steps -> VTU frames / probe CSV, the host side above the C-ABI written in C++ (the
// reference's own language). The order is the viewer backend's (src/ui/viewer.cpp:200-277):
//   load_config_from_file -> load_gmsh_file -> pre::run (material binding, preprocess.cpp:48-84,284-405)
//   -> pack::build_packed_buffers (pack.cpp:61-235: loads.cpp:87-174 at t = 0, solver.cpp:312-352 Dirichlet)
//   -> Stepper; per frame step(simulation_time), simulation_time = telemetry.simulation_time + time_step,
//   OutputManager::handle_frame (output_manager.cpp:49-87: derived fields, VTU every vtu_stride frames,
//   probe rows every frame).
// Every fold is in the order of cwf/pack.py (the Python restatement), so both drivers produce the same
// bytes; tests/test_gpu_scenario.py compares them. Errors carry the reference's texts and breadcrumbs,
// prefixed like the Python driver ("config: ", "mesh: ", "preprocess: ").
#include <sys/stat.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <string>
#include <vector>

#include "cwf_internal.hpp"
#include "yaml_lite.hpp"

struct cwf_scenario
{
    int mode = CWF_MODE_PARITY, flags = 0;
    uint64_t N = 0, E = 0;
    // config (canonical JSON of cwf_config_json, read back with the YAML flow parser)
    yl::Node cfg;
    // mesh
    std::vector<double> coords;                     // [3N]
    std::vector<uint32_t> conn;                     // [E*K] element corners
    int K = 4;                                      // 4 tet4, 8 hex8 (FAST only)
    std::vector<uint32_t> elem_group;               // [E]
    std::vector<std::vector<uint32_t>> surf_nodes;  // per surface 3 or 4 nodes
    std::vector<uint32_t> surf_group;
    std::map<std::string, uint32_t> group_id;                  // name -> first id
    std::map<uint32_t, std::vector<uint32_t>> node_groups;     // id -> tagged nodes
    // packed
    std::vector<float> grads, volume, mass32, position0, external_force, bc_value;
    std::vector<double> mass64, D36;
    std::vector<uint32_t> mat, conn8, offsets, adj_elem, bc_mask, probes;
    std::vector<uint8_t> adj_local;
    uint32_t vtu_stride = 0;
    // device
    cwf_hip_system *sys = nullptr;
    cwf_hip_stepper *st = nullptr;
    double t_sim = 0.0;
    uint32_t frame = 0;  // index of the next frame to step
    int probe_header = 0;
    std::vector<float> u, v, a, efield, nfield;
};

namespace
{
using cwf::set_error;

struct ScenErr
{
    int code;
    std::string message;
    std::string context;
};

inline float safe_f32(double v)  // pack.cpp:41-57
{
    if (!std::isfinite(v))
        return (float)v;
    if (v > (double)FLT_MAX)
        return FLT_MAX;
    if (v < -(double)FLT_MAX)
        return -FLT_MAX;
    return (float)v;
}

std::string dirname_of(const std::string &p)
{
    const size_t s = p.find_last_of('/');
    return s == std::string::npos ? std::string(".") : p.substr(0, s);
}

bool exists(const std::string &p)
{
    struct stat sb;
    return stat(p.c_str(), &sb) == 0;
}

// run.py resolve_mesh_path: as given (cwd-relative, the reference), else next to the YAML file
std::string resolve_mesh_path(const std::string &cfg_path, const std::string &mesh_path)
{
    if ((!mesh_path.empty() && mesh_path[0] == '/') || exists(mesh_path))
        return mesh_path;
    const std::string here = dirname_of(cfg_path);
    const size_t s = mesh_path.find_last_of('/');
    const std::string base = s == std::string::npos ? mesh_path : mesh_path.substr(s + 1);
    for (const std::string &c : {here + "/" + mesh_path, here + "/" + base})
        if (exists(c))
            return c;
    return mesh_path;
}

// loads.cpp:63-85 evaluate_curve with libstdc++'s std::lerp
double lerp(double a, double b, double t)
{
    if ((a <= 0 && b >= 0) || (a >= 0 && b <= 0))
        return t * b + (1 - t) * a;
    if (t == 1)
        return b;
    const double x = a + t * (b - a);
    return ((t > 1) == (b > a)) ? (b < x ? x : b) : (b > x ? x : b);
}

double evaluate_curve(const yl::Node &pts, double time)
{
    if (pts.size() == 0)
        return 1.0;
    if (time <= pts.items[0].items[0].as_double())
        return pts.items[0].items[1].as_double();
    for (size_t i = 1; i < pts.size(); ++i)
    {
        const double t0 = pts.items[i - 1].items[0].as_double(), v0 = pts.items[i - 1].items[1].as_double();
        const double t1 = pts.items[i].items[0].as_double(), v1 = pts.items[i].items[1].as_double();
        if (time <= t1)
        {
            const double span = t1 - t0;
            return lerp(v0, v1, span > 0.0 ? (time - t0) / span : 0.0);
        }
    }
    return pts.items[pts.size() - 1].items[1].as_double();
}

double curve_scale(const cwf_scenario &sc, const yl::Node &load, double time)
{
    const yl::Node &name = load["scale_curve"];
    if (!name.is_scalar())
        return 1.0;
    const yl::Node &c = sc.cfg["curves"][name.as_string()];
    return c.defined() ? evaluate_curve(c, time) : 1.0;
}

double tri_area(const double *P, uint32_t i0, uint32_t i1, uint32_t i2)
{
    const double *p0 = P + 3ull * i0, *p1 = P + 3ull * i1, *p2 = P + 3ull * i2;
    const double v1[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
    const double v2[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
    const double cr[3] = {(v1[1] * v2[2]) - (v1[2] * v2[1]), (v1[2] * v2[0]) - (v1[0] * v2[2]),
                          (v1[0] * v2[1]) - (v1[1] * v2[0])};
    return 0.5 * std::sqrt((cr[0] * cr[0]) + (cr[1] * cr[1]) + (cr[2] * cr[2]));
}

// loads.cpp:87-174 / pack.py assemble_load_vector: gravity, then tractions, then point loads
std::vector<double> assemble_loads(const cwf_scenario &sc, double time)
{
    const uint64_t N = sc.N;
    std::vector<double> L(3 * N, 0.0);
    const yl::Node &ld = sc.cfg["loads"];
    double g[3];
    for (int k = 0; k < 3; ++k)
        g[k] = ld["gravity"].items[k].as_double();
    for (uint64_t n = 0; n < N; ++n)
        for (int k = 0; k < 3; ++k)
            L[3 * n + k] += sc.mass64[n] * g[k];
    const yl::Node &tr = ld["tractions"];
    for (size_t t = 0; t < tr.size(); ++t)
    {
        const auto it = sc.group_id.find(tr.items[t]["group"].as_string());
        if (it == sc.group_id.end())
            continue;
        const double scale = curve_scale(sc, tr.items[t], time);
        double val[3];
        for (int k = 0; k < 3; ++k)
            val[k] = tr.items[t]["value"].items[k].as_double();
        for (size_t s = 0; s < sc.surf_nodes.size(); ++s)
        {
            if (sc.surf_group[s] != it->second)
                continue;
            const auto &nd = sc.surf_nodes[s];
            double area = tri_area(sc.coords.data(), nd[0], nd[1], nd[2]);
            if (nd.size() == 4)
                area = area + tri_area(sc.coords.data(), nd[0], nd[2], nd[3]);
            const double share = (area * scale) / (double)nd.size();
            for (uint32_t n : nd)
                for (int k = 0; k < 3; ++k)
                    L[3ull * n + k] += share * val[k];
        }
    }
    const yl::Node &pl = ld["points"];
    for (size_t p = 0; p < pl.size(); ++p)
    {
        const auto it = sc.group_id.find(pl.items[p]["group"].as_string());
        if (it == sc.group_id.end())
            continue;
        const auto ng = sc.node_groups.find(it->second);
        if (ng == sc.node_groups.end())
            continue;
        const double scale = curve_scale(sc, pl.items[p], time);
        for (int k = 0; k < 3; ++k)
        {
            const double add = scale * pl.items[p]["value"].items[k].as_double();
            for (uint32_t n : ng->second)
                L[3ull * n + k] += add;
        }
    }
    return L;
}

void build(cwf_scenario &sc, const std::string &cfg_path)
{
    // ---- config
    cwf_config *cfg = nullptr;
    if (cwf_config_load_file(cfg_path.c_str(), &cfg))
        throw ScenErr{CWF_ERR_PARSE, std::string("config: ") + cwf_hip_last_error(nullptr),
                      cwf_hip_last_context(nullptr)};
    const std::string json = cwf_config_json(cfg);
    cwf_config_destroy(cfg);
    sc.cfg = yl::parse(json);
    // ---- mesh
    const std::string mpath = resolve_mesh_path(cfg_path, sc.cfg["mesh_path"].as_string());
    cwf_mesh *m = nullptr;
    if (cwf_mesh_load_file(mpath.c_str(), &m))
        throw ScenErr{CWF_ERR_PARSE, std::string("mesh: ") + cwf_hip_last_error(nullptr),
                      cwf_hip_last_context(nullptr)};
    cwf_mesh_info info{};
    cwf_mesh_get_info(m, &info);
    const uint64_t N = info.node_count, E = info.element_count, S = info.surface_count;
    sc.N = N;
    sc.E = E;
    sc.coords.resize(3 * N);
    cwf_mesh_nodes(m, sc.coords.data(), nullptr);
    std::vector<uint32_t> nodes8(8 * E);
    std::vector<uint8_t> geo(E);
    sc.elem_group.resize(E);
    cwf_mesh_elements(m, nodes8.data(), geo.data(), sc.elem_group.data(), nullptr);
    std::vector<uint32_t> sn(4 * S), sgrp(S);
    std::vector<uint8_t> sgeo(S);
    cwf_mesh_surfaces(m, sn.data(), sgeo.data(), sgrp.data());
    for (uint64_t s = 0; s < S; ++s)
        sc.surf_nodes.emplace_back(sn.begin() + 4 * s, sn.begin() + 4 * s + sgeo[s]);
    sc.surf_group = sgrp;
    for (uint64_t i = 0; i < info.group_count; ++i)
    {
        uint32_t dim = 0, id = 0;
        const char *name = nullptr;
        cwf_mesh_group(m, i, &dim, &id, &name);
        sc.group_id.emplace(name ? name : "", id);  // setdefault: the first id of a name
        const uint32_t *gn = nullptr;
        uint64_t cnt = 0;
        cwf_mesh_node_group(m, id, &gn, &cnt);
        if (cnt)
            sc.node_groups[id].assign(gn, gn + cnt);
    }
    cwf_mesh_destroy(m);
    // mesh.py to_tet_mesh: the reference's tet4 only; an all-hex8 mesh runs as native hex8 in FAST mode
    if (N == 0)
        throw ScenErr{CWF_ERR_SIZE, "preprocess: mesh has zero nodes", "mesh"};
    if (E == 0)
        throw ScenErr{CWF_ERR_SIZE, "preprocess: mesh has zero elements", "mesh"};
    sc.K = sc.mode == CWF_MODE_FAST && std::all_of(geo.begin(), geo.end(), [](uint8_t g) { return g == 8; }) ? 8 : 4;
    for (uint64_t e = 0; e < E; ++e)
        if (geo[e] != sc.K)
            throw ScenErr{CWF_ERR_UNSUPPORTED, "preprocess: only tetrahedron elements supported in Phase 3",
                          "elements\n[" + std::to_string(e) + "]"};
    sc.conn.resize((uint64_t)sc.K * E);
    for (uint64_t e = 0; e < E; ++e)
        for (int a = 0; a < sc.K; ++a)
            sc.conn[sc.K * e + a] = nodes8[8 * e + a];
    // ---- materials and their binding (preprocess.cpp:48-84)
    const yl::Node &mats = sc.cfg["materials"];
    std::vector<double> density;
    for (size_t i = 0; i < mats.size(); ++i)
    {
        const double Ey = mats.items[i]["E"].as_double(), nu = mats.items[i]["nu"].as_double();
        density.push_back(mats.items[i]["rho"].as_double());
        // materials.hpp:116-134 compute_lame / make_stiffness_matrix
        const double denom = (1.0 + nu) * (1.0 - 2.0 * nu);
        const double lam = (nu * Ey) / denom, mu = Ey / (2.0 * (1.0 + nu)), c = lam + 2.0 * mu;
        const double Dm[36] = {c, lam, lam, 0, 0, 0, lam, c, lam, 0, 0, 0, lam, lam, c, 0, 0, 0,
                               0, 0, 0, mu, 0, 0, 0, 0, 0, 0, mu, 0, 0, 0, 0, 0, 0, mu};
        sc.D36.insert(sc.D36.end(), Dm, Dm + 36);
    }
    if (density.empty())
        density.push_back(0.0);
    std::map<uint32_t, uint32_t> group_to_mat;
    const yl::Node &asg = sc.cfg["assignments"];
    for (size_t i = 0; i < asg.size(); ++i)
    {
        const std::string g = asg.items[i]["group"].as_string(), mname = asg.items[i]["material"].as_string();
        const auto gi = sc.group_id.find(g);
        if (gi == sc.group_id.end())
            throw ScenErr{CWF_ERR_PARSE, "preprocess: assignment references missing physical group '" + g + "'",
                          "assignments\n[" + std::to_string(i) + "]"};
        size_t mi = mats.size();
        for (size_t k = 0; k < mats.size(); ++k)
            if (mats.items[k]["name"].as_string() == mname)
            {
                mi = k;
                break;
            }
        if (mi == mats.size())
            throw ScenErr{CWF_ERR_PARSE, "preprocess: assignment references missing material '" + mname + "'",
                          "assignments\n[" + std::to_string(i) + "]"};
        group_to_mat.emplace(gi->second, (uint32_t)mi);
    }
    sc.mat.resize(E);
    for (uint64_t e = 0; e < E; ++e)
    {
        const auto it = group_to_mat.find(sc.elem_group[e]);
        if (it == group_to_mat.end())
            throw ScenErr{CWF_ERR_MATERIAL_RANGE, "preprocess: element physical group missing assignment",
                          "elements\n[" + std::to_string(e) + "]"};
        sc.mat[e] = it->second;
    }
    // ---- geometry (native preprocess, bit-exact with pre::run for tets)
    sc.grads.assign(24 * E, 0.f);
    sc.volume.assign(E, 0.f);
    sc.mass64.assign(N, 0.0);
    sc.mass32.assign(N, 0.f);
    sc.offsets.assign(N + 1, 0);
    sc.adj_elem.assign((uint64_t)sc.K * E, 0);
    sc.adj_local.assign((uint64_t)sc.K * E, 0);
    sc.conn8.assign(8 * E, 0);
    const int pst = sc.K == 8 ? cwf_preprocess_hex8(N, E, sc.coords.data(), sc.conn.data(), sc.mat.data(),
                                                     density.data(), mats.size(), sc.grads.data(),
                                                     sc.volume.data(), sc.mass64.data(), sc.mass32.data(),
                                                     sc.offsets.data(), sc.adj_elem.data(), sc.adj_local.data(),
                                                     sc.conn8.data())
                              : cwf_preprocess_tets(N, E, sc.coords.data(), sc.conn.data(), sc.mat.data(),
                                                    density.data(), mats.size(), sc.grads.data(),
                                                    sc.volume.data(), sc.mass64.data(), sc.mass32.data(),
                                                    sc.offsets.data(), sc.adj_elem.data(), sc.adj_local.data(),
                                                    sc.conn8.data());
    if (pst)
        throw ScenErr{pst, std::string("preprocess: ") + cwf_hip_last_error(nullptr), cwf_hip_last_context(nullptr)};
    // ---- Dirichlet (solver.cpp:312-352): group nodes = tagged nodes U surface nodes (a sorted set)
    std::vector<uint8_t> fixed(3 * N, 0);
    std::vector<double> target(3 * N, 0.0);
    const yl::Node &dir = sc.cfg["dirichlet"];
    for (size_t f = 0; f < dir.size(); ++f)
    {
        const auto gi = sc.group_id.find(dir.items[f]["group"].as_string());
        if (gi == sc.group_id.end())
            continue;
        std::vector<uint32_t> nodes;
        const auto ng = sc.node_groups.find(gi->second);
        if (ng != sc.node_groups.end())
            nodes = ng->second;
        for (size_t s = 0; s < sc.surf_nodes.size(); ++s)
            if (sc.surf_group[s] == gi->second)
                nodes.insert(nodes.end(), sc.surf_nodes[s].begin(), sc.surf_nodes[s].end());
        std::sort(nodes.begin(), nodes.end());
        nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
        for (int k = 0; k < 3; ++k)
        {
            if (!dir.items[f]["constrain_axis"].items[k].as_bool())
                continue;
            const yl::Node &vk = dir.items[f]["value"].items[k];
            const double v = vk.is_scalar() ? vk.as_double() : 0.0;
            for (uint32_t n : nodes)
            {
                fixed[3ull * n + k] = 1;
                target[3ull * n + k] = v;
            }
        }
    }
    sc.bc_mask.assign(N, 0);
    sc.bc_value.assign(3 * N, 0.f);
    for (uint64_t n = 0; n < N; ++n)
        for (int k = 0; k < 3; ++k)
            if (fixed[3 * n + k])
            {
                sc.bc_mask[n] |= 1u << k;
                sc.bc_value[3 * n + k] = (float)target[3 * n + k];
            }
    // ---- loads at t = 0 (pack.cpp:61-235 evaluates them once)
    const std::vector<double> L = assemble_loads(sc, 0.0);
    sc.external_force.resize(3 * N);
    for (uint64_t d = 0; d < 3 * N; ++d)
        sc.external_force[d] = safe_f32(L[d]);
    sc.position0.resize(3 * N);
    for (uint64_t d = 0; d < 3 * N; ++d)
        sc.position0[d] = (float)sc.coords[d];
    const yl::Node &out = sc.cfg["output"];
    sc.vtu_stride = out["vtu_stride"].as_u32();
    for (size_t i = 0; i < out["probes"].size(); ++i)
        sc.probes.push_back(out["probes"].items[i].as_u32());
}

int fail(const ScenErr &e) { return set_error(nullptr, e.code, e.message, e.context); }
}  // namespace

extern "C" {

int cwf_scenario_create(const char *yaml_path, int mode, int device, int flags, cwf_scenario **out)
{
    if (!yaml_path || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    cwf_scenario *sc = new (std::nothrow) cwf_scenario();
    if (!sc)
        return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
    sc->mode = mode == CWF_MODE_FAST ? CWF_MODE_FAST : CWF_MODE_PARITY;
    sc->flags = flags;
    try
    {
        build(*sc, yaml_path);
    }
    catch (const ScenErr &e)
    {
        delete sc;
        return fail(e);
    }
    catch (const yl::Error &e)
    {
        delete sc;
        return set_error(nullptr, CWF_ERR_PARSE, std::string("config: ") + e.what());
    }
    catch (const std::bad_alloc &)
    {
        delete sc;
        return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
    }
    const uint64_t N = sc->N, E = sc->E, D = 3 * N;
    if (flags & CWF_SCENARIO_PACK_ONLY)
    {
        *out = sc;
        return 0;
    }
    cwf_system_desc d{};
    d.node_count = N;
    d.element_count = E;
    d.dof_count = D;
    d.element_connectivity = sc->conn8.data();
    d.element_gradients = sc->grads.data();
    d.element_volume = sc->volume.data();
    d.element_material_index = sc->mat.data();
    d.material_stiffness = sc->D36.data();
    d.material_count = sc->D36.size() / 36;
    d.lumped_mass = sc->mass32.data();
    d.bc_mask = sc->bc_mask.data();
    d.adjacency_offsets = sc->offsets.data();
    d.adjacency_elements = sc->adj_elem.data();
    d.adjacency_local = sc->adj_local.data();
    d.stiffness_scale = 1.0;
    d.mass_factor = 0.0;
    d.reduction_block = 256;
    d.reduction_partials = std::max<uint64_t>(1, (D + 255) / 256);
    d.mode = sc->mode;
    d.node_coords = sc->coords.data();
    if (int st = cwf_hip_system_create(&d, device, &sc->sys))
    {
        delete sc;
        return st;
    }
    const yl::Node &dm = sc->cfg["damping"], &tm = sc->cfg["time"], &sv = sc->cfg["solver"];
    const double xi = dm["xi"].as_double(), w1 = dm["w1"].as_double(), w2 = dm["w2"].as_double();
    cwf_stepper_desc s{};
    s.rayleigh_alpha = 2.0 * xi * w1 * w2 / (w1 + w2);  // materials.hpp:143-155 compute_rayleigh
    s.rayleigh_beta = 2.0 * xi / (w1 + w2);
    s.runtime_tolerance = sv["runtime_tolerance"].as_double();
    s.pause_tolerance = sv["pause_tolerance"].as_double();
    s.max_iterations = sv["max_iterations"].as_u32();
    s.initial_dt = tm["initial_dt"].as_double();
    s.adaptive = tm["adaptive"].as_bool() ? 1 : 0;
    s.warm_start = 1;
    s.min_dt = tm["min_dt"].as_double();
    s.max_dt = tm["max_dt"].as_double();
    s.low_iteration_ratio = 0.3;  // newmark_stepper.hpp:58-63 AdaptivePolicy
    s.increase_factor = 1.1;
    s.decrease_factor = 0.5;
    s.external_force = sc->external_force.data();
    s.bc_value = sc->bc_value.data();
    if (int st = cwf_hip_stepper_create(sc->sys, &s, &sc->st))
    {
        cwf_scenario_destroy(sc);
        return st;
    }
    sc->u.resize(D);
    sc->v.resize(D);
    sc->a.resize(D);
    sc->efield.resize(13 * E);
    sc->nfield.resize(13 * N);
    *out = sc;
    return 0;
}

int cwf_scenario_info(const cwf_scenario *sc, uint64_t *nodes, uint64_t *elements, uint64_t *dofs)
{
    if (!sc)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null scenario");
    if (nodes)
        *nodes = sc->N;
    if (elements)
        *elements = sc->E;
    if (dofs)
        *dofs = 3 * sc->N;
    return 0;
}

int cwf_scenario_step(cwf_scenario *sc, int paused, cwf_step_telemetry *tel)
{
    if (!sc || !tel)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (!sc->st)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "scenario was created CWF_SCENARIO_PACK_ONLY");
    if (sc->flags & CWF_SCENARIO_TIME_VARYING_LOADS)  // the viewer's custom-load path (viewer.cpp:262-266)
    {
        const std::vector<double> L = assemble_loads(*sc, sc->t_sim);
        for (uint64_t d = 0; d < 3 * sc->N; ++d)
            sc->external_force[d] = safe_f32(L[d]);
        if (int st = cwf_hip_stepper_set_external_force(sc->st, sc->external_force.data(), 3 * sc->N,
                                                        CWF_PTR_HOST))
            return st;
    }
    if (int st = cwf_hip_stepper_step(sc->st, sc->t_sim, paused, tel))
        return st;
    sc->t_sim = tel->simulation_time + tel->time_step;
    ++sc->frame;
    return 0;
}

int cwf_scenario_output_frame(cwf_scenario *sc, const char *out_root)
{
    if (!sc || !out_root)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (!sc->st)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "scenario was created CWF_SCENARIO_PACK_ONLY");
    if (sc->frame == 0)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "no frame stepped yet");
    const uint32_t idx = sc->frame - 1;
    const uint64_t D = 3 * sc->N;
    for (int w = 0; w < 3; ++w)
        if (int st = cwf_hip_stepper_get_state(sc->st, w, w == 0 ? sc->u.data() : w == 1 ? sc->v.data() : sc->a.data(),
                                               D, CWF_PTR_HOST))
            return st;
    if (int st = cwf_hip_derived_fields(sc->sys, sc->u.data(), D, CWF_PTR_HOST, sc->efield.data(), sc->nfield.data(),
                                        CWF_PTR_HOST))
        return st;
    cwf_frame_view f{};
    f.node_count = sc->N;
    f.element_count = sc->E;
    f.position0 = sc->position0.data();
    f.displacement = sc->u.data();
    f.velocity = sc->v.data();
    f.acceleration = sc->a.data();
    f.element_fields = sc->efield.data();
    f.node_fields = sc->nfield.data();
    f.connectivity = sc->conn8.data();
    const std::string root(out_root);
    if (sc->vtu_stride != 0 && idx % sc->vtu_stride == 0)  // output_manager.cpp:49-87
    {
        char name[32];
        std::snprintf(name, sizeof name, "frame_%05u.vtu", idx);
        if (int st = cwf_write_vtu((root + "/vtu/" + name).c_str(), &f, sc->t_sim, idx))
            return st;
    }
    return cwf_probe_log_frame((root + "/probes/probes.csv").c_str(), &sc->probe_header, sc->probes.data(),
                               sc->probes.size(), &f, sc->t_sim, idx);
}

int cwf_scenario_state(cwf_scenario *sc, float *u, float *v, float *a, float *element_fields, float *node_fields)
{
    if (!sc)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (!sc->st)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "scenario was created CWF_SCENARIO_PACK_ONLY");
    const uint64_t D = 3 * sc->N;
    float *out[3] = {u, v, a};
    for (int w = 0; w < 3; ++w)
        if (out[w])
            if (int st = cwf_hip_stepper_get_state(sc->st, w, out[w], D, CWF_PTR_HOST))
                return st;
    if (!element_fields && !node_fields)
        return 0;
    if (int st = cwf_hip_stepper_get_state(sc->st, 0, sc->u.data(), D, CWF_PTR_HOST))
        return st;
    if (int st = cwf_hip_derived_fields(sc->sys, sc->u.data(), D, CWF_PTR_HOST, sc->efield.data(), sc->nfield.data(),
                                        CWF_PTR_HOST))
        return st;
    if (element_fields)
        std::memcpy(element_fields, sc->efield.data(), sc->efield.size() * sizeof(float));
    if (node_fields)
        std::memcpy(node_fields, sc->nfield.data(), sc->nfield.size() * sizeof(float));
    return 0;
}

int cwf_scenario_packed(const cwf_scenario *sc, const char *name, const void **data, uint64_t *bytes)
{
    if (!sc || !name || !data || !bytes)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    const std::string n(name);
    auto view = [&](const auto &v) {
        *data = v.data();
        *bytes = v.size() * sizeof(v[0]);
        return 0;
    };
    if (n == "position0")
        return view(sc->position0);
    if (n == "external_force")
        return view(sc->external_force);
    if (n == "bc_mask")
        return view(sc->bc_mask);
    if (n == "bc_value")
        return view(sc->bc_value);
    if (n == "lumped_mass")
        return view(sc->mass32);
    if (n == "lumped_mass64")
        return view(sc->mass64);
    if (n == "connectivity")
        return view(sc->conn8);
    if (n == "gradients")
        return view(sc->grads);
    if (n == "volume")
        return view(sc->volume);
    if (n == "material_index")
        return view(sc->mat);
    if (n == "offsets")
        return view(sc->offsets);
    if (n == "element_indices")
        return view(sc->adj_elem);
    if (n == "local_indices")
        return view(sc->adj_local);
    return set_error(nullptr, CWF_ERR_ARGUMENT, "unknown packed buffer", n);
}

int cwf_scenario_external_force(const cwf_scenario *sc, double time, float *out, uint64_t n)
{
    if (!sc || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (n != 3 * sc->N)
        return set_error(nullptr, CWF_ERR_SIZE, "external force size mismatch");
    const std::vector<double> L = assemble_loads(*sc, time);
    for (uint64_t d = 0; d < n; ++d)
        out[d] = safe_f32(L[d]);
    return 0;
}

void cwf_scenario_destroy(cwf_scenario *sc)
{
    if (!sc)
        return;
    if (sc->st)
        cwf_hip_stepper_destroy(sc->st);
    if (sc->sys)
        cwf_hip_system_destroy(sc->sys);
    delete sc;
}

}  // extern "C"
