// config.cpp -- scenario YAML -> validated config (src/config/config.cpp:118-605) behind the C-ABI.
//
// Same sections, defaults, validation order, messages and context breadcrumbs as
// cwf::config::parse_config_node; yaml-cpp is replaced by yaml_lite.hpp (YAML subset). The parsed
// config is handed to the host mirrors as canonical JSON (cwf_config_json): doubles in %.17g
// (exact round trip), curves / lists in file order.
#include <cinttypes>
#include <cstdio>
#include <fstream>
#include <map>
#include <optional>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "cwf_internal.hpp"
#include "yaml_lite.hpp"

struct cwf_config
{
    std::string json;
};

namespace cwf
{
namespace
{

struct CfgError
{
    std::string message;
    std::vector<std::string> context;
};

std::string idx(size_t i) { return "[" + std::to_string(i) + "]"; }

std::string jnum(double v)
{
    if (std::isnan(v) || std::isinf(v))
        return std::isnan(v) ? "NaN" : (v > 0 ? "Infinity" : "-Infinity");
    char b[40];
    snprintf(b, sizeof b, "%.17g", v);
    return b;
}

std::string jstr(const std::string &s)
{
    std::string o = "\"";
    for (const char c : s)
    {
        if (c == '"' || c == '\\')
        {
            o.push_back('\\');
            o.push_back(c);
        }
        else if ((unsigned char)c < 0x20)
        {
            char b[8];
            snprintf(b, sizeof b, "\\u%04x", (unsigned)(unsigned char)c);
            o += b;
        }
        else
            o.push_back(c);
    }
    return o + "\"";
}

struct Vec3
{
    double v[3];
};

// node_to_vec3 (config.cpp:29-51)
Vec3 vec3(const yl::Node &n, std::vector<std::string> ctx)
{
    if (!n.defined() || !n.is_seq() || n.size() != 3)
        throw CfgError{"expected sequence[3] for vector", ctx};
    Vec3 r{};
    for (size_t i = 0; i < 3; ++i)
    {
        try
        {
            r.v[i] = n[i].as_double();
        }
        catch (const yl::Error &e)
        {
            ctx.push_back(idx(i));
            throw CfgError{e.what(), ctx};
        }
    }
    return r;
}

// node_to_optional_vec3 (config.cpp:53-83) -> JSON [v|null, ...]
std::string optional_vec3(const yl::Node &n, std::vector<std::string> ctx)
{
    if (!n.defined() || n.is_null())
        return "[null, null, null]";
    if (!n.is_seq() || n.size() != 3)
        throw CfgError{"expected sequence[3] for value override", ctx};
    std::string o = "[";
    for (size_t i = 0; i < 3; ++i)
    {
        if (i)
            o += ", ";
        if (n[i].is_null())
        {
            o += "null";
            continue;
        }
        try
        {
            o += jnum(n[i].as_double());
        }
        catch (const yl::Error &e)
        {
            ctx.push_back(idx(i));
            throw CfgError{e.what(), ctx};
        }
    }
    return o + "]";
}

// node_to_string_vec (config.cpp:85-114)
std::vector<std::string> string_vec(const yl::Node &n, std::vector<std::string> ctx)
{
    if (!n.defined() || !n.is_seq())
        throw CfgError{"expected sequence for string list", ctx};
    std::vector<std::string> items;
    for (size_t i = 0; i < n.size(); ++i)
    {
        try
        {
            items.push_back(n[i].as_string());
        }
        catch (const yl::Error &e)
        {
            ctx.push_back(idx(i));
            throw CfgError{e.what(), ctx};
        }
    }
    return items;
}

template <class F> auto guard(std::vector<std::string> ctx, F f) -> decltype(f())
{
    try
    {
        return f();
    }
    catch (const yl::Error &e)
    {
        throw CfgError{e.what(), ctx};
    }
}

// parse_config_node (config.cpp:148-605) -> canonical JSON
std::string parse_config(const yl::Node &root)
{
    if (!root.defined() || !root.is_map())
        throw CfgError{"config root must be a mapping", {}};
    std::ostringstream j;
    // mesh
    const yl::Node &mesh = root["mesh"];
    if (!mesh.defined() || !mesh.is_map())
        throw CfgError{"missing 'mesh' section", {"mesh"}};
    const yl::Node &mpath = mesh["path"];
    if (!mpath.defined() || !mpath.is_scalar())
        throw CfgError{"mesh.path must be a scalar string", {"mesh", "path"}};
    j << "{\"mesh_path\": " << jstr(mpath.as_string());
    // materials
    const yl::Node &mats = root["materials"];
    if (!mats.defined() || !mats.is_seq() || mats.size() == 0)
        throw CfgError{"materials must be a non-empty sequence", {"materials"}};
    std::set<std::string> names;
    j << ", \"materials\": [";
    for (size_t i = 0; i < mats.size(); ++i)
    {
        const yl::Node &m = mats[i];
        if (!m.is_map())
            throw CfgError{"material entry must be a map", {"materials", idx(i)}};
        std::string name;
        double E = 0, nu = 0, rho = 0;
        guard({"materials", idx(i)}, [&] {
            name = m["name"].as_string();
            E = m["E"].as_double();
            nu = m["nu"].as_double();
            rho = m["rho"].as_double();
            return 0;
        });
        if (E <= 0.0)
            throw CfgError{"material.E must be > 0", {"materials", idx(i), "E"}};
        if (nu <= -0.999 || nu >= 0.5)
            throw CfgError{"material.nu must be (-0.999, 0.5)", {"materials", idx(i), "nu"}};
        if (rho <= 0.0)
            throw CfgError{"material.rho must be > 0", {"materials", idx(i), "rho"}};
        if (names.count(name))
            throw CfgError{"material names must be unique", {"materials", idx(i), "name"}};
        names.insert(name);
        j << (i ? ", " : "") << "{\"name\": " << jstr(name) << ", \"E\": " << jnum(E) << ", \"nu\": " << jnum(nu)
          << ", \"rho\": " << jnum(rho) << "}";
    }
    j << "]";
    // assignments
    const yl::Node &asg = root["assignments"];
    if (!asg.defined() || !asg.is_seq() || asg.size() == 0)
        throw CfgError{"assignments must be a non-empty sequence", {"assignments"}};
    j << ", \"assignments\": [";
    for (size_t i = 0; i < asg.size(); ++i)
    {
        const yl::Node &a = asg[i];
        if (!a.is_map())
            throw CfgError{"assignment must be a map", {"assignments", idx(i)}};
        std::string group, material;
        guard({"assignments", idx(i)}, [&] {
            group = a["group"].as_string();
            material = a["material"].as_string();
            return 0;
        });
        if (!names.count(material))
            throw CfgError{"assignment references unknown material", {"assignments", idx(i), "material"}};
        j << (i ? ", " : "") << "{\"group\": " << jstr(group) << ", \"material\": " << jstr(material) << "}";
    }
    j << "]";
    // damping
    const yl::Node &damp = root["damping"];
    if (!damp.defined() || !damp.is_map())
        throw CfgError{"missing damping map", {"damping"}};
    double xi = 0, w1 = 0, w2 = 0;
    guard({"damping"}, [&] {
        xi = damp["xi"].as_double();
        w1 = damp["w1"].as_double();
        w2 = damp["w2"].as_double();
        return 0;
    });
    if (xi <= 0.0 || xi >= 1.0)
        throw CfgError{"damping.xi must be (0,1)", {"damping", "xi"}};
    if (w1 <= 0.0)
        throw CfgError{"damping.w1 must be > 0", {"damping", "w1"}};
    if (w2 <= w1)
        throw CfgError{"damping.w2 must be > damping.w1", {"damping", "w2"}};
    j << ", \"damping\": {\"xi\": " << jnum(xi) << ", \"w1\": " << jnum(w1) << ", \"w2\": " << jnum(w2) << "}";
    // time
    const yl::Node &tm = root["time"];
    if (!tm.defined() || !tm.is_map())
        throw CfgError{"missing time map", {"time"}};
    double dt = 0;
    bool adaptive = false;
    guard({"time"}, [&] {
        dt = tm["dt"].as_double();
        adaptive = tm["adaptive"].as_bool();
        return 0;
    });
    // config.cpp:327-329: optional clamps (conversion failures propagate as a parse error)
    const double min_dt = guard({"time"}, [&] { return tm["min_dt"].defined() ? tm["min_dt"].as_double() : 0.0; });
    const double max_dt = guard({"time"}, [&] { return tm["max_dt"].defined() ? tm["max_dt"].as_double() : dt; });
    if (dt <= 0.0)
        throw CfgError{"time.dt must be > 0", {"time", "dt"}};
    if (min_dt < 0.0)
        throw CfgError{"time.min_dt must be >= 0", {"time", "min_dt"}};
    if (max_dt < dt)
        throw CfgError{"time.max_dt must be >= time.dt", {"time", "max_dt"}};
    j << ", \"time\": {\"initial_dt\": " << jnum(dt) << ", \"adaptive\": " << (adaptive ? "true" : "false")
      << ", \"min_dt\": " << jnum(min_dt) << ", \"max_dt\": " << jnum(max_dt) << "}";
    // solver
    const yl::Node &sv = root["solver"];
    if (!sv.defined() || !sv.is_map())
        throw CfgError{"missing solver map", {"solver"}};
    std::string stype, prec;
    double tr = 0, tp = 0;
    uint32_t mi = 0;
    guard({"solver"}, [&] {
        stype = sv["type"].as_string();
        prec = sv["preconditioner"].as_string();
        tr = sv["tol_runtime"].as_double();
        tp = sv["tol_pause"].as_double();
        mi = sv["max_iters"].as_u32();
        return 0;
    });
    if (mi == 0)
        throw CfgError{"solver.max_iters must be >= 1", {"solver", "max_iters"}};
    if (tr <= 0.0 || tp <= 0.0)
        throw CfgError{"solver tolerances must be > 0", {"solver"}};
    j << ", \"solver\": {\"type\": " << jstr(stype) << ", \"preconditioner\": " << jstr(prec)
      << ", \"runtime_tolerance\": " << jnum(tr) << ", \"pause_tolerance\": " << jnum(tp)
      << ", \"max_iterations\": " << mi << "}";
    // precision
    const yl::Node &pr = root["precision"];
    if (!pr.defined() || !pr.is_map())
        throw CfgError{"missing precision map", {"precision"}};
    std::string vp, rp;
    guard({"precision"}, [&] {
        vp = pr["vectors"].as_string();
        rp = pr["reductions"].as_string();
        return 0;
    });
    j << ", \"precision\": {\"vector_precision\": " << jstr(vp) << ", \"reduction_precision\": " << jstr(rp) << "}";
    // curves (optional map)
    std::set<std::string> curves;
    j << ", \"curves\": {";
    const yl::Node &cv = root["curves"];
    if (cv.defined() && cv.is_map())
    {
        bool firstc = true;
        for (const auto &kv : cv.map)
        {
            const std::string &key = kv.first;
            const yl::Node &seq = kv.second;
            if (!seq.is_seq() || seq.size() == 0)
                throw CfgError{"curve must be non-empty sequence", {"curves", key}};
            double prev = -INFINITY;
            j << (firstc ? "" : ", ") << jstr(key) << ": [";
            firstc = false;
            for (size_t q = 0; q < seq.size(); ++q)
            {
                const yl::Node &pn = seq[q];
                if (!pn.is_seq() || pn.size() != 2)
                    throw CfgError{"curve point must be sequence[2]", {"curves", key, idx(q)}};
                double t = 0, v = 0;
                guard({"curves", key, idx(q)}, [&] {
                    t = pn[0].as_double();
                    v = pn[1].as_double();
                    return 0;
                });
                if (t < prev)
                    throw CfgError{"curve times must be non-decreasing", {"curves", key, idx(q)}};
                prev = t;
                j << (q ? ", " : "") << "[" << jnum(t) << ", " << jnum(v) << "]";
            }
            j << "]";
            curves.insert(key);
        }
    }
    j << "}";
    // loads
    const yl::Node &ld = root["loads"];
    if (!ld.defined() || !ld.is_map())
        throw CfgError{"missing loads map", {"loads"}};
    const Vec3 g = vec3(ld["gravity"], {"loads", "gravity"});
    j << ", \"loads\": {\"gravity\": [" << jnum(g.v[0]) << ", " << jnum(g.v[1]) << ", " << jnum(g.v[2]) << "]";
    for (int kind = 0; kind < 2; ++kind)  // tractions, then point loads (config.cpp:443-537)
    {
        const char *sec = kind == 0 ? "tractions" : "points";
        const yl::Node &list = ld[sec];
        j << ", \"" << sec << "\": [";
        if (list.defined() && list.is_seq())
        {
            for (size_t i = 0; i < list.size(); ++i)
            {
                const yl::Node &e = list[i];
                if (!e.is_map())
                    throw CfgError{kind == 0 ? "traction entry must be map" : "point load entry must be map",
                                   {"loads", sec, idx(i)}};
                std::string group, curve;
                guard({"loads", sec, idx(i)}, [&] {
                    group = e["group"].as_string();
                    curve = e["scale_curve"].defined() ? e["scale_curve"].as_string() : std::string();
                    return 0;
                });
                const Vec3 v = vec3(e["value"], {"loads", sec, idx(i), "value"});
                if (!curve.empty() && !curves.count(curve))
                    throw CfgError{kind == 0 ? "traction references unknown curve"
                                             : "point load references unknown curve",
                                   {"loads", sec, idx(i), "scale_curve"}};
                j << (i ? ", " : "") << "{\"group\": " << jstr(group) << ", \"value\": [" << jnum(v.v[0]) << ", "
                  << jnum(v.v[1]) << ", " << jnum(v.v[2]) << "], \"scale_curve\": " << jstr(curve) << "}";
            }
        }
        else if (list.defined())
            throw CfgError{kind == 0 ? "loads.tractions must be a sequence when present"
                                     : "loads.points must be a sequence when present",
                           {"loads", sec}};
        j << "]";
    }
    j << "}";
    // dirichlet (optional)
    j << ", \"dirichlet\": [";
    const yl::Node &dir = root["dirichlet"];
    if (dir.defined() && dir.is_map())
    {
        const yl::Node &fixes = dir["fixes"];
        if (fixes.defined() && fixes.is_seq())
            for (size_t i = 0; i < fixes.size(); ++i)
            {
                const yl::Node &e = fixes[i];
                if (!e.is_map())
                    throw CfgError{"dirichlet fixed entry must be a map", {"dirichlet", "fixes", idx(i)}};
                const std::string group =
                    guard({"dirichlet", "fixes", idx(i), "group"}, [&] { return e["group"].as_string(); });
                const auto dofs = string_vec(e["dof"], {"dirichlet", "fixes", idx(i), "dof"});
                if (dofs.empty())
                    throw CfgError{"dirichlet.dof must not be empty", {"dirichlet", "fixes", idx(i), "dof"}};
                bool ax[3] = {false, false, false};
                for (const auto &a : dofs)
                {
                    if (a == "x")
                        ax[0] = true;
                    else if (a == "y")
                        ax[1] = true;
                    else if (a == "z")
                        ax[2] = true;
                    else
                        throw CfgError{"dirichlet.dof must be subset of {x,y,z}", {"dirichlet", "fixes", idx(i), "dof"}};
                }
                const std::string val = optional_vec3(e["value"], {"dirichlet", "fixes", idx(i), "value"});
                j << (i ? ", " : "") << "{\"group\": " << jstr(group) << ", \"constrain_axis\": ["
                  << (ax[0] ? "true" : "false") << ", " << (ax[1] ? "true" : "false") << ", "
                  << (ax[2] ? "true" : "false") << "], \"value\": " << val << "}";
            }
    }
    j << "]";
    // output
    const yl::Node &out = root["output"];
    if (!out.defined() || !out.is_map())
        throw CfgError{"missing output map", {"output"}};
    const uint32_t stride = guard({"output", "vtu_stride"}, [&] { return out["vtu_stride"].as_u32(); });
    if (stride == 0)
        throw CfgError{"output.vtu_stride must be >= 1", {"output", "vtu_stride"}};
    j << ", \"output\": {\"vtu_stride\": " << stride << ", \"probes\": [";
    const yl::Node &probes = out["probes"];
    if (probes.defined() && probes.is_seq())
        for (size_t i = 0; i < probes.size(); ++i)
            j << (i ? ", " : "")
              << guard({"output", "probes", idx(i)}, [&] { return probes[i].as_u32(); });
    j << "]}}";
    return j.str();
}

std::string join_ctx(const std::vector<std::string> &c)
{
    std::string s;
    for (size_t i = 0; i < c.size(); ++i)
        s += (i ? "\n" : "") + c[i];
    return s;
}

int load(const std::string &text, const std::string *path, cwf_config **out)
{
    std::string json;
    try
    {
        const yl::Node root = yl::parse(text);
        json = parse_config(root);
    }
    catch (const CfgError &e)
    {
        return set_error(nullptr, CWF_ERR_PARSE, e.message, join_ctx(e.context));
    }
    catch (const yl::Error &e)  // config.cpp:124-128 / 137-140
    {
        return set_error(nullptr, CWF_ERR_PARSE, std::string("YAML parse error: ") + e.what(), path ? *path : "");
    }
    catch (const std::exception &e)
    {
        return set_error(nullptr, CWF_ERR_PARSE, e.what(), path ? *path : "");
    }
    *out = new cwf_config{std::move(json)};
    return 0;
}

}  // namespace
}  // namespace cwf

using namespace cwf;

extern "C" {

int cwf_config_load_string(const char *yaml_text, cwf_config **out)
{
    if (!yaml_text || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    return load(yaml_text, nullptr, out);
}

int cwf_config_load_file(const char *path, cwf_config **out)
{
    if (!path || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    std::ifstream f(path, std::ios::binary);
    if (!f)  // config.cpp:120-123 (yaml-cpp BadFile)
        return set_error(nullptr, CWF_ERR_IO, std::string("unable to open config file: bad file: ") + path, path);
    std::ostringstream ss;
    ss << f.rdbuf();
    const std::string p(path);
    return load(ss.str(), &p, out);
}

const char *cwf_config_json(const cwf_config *cfg) { return cfg ? cfg->json.c_str() : ""; }

void cwf_config_destroy(cwf_config *cfg) { delete cfg; }

}  // extern "C"
