// gmsh.cpp -- Gmsh MSH 4.1 ASCII loader (src/mesh/mesh.cpp:56-566) behind the C-ABI.
//
// Same section handling as cwf::mesh::load_gmsh_from_string: $PhysicalNames, $Entities (physical
// tags per entity), $Nodes (entity blocks; nodes of a tagged entity join that physical group's node
// list), $Elements (dim-3 tet4 / hex8 -> volume elements, dim-2 tri3 / quad4 -> surfaces, lower
// dimensions skipped; an element's group is its entity's first physical tag, else the entity tag),
// then the physical-group table. Error texts and breadcrumbs are the reference's. Groups are listed
// in ascending id (the reference's order is unordered_map iteration order).
#include <algorithm>
#include <cstdio>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "cwf_internal.hpp"

struct cwf_mesh
{
    std::vector<double> coords;        // [3N]
    std::vector<uint32_t> node_ids;    // [N] original ids
    std::vector<uint32_t> elem_nodes;  // [8E], UINT32_MAX padded
    std::vector<uint8_t> elem_geom;    // [E] 4 tet / 8 hex
    std::vector<uint32_t> elem_group;  // [E]
    std::vector<uint32_t> elem_ids;    // [E]
    std::vector<uint32_t> surf_nodes;  // [4S]
    std::vector<uint8_t> surf_geom;    // [S] 3 / 4
    std::vector<uint32_t> surf_group;  // [S]
    struct Group
    {
        uint32_t dim = 0, id = 0;
        std::string name;
    };
    std::vector<Group> groups;                                  // ascending id
    std::map<uint32_t, std::vector<uint32_t>> node_groups;      // physical id -> node indices
};

namespace cwf
{
namespace
{

struct MeshErr
{
    std::string message;
    std::vector<std::string> context;
};

using Key = uint64_t;
inline Key key(uint32_t d, uint32_t t) { return ((Key)d << 32) | t; }

std::string trim(const std::string &s)
{
    const size_t b = s.find_first_not_of(" \t\r");
    if (b == std::string::npos)
        return "";
    const size_t e = s.find_last_not_of(" \t\r");
    return s.substr(b, e - b + 1);
}

std::istringstream section(std::istringstream &in, const char *end)  // read_section (mesh.cpp:443-457)
{
    std::string contents, line;
    while (std::getline(in, line))
    {
        if (trim(line) == end)
            break;
        contents += line;
        contents.push_back('\n');
    }
    return std::istringstream(contents);
}

uint32_t stou(const std::string &s, const char *what)
{
    try
    {
        return (uint32_t)std::stoul(trim(s));
    }
    catch (const std::exception &)
    {
        throw MeshErr{std::string("invalid integer in ") + what, {what}};
    }
}

struct Entities
{
    std::unordered_map<Key, std::vector<uint32_t>> phys;
    std::map<uint32_t, uint32_t> phys_dim;  // first dimension seen per physical id
};

Entities parse_entities(std::istringstream &s)  // mesh.cpp:90-153
{
    Entities info;
    std::string line;
    if (!std::getline(s, line))
        throw MeshErr{"unexpected EOF in $Entities header", {"Entities"}};
    std::istringstream h(line);
    uint32_t cnt[4] = {0, 0, 0, 0};
    h >> cnt[0] >> cnt[1] >> cnt[2] >> cnt[3];
    for (uint32_t dim = 0; dim < 4; ++dim)
        for (uint32_t i = 0; i < cnt[dim]; ++i)
        {
            if (!std::getline(s, line))
                throw MeshErr{"unexpected EOF inside $Entities block", {"Entities", "dim" + std::to_string(dim)}};
            std::istringstream es(line);
            uint32_t tag = 0, np = 0;
            double bb[6];
            es >> tag;
            if (dim == 0)  // points carry x y z only in MSH 4.1
                es >> bb[0] >> bb[1] >> bb[2];
            else
                es >> bb[0] >> bb[1] >> bb[2] >> bb[3] >> bb[4] >> bb[5];
            es >> np;
            std::vector<uint32_t> ids;
            for (uint32_t k = 0; k < np; ++k)
            {
                uint32_t p = 0;
                es >> p;
                ids.push_back(p);
                info.phys_dim.emplace(p, dim);
            }
            if (!ids.empty())
                info.phys.emplace(key(dim, tag), std::move(ids));
        }
    return info;
}

}  // namespace

static int load_mesh(const std::string &text, cwf_mesh **out)
{
    auto m = std::make_unique<cwf_mesh>();
    try
    {
        std::unordered_map<uint32_t, size_t> id_to_index;
        std::map<Key, std::string> names;
        Entities ent;
        bool seen_nodes = false, seen_elems = false;
        std::set<uint32_t> referenced;
        std::istringstream in(text);
        std::string line;
        while (std::getline(in, line))
        {
            const std::string t = trim(line);
            if (t == "$PhysicalNames")  // mesh.cpp:56-88
            {
                auto s = section(in, "$EndPhysicalNames");
                std::string l;
                std::getline(s, l);
                const uint32_t n = stou(l, "PhysicalNames");
                for (uint32_t i = 0; i < n; ++i)
                {
                    if (!std::getline(s, l))
                        throw MeshErr{"unexpected EOF in $PhysicalNames", {"PhysicalNames"}};
                    std::istringstream ls(l);
                    uint32_t dim = 0, tag = 0;
                    std::string name;
                    ls >> dim >> tag;
                    std::getline(ls >> std::ws, name);
                    name = trim(name);
                    if (name.size() >= 2 && name.front() == '"' && name.back() == '"')
                        name = name.substr(1, name.size() - 2);
                    names.emplace(key(dim, tag), name);
                }
            }
            else if (t == "$Entities")
            {
                auto s = section(in, "$EndEntities");
                ent = parse_entities(s);
            }
            else if (t == "$Nodes")  // mesh.cpp:155-226
            {
                auto s = section(in, "$EndNodes");
                std::string l;
                if (!std::getline(s, l))
                    throw MeshErr{"unexpected EOF in $Nodes header", {"Nodes"}};
                std::istringstream h(l);
                uint64_t blocks = 0, total = 0, mn = 0, mx = 0;
                h >> blocks >> total >> mn >> mx;
                m->coords.clear();
                m->node_ids.clear();
                m->node_groups.clear();
                id_to_index.clear();
                for (uint64_t b = 0; b < blocks; ++b)
                {
                    if (!std::getline(s, l))
                        throw MeshErr{"unexpected EOF in $Nodes block header", {"Nodes"}};
                    std::istringstream bs(l);
                    uint32_t edim = 0, etag = 0, param = 0;
                    uint64_t count = 0;
                    bs >> edim >> etag >> param >> count;
                    const auto pit = ent.phys.find(key(edim, etag));
                    std::vector<uint32_t> ids(count);
                    for (uint64_t i = 0; i < count; ++i)
                    {
                        if (!std::getline(s, l))
                            throw MeshErr{"unexpected EOF reading node ids", {"Nodes"}};
                        ids[i] = stou(l, "Nodes");
                    }
                    for (uint64_t i = 0; i < count; ++i)
                    {
                        if (!std::getline(s, l))
                            throw MeshErr{"unexpected EOF reading node coordinates", {"Nodes"}};
                        std::istringstream cs(l);
                        double x = 0, y = 0, z = 0;
                        cs >> x >> y >> z;
                        id_to_index[ids[i]] = m->node_ids.size();
                        const uint32_t index = (uint32_t)m->node_ids.size();
                        m->node_ids.push_back(ids[i]);
                        m->coords.insert(m->coords.end(), {x, y, z});
                        if (pit != ent.phys.end())
                            for (uint32_t p : pit->second)
                                m->node_groups[p].push_back(index);
                    }
                }
                if (m->node_ids.size() != total)
                    throw MeshErr{"node count mismatch", {"Nodes"}};
                for (const auto &kv : m->node_groups)
                    referenced.insert(kv.first);
                seen_nodes = true;
            }
            else if (t == "$Elements")  // mesh.cpp:275-441
            {
                auto s = section(in, "$EndElements");
                std::string l;
                if (!std::getline(s, l))
                    throw MeshErr{"unexpected EOF in $Elements header", {"Elements"}};
                std::istringstream h(l);
                uint64_t blocks = 0, total = 0, mn = 0, mx = 0, processed = 0;
                h >> blocks >> total >> mn >> mx;
                for (uint64_t b = 0; b < blocks; ++b)
                {
                    if (!std::getline(s, l))
                        throw MeshErr{"unexpected EOF reading element block header", {"Elements"}};
                    std::istringstream bs(l);
                    uint32_t edim = 0, etag = 0, etype = 0;
                    uint64_t count = 0;
                    bs >> edim >> etag >> etype >> count;
                    const int nn = etype == 2 ? 3 : etype == 3 ? 4 : etype == 4 ? 4 : etype == 5 ? 8 : 0;
                    if (!nn)
                        throw MeshErr{"unsupported Gmsh element type " + std::to_string(etype),
                                      {"Elements", "entityTag=" + std::to_string(etag)}};
                    const auto pit = ent.phys.find(key(edim, etag));
                    const uint32_t group = pit != ent.phys.end() && !pit->second.empty() ? pit->second.front() : etag;
                    for (uint64_t i = 0; i < count; ++i)
                    {
                        if (!std::getline(s, l))
                            throw MeshErr{"unexpected EOF reading element data", {"Elements"}};
                        ++processed;
                        std::istringstream es(l);
                        uint32_t etag_el = 0;
                        es >> etag_el;
                        if (edim == 3 || edim == 2)
                        {
                            const bool vol = edim == 3;
                            if (vol && etype != 4 && etype != 5)
                                throw MeshErr{"unsupported volume element type " + std::to_string(etype),
                                              {"Elements", "elementTag=" + std::to_string(etag_el)}};
                            if (!vol && etype != 2 && etype != 3)
                                throw MeshErr{"unsupported surface element type " + std::to_string(etype),
                                              {"Elements", "elementTag=" + std::to_string(etag_el)}};
                            uint32_t nodes[8];
                            std::fill(nodes, nodes + 8, 0xFFFFFFFFu);
                            for (int k = 0; k < nn; ++k)
                            {
                                uint32_t tag = 0;
                                es >> tag;
                                const auto it = id_to_index.find(tag);
                                if (it == id_to_index.end())
                                    throw MeshErr{std::string(vol ? "element" : "surface") +
                                                      " references unknown node " + std::to_string(tag),
                                                  {"Elements", "elementTag=" + std::to_string(etag_el)}};
                                nodes[k] = (uint32_t)it->second;
                            }
                            referenced.insert(group);
                            if (vol)
                            {
                                m->elem_nodes.insert(m->elem_nodes.end(), nodes, nodes + 8);
                                m->elem_geom.push_back((uint8_t)nn);
                                m->elem_group.push_back(group);
                                m->elem_ids.push_back(etag_el);
                            }
                            else
                            {
                                m->surf_nodes.insert(m->surf_nodes.end(), nodes, nodes + 4);
                                m->surf_geom.push_back((uint8_t)nn);
                                m->surf_group.push_back(group);
                            }
                        }
                    }
                }
                if (processed != total)
                    throw MeshErr{"element count mismatch", {"Elements"}};
                seen_elems = true;
            }
        }
        if (!seen_nodes)
            throw MeshErr{"missing $Nodes section", {}};
        if (!seen_elems)
            throw MeshErr{"missing $Elements section", {}};
        // physical-group table (mesh.cpp:509-563)
        std::map<uint32_t, cwf_mesh::Group> gm;
        for (const auto &kv : names)
            gm[(uint32_t)(kv.first & 0xFFFFFFFFu)] =
                cwf_mesh::Group{(uint32_t)(kv.first >> 32), (uint32_t)(kv.first & 0xFFFFFFFFu), kv.second};
        for (const auto &kv : ent.phys_dim)
        {
            auto &g = gm[kv.first];
            if (g.id == 0)
                g = cwf_mesh::Group{kv.second, kv.first, ""};
            else
                g.dim = kv.second;
        }
        for (const uint32_t id : referenced)
        {
            auto &g = gm[id];
            if (g.id == 0)
            {
                const auto it = ent.phys_dim.find(id);
                g = cwf_mesh::Group{it != ent.phys_dim.end() ? it->second : 0u, id, ""};
            }
        }
        for (const auto &kv : gm)
            m->groups.push_back(kv.second);
    }
    catch (const MeshErr &e)
    {
        std::string ctx;
        for (size_t i = 0; i < e.context.size(); ++i)
            ctx += (i ? "\n" : "") + e.context[i];
        return set_error(nullptr, CWF_ERR_PARSE, e.message, ctx);
    }
    catch (const std::bad_alloc &)
    {
        return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
    }
    *out = m.release();
    return 0;
}

}  // namespace cwf

using namespace cwf;

extern "C" {

int cwf_mesh_load_string(const char *text, cwf_mesh **out)
{
    if (!text || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    return load_mesh(text, out);
}

int cwf_mesh_load_file(const char *path, cwf_mesh **out)
{
    if (!path || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    std::ifstream f(path, std::ios::binary);
    if (!f)  // mesh.cpp:461-466
        return set_error(nullptr, CWF_ERR_IO, std::string("failed to open mesh file: ") + path, path);
    std::ostringstream ss;
    ss << f.rdbuf();
    return load_mesh(ss.str(), out);
}

void cwf_mesh_destroy(cwf_mesh *m) { delete m; }

int cwf_mesh_get_info(const cwf_mesh *m, cwf_mesh_info *info)
{
    if (!m || !info)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    info->node_count = m->node_ids.size();
    info->element_count = m->elem_geom.size();
    info->surface_count = m->surf_geom.size();
    info->group_count = m->groups.size();
    return 0;
}

int cwf_mesh_nodes(const cwf_mesh *m, double *coords, uint32_t *original_ids)
{
    if (!m)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (coords)
        std::copy(m->coords.begin(), m->coords.end(), coords);
    if (original_ids)
        std::copy(m->node_ids.begin(), m->node_ids.end(), original_ids);
    return 0;
}

int cwf_mesh_elements(const cwf_mesh *m, uint32_t *nodes8, uint8_t *geometry, uint32_t *physical_group,
                      uint32_t *original_ids)
{
    if (!m)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (nodes8)
        std::copy(m->elem_nodes.begin(), m->elem_nodes.end(), nodes8);
    if (geometry)
        std::copy(m->elem_geom.begin(), m->elem_geom.end(), geometry);
    if (physical_group)
        std::copy(m->elem_group.begin(), m->elem_group.end(), physical_group);
    if (original_ids)
        std::copy(m->elem_ids.begin(), m->elem_ids.end(), original_ids);
    return 0;
}

int cwf_mesh_surfaces(const cwf_mesh *m, uint32_t *nodes4, uint8_t *geometry, uint32_t *physical_group)
{
    if (!m)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (nodes4)
        std::copy(m->surf_nodes.begin(), m->surf_nodes.end(), nodes4);
    if (geometry)
        std::copy(m->surf_geom.begin(), m->surf_geom.end(), geometry);
    if (physical_group)
        std::copy(m->surf_group.begin(), m->surf_group.end(), physical_group);
    return 0;
}

int cwf_mesh_group(const cwf_mesh *m, uint64_t index, uint32_t *dimension, uint32_t *id, const char **name)
{
    if (!m || index >= m->groups.size())
        return set_error(nullptr, CWF_ERR_ARGUMENT, "group index out of range");
    if (dimension)
        *dimension = m->groups[index].dim;
    if (id)
        *id = m->groups[index].id;
    if (name)
        *name = m->groups[index].name.c_str();
    return 0;
}

int cwf_mesh_node_group(const cwf_mesh *m, uint32_t group_id, const uint32_t **nodes, uint64_t *count)
{
    if (!m || !count)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    const auto it = m->node_groups.find(group_id);
    *count = it == m->node_groups.end() ? 0 : it->second.size();
    if (nodes)
        *nodes = it == m->node_groups.end() ? nullptr : it->second.data();
    return 0;
}

}  // extern "C"
