// frontend_api_test.cpp -- the scenario front-end and writers through the C++ mirror include/cwf_hip.hpp
// (no GPU needed): the reference fixture tests/data/cantilever.{yaml,msh} (copied under tests/golden/data)
// as in tests/config_validation_test.cpp:67-73 and tests/mesh_loader_test.cpp:48-77, one validation error
// with its breadcrumbs, and a VTU + probe frame written from host data.
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/cwf_hip.hpp"

static int failures = 0;
#define EXPECT(c)                                                   \
    do                                                              \
    {                                                               \
        if (!(c))                                                   \
        {                                                           \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                             \
        }                                                           \
    } while (0)

int main(int argc, char **argv)
{
    const std::string data = argc > 1 ? argv[1] : "tests/golden/data";
    const std::string tmp = argc > 2 ? argv[2] : "/tmp";
    namespace ch = cwf::hip;
    auto cfg = ch::config::load_config_from_file(data + "/cantilever.yaml");
    EXPECT(cfg.has_value());
    if (cfg)
        EXPECT(cfg.value().find("\"mesh_path\": \"tests/data/cantilever.msh\"") != std::string::npos);
    auto bad = ch::config::load_config_from_string("mesh:\n  path: a.msh\nmaterials:\n  - name: c\n    E: -1\n"
                                                   "    nu: 0.2\n    rho: 1\n");
    EXPECT(!bad.has_value());
    if (!bad)
    {
        EXPECT(bad.error().message == "material.E must be > 0");
        EXPECT((bad.error().context == std::vector<std::string>{"materials", "[0]", "E"}));
    }
    auto m = ch::mesh::load_gmsh_file(data + "/cantilever.msh");
    EXPECT(m.has_value());
    if (m)
    {
        const auto &mesh = m.value();
        EXPECT(mesh.positions.size() == 12 && mesh.positions[3] == 1.0);
        EXPECT(mesh.geometry.size() == 1 && mesh.geometry[0] == 4);
        EXPECT(mesh.elements[0] == 0 && mesh.elements[3] == 3 && mesh.elements[4] == 0xFFFFFFFFu);
        EXPECT(mesh.surface_group.size() == 2);
        bool solid = false;
        for (const auto &g : mesh.physical_groups)
            solid |= g.id == 3 && g.name == "SOLID";
        EXPECT(solid);
    }
    auto missing = ch::mesh::load_gmsh_file(data + "/definitely_missing.msh");
    EXPECT(!missing.has_value() && missing.error().message.find("failed to open mesh file") == 0);

    // one frame of the unit tet through the writers (host-only path)
    std::vector<float> pos{0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1}, u(12, 0.0f), v(12, 0.5f), a(12, -1.0f);
    std::vector<std::uint32_t> conn{0, 1, 2, 3, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    ch::post::DerivedFieldSet d;
    d.elements.resize(1);
    d.nodes.resize(4);
    d.elements[0].von_mises = 7.0f;
    ch::post::FrameData f{pos, u, v, a, conn};
    EXPECT(ch::post::write_vtu(tmp + "/cpp_frame.vtu", f, d, 0.01, 3).has_value());
    std::ifstream vtu(tmp + "/cpp_frame.vtu", std::ios::binary);
    std::string head(200, '\0');
    vtu.read(head.data(), 200);
    EXPECT(head.find("<VTKFile type=\"UnstructuredGrid\"") != std::string::npos);
    ch::post::ProbeLogger lg(tmp + "/cpp_probes.csv", {3});
    EXPECT(lg.log_frame(0.01, 3, f, d).has_value());
    ch::post::ProbeLogger badp(tmp + "/cpp_probes_bad.csv", {9});
    auto r = badp.log_frame(0.0, 0, f, d);
    EXPECT(!r.has_value() && r.error().message == "probe index out of range");

    // the native scenario driver: packing only (no device), then a step is refused
    auto sc = ch::scenario::Scenario::create(data + "/cantilever.yaml", CWF_MODE_PARITY, 0, CWF_SCENARIO_PACK_ONLY);
    EXPECT(sc.has_value());
    if (sc)
    {
        EXPECT(sc.value().dof_count() == 12);
        auto st = sc.value().step();
        EXPECT(!st.has_value() && st.error().message.find("PACK_ONLY") != std::string::npos);
    }
    auto nosc = ch::scenario::Scenario::create(data + "/definitely_missing.yaml");
    EXPECT(!nosc.has_value() && nosc.error().message.find("config: ") == 0);
    std::printf("%s\n", failures ? "FAILED" : "OK");
    return failures ? 1 : 0;
}
