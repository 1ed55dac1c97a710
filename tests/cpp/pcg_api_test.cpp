// pcg_api_test.cpp -- the reference's single-tet fixture (tests/pcg_test.cpp:35-121,
// tests/newmark_stepper_test.cpp:41-127) driven through the C++ mirror include/cwf_hip.hpp.
// Expected values are the reference outputs recorded in SURVEY.md section 8c.
#include <array>
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/cwf_hip.hpp"

static int failures = 0;
#define EXPECT(c)                                                       \
    do                                                                  \
    {                                                                   \
        if (!(c))                                                       \
        {                                                               \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
            ++failures;                                                 \
        }                                                               \
    } while (0)

static std::string g9(float v)
{
    char b[64];
    std::snprintf(b, sizeof b, "%.9g", v);
    return b;
}

int main()
{
    using namespace cwf::hip;
    const std::vector<double> coords = {0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1};
    const std::vector<uint32_t> tets = {0, 1, 2, 3};
    const std::vector<uint32_t> mat = {0};
    const double density = 2500.0;
    std::vector<float> grads(24), vol(1), mass32(4);
    std::vector<double> mass64(4);
    std::vector<uint32_t> off(5), ae(4), conn(8);
    std::vector<uint8_t> al(4);
    EXPECT(cwf_preprocess_tets(4, 1, coords.data(), tets.data(), mat.data(), &density, 1, grads.data(), vol.data(),
                               mass64.data(), mass32.data(), off.data(), ae.data(), al.data(), conn.data()) == 0);
    // materials.hpp:116-134, E = 30 GPa, nu = 0.2; Rayleigh xi = 0.02, w = 5..50; dt = 0.01
    const double E = 30.0e9, nu = 0.2;
    const double lam = (nu * E) / ((1.0 + nu) * (1.0 - 2.0 * nu)), mu = E / (2.0 * (1.0 + nu)), c = lam + 2.0 * mu;
    const std::array<double, 36> D = {c, lam, lam, 0, 0, 0, lam, c, lam, 0, 0, 0, lam, lam, c, 0, 0, 0,
                                      0, 0, 0, mu, 0, 0, 0, 0, 0, 0, mu, 0, 0, 0, 0, 0, 0, mu};
    const double ra = 2.0 * 0.02 * 5.0 * 50.0 / 55.0, rb = 2.0 * 0.02 / 55.0;
    const double dt = 0.01, a0 = 1.0 / (0.25 * dt * dt), a1 = 0.5 / (0.25 * dt);
    const std::vector<uint32_t> bc = {7, 7, 7, 0};
    std::array<std::array<double, 36>, 1> mats{D};
    pcg::MatrixFreeSystem sys{conn, grads, vol, mat, mats, mass32, bc, 4, 1, 12, 1.0 + a1 * rb, a0 + a1 * ra, 256, 1};

    pcg::MatrixFreeWorkspace ws;
    std::vector<float> in(12), out(12);
    for (int i = 0; i < 12; ++i)
        in[i] = static_cast<float>(0.1 * static_cast<double>(i + 1));
    auto st = pcg::apply_keff(sys, in, out, ws);
    EXPECT(st.has_value());
    EXPECT(g9(out[9]) == "2.39053414e+09" && g9(out[10]) == "2.62958771e+09" && g9(out[11]) == "7.64136858e+09");
    for (int i = 0; i < 9; ++i)
        EXPECT(out[i] == in[i]);  // Dirichlet identity rows

    std::vector<float> rhs(12, 0.0f), x(12, 0.0f), r(12, 0.0f);
    rhs[11] = -500.0f;
    auto tel = pcg::solve_pcg(sys, rhs, {64, 3.0e-4, false}, {x, r, {}, {}, {}, {}}, ws);
    EXPECT(tel.has_value() && tel->converged && tel->iterations == 1);
    EXPECT(g9(x[11]) == "-7.85199674e-08");

    std::vector<float> inv(36);
    EXPECT(pcg::build_block_jacobi_inverse(sys, ws, inv).has_value());
    EXPECT(inv[0] == 1.0f && inv[1] == 0.0f);  // constrained rows -> identity

    auto bad = pcg::solve_pcg(sys, rhs, {0, 3.0e-4, false}, {x, r, {}, {}, {}, {}}, ws);
    EXPECT(!bad.has_value() && bad.error().message == "max_iterations must be >= 1");

    std::vector<float> f(12, 0.0f), bcv(12, 0.0f);
    f[11] = -500.0f;
    newmark::Stepper stepper(sys, f, bcv, {ra, rb}, {3.0e-4, 1.0e-5, 64}, {dt, false, 0.0, 0.0});
    auto s1 = stepper.step(0.0, false);
    EXPECT(s1.has_value() && s1->pcg.iterations == 1);
    std::vector<float> u(12);
    EXPECT(stepper.state(0, u));
    EXPECT(g9(u[11]) == "-7.85199674e-08");  // from rest: u = u_pred + x = x
    auto s2 = stepper.step(stepper.current_time(), true);
    EXPECT(s2.has_value() && s2->paused_mode && s2->applied_tolerance == 1.0e-5);
    // the device-side load rewrite: external_force = f32(base + c * pattern)
    std::vector<double> base(12, 0.0), pattern(12, 0.0);
    base[2] = -9.81;
    pattern[11] = -500.0;
    EXPECT(stepper.set_load_pattern(base, pattern) && stepper.set_load_scale(0.5));
    std::vector<float> fe(12);
    EXPECT(stepper.state(4, fe));
    EXPECT(fe[2] == (float)-9.81 && fe[11] == -250.0f && fe[0] == 0.0f);

    // two-entry breadcrumbs come back as two entries (pcg.cpp:566-570, 609-613), so a caller rebuilds a
    // PcgError equal to the reference's
    const std::vector<uint32_t> bad_mat = {1};
    pcg::MatrixFreeSystem sys_m{conn, grads, vol, bad_mat, mats, mass32, bc, 4, 1, 12, 1.0, 0.0, 256, 1};
    pcg::MatrixFreeWorkspace ws_m;
    auto em = pcg::apply_keff(sys_m, in, out, ws_m);
    EXPECT(!em.has_value() && em.error().message == "element references material out of range");
    EXPECT(!em.has_value() && em.error().context == std::vector<std::string>({"element=0", "material_index=1"}));
    std::vector<uint32_t> bad_conn = conn;
    bad_conn[2] = 9;
    pcg::MatrixFreeSystem sys_n{bad_conn, grads, vol, mat, mats, mass32, bc, 4, 1, 12, 1.0, 0.0, 256, 1};
    pcg::MatrixFreeWorkspace ws_n;
    auto en = pcg::apply_keff(sys_n, in, out, ws_n);
    EXPECT(!en.has_value() && en.error().message == "element connectivity references node out of range");
    EXPECT(!en.has_value() && en.error().context == std::vector<std::string>({"element=0", "node=9"}));
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
    return failures ? 1 : 0;
}
