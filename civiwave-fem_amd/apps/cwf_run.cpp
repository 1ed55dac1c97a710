// cwf_run -- native scenario runner over the C-ABI:
//
//   cwf_run scenario.yaml [--steps N] [--out DIR] [--mode parity|fast] [--device K] [--paused]
//                         [--time-varying-loads]
//
// The reference has no such executable (its only binary is the viewer demo); this drives the viewer
// backend's sequence (src/ui/viewer.cpp:200-277) through cwf_scenario_*: one JSON line per frame
// (frame, time, dt, iterations, residual, converged, dt_increased, dt_decreased), then a summary line.
// Same flags and output as `python -m cwf.run`; exit status 1 with "error: <message> <context>" on stderr.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "cwf_hip.h"

static int usage()
{
    std::fprintf(stderr,
                 "usage: cwf_run scenario.yaml [--steps N] [--out DIR] [--mode parity|fast] [--device K]\n"
                 "               [--paused] [--time-varying-loads]\n");
    return 2;
}

static int fail(const char *what)
{
    std::string ctx = cwf_hip_last_context(nullptr);
    for (char &c : ctx)
        if (c == '\n')
            c = ' ';
    std::fprintf(stderr, "error: %s%s %s\n", what, cwf_hip_last_error(nullptr), ctx.c_str());
    return 1;
}

int main(int argc, char **argv)
{
    const char *scenario = nullptr, *out = nullptr;
    long steps = 10;
    int mode = CWF_MODE_PARITY, device = 0, paused = 0, flags = 0;
    for (int i = 1; i < argc; ++i)
    {
        const std::string a = argv[i];
        const bool has_val = i + 1 < argc;
        if (a == "--steps" && has_val)
            steps = std::strtol(argv[++i], nullptr, 10);
        else if (a == "--out" && has_val)
            out = argv[++i];
        else if (a == "--mode" && has_val)
        {
            const std::string m = argv[++i];
            if (m != "parity" && m != "fast")
                return usage();
            mode = m == "fast" ? CWF_MODE_FAST : CWF_MODE_PARITY;
        }
        else if (a == "--device" && has_val)
            device = std::atoi(argv[++i]);
        else if (a == "--paused")
            paused = 1;
        else if (a == "--time-varying-loads")
            flags |= CWF_SCENARIO_TIME_VARYING_LOADS;
        else if (!a.empty() && a[0] != '-' && !scenario)
            scenario = argv[i];
        else
            return usage();
    }
    if (!scenario || steps < 0)
        return usage();
    cwf_scenario *sc = nullptr;
    if (cwf_scenario_create(scenario, mode, device, flags, &sc))
        return fail("");
    uint64_t N = 0, E = 0, D = 0;
    cwf_scenario_info(sc, &N, &E, &D);
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t total_iters = 0;
    double t_sim = 0.0;
    for (long frame = 0; frame < steps; ++frame)
    {
        cwf_step_telemetry tel{};
        if (cwf_scenario_step(sc, paused, &tel))
        {
            char what[64];
            std::snprintf(what, sizeof what, "step %ld: ", frame);
            const int rc = fail(what);
            cwf_scenario_destroy(sc);
            return rc;
        }
        t_sim = tel.simulation_time + tel.time_step;
        total_iters += tel.pcg.iterations;
        if (out && cwf_scenario_output_frame(sc, out))
        {
            char what[64];
            std::snprintf(what, sizeof what, "output frame %ld: ", frame);
            const int rc = fail(what);
            cwf_scenario_destroy(sc);
            return rc;
        }
        std::printf("{\"frame\": %ld, \"time\": %.17g, \"dt\": %.17g, \"iterations\": %llu, \"residual\": %.17g, "
                    "\"converged\": %s, \"dt_increased\": %s, \"dt_decreased\": %s}\n",
                    frame, t_sim, tel.time_step, (unsigned long long)tel.pcg.iterations, tel.pcg.residual_norm,
                    tel.pcg.converged ? "true" : "false", tel.dt_increased ? "true" : "false",
                    tel.dt_decreased ? "true" : "false");
        std::fflush(stdout);
    }
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("{\"summary\": {\"scenario\": \"%s\", \"nodes\": %llu, \"elements\": %llu, \"dofs\": %llu, "
                "\"steps\": %ld, \"pcg_iterations\": %llu, \"wall_s\": %.6f, \"final_time\": %.17g, "
                "\"mode\": \"%s\"}}\n",
                scenario, (unsigned long long)N, (unsigned long long)E, (unsigned long long)D, steps,
                (unsigned long long)total_iters, wall, t_sim, mode == CWF_MODE_FAST ? "fast" : "parity");
    cwf_scenario_destroy(sc);
    return 0;
}
