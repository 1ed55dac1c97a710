/*
 * cwf_oracle.h -- CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY
 * (see cwf_oracle.c header). Plain C99, no GPU, no dependency on the product library.
 */
#ifndef CWF_ORACLE_H
#define CWF_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum
{
    ORC_OK = 0,
    ORC_ERR_SIZE = -1,
    ORC_ERR_NODE_RANGE = -2,
    ORC_ERR_MATERIAL_RANGE = -3,
    ORC_ERR_MATERIALS = -4,
    ORC_ERR_REDUCTION = -5,
    ORC_ERR_MAX_ITERATIONS = -6,
    ORC_ERR_RHO_ZERO = -7,
    ORC_ERR_DENOM_ZERO = -8,
    ORC_ERR_ALLOC = -9,
    ORC_ERR_VOLUME = -10
};

/* mirrors cwf::gpu::pcg::MatrixFreeSystem (include/cwf/gpu/pcg.hpp:67-86) */
typedef struct orc_system
{
    uint64_t node_count, element_count, dof_count;
    const uint32_t *connectivity;   /* [E*8] */
    const float *gradients;         /* [E*24] */
    const float *volume;            /* [E] */
    const uint32_t *material_index; /* [E] */
    const double *stiffness;        /* [M*36] */
    uint64_t material_count;
    const float *lumped_mass; /* [N] */
    const uint32_t *bc_mask;  /* [N] */
    double stiffness_scale, mass_factor;
    uint64_t reduction_block, reduction_partials;
} orc_system;

/* mirrors PcgTelemetry (pcg.hpp:125-133) */
typedef struct orc_telemetry
{
    uint64_t iterations;
    double residual_norm, rhs_norm, alpha_last, beta_last;
    int32_t converged;
    int32_t pad;
} orc_telemetry;

typedef struct orc_step_telemetry
{
    double simulation_time, time_step, applied_tolerance;
    int32_t paused_mode, dt_increased, dt_decreased, dt_clamped_min, dt_clamped_max, pad;
    orc_telemetry pcg;
} orc_step_telemetry;

/* state of the Stepper CPU branch (newmark_stepper.hpp:145-179), interleaved dof = 3n+k */
typedef struct orc_stepper
{
    const orc_system *system;
    double rayleigh_alpha, rayleigh_beta;
    double runtime_tolerance, pause_tolerance;
    uint64_t max_iterations;
    int32_t adaptive, warm_start;
    double min_dt, max_dt;
    double low_iteration_ratio, increase_factor, decrease_factor;
    double dt, beta, gamma, accumulated_time;
    uint64_t frame_index;
    float *u, *v, *a;               /* nodes.displacement/velocity/acceleration */
    const float *external_force;    /* nodes.external_force */
    const float *bc_value;          /* nodes.bc_value */
    float *u_pred, *v_pred;         /* predicted_displacement_/velocity_ */
    float *rhs, *damping_rhs, *damping_out;
    float *x, *r, *p, *z, *Ap;      /* solver buffers (x persists for warm start) */
    double *partials;
} orc_stepper;

typedef struct orc_dense_stats
{
    uint64_t iterations;
    double residual_norm;
    int32_t converged, pad;
} orc_dense_stats;

const char *orc_last_message(void);
const char *orc_last_context(void);

void orc_make_stiffness(double E, double nu, double *D36);
void orc_rayleigh(double xi, double w1, double w2, double *alpha, double *beta);
void orc_newmark_coefficients(double dt, double beta, double gamma, double *a, double *upd);

int orc_preprocess_tets(uint64_t node_count, uint64_t element_count, const double *coords, const uint32_t *tets,
                        const uint32_t *material_index, const double *density, float *grads24, float *volume,
                        double *mass64, float *mass32, uint32_t *offsets, uint32_t *adj_elem, uint8_t *adj_local,
                        uint32_t *conn8);
double orc_evaluate_curve(const double *t, const double *v, uint64_t n, double time);
void orc_gravity_loads(uint64_t node_count, const double *mass64, const double *gravity, double *loads);
void orc_point_loads(uint64_t count, const uint32_t *nodes, const double *value, double scale, double *loads);

int orc_apply_keff(const orc_system *s, const float *in, float *out);
int orc_block_jacobi(const orc_system *s, float *inv_out);
double orc_dot(const orc_system *s, const float *a, const float *b, double *partials);
int orc_solve_pcg(const orc_system *s, const float *rhs, uint64_t max_iterations, double relative_tolerance,
                  int warm_start, float *x, float *r, float *p, float *z, float *Ap, double *partials,
                  orc_telemetry *tel, double *residual_history);
int orc_stepper_step(orc_stepper *t, double sim_time, int paused, orc_step_telemetry *out);
/* src/post/derived_fields.cpp:139-211; outputs 13 floats per element / node (either may be NULL) */
int orc_derived_fields(const orc_system *s, const float *u, float *elem_out, float *node_out);

int orc_dense_assemble(uint64_t node_count, uint64_t element_count, const uint32_t *tets, const double *grads64,
                       const double *volume64, const uint32_t *material_index, const double *stiffness, double *K);
int orc_dense_newmark_step(uint64_t n, const double *K, const double *mass_diag, const double *load,
                           const uint8_t *mask, const double *targets, double r_alpha, double r_beta,
                           const double *coef, const double *u0, const double *v0, const double *acc0,
                           double tolerance, uint64_t max_iterations, double *u1, double *v1, double *acc1,
                           orc_dense_stats *stats);

/* native hex8 (hex8_oracle.c; parity unpinned: the reference rejects hex8) */
int orc_hex8_preprocess(uint64_t N, uint64_t E, const double *coords, const uint32_t *conn8,
                        const uint32_t *material_index, const double *density, uint64_t material_count,
                        double *volume, double *mass64, float *grads24);
int orc_hex8_apply(uint64_t N, uint64_t E, const double *coords, const uint32_t *conn8, const uint32_t *material_index,
                   const double *D36, double sK, double sM, const float *mass, const uint32_t *mask, const float *x,
                   float *y, double *acc);
int orc_hex8_apply64(uint64_t N, uint64_t E, const double *coords, const uint32_t *conn8,
                     const uint32_t *material_index, const double *D36, double sK, double sM, const float *mass,
                     const uint32_t *mask, const double *x, double *y);
int orc_hex8_diag_blocks(uint64_t N, uint64_t E, const double *coords, const uint32_t *conn8,
                         const uint32_t *material_index, const double *D36, double sK, double *blocks);

#ifdef __cplusplus
}
#endif
#endif
