// bioim_device.h — device-side model image (compute precision) built from a
// ModelPack at bioim_create() time.  Same information as the pack, with the
// reals converted to the kernel's precision and a few derived constants
// precomputed; the structural indices live in the compile-time topology
// (topologies.h) and are not repeated here.
#pragma once

#include <stdint.h>

#include "bioim_modelpack.h"

#define BIOIM_OBS_MAX 256

#define BIOIM_UTAB 32 /* intervals of the per-segment u(x) initial-guess table */

template <typename Real>
struct DCurve {
    Real x[BIOIM_MAX_CURVESEG][6];
    Real y[BIOIM_MAX_CURVESEG][6];
    Real ut[BIOIM_MAX_CURVESEG][BIOIM_UTAB + 1]; /* u at uniform x nodes of each segment */
    Real inv_h[BIOIM_MAX_CURVESEG];               /* BIOIM_UTAB / (x_end - x_start)       */
    Real x0, y0, dydx0, x1, y1, dydx1;
    int32_t nseg, pad;
};

template <typename Real>
struct DMuscle {
    Real fiso, lopt, inv_lopt, lts, inv_lts, lv; /* lv = lopt * vmax */
    Real tau_act, tau_deact, amin, beta, width, lmin, slow, mass, default_act;
    int32_t pt_off, npt;
    DCurve<Real> fal, fv, fpe, fse;
};

template <typename Real>
struct DPathPt {
    int32_t type, cbody, cond_coord, mcoord; /* mcoord: moving point coordinate (-1 none) */
    int32_t mdof;                             /* its dof (-1 locked/none)                 */
    uint32_t dofmask;                         /* dofs moving this point                   */
    int32_t fn[3];
    int32_t pad;
    Real loc[3], R[9], p[3];
    Real lo, hi;
};

template <typename Real>
struct DModel {
    /* composite bodies */
    Real R_pf[BIOIM_MAX_CBODY][9], p_pf[BIOIM_MAX_CBODY][3];
    Real R_mb[BIOIM_MAX_CBODY][9], p_mb[BIOIM_MAX_CBODY][3];
    Real axis[BIOIM_MAX_CBODY][6][3];
    Real mass[BIOIM_MAX_CBODY], com[BIOIM_MAX_CBODY][3], inertia[BIOIM_MAX_CBODY][6];
    int32_t fn[BIOIM_MAX_CBODY][6];
    /* functions */
    int32_t fn_type[BIOIM_MAX_FN], fn_coord[BIOIM_MAX_FN], fn_off[BIOIM_MAX_FN], fn_n[BIOIM_MAX_FN];
    Real fn_a[BIOIM_MAX_FN], fn_b[BIOIM_MAX_FN];
    Real kx[BIOIM_MAX_KNOTS], ky[BIOIM_MAX_KNOTS], kb[BIOIM_MAX_KNOTS], kc[BIOIM_MAX_KNOTS], kd[BIOIM_MAX_KNOTS];
    Real coord_default[BIOIM_MAX_COORD];
    int32_t coord_dof[BIOIM_MAX_COORD];
    Real os_R[BIOIM_MAX_OSBODY][9], os_p[BIOIM_MAX_OSBODY][3];
    /* muscles */
    DMuscle<Real> mus[BIOIM_MAX_MUSCLE];
    DPathPt<Real> pt[BIOIM_MAX_PATHPT];
    /* contact / limits / actuators */
    Real sph_loc[BIOIM_MAX_SPHERE][3], sph_r[BIOIM_MAX_SPHERE];
    Real cf_kk[BIOIM_MAX_CFORCE], cf_c[BIOIM_MAX_CFORCE], cf_ms[BIOIM_MAX_CFORCE], cf_md[BIOIM_MAX_CFORCE],
        cf_mv[BIOIM_MAX_CFORCE], cf_vt[BIOIM_MAX_CFORCE];
    Real lim_qup[BIOIM_MAX_LIMIT], lim_qlow[BIOIM_MAX_LIMIT], lim_kup[BIOIM_MAX_LIMIT], lim_klow[BIOIM_MAX_LIMIT],
        lim_damp[BIOIM_MAX_LIMIT], lim_trans[BIOIM_MAX_LIMIT];
    Real ca_opt[BIOIM_MAX_ACT], ca_min[BIOIM_MAX_ACT], ca_max[BIOIM_MAX_ACT];
    Real kp[BIOIM_MAX_ACT], kv[BIOIM_MAX_ACT];
    /* lane-parallel index tables (runtime copies of the topology) */
    uint32_t anc[BIOIM_MAX_CBODY], dofmask[BIOIM_MAX_CBODY];
    int32_t dof_cb[BIOIM_MAX_COORD];
    int32_t e_l[BIOIM_MAX_COORD * (BIOIM_MAX_COORD + 1) / 2], e_k[BIOIM_MAX_COORD * (BIOIM_MAX_COORD + 1) / 2],
        e_c[BIOIM_MAX_COORD * (BIOIM_MAX_COORD + 1) / 2];
    int32_t sph_cb[BIOIM_MAX_SPHERE], sph_force[BIOIM_MAX_SPHERE];
    int32_t lim_coord[BIOIM_MAX_LIMIT], lim_dof[BIOIM_MAX_LIMIT];
    int32_t act_dof[BIOIM_MAX_ACT];
    int32_t float_origin, pad1;
    /* env semantics */
    Real w_imitate, w_effort, w_action, action_r_scale, max_actuation, total_mass, weight, moment;
    Real torso_y_min, limit_force_max, acc_max;
    Real gravity[3];
    int32_t horizon, cycle, n_episode, reset_hi, nsub, nrows, obs_dim, info_dim;
    uint32_t env_flags;
    int32_t pad0;
    double step_size;
    /* reference motion */
    double ref_time[BIOIM_MAX_REFROWS];
    int32_t ref_istep[BIOIM_MAX_REFROWS];
    Real ref_q[BIOIM_MAX_REFROWS][BIOIM_MAX_COORD];
    Real ref_u[BIOIM_MAX_REFROWS][BIOIM_MAX_COORD];
    Real ref_x[BIOIM_MAX_REFROWS][BIOIM_NREFBODY][3];
};

/* Per-launch state pointers (SoA, env index fastest). */
template <typename Real>
struct DState {
    Real *q, *u, *act, *lce, *hist, *last, *old_px; /* [ndof][N] [ndof][N] [nm][N] [nm][N] [H][nact][N] [nact][N] [N] */
    double *t;
    int32_t *istep, *has_last, *done, *resets;
};
