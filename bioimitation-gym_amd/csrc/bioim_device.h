// bioim_device.h — device-side model image (compute precision) built from a
// ModelPack at bioim_create() time.  Same information as the pack, with the
// reals converted to the kernel's precision and a few derived constants
// precomputed; the structural indices live in the compile-time topology
// (topologies.h) and are not repeated here.
#pragma once

#include <stdint.h>

#include "bioim_modelpack.h"

#define BIOIM_OBS_MAX 256

#define BIOIM_MAX_SPAN 8 /* muscle span: non-root dofs per muscle (max) */

#define BIOIM_UTAB 32 /* intervals of the per-segment u(x) initial-guess table */

template <typename Real>
struct DCurve {
    /* per quintic segment: x(u), y(u) in the power basis (Horner), from the
     * pack's Bernstein control points; x/y at u = 0 and u = 1 */
    Real cx[BIOIM_MAX_CURVESEG][6];
    Real cy[BIOIM_MAX_CURVESEG][6];
    Real xa[BIOIM_MAX_CURVESEG], xb[BIOIM_MAX_CURVESEG], ya[BIOIM_MAX_CURVESEG], yb[BIOIM_MAX_CURVESEG];
    /* segment search keys: xsep[s] = end x of segment s for s < nseg - 1,
     * +inf after (so the search needs no segment count); xa of unused
     * segments is +inf too (never bracketed by the fiber-velocity search) */
    Real xsep[BIOIM_MAX_CURVESEG];
    /* u at uniform x nodes of each segment, and du/dt at the same nodes
     * (t = (x - xa) inv_h, the table coordinate): the cubic Hermite start of
     * curve_eval (error <= 3.1e-5 before Newton, vs 1.2e-3 for linear
     * interpolation of ut).  Only starting guesses, so float in both
     * precisions (rounding 6e-8, far below the start error; keeps the fp64
     * 3D image inside 160 KiB of LDS) */
    float ut[BIOIM_MAX_CURVESEG][BIOIM_UTAB + 1];
    float mt[BIOIM_MAX_CURVESEG][BIOIM_UTAB + 1];
    Real inv_h[BIOIM_MAX_CURVESEG];               /* BIOIM_UTAB / (x_end - x_start)       */
    Real x0, y0, dydx0, x1, y1, dydx1;
    Real y_at0; /* y(0), host-evaluated: the fiber-velocity curve at rest (clamped fiber) */
    int32_t nseg, pad;
};

/* ------------------------------------------------------------------
 * Shared model image (SModel): the model data that lanes index at run time
 * (lane = body, muscle, path point, sphere).  One copy per workgroup is
 * staged into LDS at kernel start, so these lookups are ds_reads (~50 cycles)
 * instead of lane-divergent global loads (~200+ cycles at one wave per SIMD).
 * Curves are deduplicated (all muscles of the shipped models share one set). */
/* LDS bank padding of the lane-indexed model structs (lane l reads element
 * m(l) of an array of them): a stride of 50 dwords (fp64: 64-bit reads hit
 * bank (a/4) mod 64, lanes 0..15 on 16 distinct bank pairs) or 33 dwords
 * (fp32: 32-bit reads, bank (a/4) mod 32, an odd stride is conflict-free);
 * unpadded, SMuscle is 48 / 32 dwords: 4-way / 16-way conflicts. */
#ifndef BIOIM_LDS_PAD
#define BIOIM_LDS_PAD 1
#endif
template <typename Real>
struct SMuscle {
    Real fiso, lopt, inv_lopt, lts, inv_lts, lv; /* lv = lopt * vmax */
    Real tau_act, tau_deact, amin, beta, width, lmin, slow, mass, default_act, pad;
#if BIOIM_LDS_PAD
    Real pad_bank;    /* 17 reals + 16 ints: 50 dwords (fp64), 33 (fp32) */
#endif
    int32_t pt_off, npt;
    int32_t cv[4]; /* curve indices: fal, fv, fpe, fse */
    /* non-root dofs the path can move (union of its points' dofmasks minus
     * the floating base: a muscle's force is internal, so its generalized
     * force on the root dofs is zero) */
    int32_t nspan, pad2;
    int32_t span[BIOIM_MAX_SPAN];
};

template <typename Real>
struct DPathPt {
    int32_t type, cbody, cond_coord, mcoord; /* mcoord: moving point coordinate (-1 none) */
    int32_t mdof;                             /* its dof (-1 locked/none)                 */
    uint32_t dofmask;                         /* dofs moving this point                   */
    int32_t mf[3];                            /* moving point: slot of each axis' function (-1: loc) */
    int32_t pad;
#if BIOIM_LDS_PAD
    int32_t pad_bank[2];                      /* 12 ints + 17 reals: 46 dwords (fp64), 29 (fp32) */
#endif
    Real loc[3], R[9], p[3];
    Real lo, hi;
};

/* composite body: joint-local constants (lane = body in the kinematics) */
template <typename Real>
struct SBody {
    Real R_pf[9], p_pf[3], R_mb[9], p_mb[3];
    Real axis[6][3];
    Real mass, com[3], inertia[6];
    Real fa[6], fb[6];      /* linear / constant axis function: a q + b, b (the
                             * kind, coordinate and spline slot per axis are
                             * compile-time: T::axis_kind / axis_coord,
                             * TopoInfo::jslot) */
    int32_t pslot, pad;     /* the parent's frame slot (ground: NB)            */
};

template <typename Real>
struct SFn {
    int32_t type, coord, off, n;
    Real a, b;
};

/* compile-time facts of a topology (topologies.h) */
template <class T> struct TopoInfo {
    /* spatial-transform axes used by any body */
    static constexpr unsigned axes_used() {
        unsigned m = 0;
        for (int c = 0; c < T::NB; ++c)
            for (int a = 0; a < 6; ++a)
                if (T::axis_kind[c * 6 + a] >= 0) m |= 1u << a;
        return m;
    }
    /* function kinds at axis a over all bodies: bit (kind + 1), kind -1 = absent */
    static constexpr unsigned axis_kinds(int a) {
        unsigned m = 0;
        for (int c = 0; c < T::NB; ++c) m |= 1u << (T::axis_kind[c * 6 + a] + 1);
        return m;
    }
    /* (body, axis) pairs whose function is a spline: evaluated lane-parallel
     * before the joint kinematics, like the moving-point functions */
    static constexpr int njs() {
        int n = 0;
        for (int c = 0; c < T::NB; ++c)
            for (int a = 0; a < 6; ++a) n += T::axis_kind[c * 6 + a] == BIOIM_FN_SPLINE ? 1 : 0;
        return n;
    }
    /* function slots per dynamics call: moving-point functions, then joint splines */
    static constexpr int nslot() { return T::NMF + njs(); }
    /* function slot of body c's spline axis a (build_smodel assigns them in
     * body-major order after the moving-point slots), -1 if not a spline */
    static constexpr int jslot(int c, int a) {
        if (T::axis_kind[c * 6 + a] != BIOIM_FN_SPLINE) return -1;
        int n = T::NMF;
        for (int k = 0; k < c * 6 + a; ++k) n += T::axis_kind[k] == BIOIM_FN_SPLINE ? 1 : 0;
        return n;
    }
    static constexpr int depth_of(int c) {
        int l = 1;
        for (int p = T::parent[c]; p >= 0; p = T::parent[p]) ++l;
        return l;
    }
    static constexpr int depth() {
        int d = 0;
        for (int c = 0; c < T::NB; ++c) d = depth_of(c) > d ? depth_of(c) : d;
        return d;
    }
};

template <class T> struct SDim {
    static constexpr int NCV = T::NCURVE > 0 ? T::NCURVE : 1, NMU = T::NM > 0 ? T::NM : 1;
    static constexpr int NPT = T::NPT > 0 ? T::NPT : 1, NFN = T::NFN > 0 ? T::NFN : 1;
    static constexpr int NK = T::NKNOT > 0 ? T::NKNOT : 1, NCD = T::NC > 0 ? T::NC : 1, NDD = T::ND > 0 ? T::ND : 1;
    static constexpr int NP = NDD * (NDD + 1) / 2, NSD = T::NS > 0 ? T::NS : 1, NFD = T::NF > 0 ? T::NF : 1;
    static constexpr int NLD = T::NL > 0 ? T::NL : 1, NAD = T::NA > 0 ? T::NA : 1;
};

template <class T, typename Real>
struct SModel {
    using D = SDim<T>;
    DCurve<Real> curve[D::NCV];
    SMuscle<Real> mus[D::NMU];
    DPathPt<Real> pt[D::NPT];
    SBody<Real> body[T::NB];
    SFn<Real> fn[D::NFN];
    Real kx[D::NK], ky[D::NK], kb[D::NK], kc[D::NK], kd[D::NK];
    /* contact spheres and Hunt-Crossley parameters (lane = sphere) */
    Real sph_loc[D::NSD][3], sph_r[D::NSD];
    Real cf_kk[D::NFD], cf_c[D::NFD], cf_ms[D::NFD], cf_md[D::NFD], cf_mv[D::NFD], cf_vt[D::NFD];
    /* coordinate limit forces (lane = limit) */
    Real lim_qup[D::NLD], lim_qlow[D::NLD], lim_kup[D::NLD], lim_klow[D::NLD], lim_damp[D::NLD], lim_trans[D::NLD];
    Real lim_itrans[D::NLD];   /* 1 / transition width */
    /* coordinate actuators / PD gains (lane = actuator) */
    Real ca_opt[D::NAD], ca_min[D::NAD], ca_max[D::NAD], kp[D::NAD], kv[D::NAD];
    /* index tables */
    int32_t coord_dof[D::NCD], dof_cb[D::NDD], dof_coord[D::NDD];
    uint32_t dofmask[T::NB];
    /* moving-point location functions: evaluated lane-parallel once per
     * dynamics call into the env's MF slots (function index, coordinate) */
    int32_t mf_fn[TopoInfo<T>::nslot() > 0 ? TopoInfo<T>::nslot() : 1];
    int32_t mf_coord[TopoInfo<T>::nslot() > 0 ? TopoInfo<T>::nslot() : 1];
    /* OpenSim bodies reported in observations / rewards (lane = body) */
    Real os_p[T::NOS][3];
    int32_t os_cb[T::NOS];
    int32_t obs_slot[T::NOBP + T::NOBV]; /* report slots of the observed bodies (NOS = COM) */
    int32_t rw_slot[BIOIM_NREFBODY];     /* report slots of the reward's reference bodies  */
    /* root-to-body joint chain, front-padded with the identity joint slot NB */
    int32_t chain[T::NB][TopoInfo<T>::depth()];
    int32_t sph_cb[D::NSD], sph_force[D::NSD], lim_coord[D::NLD], lim_dof[D::NLD], act_dof[D::NAD];
    /* muscle torque gather (lane = dof): the TAU slots (muscle slot s, span
     * entry k -> s * MAXSPAN + k) holding -F_t dL/dq_d, padded with the zero
     * slot */
    uint8_t tau_src[D::NDD][T::MAXARM];
    /* force-report body of each contact sphere (its OpenSim body, a report
     * slot); last and byte-sized so that it lands in the image's 16-byte
     * round-up and leaves every other offset where it was */
    uint8_t sph_ob[D::NSD];
};

/* bytes of the LDS image (16-byte granules for the cooperative copy) */
template <class T, typename Real> constexpr size_t smodel_bytes() { return (sizeof(SModel<T, Real>) + 15) & ~size_t(15); }

template <typename Real>
struct DModel {
    /* composite bodies (wave-uniform reads: observation / reward reporting) */
    Real mass[BIOIM_MAX_CBODY], com[BIOIM_MAX_CBODY][3];
    Real coord_default[BIOIM_MAX_COORD];
    int32_t coord_dof[BIOIM_MAX_COORD];
    Real os_R[BIOIM_MAX_OSBODY][9], os_p[BIOIM_MAX_OSBODY][3];
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
    double *hrk;   /* [N] RK-Merson step size carried to the next env step (0: none yet) */
    /* budgeted RK launches (bioim_set_rk_budget): an env whose step is not
     * finished within the launch's attempt budget is suspended at an accepted
     * RK point and resumed by the next launch */
    int32_t *pend;  /* [N] 1: suspended mid-step                                      */
    double *rkt, *rkh; /* [N] its integration time and proposed step size            */
    int32_t *rka;   /* [N] attempts spent on the step so far                          */
    Real *ctl, *cur; /* [nact][N] its held controls and smoothed actions               */
    Real *vnw;      /* [nm][N] fiber-velocity warm starts (the last call's roots)      */
    /* [N] RK kernels' counters: low 32 bits the dynamics evaluations so far
     * (bioim_eval_count), high 32 the env steps finished (bioim_finished_count);
     * one 64-bit update per launch */
    uint64_t *rkev;
    /* the realize cache (step kernels of the planar muscle models, DESIGN.md
     * 5.10): [N][cache_dim] per env, written by every realize for the next
     * launch's first substep — the packed lower M + h C + h^2 K and the
     * implicit right-hand side at that substep's h (the state does not change
     * between the realize and that substep; muscle forces do not depend on
     * the excitations), per muscle the fiber-velocity root, dv/dl and the
     * clamp flag, then that h; valid[N] = 1 when the row belongs to the
     * current state (every other writer of the state clears it) */
    Real *cache;
    int32_t *cache_ok;
};
