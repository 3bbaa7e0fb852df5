/*
 * bioim_modelpack.h — the flat, pointer-free ModelPack consumed at the C-ABI.
 *
 * A ModelPack is the compiled form of one registered environment ID: the
 * OpenSim model after the reference's load-time transforms
 * (construct_predictive_model  opensim_utils.py:204-222,
 *  convert_model_to_torque_actuated opensim_utils.py:238-270,
 *  convert_model_to_prosthetic muscle_locked_knee_imitation_env3D.py:104-126),
 * welded bodies merged into composite bodies, every function pre-fitted
 * (SimmSpline coefficients, Millard quintic-Bezier control points), plus the
 * env-level semantics (obs layout, reward, termination) and the reference
 * motion tables (q_d, u_d, x_d of muscle_walking_imitation_env2D.py:61-71).
 *
 * The pack is produced on the host by bioimitation/modelpack.py and is the
 * only model input of bioim_create() (include/bioim.h).  All reals are
 * float64; the device path converts to its compute precision at create time.
 *
 * Frame conventions: a transform (R, p) maps child coordinates to parent
 * coordinates, x_parent = R x_child + p; R is row-major 3x3.
 */
#ifndef BIOIM_MODELPACK_H
#define BIOIM_MODELPACK_H

#include <stdint.h>

#define BIOIM_PACK_MAGIC   0x4D4F4942u /* "BIOM" */
#define BIOIM_PACK_VERSION 3 /* 3: bioim_sphere_t carries obody (40 -> 48 bytes) */

#define BIOIM_MAX_COORD    24
#define BIOIM_MAX_CBODY    12
#define BIOIM_MAX_OSBODY   24
#define BIOIM_MAX_FN       96
#define BIOIM_MAX_KNOTS    1536
#define BIOIM_MAX_MUSCLE   24
#define BIOIM_MAX_PATHPT   160
#define BIOIM_MAX_SPHERE   8
#define BIOIM_MAX_CFORCE   4
#define BIOIM_MAX_LIMIT    12
#define BIOIM_MAX_ACT      24
#define BIOIM_MAX_CURVESEG 6
#define BIOIM_MAX_OBSBODY  12
#define BIOIM_MAX_REFROWS  512
#define BIOIM_NREFBODY     9   /* center_of_mass, femur_r, femur_l, tibia_r, tibia_l, talus_r, talus_l, calcn_r, calcn_l */
#define BIOIM_MAX_HORIZON  8

/* function kinds (OpenSim Function subclasses used by the shipped models) */
#define BIOIM_FN_CONST   0 /* value = b                                  */
#define BIOIM_FN_LINEAR  1 /* value = a*q + b   (LinearFunction)          */
#define BIOIM_FN_SPLINE  2 /* value = a*S(q)    (SimmSpline / MultiplierFunction(SimmSpline)) */

/* path point kinds (PathPoint / ConditionalPathPoint / MovingPathPoint) */
#define BIOIM_PT_FIXED   0
#define BIOIM_PT_COND    1
#define BIOIM_PT_MOVING  2

/* env_flags */
#define BIOIM_ENV_MUSCLE       (1u << 0) /* muscle-actuated (else coordinate actuators)      */
#define BIOIM_ENV_HAS_TZ       (1u << 1) /* pelvis_tz exists: 3D relative body positions      */
#define BIOIM_ENV_REWARD_FEET  (1u << 2) /* reward multiplies imitation by (foot_l+foot_r)    */
#define BIOIM_ENV_DONE_CROSS   (1u << 3) /* done when calcn_r.z - calcn_l.z < 0               */
#define BIOIM_ENV_RAW_ACTION   (1u << 4) /* physics gets the raw action, not the mean (palsy) */
#define BIOIM_ENV_TARGET_OBS   (1u << 5) /* config use_target_obs                             */
#define BIOIM_ENV_GRF_OBS      (1u << 6) /* config use_GRF                                    */
#define BIOIM_ENV_PD           (1u << 7) /* torque env: PD law on the action                  */
#define BIOIM_ENV_PHASE_ISTEP  (1u << 8) /* informational only: phase from istep (all envs)   */

typedef struct {
    int32_t type;     /* BIOIM_FN_*                                           */
    int32_t coord;    /* index into the full coordinate vector, -1 = none     */
    int32_t knot_off; /* spline: first knot in knot_* arrays                  */
    int32_t nknots;   /* spline: number of knots                              */
    double  a, b;
} bioim_fn_t;

/* A composite body: one moving OpenSim body plus every body welded to it. */
typedef struct {
    int32_t parent;   /* composite index, -1 = ground                          */
    int32_t fn[6];    /* transform-axis functions rot1..3, trans1..3; -1 = none */
    int32_t pad;
    double  R_pf[9], p_pf[3]; /* joint frame F expressed in the parent composite frame */
    double  R_mb[9], p_mb[3]; /* composite body frame expressed in the joint frame M   */
    double  axis[6][3];       /* rotation axes (body-fixed sequence) then translation axes (in F) */
    double  mass, com[3];     /* merged mass properties, composite frame           */
    double  inertia[6];       /* about the COM: xx yy zz xy xz yz                  */
} bioim_cbody_t;

typedef struct {
    int32_t motion;   /* 0 rotational, 1 translational                         */
    int32_t locked;
    int32_t dof;      /* index into the free-DOF vector, -1 when locked         */
    int32_t cbody;    /* composite body whose inboard joint owns the coordinate */
    double  default_value, range_min, range_max;
} bioim_coord_t;

/* OpenSim body -> composite body (reported body kinematics). */
typedef struct {
    int32_t cbody, pad;
    double  R[9], p[3];       /* OpenSim body frame expressed in the composite frame */
    double  mass, com[3];     /* own mass properties in the OpenSim body frame       */
} bioim_osbody_t;

typedef struct {
    int32_t cbody;
    int32_t type;             /* BIOIM_PT_*                                     */
    int32_t cond_coord;       /* conditional: coordinate index                   */
    int32_t fn[3];            /* moving: x/y/z location functions, -1 = use loc[] */
    double  loc[3];           /* fixed/conditional: composite frame; moving: OpenSim body frame */
    double  R[9], p[3];       /* moving: OpenSim body frame in composite frame   */
    double  range_lo, range_hi;
} bioim_pathpt_t;

/* SmoothSegmentedFunction: nseg quintic Bezier segments + linear extrapolation. */
typedef struct {
    int32_t nseg, pad;
    double  x[BIOIM_MAX_CURVESEG][6];
    double  y[BIOIM_MAX_CURVESEG][6];
    double  x0, y0, dydx0;    /* left end, left extrapolation slope   */
    double  x1, y1, dydx1;    /* right end, right extrapolation slope */
} bioim_curve_t;

/* Millard2012EquilibriumMuscle (damped, compliant tendon, fixed-width pennation). */
typedef struct {
    int32_t pt_off, npt;
    double  fiso, lopt, lts, alpha_opt, vmax;
    double  tau_act, tau_deact, amin, damping, default_act;
    double  width;            /* lopt * sin(alpha_opt) (fixed-width pennation)  */
    double  lmin;             /* minimum fiber length                           */
    double  slow_twitch;      /* cost-of-transport slow-twitch ratio            */
    double  mass;             /* fiso / 0.25e6 * 1059.7 * lopt                  */
    bioim_curve_t fal, fv, fpe, fse;
} bioim_muscle_t;

typedef struct {
    int32_t cbody, force;     /* composite body, owning HuntCrossleyForce        */
    double  loc[3];           /* center in composite frame                       */
    double  radius;
    int32_t obody, pad_;      /* the OpenSim body (osbody index) the sphere is on:
                                 its ForceReporter record entry (foot side)       */
} bioim_sphere_t;

typedef struct {
    double stiffness, dissipation, static_friction, dynamic_friction,
           viscous_friction, transition_velocity;
} bioim_cforce_t;

typedef struct {
    int32_t coord, dof;
    double  qup, qlow;        /* radians (or m)                                  */
    double  kup, klow;        /* stiffness already scaled per radian (x 180/pi)  */
    double  damping;          /* already scaled per radian/s                     */
    double  trans;            /* transition width, radians                       */
} bioim_limit_t;

typedef struct {
    int32_t coord, dof;
    double  optimal_force, min_control, max_control;
} bioim_coordact_t;

typedef struct {
    uint32_t magic, version;
    char     env_id[48];

    /* model sizes */
    int32_t ncoord, ndof, ncbody, nosbody;
    int32_t nfn, nknots, nmuscle, npathpt;
    int32_t nsphere, ncforce, nlimit, ncoordact;

    /* env-level semantics */
    uint32_t env_flags;
    int32_t nact, obs_dim, info_dim;
    int32_t nsub;             /* fixed integrator substeps per env step          */
    int32_t horizon;          /* action smoothing deque length                  */
    int32_t cycle;            /* gait cycle length (phase)                       */
    int32_t n_episode;        /* N: done when istep >= N                         */
    int32_t reset_hi;         /* reset index ~ randint(0, reset_hi) (inclusive)   */
    int32_t coord_tx, coord_ty, coord_tz;
    int32_t torso_body, calcn_r_body, calcn_l_body;
    int32_t n_obs_bpos, n_obs_bvel;
    int32_t obs_bpos[BIOIM_MAX_OBSBODY];   /* OpenSim body index, -1 = center of mass */
    int32_t obs_bvel[BIOIM_MAX_OBSBODY];
    int32_t rw_body[BIOIM_NREFBODY];       /* sim body per ref slot, -1 = center of mass */
    int32_t pd_coord[BIOIM_MAX_ACT];       /* PD: position coordinate per action entry */
    int32_t pd_vcoord[BIOIM_MAX_ACT];      /* PD: speed coordinate per action entry (the 3D torque
                                              envs index q and q' differently,
                                              torque_walking_imitation_env3D.py:130-131) */
    int32_t pad0;

    double  step_size;
    double  w_imitate, w_effort, w_action;
    double  action_r_scale;   /* 1 (2D) or 0.5 (3D)                                    */
    double  max_actuation;
    double  total_mass, gravity[3], height;
    double  torso_y_min, limit_force_max, acc_max;
    double  kp[BIOIM_MAX_ACT], kv[BIOIM_MAX_ACT];

    /* model tables */
    bioim_coord_t    coord[BIOIM_MAX_COORD];
    bioim_cbody_t    cbody[BIOIM_MAX_CBODY];
    bioim_osbody_t   osbody[BIOIM_MAX_OSBODY];
    bioim_fn_t       fn[BIOIM_MAX_FN];
    double           knot_x[BIOIM_MAX_KNOTS], knot_y[BIOIM_MAX_KNOTS];
    double           knot_b[BIOIM_MAX_KNOTS], knot_c[BIOIM_MAX_KNOTS], knot_d[BIOIM_MAX_KNOTS];
    bioim_muscle_t   muscle[BIOIM_MAX_MUSCLE];
    bioim_pathpt_t   pathpt[BIOIM_MAX_PATHPT];
    bioim_sphere_t   sphere[BIOIM_MAX_SPHERE];
    bioim_cforce_t   cforce[BIOIM_MAX_CFORCE];
    bioim_limit_t    limit[BIOIM_MAX_LIMIT];
    bioim_coordact_t coordact[BIOIM_MAX_ACT];

    /* reference motion (resampled at step_size) */
    int32_t nrows, pad1;
    int32_t ref_istep[BIOIM_MAX_REFROWS];  /* int(time/step_size), float64 truncation */
    double  ref_time[BIOIM_MAX_REFROWS];
    double  ref_q[BIOIM_MAX_REFROWS][BIOIM_MAX_COORD];
    double  ref_u[BIOIM_MAX_REFROWS][BIOIM_MAX_COORD];
    double  ref_x[BIOIM_MAX_REFROWS][BIOIM_NREFBODY][3];
} bioim_modelpack_t;

#endif /* BIOIM_MODELPACK_H */
