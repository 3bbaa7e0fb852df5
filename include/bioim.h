/*
 * bioim.h — C-ABI of the MI355X-native vectorized env step (libbioim.so).
 *
 * This is the drop-in boundary for the reference's physics facade
 * `OsimModel` (bioimitation/imitation_envs/utils/opensim_wrapper.py:6-338)
 * plus the per-step env arithmetic layered on it by the task envs
 * (muscle_walking_imitation_env2D.py:115-403, torque_walking_imitation_env2D.py:117-366)
 * and by `OsimEnv.step/reset` (opensim_environment.py:86-113).  One handle
 * owns N independent environment instances of one registered env ID on one
 * GPU; every call advances/reads all of them (a batched `env.step`).
 *
 * Each entry point cites the reference interface it replaces:
 *
 *   bioim_create   <- OsimEnv.__init__ -> OsimModel.__init__ (opensim_wrapper.py:7-90),
 *                     per instance, N times
 *   bioim_reset    <- Env.reset (muscle_walking_imitation_env2D.py:133-156) =
 *                     OsimModel.reset/set_time/set_coordinates/set_velocities
 *                     (opensim_wrapper.py:293-332) + get_observation
 *   bioim_step     <- Env.step (muscle_walking_imitation_env2D.py:115-131) ->
 *                     OsimEnv.step (opensim_environment.py:100-113) =
 *                     actuate (opensim_wrapper.py:92-107) + integrate (:299-301)
 *                     + get_state_dict/get_reward/is_done
 *   bioim_get_state/bioim_set_state <- (no reference equivalent; the env
 *                     state is not checkpointable upstream) parity re-sync,
 *                     checkpoint/resume
 *   bioim_destroy  <- garbage collection of the OsimModel instances
 *
 * Conventions
 *   - Real-valued buffers are float (precision 32) or double (precision 64),
 *     fixed at create time.  All buffers passed to reset/step are DEVICE
 *     pointers on the handle's device; the caller owns them.
 *   - obs is [N][obs_dim] row-major, reward [N], done [N] (uint8 0/1),
 *     info [N][info_dim] (the reference's info['all_rewards']).
 *   - Calls are asynchronous on the handle's HIP stream (bioim_stream /
 *     bioim_set_stream); bioim_sync waits.  Not re-entrant per handle.
 *   - Every entry returns 0 on success, < 0 on error; bioim_last_error()
 *     returns the thread-local message.  A missing GPU or a pack whose
 *     topology has no compiled kernel is an error (there is no CPU fallback).
 *
 * Flat per-env state (bioim_get_state/set_state, doubles), matching the
 * oracle's layout: [t, istep, has_last, old_pelvis_x, done, q[ndof], u[ndof],
 * activation[nmuscle], fiber_length[nmuscle], hist[horizon][nact],
 * last_action[nact], rk_step_size, controls[nact]] — controls are the held
 * actuator controls (the PrescribedController's Constant functions, set by
 * each step's actuate and kept through resets).
 */
#ifndef BIOIM_H
#define BIOIM_H

#include <stdint.h>

#include "bioim_modelpack.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bioim_handle bioim_handle_t;

enum {
    BIOIM_OK = 0,
    BIOIM_E_ARG = -1,
    BIOIM_E_DEVICE = -2,
    BIOIM_E_PACK = -3,
    BIOIM_E_NOKERNEL = -4,
    BIOIM_E_LAUNCH = -5,
};

/* Create N env instances of the pack's env ID on `device`; precision 32|64.
 * `seed` drives reset indices drawn on the device (randint(0, reset_hi)). */
int bioim_create(const bioim_modelpack_t *pack, int n_envs, int device, int precision, uint64_t seed,
                 bioim_handle_t **out);
int bioim_destroy(bioim_handle_t *h);

/* Reset `n` envs.  env_ids: device int32[n] (NULL = all envs, n ignored).
 * ref_index: device int32[n] reference-row indices (NULL = draw
 * randint(0, reset_hi) per env from the handle's counter-based RNG).
 * obs (may be NULL): device [N][obs_dim] — rows of the reset envs are written. */
int bioim_reset(bioim_handle_t *h, const int32_t *env_ids, const int32_t *ref_index, int n, void *obs);

/* One env step for all N envs.  actions: device [N][nact].  Outputs may be
 * NULL except done.  With auto-reset on, envs that finish are reset in the
 * same launch and their obs row is the post-reset observation. */
int bioim_step(bioim_handle_t *h, const void *actions, void *obs, void *reward, uint8_t *done, void *info);
int bioim_set_auto_reset(bioim_handle_t *h, int on);
/* In-kernel auto-resets (default step kernels: no push table, semi-implicit
 * or RK-Merson, no force report / state storage) read the reset state
 * and observation of the drawn reference row from a per-handle table (torque
 * models: with M^-1 at the row, for the held torques' share of q'')
 * instead of running the reset realize with fiber equilibrium in the step
 * launch (that realize made every launch wait for its slowest wave).  The
 * table is built once, on the first such step, by that same reset realize
 * (one scratch env per reference row); that step blocks while it is built
 * (milliseconds).  on = 1 (default) uses it, 0 runs the
 * realize in the launch as before, with the same results bit for bit (both
 * start the fiber-velocity roots cold; the row also carries the reset
 * realize's cache for the next step's first substep).  Replaces nothing in the
 * reference (OsimModel.reset + equilibrateMuscles per reset,
 * opensim_wrapper.py:293-297). */
int bioim_set_reset_table(bioim_handle_t *h, int on);
/* rows of the handle's built reset table (0: none built yet or none wanted) */
int bioim_reset_table_rows(const bioim_handle_t *h);
/* Row strides (in elements) of the actions / obs / info buffers this handle
 * reads and writes (default nact, obs_dim, info_dim).  Larger strides let
 * handles of different env IDs share padded buffers. */
int bioim_set_io_strides(bioim_handle_t *h, int act_stride, int obs_stride, int info_stride);
/* One env step of a mixed batch (BASELINE config C5): handle i
 * owns rows [sum(n_<i), sum(n_<=i)) of the padded buffers (all handles on one
 * device, same precision and strides; auto-reset per handle).  Segment 0 runs
 * on hs[0]'s stream, the others concurrently on private per-handle streams
 * forked from and joined back into it (events), so the call is ordered on
 * hs[0]'s stream like bioim_step.  Two segments whose topologies form a fused
 * pair (the spatial prosthetic and full muscle models, config C5) and that
 * run the default step (no push table, semi-implicit) go in ONE launch of a
 * fused two-topology kernel on hs[0]'s stream instead (bioim_set_group_fusion).  Later calls on a member handle's own
 * stream must be ordered after hs[0]'s stream (share one stream, as
 * VectorEnv does).  Replaces nothing in the reference
 * (one OsimModel per Ray worker); the batch is the RLlib VectorEnv over
 * heterogeneous sub-envs. */
int bioim_step_group(bioim_handle_t **hs, int nh, const void *actions, void *obs, void *reward, uint8_t *done,
                     void *info);
/* Process-wide switch of the fused two-topology launch in bioim_step_group
 * (default on; off: one concurrent launch per segment).  Results are the
 * same bit for bit either way. */
int bioim_set_group_fusion(int on);
/* 1 if the last bioim_step_group call with h as its first handle ran as ONE
 * fused two-topology launch, 0 if it ran one launch per segment (or no group
 * step yet); -1 for a null handle.  Lets callers and tests see that the
 * fused kernel really ran (it falls back to per-segment launches for fp32,
 * a push table, RK-Merson or a pair without a fused kernel). */
int bioim_group_fused(const bioim_handle_t *h);
/* apply_perturbations (muscle_walking_imitation_env2D.py:83-100 and the same
 * block in every task env): a PrescribedForce on the torso whose ground-frame
 * x force is a PiecewiseConstantFunction of simulation time.  Here: a
 * zero-order-hold table per env — force y[e][k] on [x[k], x[k+1]) (y[e][0]
 * before x[0]) along ground x, applied at the origin of OpenSim body
 * `os_body` (ModelPack osbody index) at every substep and realize.  x: host
 * double[npts], strictly increasing, shared by all envs; y: host double
 * [N][npts].  npts = 0 removes the force.  Synchronous (copies to device). */
int bioim_set_perturbation(bioim_handle_t *h, int os_body, int npts, const double *x, const double *y);
/* Inverse-dynamics primitives of the reference's InverseDynamics helper
 * (bioimitation/imitation_envs/inverse_dynamics/inverse_dynamics.cpp:45-205;
 * Boost.Python, built against OpenSim) on the handle's model, batched over n
 * states: muscles disabled, actuator controls 0, the model's gravity,
 * Hunt-Crossley contact and coordinate limit forces.  q, u, v, out: device
 * [n][ndof] in the handle's precision, dof order (locked coordinates are not
 * dofs).  `u` is read by CORIOLIS/RESIDUAL/TOTAL, `v` by MULT_M/MULT_MINV/
 * RESIDUAL.  Conventions (inverse_dynamics.cpp comments): M q'' + c = g + tau;
 * RESIDUAL = M v + c - f_applied (calculateResidualForces, :63-94); TOTAL =
 * c - f_applied, i.e. M q'' + f = tau (calculateTotalForces, :96-125);
 * GRAVITY = g (:127-141); CORIOLIS = c (:143-158); MULT_M = M v (:160-175);
 * MULT_MINV = M^-1 v (:177-192).  Asynchronous on the handle's stream. */
enum {
    BIOIM_ID_GRAVITY = 0,
    BIOIM_ID_CORIOLIS = 1,
    BIOIM_ID_MULT_M = 2,
    BIOIM_ID_MULT_MINV = 3,
    BIOIM_ID_RESIDUAL = 4,
    BIOIM_ID_TOTAL = 5,
};
int bioim_id_eval(bioim_handle_t *h, int op, int n, const void *q, const void *u, const void *v, void *out);
/* OsimModel calls on single envs (the reference's physics facade,
 * opensim_wrapper.py:92-332), for callers that drive the model directly
 * (tests/example_position_control.py:203-223; the env methods
 * get_state_dict / get_limit_forces / calc_cost_of_transport).  For the n
 * listed envs (env_ids: device int32[n]):
 *   controls (device [n][nact], may be NULL): OsimModel.actuate first —
 *     NaN -> 0, clip to [min_control, max_control], held from then on;
 *   op BIOIM_OSIM_REALIZE: nothing else (the calc_* realizations);
 *   op BIOIM_OSIM_EQUILIBRATE: reset_manager (:287-291) — a new integrator
 *     and equilibrateMuscles: each muscle's static fiber equilibrium at the
 *     held activation; the caller writes time / coordinates / speeds with
 *     bioim_set_state first (set_time :303-307, set_coordinates :309-319,
 *     set_velocities :321-332, reset :293-297);
 *   op BIOIM_OSIM_INTEGRATE: integrate (:299-301) — istep += 1, then the
 *     handle's integrator to step_size * istep with the held controls;
 * then the state is realized: obs (device [N][obs_stride], may be NULL)
 * gets the env's observation row, report (device [N][bioim_osim_report_dim],
 * may be NULL) the realized quantities (rows indexed by env):
 *   [time, istep, q[nc], u[nc], qdd[nc] (CoordinateSet order),
 *    per OpenSim body: origin pos[3], vel[3], acc[3], body-fixed XYZ angles[3],
 *      angular vel[3], angular acc[3] (ground frame); then the system COM
 *      pos[3], vel[3], acc[3],
 *    per muscle: activation, fiber_length, fiber_velocity, fiber_force,
 *      active_fiber_force, excitation, tendon_force,
 *    per actuator: actuation,
 *    per Hunt-Crossley force: force[3], moment about the ground origin[3] on the feet,
 *    per CoordinateLimitForce: its generalized force,
 *    calc_cost_of_transport() (0 for torque models)].
 * Env-level state (action deque, last action, old pelvis x, done) is left
 * alone.  Refused while envs are suspended mid-step (bioim_set_rk_budget).
 * Asynchronous on the handle's stream. */
enum {
    BIOIM_OSIM_REALIZE = 0,
    BIOIM_OSIM_EQUILIBRATE = 1,
    BIOIM_OSIM_INTEGRATE = 2,
};
int bioim_osim_report_dim(const bioim_handle_t *h);
int bioim_osim(bioim_handle_t *h, int op, const int32_t *env_ids, int n, const void *controls, void *obs, void *report);
/* Global index of this handle's env 0 (multi-GPU sharding): device-drawn
 * reset indices depend on the global env index, so a sharded run is
 * bit-identical to an unsharded one. */
int bioim_set_env_offset(bioim_handle_t *h, int offset);

/* Host-side state transfer (synchronous). */
int bioim_state_dim(const bioim_handle_t *h);
int bioim_get_state(bioim_handle_t *h, double *host_state /* [N][state_dim] */);
int bioim_set_state(bioim_handle_t *h, const double *host_state);
/* The same rows as bioim_get_state, written as doubles into a device buffer
 * [N][state_dim] on the handle's stream, without synchronizing (the
 * single-env recorder copies them with the step's outputs in one transfer).
 * Rows of envs suspended mid-step by the RK budget are not at a step
 * boundary (bioim_get_state refuses them; this call does not check).  No
 * reference counterpart. */
int bioim_copy_state(bioim_handle_t *h, void *device_out);

/* Integrator of the physics between env steps.  kind 0: the fixed
 * semi-implicit substeps (the pack's nsub; default).  kind 1: the reference's
 * integrator, an adaptive Kutta-Merson 4(5) at `accuracy` (OpenSim's
 * Manager, opensim_wrapper.py:287-301, accuracy 1e-3 from
 * muscle_walking_imitation_env2D.py:42), restated in
 * oracle/bioim_oracle.c integrate_rk_merson.  Replaces the integrator
 * choice inside OsimModel.reset_manager. */
int bioim_set_integrator(bioim_handle_t *h, int kind, double accuracy);
/* Budgeted steps for the adaptive integrator (kind 1).  attempts > 0: each
 * bioim_step gives every env at most `attempts` Kutta-Merson step attempts
 * (5 dynamics evaluations each);
 * an env whose env step is not finished by then is suspended at its last
 * accepted integration point and resumed by the next bioim_step (its action
 * row is ignored until it finishes).  ready_out (device [n], may be NULL)
 * receives 1 for the envs whose step finished in this launch — only their
 * obs / reward / done / info rows are written (done is 0 for the others).
 * A resumed step continues bit for bit as if it had never been suspended
 * (state, step size, attempt count and the fiber-velocity warm starts are
 * saved), so the trajectories equal the unbudgeted run's; what changes is
 * that one stiff env no longer holds the whole launch.  The consumer pattern
 * is RLlib's BaseEnv.poll() / send_actions(): new actions only for ready
 * envs.  attempts = 0 restores one-step-per-launch.  No reference
 * counterpart (OpenSim steps one env at a time). */
int bioim_set_rk_budget(bioim_handle_t *h, int attempts, uint8_t *ready_out);
/* Dynamics evaluations the adaptive integrator (kind 1) has spent so far,
 * summed over the handle's envs (5 per Kutta-Merson attempt, 1 per realize
 * after a step or reset).  Synchronizes the handle's streams.
 * 0 for handles that never ran the adaptive integrator.  No reference
 * counterpart (bench.py's evaluations per env step). */
int bioim_eval_count(bioim_handle_t *h, uint64_t *total);
/* Env steps the adaptive integrator (kind 1) has finished so far, summed
 * over the handle's envs: the count of bioim_step rows whose ready flag was
 * 1 (bioim_set_rk_budget).  Synchronizes the handle's streams.  No reference
 * counterpart (bench.py counts the reference-integrator rate with it instead
 * of reading ready[] after every launch). */
int bioim_finished_count(bioim_handle_t *h, uint64_t *total);
/* Sets every env's two RK counters (the evaluations and the finished steps
 * that bioim_eval_count / bioim_finished_count sum) to the given values,
 * e.g. to restart the counting of a measurement window or to carry counts
 * across a handle re-creation.  Each counter is 32 bits per env and wraps on
 * its own (no carry into the other).  Synchronizes the handle's streams.  No
 * reference counterpart. */
int bioim_set_rk_counters(bioim_handle_t *h, uint32_t evals, uint32_t finished);
/* envs suspended mid-step (synchronizes the handle's stream) */
int bioim_pending_count(bioim_handle_t *h);
/* Optional per-env step mask (device [n], NULL = every env steps): an env
 * with 0 is left untouched by bioim_step (state, outputs, ready flag) unless
 * it is finishing a suspended RK step.  Lets an asynchronous consumer step
 * only the envs it sent actions to (RLlib BaseEnv.send_actions). */
int bioim_set_active_mask(bioim_handle_t *h, const uint8_t *active);
/* Optional terminal-observation output: when set (a device buffer with the
 * handle's obs row stride), every step also writes each env's observation
 * as computed by that step *before* an in-kernel auto-reset replaces it, so
 * a done env's terminal observation survives (gym's final_observation;
 * bootstrapping in the reference's jaxrl SAC loop,
 * tests/sample_baselines_training.py:69-91).  NULL disables it. */
int bioim_set_final_obs(bioim_handle_t *h, void *final_obs);
/* Optional per-force-element report (the reference's ForceReporter analysis,
 * opensim_wrapper.py:10-15, printed by save_simulation :334-338): when set,
 * every realize writes per env a row of bioim_force_report_dim() values:
 * [actuation of each muscle (tendon force, N) or coordinate actuator
 * (control x optimal force)] [per Hunt-Crossley force: force (3) and moment
 * about the ground origin (3) on the feet] [per CoordinateLimitForce: its
 * generalized force] [per contact sphere, pack order: its force (3) on its
 * OpenSim body and the moment (3) about that body's origin, in ground — the
 * HuntCrossleyForce record's foot-side entries sum these per body].  NULL
 * disables it. */
int bioim_force_report_dim(const bioim_handle_t *h);
/* Optional state storage of the adaptive integrator (kind 1): OpenSim's
 * Manager stores the state at every accepted integration step, which
 * save_simulation prints (opensim_wrapper.py:334-337).  When set, each env
 * step (bioim_step, or bioim_osim INTEGRATE) writes per env one row per
 * accepted Kutta-Merson step: rows [n][capacity][1 + 2 ndof + 2 nmuscle] =
 * (time, q, u in dof order, activation, fiber length); count[n] receives the
 * number of accepted steps of the env's last env step (rows beyond capacity
 * are counted, not stored; a budgeted step's count spans its launches).
 * Device buffers owned by the caller; rows = NULL disables it. */
int bioim_set_state_storage(bioim_handle_t *h, void *rows, int capacity, int32_t *count);
int bioim_set_force_report(bioim_handle_t *h, void *force_out);
/* Sum over the handle's envs of their reset counters (explicit resets and
 * in-kernel auto-resets); synchronizes the handle's streams.  Lets a caller
 * count terminations over a stretch of steps without touching the step
 * launches (bench.py's done rate).  No reference counterpart. */
int bioim_reset_count(bioim_handle_t *h, uint64_t *total);
/* out[0..7] = n_envs, obs_dim, nact, info_dim, precision, lanes_per_env, nsub, state_dim */
int bioim_query(const bioim_handle_t *h, int32_t *out);
/* out[0..4] = lanes per env, threads per workgroup, envs per workgroup,
 * LDS bytes per workgroup (model image + env regions), workgroups per step */
int bioim_query_launch(const bioim_handle_t *h, int32_t *out);
void *bioim_stream(bioim_handle_t *h);
int bioim_set_stream(bioim_handle_t *h, void *hip_stream);
int bioim_sync(bioim_handle_t *h);
const char *bioim_last_error(void);
/* sizeof(bioim_modelpack_t) as compiled into the library (layout check). */
uint64_t bioim_modelpack_size(void);
/* Build id: sha256 (16 hex digits) over the kernel sources and hipcc flags the
 * library was compiled from (bioimitation/_buildinfo.py); the Python host
 * refuses a library whose id differs from its source tree's.  No reference
 * counterpart (build hygiene). */
const char *bioim_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* BIOIM_H */
