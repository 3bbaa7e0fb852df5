// bioim_step.hip — MI355X (gfx950) batched env step for bioimitation-gym.
//
// One launch advances N environments by one env step (0.01 s): action
// pre-processing, nsub semi-implicit substeps of the musculoskeletal
// forward dynamics, the realize at the end state, and the observation,
// reward and termination of the reference's task envs.
//
// Work decomposition (CDNA4, wave64): an environment is a
// group of G = 16 lanes for every topology, 4 envs per wave, 16 envs per
// 256-thread workgroup, one wave per SIMD.
//   - lanes take roles per phase: composite body (joint kinematics, frame
//     composition, inertias, subtree sums), dof (lane d owns coordinate d's
//     value and speed in registers, M entries, rhs), muscle (path geometry,
//     moment arms over its span, Millard damped equilibrium; lane l also
//     takes muscle l + 16 where a topology has more than 16), contact sphere,
//     limit force, report slot;
//   - lanes of one env exchange data through its per-env LDS region (frames,
//     Plücker columns, packed M, torque slots) with wave-scope fences: the env
//     never leaves its wave; group sums are xor-butterflies (bitwise identical
//     totals on every lane);
//   - the tree-sparse LTL solve runs redundantly on every lane in registers;
//   - the lane-indexed model image (muscles, path points, joints, splines,
//     spheres) is staged into LDS once per workgroup; uniform constants and
//     the reference-motion tables are scalar loads.
// Per-env state is SoA in HBM (env index fastest).  Reference semantics: see
// oracle/bioim_oracle.c, which this kernel must match (tests/test_gpu_*.py).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <type_traits>
#include <vector>

#include "bioim.h"
#include "bioim_device.h"
#include "topologies.h"

#define DEV __device__ __forceinline__
#define BIOIM_EPB 16 /* envs per workgroup (BIOIM_EPB * G threads) share one LDS model image */
/* env flags baked into a kernel (topologies.h FLAGS); RAW_ACTION, TARGET_OBS, GRF_OBS are run-time */
#define BIOIM_STRUCT_FLAGS (BIOIM_ENV_MUSCLE | BIOIM_ENV_HAS_TZ | BIOIM_ENV_REWARD_FEET | BIOIM_ENV_DONE_CROSS | BIOIM_ENV_PD)

#ifndef BIOIM_CHECK
#define BIOIM_CHECK 0
#endif
/* BIOIM_CHECK=1 (a diagnostic build, never shipped): every global load and
 * store of the env kernel goes through a bounds check that prints the source
 * line, the index, the bound, the workgroup and the thread, then traps — the
 * stale-lane class of DESIGN.md 5.5 then ends as a named trap instead of an
 * anonymous illegal-address fault.  With BIOIM_CHECK=0 the accessors expand to
 * plain subscripts (the shipped kernels are unchanged). */
DEV size_t bioim_chk(size_t i, size_t n, int line) {
    if (i >= n) {
        printf("BIOIM_CHECK bioim_step.hip:%d index %llu outside [0, %llu) workgroup %u thread %u\n", line,
               (unsigned long long)i, (unsigned long long)n, blockIdx.x, threadIdx.x);
        __builtin_trap();
    }
    return i;
}
#if BIOIM_CHECK
#define GAT(p, i, n) ((p)[bioim_chk((size_t)(i), (size_t)(n), __LINE__)])
#define GIDX(i, n) bioim_chk((size_t)(i), (size_t)(n), __LINE__)
#else
#define GAT(p, i, n) ((p)[i])
#define GIDX(i, n) (i)
#endif

template <int I, int N, class F>
DEV void sfor(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

#ifndef BIOIM_ENV_MOD
#define BIOIM_ENV_MOD -1
#endif
#ifndef BIOIM_BF3
#define BIOIM_BF3 122
#endif
#ifndef BIOIM_BF_SPATIAL
#define BIOIM_BF_SPATIAL 0
#endif
/* BIOIM_BF3_RK=1 (shipped): the BIOIM_BF3 pieces in the spatial RK-Merson
 * kernels too — no scratch, hazard gate clean, same-box Running3D RK launch
 * 0.7826 -> 0.7452 ms, LockedKnee3D 0.7289 -> 0.6989 ms (profiles/r04/r04g/ab_rk.log) */
#ifndef BIOIM_BF3_RK
#define BIOIM_BF3_RK 1
#endif
/* fiber-velocity warm start (round-5 experiments): BIOIM_FV_HERMITE = cubic
 * Hermite u(v) start from the table slopes instead of linear interpolation;
 * BIOIM_FV_PRED = linear extrapolation of the previous two substeps' roots
 * in the semi-implicit substep loop */
#ifndef BIOIM_FV_HERMITE
#define BIOIM_FV_HERMITE 0
#endif
#ifndef BIOIM_FV_PRED
#define BIOIM_FV_PRED 0
#endif
/* the substep's fiber-length update through fast_rcp instead of the IEEE
 * division (round-5 experiment, off: the oracle divides, and after 6 steps
 * the realize report drifted to 1.4e-9 of it, past the 1e-9 report test,
 * profiles/r05/r05p/gpu_tests.log) */
#ifndef BIOIM_SUBSTEP_RCP
#define BIOIM_SUBSTEP_RCP 0
#endif
/* BIOIM_SGB: sched_group_barrier pipelines in the muscle eval (round-5
 * experiment, off; same box C3 +1.3 % / +1.8 %: profiles/r05/r05o) */
#ifndef BIOIM_SGB
#define BIOIM_SGB 0
#endif
/* solve_fv: a lane whose root lies past the curve's end leaves the Newton
 * loop after one step (0: it iterates to the segment end as before) */
#ifndef BIOIM_FV_PAST_END
#define BIOIM_FV_PAST_END 1
#endif
#ifndef BIOIM_FV_PE_PLANAR
#define BIOIM_FV_PE_PLANAR 0
#endif
/* the reset table (LaunchArgs::reset_tab) in the planar RK-Merson step
 * kernels too, and (round 6) in the spatial ones: they fit it at 486-512
 * registers with no scratch; same-box reference-integrator legs C4 +3.9 %,
 * LockedKnee3D +4.4 %, Palsy3D +5.6 % (profiles/r06/r06e/ab_rk.txt) */
#ifndef BIOIM_RESET_TAB_RK_SPATIAL
#define BIOIM_RESET_TAB_RK_SPATIAL 1
#endif
#ifndef BIOIM_RESET_TAB_RK
#define BIOIM_RESET_TAB_RK 1
#endif
template <typename Real> struct Eps;
template <> struct Eps<float> {
    static constexpr float u_tol = 2e-7f;   /* Bezier parameter tolerance  */
    static constexpr float u_stop = 2e-7f;  /* Newton step after which the root is converged */
    static constexpr float v_tol = 1e-7f;   /* normalized velocity         */
    static constexpr float l_tol = 1e-9f;   /* fiber length (m)            */
    static constexpr float l_stop = 1e-9f;  /* Newton step after which the length is converged */
    static constexpr float h_stop = 0.0f;   /* fiber-equilibrium residual stop (off in fp32) */
    static constexpr int it_max = 24;
    static constexpr int curve_newton = 1; /* from the Hermite start: 5.9e-9 < fp32 rounding */
};
template <> struct Eps<double> {
    static constexpr double u_tol = 1e-15;
    /* a Newton step of at most 1e-11 leaves an error ~ |g''/2g'| 1e-22 in u
     * (quadratic convergence; the smooth curves have |g''/g'| = O(10)) */
    static constexpr double u_stop = 1e-11;
    static constexpr double v_tol = 1e-15;
    static constexpr double l_tol = 1e-15;
    static constexpr double l_stop = 1e-10;
    /* the oracle's residual stop of the reset fiber equilibrium
     * (oracle/bioim_oracle.c muscle_equilibrium, |H| < 1e-12): where the root is
     * ill-conditioned (a tendon at its slack length: H nearly flat in l) the
     * iterate that stop returns is the oracle's, instead of one converged
     * further (round 6: Palsy3D tib_ant_r at reset row 46, 9.2e-12 apart;
     * DESIGN.md 2) */
    static constexpr double h_stop = 1e-12;
    static constexpr int it_max = 60;
    static constexpr int curve_newton = 2; /* from the Hermite start: 8.9e-16 */
};

/* ------------------------------------------------------------- vec3 */
template <typename Real> DEV void cross3(const Real *a, const Real *b, Real *o) {
    Real x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
template <typename Real> DEV Real dot3(const Real *a, const Real *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <typename Real> DEV void mv3(const Real *R, const Real *v, Real *o) {
    Real x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    Real y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    Real z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}
template <typename Real> DEV void mm3(const Real *A, const Real *B, Real *C) {
    Real T[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = T[i];
}
/* The same products with compile-time zero masks (bit i: operand entry i
 * is known to be zero): a term with a known-zero factor is left out, so
 * planar models (Planar below) run the 2-D arithmetic through the same
 * code; with empty masks these are exactly mv3 / mm3 / cross3 / dot3
 * (same terms, same order). */
template <unsigned ZA, unsigned ZB, int N, typename Real>
DEV Real sum_m(const Real *a, const Real *b, const int (&ia)[N], const int (&ib)[N], const int (&sg)[N]) {
    Real acc = 0;
    bool first = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (((ZA >> ia[k]) & 1u) || ((ZB >> ib[k]) & 1u)) continue;
        const Real t = a[ia[k]] * b[ib[k]];
        acc = first ? (sg[k] > 0 ? t : -t) : (sg[k] > 0 ? acc + t : acc - t);
        first = false;
    }
    return acc;
}
template <unsigned ZA, unsigned ZB, typename Real> DEV void mv3m(const Real *R, const Real *v, Real *o) {
    Real r[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int ia[3] = {3 * i, 3 * i + 1, 3 * i + 2}, ib[3] = {0, 1, 2}, sg[3] = {1, 1, 1};
        r[i] = sum_m<ZA, ZB, 3>(R, v, ia, ib, sg);
    }
    o[0] = r[0]; o[1] = r[1]; o[2] = r[2];
}
template <unsigned ZA, unsigned ZB, typename Real> DEV void mm3m(const Real *A, const Real *B, Real *C) {
    Real T[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int ia[3] = {3 * i, 3 * i + 1, 3 * i + 2}, ib[3] = {j, 3 + j, 6 + j}, sg[3] = {1, 1, 1};
            T[3 * i + j] = sum_m<ZA, ZB, 3>(A, B, ia, ib, sg);
        }
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = T[i];
}
template <unsigned ZA, unsigned ZB, typename Real> DEV void cross3m(const Real *a, const Real *b, Real *o) {
    const int sg[2] = {1, -1};
    const int ia0[2] = {1, 2}, ib0[2] = {2, 1}, ia1[2] = {2, 0}, ib1[2] = {0, 2}, ia2[2] = {0, 1}, ib2[2] = {1, 0};
    Real x = sum_m<ZA, ZB, 2>(a, b, ia0, ib0, sg), y = sum_m<ZA, ZB, 2>(a, b, ia1, ib1, sg),
         z = sum_m<ZA, ZB, 2>(a, b, ia2, ib2, sg);
    o[0] = x; o[1] = y; o[2] = z;
}
template <unsigned ZA, unsigned ZB, typename Real> DEV Real dot3m(const Real *a, const Real *b) {
    const int ia[3] = {0, 1, 2}, sg[3] = {1, 1, 1};
    return sum_m<ZA, ZB, 3>(a, b, ia, ia, sg);
}

/* Planar topologies (T::PLANAR; the host checks each pack, pack_is_planar):
 * frames rotate about z only, so R13 = R23 = R31 = R32 = 0 and R33 = 1,
 * angular velocities and accelerations lie along z, linear ones in the x-y
 * plane.  These helpers write those zeros over values just read from LDS;
 * in the functions that use them the products with the known zeros then fold
 * away (those functions are compiled without signed zeros / NaN semantics:
 * `#pragma float_control(precise, off)`), so a planar model runs 2-D
 * arithmetic through the same source.  No-ops for spatial topologies. */
template <class T> struct Planar {
    /* zero masks (mv3m / mm3m / cross3m / dot3m): rotation, angular, linear */
    static constexpr unsigned ZR = T::PLANAR ? 0xE4u : 0u, ZW = T::PLANAR ? 0x3u : 0u, ZV = T::PLANAR ? 0x4u : 0u;
    template <typename Real> static DEV void rot(Real *R) {
        if constexpr (T::PLANAR) { R[2] = R[5] = R[6] = R[7] = Real(0); R[8] = Real(1); }
    }
    template <typename Real> static DEV void ang(Real *w) {
        if constexpr (T::PLANAR) { w[0] = w[1] = Real(0); }
    }
    template <typename Real> static DEV void lin(Real *v) {
        if constexpr (T::PLANAR) { v[2] = Real(0); }
    }
    /* frame slot KB: R9 o3 w3 vO3 */
    template <typename Real> static DEV void frame(Real *kb) { rot(kb); ang(kb + 12); lin(kb + 15); }
    /* joint-local slot LOC: R9 p3 wrel3 vrel3 arel3 aa3 */
    template <typename Real> static DEV void loc(Real *lc) { rot(lc); ang(lc + 12); lin(lc + 15); ang(lc + 18); lin(lc + 21); }
    /* acceleration slot AL: alpha3 aO3 */
    template <typename Real> static DEV void acc(Real *ab) { ang(ab); lin(ab + 3); }
    /* Plucker column: Omega3 V3 */
    template <typename Real> static DEV void col(Real *s) { ang(s); lin(s + 3); }
};

DEV void sincos_rt(double x, double &s, double &c);
DEV void sincos_rt(float x, float &s, float &c);
template <typename Real> DEV void axis_rot(const Real *a, Real th, Real *R) {
    Real s, c;
    sincos_rt(th, s, c);
    Real t = Real(1) - c, x = a[0], y = a[1], z = a[2];
    R[0] = t * x * x + c;     R[1] = t * x * y - s * z; R[2] = t * x * z + s * y;
    R[3] = t * x * y + s * z; R[4] = t * y * y + c;     R[5] = t * y * z - s * x;
    R[6] = t * x * z - s * y; R[7] = t * y * z + s * x; R[8] = t * z * z + c;
}

template <int G, typename Real> DEV Real group_sum(Real x) {
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) x += __shfl_xor(x, off, G);
    return x;
}
template <int G, typename Real> DEV Real group_max(Real x) {
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) x = fmax(x, __shfl_xor(x, off, G));
    return x;
}
template <int G> DEV bool group_any(bool p) {
    unsigned long long b = __ballot(p);
    int base = (threadIdx.x & 63) & ~(G - 1);
    unsigned long long m = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
    return ((b >> base) & m) != 0ull;
}

#ifdef BIOIM_STAMPS
__device__ unsigned long long g_stamps[24];
#endif
/* Diagnostic build only (-DBIOIM_WAVETIME, single translation unit,
 * tools/wavetime.py): shader cycles of every wave of the last step launch */
#ifdef BIOIM_WAVETIME
#define BIOIM_WAVETIME_N 65536
__device__ unsigned long long g_wavetime[BIOIM_WAVETIME_N];
/* per thread of the last launch: fiber-velocity Newton iterations (sum over
 * the launch's solves), the most of one solve, bisection fallbacks */
__device__ unsigned g_fvit[BIOIM_WAVETIME_N * 4], g_fvmax[BIOIM_WAVETIME_N * 4], g_fvbis[BIOIM_WAVETIME_N * 4];
DEV unsigned diag_tid() { return blockIdx.x * blockDim.x + threadIdx.x; }
#endif

/* ------------------------------------------------------------ functions */
template <class T, typename Real>
DEV void spline_eval(const SModel<T, Real> &SM, int off, int n, Real q, Real &f, Real &f1, Real &f2) {
    Real x0 = SM.kx[off], xn = SM.kx[off + n - 1];
    if (q < x0) { f = SM.ky[off] + (q - x0) * SM.kb[off]; f1 = SM.kb[off]; f2 = 0; return; }
    if (q > xn) {
        int j = off + n - 1;
        f = SM.ky[j] + (q - xn) * SM.kb[j]; f1 = SM.kb[j]; f2 = 0; return;
    }
    /* interval search: fixed trip count, all loads independent (one LDS wait) */
    int k = 0;
#pragma unroll
    for (int i = 1; i < T::NKMAX - 1; ++i) {
        Real xi = SM.kx[off + (i < n - 1 ? i : 0)];
        k += (i < n - 1 && q > xi) ? 1 : 0;
    }
    int j = off + k;
    Real dx = q - SM.kx[j], b = SM.kb[j], c = SM.kc[j], d = SM.kd[j];
    f = SM.ky[j] + dx * (b + dx * (c + dx * d));
    f1 = b + dx * (Real(2) * c + Real(3) * dx * d);
    f2 = Real(2) * c + Real(6) * dx * d;
}

/* value and first two derivatives of function fi (fi < 0: absent axis, 0) */
template <class T, typename Real>
DEV void fn_eval(const SModel<T, Real> &SM, int fi, Real q, Real &f, Real &f1, Real &f2) {
    f = 0; f1 = 0; f2 = 0;
    if (fi < 0) return;
    const SFn<Real> &F = SM.fn[fi];
    if (F.type == BIOIM_FN_CONST) { f = F.b; }
    else if (F.type == BIOIM_FN_LINEAR) { f = F.a * q + F.b; f1 = F.a; }
    else {
        Real s, s1, s2;
        spline_eval<T, Real>(SM, F.off, F.n, q, s, s1, s2);
        f = F.a * s; f1 = F.a * s1; f2 = F.a * s2;
    }
}

/* fn_eval without branches (phase 0b's function slots): the spline is
 * evaluated at the argument clamped to its knots (interval search and
 * coefficients as in spline_eval) and the linear extrapolation, constant and
 * linear kinds are selected; the same values as fn_eval, in one basic block
 * so the slot's dependent LDS loads are not split by branches */
template <bool BFK, class T, typename Real>
DEV void fn_eval_bf(const SModel<T, Real> &SM, int fi, Real q, Real &f, Real &f1, Real &f2) {
    const SFn<Real> &F = SM.fn[fi < 0 ? 0 : fi];
    const int type = F.type, oo = F.off >= 0 ? F.off : 0, nn = F.n > 1 ? F.n : 1;
    const Real a = F.a, b = F.b;
    const Real x0 = SM.kx[oo], xn = SM.kx[oo + nn - 1];
    const Real qc = q < x0 ? x0 : (q > xn ? xn : q);
    int k = 0;
#pragma unroll
    for (int i = 1; i < T::NKMAX - 1; ++i) {
        const Real xi = SM.kx[oo + (i < nn - 1 ? i : 0)];
        k += (i < nn - 1 && qc > xi) ? 1 : 0;
    }
    const int j = oo + k, jn = oo + nn - 1;
    const Real dx = qc - SM.kx[j], kb = SM.kb[j], kc = SM.kc[j], kd = SM.kd[j];
    Real s0 = SM.ky[j] + dx * (kb + dx * (kc + dx * kd));
    Real s1 = kb + dx * (Real(2) * kc + Real(3) * dx * kd);
    Real s2 = Real(2) * kc + Real(6) * dx * kd;
    const Real ylo = SM.ky[oo], blo = SM.kb[oo], yhi = SM.ky[jn], bhi = SM.kb[jn];
    const bool lo = q < x0, hi = q > xn;
    /* every ?: below picks between plain locals: clang emits a ?: whose arms
     * are expressions as a branch, the loads feeding an arm then sink into
     * it and the branch can no longer be folded into a select */
    const bool con = type == BIOIM_FN_CONST, lin = type == BIOIM_FN_LINEAR, present = fi >= 0;
    if constexpr (BFK) {
        const Real elo = ylo + (q - x0) * blo, ehi = yhi + (q - xn) * bhi, zero = 0;
        s0 = lo ? elo : (hi ? ehi : s0);
        s1 = lo ? blo : (hi ? bhi : s1);
        s2 = lo || hi ? zero : s2;
        const Real vl = a * q + b, vs = a * s0, vs1 = a * s1, vs2 = a * s2;
        f = !present ? zero : (con ? b : (lin ? vl : vs));
        f1 = !present || con ? zero : (lin ? a : vs1);
        f2 = !present || con || lin ? zero : vs2;
    } else {
        s0 = lo ? ylo + (q - x0) * blo : (hi ? yhi + (q - xn) * bhi : s0);
        s1 = lo ? blo : (hi ? bhi : s1);
        s2 = lo || hi ? Real(0) : s2;
        f = !present ? Real(0) : (con ? b : (lin ? a * q + b : a * s0));
        f1 = !present || con ? Real(0) : (lin ? a : a * s1);
        f2 = !present || con || lin ? Real(0) : a * s2;
    }
}

/* fn_eval specialised to the function kinds KM (bit kind+1; bit 0 = absent
 * axis) that can occur at this call site (compile-time, per topology axis) */
template <unsigned KM, class T, typename Real>
DEV void fn_eval_km(const SModel<T, Real> &SM, int fi, Real q, Real &f, Real &f1, Real &f2) {
    constexpr bool ABS = (KM & 1u) != 0, CON = (KM & 2u) != 0, LIN = (KM & 4u) != 0, SPL = (KM & 8u) != 0;
    f = 0; f1 = 0; f2 = 0;
    if constexpr (!CON && !LIN && !SPL) return;
    const SFn<Real> &F = SM.fn[ABS ? (fi < 0 ? 0 : fi) : fi];
    const Real a = F.a, b = F.b;
    const int type = F.type;
    Real v = 0, v1 = 0, v2 = 0;
    if constexpr (LIN && CON) { const bool lin = type == BIOIM_FN_LINEAR; v = lin ? a * q + b : b; v1 = lin ? a : Real(0); }
    else if constexpr (LIN) { v = a * q + b; v1 = a; }
    else if constexpr (CON) { v = b; }
    if constexpr (SPL) {
        if (type == BIOIM_FN_SPLINE) {
            Real s0, s1, s2;
            spline_eval<T, Real>(SM, F.off, F.n, q, s0, s1, s2);
            v = a * s0; v1 = a * s1; v2 = a * s2;
        }
    }
    const bool present = !ABS || fi >= 0;
    f = present ? v : Real(0); f1 = present ? v1 : Real(0); f2 = present ? v2 : Real(0);
}

/* sin and cos with one shared range reduction.  fp64: Cody-Waite reduction
 * by pi/2 (three-part constant, exact for |x| < 1e5, far beyond joint
 * angles) and Taylor polynomials on [-pi/4, pi/4] (truncation < 1e-19);
 * agrees with libm to ~1 ulp.  fp32: the device sincosf. */
DEV void sincos_rt(double x, double &s, double &c) {
    const double k = rint(x * 0.63661977236758134308);
    double r = fma(-k, 1.57079632679489655800e+00, x);
    r = fma(-k, 6.12323399573676603587e-17, r);
    r = fma(-k, -1.4973849048591698e-33, r);
    const double r2 = r * r;
    double ps = 2.8114572543455208e-15;                /* 1/17! */
    ps = fma(ps, r2, -7.6471637318198164e-13);         /* -1/15! */
    ps = fma(ps, r2, 1.6059043836821613e-10);          /* 1/13! */
    ps = fma(ps, r2, -2.5052108385441720e-08);         /* -1/11! */
    ps = fma(ps, r2, 2.7557319223985893e-06);          /* 1/9! */
    ps = fma(ps, r2, -1.9841269841269841e-04);         /* -1/7! */
    ps = fma(ps, r2, 8.3333333333333333e-03);          /* 1/5! */
    ps = fma(ps, r2, -1.6666666666666667e-01);         /* -1/3! */
    const double sr = fma(ps * r2, r, r);
    double pc = 1.5619206968586225e-16;                /* 1/18! */
    pc = fma(pc, r2, -4.7794773323873853e-14);         /* -1/16! */
    pc = fma(pc, r2, 1.1470745597729725e-11);          /* 1/14! */
    pc = fma(pc, r2, -2.0876756987868099e-09);         /* -1/12! */
    pc = fma(pc, r2, 2.7557319223985891e-07);          /* 1/10! */
    pc = fma(pc, r2, -2.4801587301587302e-05);         /* -1/8! */
    pc = fma(pc, r2, 1.3888888888888889e-03);          /* 1/6! */
    pc = fma(pc, r2, -4.1666666666666667e-02);         /* -1/4! */
    pc = fma(pc, r2, 0.5);
    const double cr = fma(-pc, r2, 1.0);
    const int q = (int)k & 3;
    const double ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
    s = (q & 2) ? -ss : ss;
    c = ((q + 1) & 2) ? -cc : cc;
}
DEV void sincos_rt(float x, float &s, float &c) { sincosf(x, &s, &c); }

/* ----------------------------------------------------- smooth curves */
/* BIOIM_EXACT_RCP=1: a diagnostic build (never shipped) whose reciprocals
 * and inverse square roots below are IEEE divisions and square roots, the
 * oracle's operations — to attribute the GPU's operation-level distance from
 * the oracle */
#ifndef BIOIM_EXACT_RCP
#define BIOIM_EXACT_RCP 0
#endif
#if BIOIM_EXACT_RCP
DEV double newton_rcp(double x) { return 1.0 / x; }
DEV float newton_rcp(float x) { return 1.0f / x; }
DEV double fast_rcp(double x) { return 1.0 / x; }
DEV float fast_rcp(float x) { return 1.0f / x; }
DEV double fast_rsqrt(double x) { return 1.0 / sqrt(x); }
DEV float fast_rsqrt(float x) { return 1.0f / sqrtf(x); }
#else
/* reciprocal for Newton updates (a self-correcting iteration tolerates a
 * last-bits error in the step): hardware rcp plus one refinement */
DEV double newton_rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    const double e = fma(-x, r, 1.0);
    return fma(r, e, r);
}
DEV float newton_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
/* reciprocal to (about) the last bit: hardware rcp plus two refinements —
 * a shorter dependency chain than the IEEE division sequence; used where the
 * divisor is a well-scaled positive quantity (lengths, cosines, time
 * constants, slip speeds) */
DEV double fast_rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}
DEV float fast_rcp(float x) {
    float r = __builtin_amdgcn_rcpf(x);
    return fmaf(r, fmaf(-x, r, 1.0f), r);
}
/* 1/sqrt(x) for x > 0: hardware rsq plus two Newton refinements; a length
 * and its inverse then cost one rsq (len = x * rsqrt(x)) instead of an IEEE
 * sqrt and a reciprocal */
DEV double fast_rsqrt(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double hx = 0.5 * x;
    y = fma(y, fma(-hx * y, y, 0.5), y);
    return fma(y, fma(-hx * y, y, 0.5), y);
}
DEV float fast_rsqrt(float x) {
    float y = __builtin_amdgcn_rsqf(x);
    return fmaf(y, fmaf(-0.5f * x * y, y, 0.5f), y);
}
#endif

/* a quintic segment in the power basis c[0] + c[1] u + ... + c[5] u^5
 * (converted from the Bezier control points at create time, convert_curve):
 * Horner, 5 FMAs; the derivative 4 */
template <typename Real> DEV Real bez5(const Real *c, Real u) {
    return fma(fma(fma(fma(fma(c[5], u, c[4]), u, c[3]), u, c[2]), u, c[1]), u, c[0]);
}
template <typename Real> DEV Real dbez5(const Real *c, Real u) {
    return fma(fma(fma(fma(Real(5) * c[5], u, Real(4) * c[4]), u, Real(3) * c[3]), u, Real(2) * c[2]), u, c[1]);
}

/* y(x), dy/dx of a SmoothSegmentedFunction.  Branch-free with a fixed trip
 * count (no lane divergence): segment located by comparisons, u(x) started
 * from the segment's 32-interval table by cubic Hermite interpolation (node
 * values ut and slopes mt; start error <= 3.1e-5 over every shipped curve),
 * then Newton steps on the quintic x(u): two reach machine precision in
 * fp64, one is below fp32 rounding (tests/test_curves.py); linear
 * extrapolation outside [x0, x1]. */
template <bool BF = true, typename Real>
DEV void curve_eval(const DCurve<Real> &C, Real x, Real &y, Real &dydx) {
    Real xc = x < C.x0 ? C.x0 : (x > C.x1 ? C.x1 : x);
    int k = 0;
#pragma unroll
    for (int s = 0; s < BIOIM_MAX_CURVESEG - 1; ++s) k += xc > C.xsep[s] ? 1 : 0;
    Real px[6], py[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) { px[i] = C.cx[k][i]; py[i] = C.cy[k][i]; }
    Real tt = (xc - C.xa[k]) * C.inv_h[k];
    int i0 = (int)tt;
    i0 = i0 < 0 ? 0 : (i0 > BIOIM_UTAB - 1 ? BIOIM_UTAB - 1 : i0);
    Real fr = tt - Real(i0);
    /* Hermite basis in the form u0 + f (m0 + f (c2 + f c3)) */
    const Real u0 = Real(C.ut[k][i0]), u1 = Real(C.ut[k][i0 + 1]), m0 = Real(C.mt[k][i0]), m1 = Real(C.mt[k][i0 + 1]);
    const Real du = u1 - u0;
    const Real c2 = Real(3) * du - Real(2) * m0 - m1, c3 = m0 + m1 - Real(2) * du;
    Real u = fma(fr, fma(fr, fma(fr, c3, c2), m0), u0);
#pragma unroll
    for (int it = 0; it < Eps<Real>::curve_newton; ++it) u -= (bez5(px, u) - xc) * newton_rcp(dbez5(px, u));
    y = bez5(py, u);
    dydx = dbez5(py, u) * fast_rcp(dbez5(px, u));
    /* linear extrapolation blended in by 0 / 1 weights (every term finite):
     * a load under the condition, or a select of loaded values, made the
     * compiler branch, which split the muscle eval's three independent curve
     * chains into separate basic blocks */
    if constexpr (BF) {
        const Real x0 = C.x0, y0 = C.y0, d0 = C.dydx0, x1 = C.x1, y1 = C.y1, d1 = C.dydx1;
        const Real ylo = y0 + d0 * (x - x0), yhi = y1 + d1 * (x - x1);
        const Real wb = x < x0 ? Real(1) : Real(0), wa = x > x1 ? Real(1) : Real(0), wm = Real(1) - wb - wa;
        y = fma(wb, ylo, fma(wa, yhi, wm * y));
        dydx = fma(wb, d0, fma(wa, d1, wm * dydx));
    } else {   /* the branching form: separate blocks, fewer values live at once */
        if (x < C.x0) { y = C.y0 + C.dydx0 * (x - C.x0); dydx = C.dydx0; }
        if (x > C.x1) { y = C.y1 + C.dydx1 * (x - C.x1); dydx = C.dydx1; }
    }
}

/* root of a*fal*fv(v) + beta*v = rhs (strictly increasing in v), solved in the
 * Bezier parameter of the bracketing segment, warm-started from v0 (the
 * previous substep's root) through the segment's u(x) table; returns v, fv,
 * dfv/dv.  At least two safeguarded Newton steps, then more until
 * converged. */
template <bool BF = true, bool PE = true, typename Real>
DEV void solve_fv(const DCurve<Real> &C, Real afal, Real beta, Real rhs, Real v0, Real &v, Real &fv, Real &dfv) {
    Real g0 = afal * C.y0 + beta * C.x0 - rhs;
    Real g1 = afal * C.y1 + beta * C.x1 - rhs;
    int k = 0;
#pragma unroll
    for (int s = 1; s < BIOIM_MAX_CURVESEG; ++s) k += afal * C.ya[s] + beta * C.xa[s] - rhs <= 0 ? 1 : 0;
    Real px[6], py[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) { px[i] = C.cx[k][i]; py[i] = C.cy[k][i]; }
    const Real xa = C.xa[k], xb = C.xb[k];
    Real ga = afal * C.ya[k] + beta * xa - rhs, gb = afal * C.yb[k] + beta * xb - rhs;
    /* both starts computed, one selected (no branch: the table loads and the
     * division stay in the muscle eval's basic block) — the warm start
     * through the segment's u(x) table, or the secant of g over the segment */
    Real u;
    if constexpr (!BF) {
        if (v0 > xa && v0 < xb) {
            Real tt = (v0 - xa) * C.inv_h[k];
            int i0 = (int)tt;
            i0 = i0 < 0 ? 0 : (i0 > BIOIM_UTAB - 1 ? BIOIM_UTAB - 1 : i0);
            Real fr = tt - Real(i0);
            u = C.ut[k][i0] + fr * (C.ut[k][i0 + 1] - C.ut[k][i0]);
        } else {
            u = ga / (ga - gb);
        }
    } else {
        const Real vc = v0 > xa ? (v0 < xb ? v0 : xb) : xa;
        Real tt = (vc - xa) * C.inv_h[k];
        int i0 = (int)tt;
        i0 = i0 < 0 ? 0 : (i0 > BIOIM_UTAB - 1 ? BIOIM_UTAB - 1 : i0);
        Real fr = tt - Real(i0);
        const Real ua = C.ut[k][i0], ub = C.ut[k][i0 + 1];
#if BIOIM_FV_HERMITE
        /* the cubic Hermite start of curve_eval (table slopes mt) */
        const Real ma = C.mt[k][i0], mb = C.mt[k][i0 + 1], dua = ub - ua;
        const Real h2 = Real(3) * dua - Real(2) * ma - mb, h3 = ma + mb - Real(2) * dua;
        const Real ut = fma(fr, fma(fr, fma(fr, h3, h2), ma), ua), us = ga * newton_rcp(ga - gb);
#else
        const Real ut = ua + fr * (ub - ua), us = ga * newton_rcp(ga - gb);
#endif
        u = ((v0 > xa) & (v0 < xb)) ? ut : us;
    }
    const Real half = 0.5;
    u = ((u > Real(0)) & (u < Real(1))) ? u : half;
    /* g(u) = a fal y(u) + beta x(u) - rhs is one quintic in u */
    Real pg[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) pg[i] = afal * py[i] + beta * px[i];
    pg[0] -= rhs;
    Real lo = 0, hi = 1, dprev = 1;
    /* the root lies past an end of the curve (g keeps one sign over it): the
     * result is the linear extrapolation below, whatever the loop finds, so
     * the lane leaves the loop after its first step.  Before round 5 such a
     * lane ran the Newton loop down to the segment's end by bisections (up to
     * ~40 iterations) and its wave — and the launch — waited for it: the
     * raw-action Palsy3D model hit it in 10 % of its waves.
     * PE: the spatial models only (same-box Palsy3D -15 %, C5 -13 %,
     * Running3D -1.5 %; the planar kernels, which rarely meet it, measured
     * +0.5 % with it: profiles/r05/r05k) */
    const bool past_end = PE && BIOIM_FV_PAST_END && ((g0 >= 0) | (g1 <= 0));
    for (int it = 0; it < Eps<Real>::it_max; ++it) {
        Real g = bez5(pg, u);
        if (g > 0) hi = u; else lo = u;
        Real dg = dbez5(pg, u);
        Real un = u - g * newton_rcp(dg);
        /* inclusive bracket: a converged step (un == u == lo or hi after
         * rounding) must not trigger the bisection fallback */
        if (!(un >= lo && un <= hi)) un = Real(0.5) * (lo + hi);
#ifdef BIOIM_WAVETIME
        if (!(u - g * newton_rcp(dg) >= lo && u - g * newton_rcp(dg) <= hi) && diag_tid() < BIOIM_WAVETIME_N * 4) g_fvbis[diag_tid()] += 1;
#endif
        Real du = fabs(un - u);
        u = un;
        /* converged, or stagnating at the rounding level of g */
        if (past_end || (it >= 1 && (du <= Eps<Real>::u_stop || (du <= Real(1e3) * Eps<Real>::u_tol && du >= Real(0.5) * dprev)))) {
#ifdef BIOIM_WAVETIME
            if (diag_tid() < BIOIM_WAVETIME_N * 4) {
                g_fvit[diag_tid()] += it + 1;
                if ((unsigned)(it + 1) > g_fvmax[diag_tid()]) g_fvmax[diag_tid()] = it + 1;
            }
#endif
#ifdef BIOIM_STAMPS
            if (blockIdx.x == 0 && threadIdx.x < 14) atomicAdd(&g_stamps[12], (unsigned long long)(it + 1));
            if (blockIdx.x == 0 && threadIdx.x < 14) atomicAdd(&g_stamps[13], 1ull);
#endif
            break;
        }
#ifdef BIOIM_STAMPS
        if (it == Eps<Real>::it_max - 1 && blockIdx.x == 0 && threadIdx.x < 14) atomicAdd(&g_stamps[14], 1ull);
#endif
        dprev = du;
    }
    v = bez5(px, u);
    fv = bez5(py, u);
    dfv = dbez5(py, u) * fast_rcp(dbez5(px, u));
    if constexpr (!BF) {
        if (g0 >= 0) {
            v = (rhs - afal * (C.y0 - C.dydx0 * C.x0)) / (afal * C.dydx0 + beta);
            fv = C.y0 + C.dydx0 * (v - C.x0); dfv = C.dydx0;
        } else if (g1 <= 0) {
            v = (rhs - afal * (C.y1 - C.dydx1 * C.x1)) / (afal * C.dydx1 + beta);
            fv = C.y1 + C.dydx1 * (v - C.x1); dfv = C.dydx1;
        }
    } else {   /* linear extrapolation past an end (one reciprocal, selected).
                * Reciprocals instead of IEEE divisions here and in the secant
                * start: same-box 2D 0.2772 -> 0.2762 ms, 3D 0.5176 -> 0.5145 ms,
                * C5 unchanged (profiles/r04/r04y; computing this before the
                * Newton loop instead was 2D -0.6 % but C5 +1.2 %) */
        const Real y0 = C.y0, d0 = C.dydx0, x0 = C.x0, y1 = C.y1, d1 = C.dydx1, x1 = C.x1;
        const bool e0 = g0 >= 0, e1 = g1 <= 0;
        const Real yE = e0 ? y0 : y1, dE = e0 ? d0 : d1, xE = e0 ? x0 : x1;
        const Real vE = (rhs - afal * (yE - dE * xE)) * fast_rcp(afal * dE + beta);
        const Real fvE = yE + dE * (vE - xE);
        const bool ext = e0 | e1;
        v = ext ? vE : v; fv = ext ? fvE : fv; dfv = ext ? dE : dfv;
    }
}

/* muscle of lane slot s (slot = lane + j * G): when the muscles take two
 * passes over the lanes, the second, partly idle pass holds the cheapest
 * paths (T::mperm, tools/build_packs.py); a bijection of [0, NM), the
 * identity elsewhere, so slot-range checks stay valid */
template <class T> DEV int mslot(int s) {
    int r = s;
    if constexpr (T::NM > T::G) {
        sfor<0, T::NM>([&](auto iI) {
            constexpr int i = decltype(iI)::value;
            r = s == i ? T::mperm[i] : r;
        });
    }
    return r;
}

/* ---------------------------------------------------------- LDS layout
 * Per workgroup: the shared model image (SModel, bioim_device.h), then one
 * region per env.  Phase 1 (lane-parallel kinematics) publishes frames,
 * Plucker columns, per-body inertias and Newton-Euler wrenches; the force
 * phases read them and publish per-lane slots that are reduced in a fixed
 * order (bitwise deterministic).  The union region U is reused by phase 1
 * (joint-local data), phases 2-3 (force slots) and the observation staging. */
template <class T, typename Real> struct Lay {
    static constexpr int NB = T::NB, ND = T::ND > 0 ? T::ND : 1, NC = T::NC, NP = ND * (ND + 1) / 2;
    static constexpr int NMS = T::NM > T::NA ? T::NM : T::NA;
    static constexpr int MPL = (NMS + T::G - 1) / T::G;      /* muscles (actions) per lane            */
    static constexpr int NS = T::NS > 0 ? T::NS : 1, NL = T::NL > 0 ? T::NL : 1;
    static constexpr int CJN = 10;               /* per sphere: P3, F3 (implicit), C4 (xx xz yy zz)  */
    static constexpr int NTR = (T::TX >= 0) + (T::TY >= 0) + (T::TZ >= 0);
    /* largest observation of the topology (target obs and GRF on) */
    static constexpr int OBSMAX = 1 + (NC - NTR) + 2 * NC + 2 * (NC - 1) + 3 * (T::NOBP + T::NOBV) + 3 * T::NM +
                                  6 * T::NF;
    static constexpr int KB = 0;                 /* [NB+1][18]: R9 o3 w3 vO3 (slot NB: ground)      */
    static constexpr int AL = KB + 18 * (NB + 1); /* [NB+1][6]: alpha3, aO3 (velocity-product accels) */
    static constexpr int S = AL + 6 * (NB + 1);  /* [ND][6]: Plucker columns (Omega, V at origin)   */
    static constexpr int QF = S + 6 * ND;        /* [NC] coordinate values                          */
    static constexpr int UF = QF + NC;           /* [NC] coordinate speeds                          */
    static constexpr int IC = UF + NC;           /* [NB][10]: m, h3, J6; then in place: subtree sums */
    static constexpr int WB = IC + 10 * NB;      /* [NB][6]: n3, f3; then in place: subtree sums     */
    static constexpr int MP = WB + 6 * NB;       /* [NP] packed lower M (+implicit)                 */
    static constexpr int RHS = MP + NP;          /* [ND]                                            */
    static constexpr int CW = RHS + ND;          /* [NS][8]: F3, Mo3, active                        */
    static constexpr int LIM = CW + 8 * NS;      /* [NL][4]: f, diag add, tau add                   */
    static constexpr int NSLOT = TopoInfo<T>::nslot();
    static constexpr int MF = LIM + 4 * NL;      /* [NSLOT][3]: function slots f, f', f''           */
    static constexpr int U = ((MF + 3 * (NSLOT > 0 ? NSLOT : 1) + 1) / 2) * 2;
    static constexpr int LOC = U;                /* phase 1: [NB+1][24] joint-local data (NB: identity) */
    static constexpr int SL = LOC + 24 * (NB + 1); /* phase 1: [ND][6] joint-local Plucker columns, + sink row */
    /* phases 2-3: [MPL * G][MAXSPAN] per muscle slot, -F_t dL/dq over its
     * span (actuator slot: its torque), then one zero slot (TZ) */
    static constexpr int TZ = MPL * T::G * T::MAXSPAN;
    static constexpr int TAUN = TZ + 1;
    static constexpr int TAU = U;
    static constexpr int CJ = TAU + TAUN;        /* phases 2-3: [NS][CJN] contact slots             */
    static constexpr int OBS = U;                /* report: observation staging                     */
    static constexpr int REP = OBS + OBSMAX;     /* report: [NOS+1][6] body pos/vel (NOS: COM)      */
    static constexpr int U1 = 24 * (NB + 1) + 6 * (ND + 1), U2 = TAUN + NS * CJN;
    static constexpr int U3 = OBSMAX + 6 * (T::NOS + 1);
    static constexpr int USZ = U1 > U2 ? (U1 > U3 ? U1 : U3) : (U2 > U3 ? U2 : U3);
    static constexpr int SIZE0 = ((U + USZ + 1) / 2) * 2;
    /* per-env stride residue mod 32 doubles (BIOIM_ENV_MOD >= 0, planar
     * topologies; the spatial ones have no LDS to spare): it sets which banks
     * the other env of a 32-lane group hits (ds_read_b64: 2 x 32 lanes;
     * ds_read_b128: 16-lane groups mixing both envs) */
    static constexpr int SIZE = (BIOIM_ENV_MOD >= 0 && T::PLANAR) ? SIZE0 + ((BIOIM_ENV_MOD - SIZE0 % 32) + 32) % 32 : SIZE0;
};

/* The realize cache (DState::cache): a step's realize runs at
 * the state the next step's first substep starts from, and a muscle model's
 * forces there do not depend on the excitations the policy sends next (they
 * enter only the activation rate).  So the realize also forms the implicit
 * system of that substep (h = the next step's substep length: M + h C + h^2 K
 * and its right-hand side, CJ / LIM at that h) and the muscles' fiber-velocity
 * roots, and stores them per env; the next launch's first substep loads them
 * and goes straight to the solve instead of a whole dynamics call.  Torque
 * models: the actuator torques are the controls, so their cached right-hand
 * side stops short of them and the cached substep adds this step's. */
#ifndef BIOIM_REALIZE_CACHE
#define BIOIM_REALIZE_CACHE 1
#endif
#ifndef BIOIM_REALIZE_CACHE_SPATIAL
#define BIOIM_REALIZE_CACHE_SPATIAL 1
#endif
#ifndef BIOIM_REALIZE_CACHE_TORQUE
#define BIOIM_REALIZE_CACHE_TORQUE 1
#endif
/* the spatial kernels load the cache row at the substep (0) or at kernel
 * start like the planar ones (1) */
#ifndef BIOIM_CACHE_PREFETCH_SPATIAL
#define BIOIM_CACHE_PREFETCH_SPATIAL 0
#endif
template <class T> struct CacheLay {
    /* torque models: the cached right-hand side leaves out the actuator
     * torques (the controls), which the cached substep adds */
    static constexpr bool ON = BIOIM_REALIZE_CACHE &&
                               (T::NM > 0 ? (T::PLANAR || BIOIM_REALIZE_CACHE_SPATIAL) : BIOIM_REALIZE_CACHE_TORQUE);
    /* planar kernels load the row at kernel start, ahead of the action
     * pre-processing; the spatial ones (no register headroom) at the substep */
    static constexpr bool PREFETCH = T::PLANAR || BIOIM_CACHE_PREFETCH_SPATIAL;
    static constexpr int ND = T::ND > 0 ? T::ND : 1, NP = ND * (ND + 1) / 2;
    static constexpr int SYS = NP + ND;          /* [NP] packed lower M(h), [ND] rhs(h): LDS MP..RHS order */
    static constexpr int MUS = SYS;              /* [NM][3] fiber-velocity root, dv/dl, clamped (0 / 1) */
    static constexpr int H = MUS + 3 * T::NM;    /* the h the system was formed at */
    static constexpr int DIM = ON ? H + 1 : 0;
    static constexpr int PF = (SYS + T::G - 1) / T::G;   /* system values per lane */
};

/* apply_perturbations kernels only: per env 5 doubles after all env regions
 * (call time base, substep length, cursor segment [lo, hi), its force) */
constexpr int PERT_SLOT = 5;

DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
/* the same fence inside a lane-divergent region: orders this wave's LDS
 * accesses (the active lanes' reads before their writes); lanes of one wave
 * execute in lockstep, so no lane can be behind */
DEV void wave_sync_lanes() { wave_sync(); }

/* Diagnostic build only (-DBIOIM_STAMPS, tools/stamps.py): per-phase shader
 * cycles of the first env of workgroup 0, accumulated over one launch. */
#ifdef BIOIM_STAMPS
#define STAMP(i)                                                                      \
    do {                                                                              \
        __builtin_amdgcn_sched_barrier(0);                                            \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();                         \
        __builtin_amdgcn_s_waitcnt(0xC07F);                                           \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[i] += t_ - stamp_prev;      \
        stamp_prev = t_;                                                              \
        __builtin_amdgcn_sched_barrier(0);                                            \
    } while (0)
#define STAMP_DECL unsigned long long stamp_prev = __builtin_amdgcn_s_memtime();
#else
#define STAMP(i) do {} while (0)
#define STAMP_DECL
#endif

template <int I> DEV constexpr int tri(int k, int l) { return k * (k + 1) / 2 + l; }

/* publish the coordinate values/speeds to LDS (QF/UF): dof lane d writes its
 * coordinate, lane 0 the locked coordinates (default value, zero speed) */
template <class T, typename Real>
DEV void publish_coords(const DModel<Real> &M, const SModel<T, Real> &SM, Real *lds, int lane, Real qd, Real ud) {
    using LY = Lay<T, Real>;
    if (lane < T::ND) {
        const int c = SM.dof_coord[lane];
        lds[LY::QF + c] = qd;
        lds[LY::UF + c] = ud;
    }
    if (lane == 0) {
        sfor<0, T::NC>([&](auto cI) {
            constexpr int c = decltype(cI)::value;
            if constexpr (T::coord_dof[c] < 0) { lds[LY::QF + c] = M.coord_default[c]; lds[LY::UF + c] = 0; }
        });
    }
}

/* ---------------------------------------------------------- kinematics
 * Phase 1a (lane = composite body c): the joint-local part, which depends
 * only on c's own coordinates — the spatial-transform axes (function
 * values and derivatives, the body-fixed rotation sequence, translations),
 * giving the child-in-parent transform, the joint's relative velocity and
 * velocity-product acceleration in the parent frame, and the joint's
 * Plucker columns about the parent origin (accumulated per dof into SL). */
template <class T, typename Real>
DEV void kin_local(const SModel<T, Real> &SM, Real *lds, int c) {
    using LY = Lay<T, Real>;
    using PL = Planar<T>;
    constexpr unsigned ZR = PL::ZR, ZW = PL::ZW, ZV = PL::ZV;
    constexpr unsigned USED = TopoInfo<T>::axes_used();
    const SBody<Real> &b = SM.body[c];
    Real RFM[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    Real wrel[3] = {0, 0, 0}, arel[3] = {0, 0, 0}, pFM[3] = {0, 0, 0}, pd[3] = {0, 0, 0}, pdd[3] = {0, 0, 0};
    Real col[6][3];
    int cd[6];
    sfor<0, 6>([&](auto aI) {
        constexpr int ax = decltype(aI)::value;
        cd[ax] = -1;
        if constexpr (((USED >> ax) & 1u) != 0) {
            /* the axis function's kind, coordinate, dof and spline slot are
             * compile-time facts of (body, axis) (topology_matches checks kind
             * and coordinate per pack): selected by the lane instead of read
             * through the function table, so the coordinate and coefficient
             * loads do not wait on one another */
            int kind = -1, cc = -1, dof = -1, js = -1;
            /* spatial models: an opaque copy of the lane's body, so the
             * selects are recomputed per call (a few VALU ops) instead of
             * hoisted out of the substep loop into 24 registers live across
             * it (the 3D push + RK-Merson kernel otherwise spills 16 B; 1 %
             * slower in 3D, so the planar kernels, far from the register
             * limit, keep the hoisted copies) */
            int cb = c;
            if constexpr (!T::PLANAR) asm volatile("" : "+v"(cb));
            sfor<0, T::NB>([&](auto bI) {
                constexpr int bb = decltype(bI)::value;
                constexpr int k = T::axis_kind[bb * 6 + ax], co = T::axis_coord[bb * 6 + ax];
                constexpr int dc = co >= 0 ? T::coord_dof[co] : -1, jsl = TopoInfo<T>::jslot(bb, ax);
                kind = cb == bb ? k : kind;
                cc = cb == bb ? co : cc;
                dof = cb == bb ? dc : dof;
                js = cb == bb ? jsl : js;
            });
            const int cs = cc >= 0 ? cc : 0;
            Real qc = lds[LY::QF + cs], uc = lds[LY::UF + cs];
            qc = cc >= 0 ? qc : Real(0);
            uc = cc >= 0 ? uc : Real(0);
            constexpr unsigned KM = TopoInfo<T>::axis_kinds(ax);
            const Real fa = b.fa[ax], fb = b.fb[ax];
            Real f = 0, f1 = 0, f2 = 0;
            if constexpr ((KM & (1u << (BIOIM_FN_LINEAR + 1))) != 0) {
                if (kind == BIOIM_FN_LINEAR) { f = fa * qc + fb; f1 = fa; }
            }
            if constexpr ((KM & (1u << (BIOIM_FN_CONST + 1))) != 0) {
                if (kind == BIOIM_FN_CONST) f = fb;
            }
            if constexpr ((KM & (1u << (BIOIM_FN_SPLINE + 1))) != 0) {
                /* spline axes: evaluated in phase 0b.  Planar: loaded
                 * unconditionally (slot 0 for the other kinds) and selected,
                 * no branch (same-box Torque2D -3 %, 2D -0.7 % with the
                 * branch-free SL and subtree sums; no gain in 3D, where it
                 * costs registers: profiles/r03/ab_subtree.txt) */
                const int jj = js >= 0 ? js : 0;
                if constexpr (T::PLANAR) {
                    const bool sp = kind == BIOIM_FN_SPLINE;
                    const Real sf = lds[LY::MF + 3 * jj], sf1 = lds[LY::MF + 3 * jj + 1], sf2 = lds[LY::MF + 3 * jj + 2];
                    f = sp ? sf : f; f1 = sp ? sf1 : f1; f2 = sp ? sf2 : f2;
                } else if (kind == BIOIM_FN_SPLINE) {
                    f = lds[LY::MF + 3 * jj]; f1 = lds[LY::MF + 3 * jj + 1]; f2 = lds[LY::MF + 3 * jj + 2];
                }
            }
            cd[ax] = dof;
            Real a[3] = {b.axis[ax][0], b.axis[ax][1], b.axis[ax][2]};
            if constexpr (ax < 3) {
                PL::ang(a);
                Real ucol[3], cr[3];
                mv3m<ZR, ZW>(RFM, a, ucol);
                Real thd = f1 * uc;
                cross3m<ZW, ZW>(wrel, ucol, cr);
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    arel[i] += ucol[i] * (f2 * uc * uc) + cr[i] * thd;
                    wrel[i] += ucol[i] * thd;
                    col[ax][i] = ucol[i] * f1;
                }
                PL::ang(arel); PL::ang(wrel); PL::ang(col[ax]);
                Real Rk[9];
                if constexpr (T::PLANAR) {   /* about (0, 0, a_z), a_z = +-1 */
                    Real sn, cn;
                    sincos_rt(f, sn, cn);
                    Rk[0] = cn; Rk[1] = -sn * a[2]; Rk[3] = sn * a[2]; Rk[4] = cn;
                    PL::rot(Rk);
                } else {
                    axis_rot(a, f, Rk);  /* f == 0 (absent axis): identity */
                }
                mm3m<ZR, ZR>(RFM, Rk, RFM);
            } else {
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    pFM[i] += a[i] * f; pd[i] += a[i] * (f1 * uc); pdd[i] += a[i] * (f2 * uc * uc);
                    col[ax][i] = a[i] * f1;
                }
                PL::lin(pd); PL::lin(pdd); PL::lin(col[ax]);
            }
        }
    });
    Real Rpf[9], Rmb[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) { Rpf[i] = b.R_pf[i]; Rmb[i] = b.R_mb[i]; }
    PL::rot(Rpf); PL::rot(Rmb);
    Real dF[3], T9[9], RPB[9], pm[3], pPB[3];
    mv3m<ZR, 0>(RFM, b.p_mb, dF);
    mm3m<ZR, ZR>(Rpf, RFM, T9);
    mm3m<ZR, ZR>(T9, Rmb, RPB);
#pragma unroll
    for (int i = 0; i < 3; ++i) pm[i] = pFM[i] + dF[i];
    mv3m<ZR, 0>(Rpf, pm, pPB);
    Real *lc = lds + LY::LOC + 24 * c;
#pragma unroll
    for (int i = 0; i < 9; ++i) lc[i] = RPB[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) lc[9 + i] = pPB[i] + b.p_pf[i];
    Real t1[3], t2[3], t3[3], o[3];
    mv3m<ZR, ZW>(Rpf, wrel, o);
#pragma unroll
    for (int i = 0; i < 3; ++i) lc[12 + i] = o[i];
    cross3m<ZW, 0>(wrel, dF, t1);
#pragma unroll
    for (int i = 0; i < 3; ++i) t2[i] = pd[i] + t1[i];
    mv3m<ZR, ZV>(Rpf, t2, o);
#pragma unroll
    for (int i = 0; i < 3; ++i) lc[15 + i] = o[i];
    mv3m<ZR, ZW>(Rpf, arel, o);
#pragma unroll
    for (int i = 0; i < 3; ++i) lc[18 + i] = o[i];
    cross3m<ZW, 0>(arel, dF, t2);
    cross3m<ZW, ZV>(wrel, t1, t3);
#pragma unroll
    for (int i = 0; i < 3; ++i) t2[i] = pdd[i] + t2[i] + t3[i];
    mv3m<ZR, ZV>(Rpf, t2, o);
#pragma unroll
    for (int i = 0; i < 3; ++i) lc[21 + i] = o[i];
    /* Plucker columns in the parent frame, linear part at the parent origin;
     * rotations act about the M origin pM = p_pf + R_pf pFM */
    Real pM[3];
    mv3m<ZR, 0>(Rpf, pFM, pM);
#pragma unroll
    for (int i = 0; i < 3; ++i) pM[i] += b.p_pf[i];
    sfor<0, 6>([&](auto aI) {
        constexpr int ax = decltype(aI)::value;
        if constexpr (((USED >> ax) & 1u) != 0) {
            /* planar: an axis without a dof accumulates into the sink row
             * SL[ND] (no branch) */
            if (T::PLANAR || cd[ax] >= 0) {
                Real *sl = lds + LY::SL + 6 * (cd[ax] >= 0 ? cd[ax] : LY::ND);
                Real v[3];
                if constexpr (ax < 3) {
                    mv3m<ZR, ZW>(Rpf, col[ax], v);
                    Real lin[3];
                    cross3m<0, ZW>(pM, v, lin);
#pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        if (!((ZW >> i) & 1u)) sl[i] += v[i];
                        if (!((ZV >> i) & 1u)) sl[3 + i] += lin[i];
                    }
                } else {
                    mv3m<ZR, ZV>(Rpf, col[ax], v);
#pragma unroll
                    for (int i = 0; i < 3; ++i)
                        if (!((ZV >> i) & 1u)) sl[3 + i] += v[i];
                }
            }
        }
    });
}

/* body frame and motion: orientation, origin, angular velocity, spatial
 * velocity at the (shifted) ground origin, and the velocity-product
 * accelerations (zero q'') */
template <typename Real> struct Frame {
    Real R[9], o[3], w[3], vO[3], al[3], aO[3];
};

/* F := F composed with the joint whose parent-frame data is lc (LOC slot).
 * Zero masks: R rotations, w/wrg/al angular, vO/vrel/aO/aa linear (Planar) */
template <class T, typename Real> DEV void compose(Frame<Real> &F, const Real *lc) {
    using PL = Planar<T>;
    constexpr unsigned ZR = PL::ZR, ZW = PL::ZW, ZV = PL::ZV;
    Real R[9], oB[3], w[3], wrg[3], vrel[3], vO[3], al[3], t[3], t2[3], t3[3];
    mm3m<ZR, ZR>(F.R, lc, R);
    mv3m<ZR, 0>(F.R, lc + 9, t);
#pragma unroll
    for (int i = 0; i < 3; ++i) oB[i] = F.o[i] + t[i];
    mv3m<ZR, ZW>(F.R, lc + 12, wrg);
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = F.w[i] + wrg[i];
    mv3m<ZR, ZV>(F.R, lc + 15, vrel);
    cross3m<ZW, 0>(wrg, oB, t);
#pragma unroll
    for (int i = 0; i < 3; ++i) vO[i] = F.vO[i] + vrel[i] - t[i];
    mv3m<ZR, ZW>(F.R, lc + 18, t);
    cross3m<ZW, ZW>(F.w, wrg, t2);
#pragma unroll
    for (int i = 0; i < 3; ++i) al[i] = F.al[i] + t2[i] + t[i];
    /* acceleration of the new origin: parent point acceleration
     * + Coriolis 2 wP x vrel + relative acceleration */
    Real vpt[3], aB[3], aa[3];
    cross3m<ZW, 0>(F.w, oB, t);
#pragma unroll
    for (int i = 0; i < 3; ++i) vpt[i] = F.vO[i] + t[i];
    cross3m<ZW, 0>(F.al, oB, t);
    cross3m<ZW, ZV>(F.w, vpt, t2);
    cross3m<ZW, ZV>(F.w, vrel, t3);
    mv3m<ZR, ZV>(F.R, lc + 21, aa);
#pragma unroll
    for (int i = 0; i < 3; ++i) aB[i] = F.aO[i] + t[i] + t2[i] + Real(2) * t3[i] + aa[i];
    Real vB[3];
    cross3m<ZW, 0>(w, oB, t);
#pragma unroll
    for (int i = 0; i < 3; ++i) vB[i] = vO[i] + t[i];
    cross3m<ZW, 0>(al, oB, t);
    cross3m<ZW, ZV>(w, vB, t2);
#pragma unroll
    for (int i = 0; i < 9; ++i) F.R[i] = R[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        F.aO[i] = aB[i] - t[i] - t2[i];
        F.o[i] = oB[i]; F.w[i] = w[i]; F.vO[i] = vO[i]; F.al[i] = al[i];
    }
    PL::rot(F.R); PL::ang(F.w); PL::lin(F.vO); PL::ang(F.al); PL::lin(F.aO);
}

/* identity joint (LOC slot NB) and the ground frame (KB/AL slot NB) */
template <class T, typename Real> DEV void kin_ground(Real *lds, Real x0) {
    using LY = Lay<T, Real>;
    Real *lc = lds + LY::LOC + 24 * T::NB, *kb = lds + LY::KB + 18 * T::NB, *ab = lds + LY::AL + 6 * T::NB;
#pragma unroll
    for (int i = 0; i < 24; ++i) lc[i] = (i < 9 && (i % 4) == 0) ? Real(1) : Real(0);
#pragma unroll
    for (int i = 0; i < 18; ++i) kb[i] = (i < 9 && (i % 4) == 0) ? Real(1) : Real(0);
    kb[9] = -x0;
#pragma unroll
    for (int i = 0; i < 6; ++i) ab[i] = 0;
}

/* Phase 1b (lane = body c): compose c's root-to-body joint chain in
 * registers (front-padded with the identity joint, so every lane runs the
 * same DEPTH compositions with no inter-lane dependency) */
template <class T, typename Real>
DEV void kin_chain(const SModel<T, Real> &SM, Real *lds, int c, Real x0) {
    using LY = Lay<T, Real>;
    Frame<Real> F;
#pragma unroll
    for (int i = 0; i < 9; ++i) F.R[i] = (i % 4) == 0 ? Real(1) : Real(0);
#pragma unroll
    for (int i = 0; i < 3; ++i) { F.o[i] = i == 0 ? -x0 : Real(0); F.w[i] = 0; F.vO[i] = 0; F.al[i] = 0; F.aO[i] = 0; }
    sfor<0, TopoInfo<T>::depth()>([&](auto lI) {
        constexpr int lvl = decltype(lI)::value;
        const Real *src = lds + LY::LOC + 24 * SM.chain[c][lvl];
        Real lc[24];
#pragma unroll
        for (int i = 0; i < 24; ++i) lc[i] = src[i];
        Planar<T>::loc(lc);
        compose<T, Real>(F, lc);
    });
    Real *kb = lds + LY::KB + 18 * c, *ab = lds + LY::AL + 6 * c;
#pragma unroll
    for (int i = 0; i < 9; ++i) kb[i] = F.R[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        kb[9 + i] = F.o[i]; kb[12 + i] = F.w[i]; kb[15 + i] = F.vO[i];
        ab[i] = F.al[i]; ab[3 + i] = F.aO[i];
    }
}

/* Phase 0b: the function slots (Lay::MF), one lane each — moving path
 * points' location functions and the joints' spline axes — from the
 * published coordinates; ends with a wave sync when there are any */
template <bool BFK, class T, typename Real>
DEV void fn_slots(const SModel<T, Real> &SM, Real *lds, int lane) {
    using LY = Lay<T, Real>;
    if constexpr (LY::NSLOT > 0) {
        sfor<0, (LY::NSLOT + T::G - 1) / T::G>([&](auto pI) {
            const int f = lane + decltype(pI)::value * T::G;
            if (f < LY::NSLOT) {
                Real v, d1, d2;
                fn_eval_bf<BFK, T, Real>(SM, SM.mf_fn[f], lds[LY::QF + SM.mf_coord[f]], v, d1, d2);
                lds[LY::MF + 3 * f] = v;
                lds[LY::MF + 3 * f + 1] = d1;
                lds[LY::MF + 3 * f + 2] = d2;
            }
        });
        wave_sync();
    }
}

/* Phase 1c (lane = dof): ground Plucker column from the parent frame */
template <class T, typename Real>
DEV void kin_column(const SModel<T, Real> &SM, Real *lds, int d) {
    using LY = Lay<T, Real>;
    using PL = Planar<T>;
    constexpr unsigned ZR = PL::ZR, ZW = PL::ZW, ZV = PL::ZV;
    const Real *kp = lds + LY::KB + 18 * SM.body[SM.dof_cb[d]].pslot;
    const Real *sl = lds + LY::SL + 6 * d;
    Real K[12], sc[6];
#pragma unroll
    for (int i = 0; i < 12; ++i) K[i] = kp[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) sc[i] = sl[i];
    PL::rot(K); PL::col(sc);
    Real Sa[3], Sl[3], t[3];
    mv3m<ZR, ZW>(K, sc, Sa);
    mv3m<ZR, ZV>(K, sc + 3, Sl);
    cross3m<ZW, 0>(Sa, K + 9, t);
    Real *S = lds + LY::S + 6 * d;
#pragma unroll
    for (int i = 0; i < 3; ++i) { S[i] = Sa[i]; S[3 + i] = Sl[i] - t[i]; }
}

/* Phase 1c (lane = body): spatial inertia at the ground origin and the
 * Newton-Euler (velocity-product + gravity) wrench */
template <class T, typename Real>
DEV void body_inertia(const SModel<T, Real> &SM, const DModel<Real> &M, Real *lds, int c) {
    using LY = Lay<T, Real>;
    using PL = Planar<T>;
    constexpr unsigned ZR = PL::ZR, ZW = PL::ZW, ZV = PL::ZV;
    const SBody<Real> &b = SM.body[c];
    const Real *kb = lds + LY::KB + 18 * c, *ab = lds + LY::AL + 6 * c;
    Real K[18], A[6];
#pragma unroll
    for (int i = 0; i < 18; ++i) K[i] = kb[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) A[i] = ab[i];
    PL::frame(K); PL::acc(A);
    const Real *R = K, *o = K + 9, *w = K + 12, *vO = K + 15, *al = A, *aO = A + 3;
    Real cl[3], cG[3];
    mv3m<ZR, 0>(R, b.com, cl);
#pragma unroll
    for (int i = 0; i < 3; ++i) cG[i] = o[i] + cl[i];
    Real Ib[9] = {b.inertia[0], b.inertia[3], b.inertia[4], b.inertia[3], b.inertia[1],
                  b.inertia[5], b.inertia[4], b.inertia[5], b.inertia[2]};
    Real Tm[9], RT[9], IG[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) RT[3 * i + j] = R[3 * j + i];
    mm3m<ZR, 0>(R, Ib, Tm);
    mm3m<0, ZR>(Tm, RT, IG);
    Real m = b.mass, ccd = dot3(cG, cG);
    Real *ic = lds + LY::IC + 10 * c;
    ic[0] = m;
#pragma unroll
    for (int i = 0; i < 3; ++i) ic[1 + i] = m * cG[i];
    ic[4] = IG[0] + m * (ccd - cG[0] * cG[0]);
    ic[5] = IG[4] + m * (ccd - cG[1] * cG[1]);
    ic[6] = IG[8] + m * (ccd - cG[2] * cG[2]);
    ic[7] = IG[1] - m * cG[0] * cG[1];
    ic[8] = IG[2] - m * cG[0] * cG[2];
    ic[9] = IG[5] - m * cG[1] * cG[2];
    Real vc[3], ac[3], t[3], t2[3];
    cross3m<ZW, 0>(w, cG, t);
#pragma unroll
    for (int i = 0; i < 3; ++i) vc[i] = vO[i] + t[i];
    cross3m<ZW, 0>(al, cG, t);
    cross3m<ZW, ZV>(w, vc, t2);
#pragma unroll
    for (int i = 0; i < 3; ++i) ac[i] = aO[i] + t[i] + t2[i];
    Real f[3], Iw[3], Ia[3], n[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) f[i] = m * (ac[i] - M.gravity[i]);
    mv3m<0, ZW>(IG, w, Iw);
    mv3m<0, ZW>(IG, al, Ia);
    cross3m<ZW, 0>(w, Iw, t);
#pragma unroll
    for (int i = 0; i < 3; ++i) n[i] = Ia[i] + t[i];
    cross3(cG, f, t);
    Real *wb = lds + LY::WB + 6 * c;
#pragma unroll
    for (int i = 0; i < 3; ++i) { wb[i] = n[i] + t[i]; wb[3 + i] = f[i]; }
}

/* symmetric 3x3 (xx yy zz xy xz yz) times v, v's known zeros masked (ZB) */
template <unsigned ZB, typename Real> DEV void symvm(const Real *J, const Real *v, Real *o) {
    const int r0[3] = {0, 3, 4}, r1[3] = {3, 1, 5}, r2[3] = {4, 5, 2}, iv[3] = {0, 1, 2}, sg[3] = {1, 1, 1};
    Real x = sum_m<0, ZB, 3>(J, v, r0, iv, sg), y = sum_m<0, ZB, 3>(J, v, r1, iv, sg), z = sum_m<0, ZB, 3>(J, v, r2, iv, sg);
    o[0] = x; o[1] = y; o[2] = z;
}
/* symmetric 3x3 (xx yy zz xy xz yz) times v */
template <typename Real> DEV void symv(const Real *J, const Real *v, Real *o) {
    Real x = J[0] * v[0] + J[3] * v[1] + J[4] * v[2];
    Real y = J[3] * v[0] + J[1] * v[1] + J[5] * v[2];
    Real z = J[4] * v[0] + J[5] * v[1] + J[2] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}

/* Tree-sparse LTL factorization M = L^T L and solve (Featherstone, Rigid
 * Body Dynamics Algorithms 6.3), unrolled at compile time over the
 * topology's dof tree: entry (k, i) of M is structurally non-zero only when
 * i is k or an ancestor dof of k, and factoring from the leaves up creates
 * no fill-in, so only those entries are touched (2D: 53 of the dense 121
 * multiply-adds, 3D: 257 of 457).  In place on the packed lower M; returns
 * false if not SPD. */
template <class T> struct DofTree {
    /* parent dof: the previous dof of the same body, else the last dof of
     * the nearest ancestor body that has one, else -1 */
    static constexpr int par(int d) {
        for (int e = d - 1; e >= 0; --e)
            if (T::dof_cb[e] == T::dof_cb[d]) return e;
        for (int b = T::parent[T::dof_cb[d]]; b >= 0; b = T::parent[b]) {
            int last = -1;
            for (int e = 0; e < T::ND; ++e)
                if (T::dof_cb[e] == b) last = e;
            if (last >= 0) return last;
        }
        return -1;
    }
    /* i is a proper ancestor dof of k */
    static constexpr bool anc(int k, int i) {
        for (int j = par(k); j >= 0; j = par(j))
            if (j == i) return true;
        return false;
    }
    /* bit l set: l is k or an ancestor dof of k (the structurally non-zero
     * entries (k, l) of row k of M) */
    static constexpr unsigned path_mask(int k) {
        unsigned m = 1u << k;
        for (int j = par(k); j >= 0; j = par(j)) m |= 1u << j;
        return m;
    }
    /* dof 0 is on every dof's root path (phase 3's row stores rely on it) */
    static constexpr bool root_common() {
        for (int k = 0; k < T::ND; ++k)
            if (!(path_mask(k) & 1u)) return false;
        return true;
    }
};

template <class T, int N, typename Real> DEV bool ltl_solve(Real *A, Real *b) {
    using DT = DofTree<T>;
    bool ok = true;
    Real inv[N];
    /* factor: for k = N-1 .. 0 */
    sfor<0, N>([&](auto kk) {
        constexpr int k = N - 1 - decltype(kk)::value;
        Real s = A[tri<0>(k, k)];
        ok = ok && (s > 0);
        const Real sp = s > 0 ? s : Real(1e-30);
        const Real id = fast_rsqrt(sp), d = sp * id;
        inv[k] = id;
        A[tri<0>(k, k)] = d;
        sfor<0, N>([&](auto iI) {
            constexpr int i = decltype(iI)::value;
            if constexpr (DT::anc(k, i)) A[tri<0>(k, i)] *= id;
        });
        sfor<0, N>([&](auto iI) {
            constexpr int i = decltype(iI)::value;
            if constexpr (DT::anc(k, i)) {
                sfor<0, N>([&](auto jI) {
                    constexpr int j = decltype(jI)::value;
                    if constexpr (j == i || DT::anc(i, j)) A[tri<0>(i, j)] -= A[tri<0>(k, i)] * A[tri<0>(k, j)];
                });
            }
        });
    });
    /* L^T y = b, leaves first */
    sfor<0, N>([&](auto ii) {
        constexpr int i = N - 1 - decltype(ii)::value;
        b[i] *= inv[i];
        sfor<0, N>([&](auto jI) {
            constexpr int j = decltype(jI)::value;
            if constexpr (DT::anc(i, j)) b[j] -= A[tri<0>(i, j)] * b[i];
        });
    });
    /* L x = y, root first */
    sfor<0, N>([&](auto iI) {
        constexpr int i = decltype(iI)::value;
        sfor<0, N>([&](auto jI) {
            constexpr int j = decltype(jI)::value;
            if constexpr (DT::anc(i, j)) b[i] -= A[tri<0>(i, j)] * b[j];
        });
        b[i] *= inv[i];
    });
    return ok;
}

/* ---------------------------------------------------- contact + limits */
/* branch-free: the transition polynomial is evaluated everywhere and
 * selected (finite for any x) */
template <bool BF, typename Real> DEV Real smooth_step(Real y0, Real y1, Real x0, Real x1, Real iw, Real x) {
    if constexpr (!BF) {
        if (x <= x0) return y0;
        if (x >= x1) return y1;
    }
    Real t = (x - x0) * iw;   /* iw = 1 / (x1 - x0) */
    const Real v = y0 + (y1 - y0) * t * t * t * (Real(10) + t * (Real(6) * t - Real(15)));
    return x <= x0 ? y0 : (x >= x1 ? y1 : v);
}
template <bool BF, typename Real> DEV Real smooth_step_d(Real y0, Real y1, Real x0, Real x1, Real iw, Real x) {
    if constexpr (!BF) {
        if (x <= x0 || x >= x1) return 0;
    }
    Real t = (x - x0) * iw;
    const Real v = (y1 - y0) * Real(30) * t * t * (Real(1) - t) * (Real(1) - t) * iw, zero = 0;
    return ((x <= x0) | (x >= x1)) ? zero : v;
}

/* Hunt-Crossley sphere s (this lane) vs the ground plane.  Publishes the
 * sphere's wrench about the (shifted) ground origin (CW) and, for the
 * generalized force / implicit matrix, the contact point P, the force F
 * (normal component at the implicitly advanced position) and the 3x3
 * implicit damping/stiffness block C (h > 0) into CJ.  Phase 3 forms the
 * contact-point Jacobian J_d = S_d.ang x P + S_d.lin from the Plucker
 * columns it already holds: M_lk += J_l.C J_k, rhs_d += S_d.(P x F, F). */
/* One sphere's Hunt-Crossley contact (lane = sphere s): the force and its
 * moment about the ground origin (CW slot: F3, Mo3, active), and for the
 * implicit step the contact point, the force with the -h Kn v_y term and
 * the 3x3 damping/stiffness block (CJ slot).  Branch-free (selects only), so
 * the muscle lanes can evaluate it inside the muscle block where the
 * scheduler interleaves it with the curve evaluations' dependency chains
 * (contact_store writes it); an inactive sphere's CJ values are unused. */
template <typename Real> struct ContactOut {
    Real cw[7], cj[10];
};
template <bool BFK, class T, typename Real>
DEV void contact_compute(const SModel<T, Real> &SM, const Real *lds, int s, Real h, ContactOut<Real> &o) {
    using LY = Lay<T, Real>;
    using PL = Planar<T>;
    const int cb = SM.sph_cb[s], fo = SM.sph_force[s];
    const Real *kbp = lds + LY::KB + 18 * cb;
    Real kb[18];
#pragma unroll
    for (int i = 0; i < 18; ++i) kb[i] = kbp[i];
    PL::frame(kb);
    Real Cn[3];
    mv3m<PL::ZR, 0>(kb, SM.sph_loc[s], Cn);
#pragma unroll
    for (int i = 0; i < 3; ++i) Cn[i] += kb[9 + i];
    const Real rad = SM.sph_r[s];
    const Real depth = rad - Cn[1];
    const bool pen = depth > 0;
    const Real P[3] = {Cn[0], Cn[1] - (rad - Real(0.5) * depth), Cn[2]};
    Real t[3], vs[3];
    cross3m<PL::ZW, 0>(kb + 12, P, t);
#pragma unroll
    for (int i = 0; i < 3; ++i) vs[i] = kb[15 + i] + t[i];
    PL::lin(vs);
    const Real vn = -vs[1];
    const Real kk = SM.cf_kk[fo], cc = SM.cf_c[fo];
    const Real dps = pen ? depth : Real(1), zero = 0;
    const Real rkd = rad * kk * dps;
    /* ?: arms are plain locals: an expression arm makes clang emit a branch */
    constexpr bool BF = BFK;
    Real fH;
    if constexpr (BF) {
        const Real fHp = Real(4.0 / 3.0) * kk * dps * (rkd * fast_rsqrt(rkd));
        fH = pen ? fHp : zero;
    } else {
        fH = pen ? Real(4.0 / 3.0) * kk * dps * (rkd * fast_rsqrt(rkd)) : Real(0);
    }
    const Real fn = fH * (Real(1) + Real(1.5) * cc * vn);
    const bool active = pen && fn > 0;
    const Real vt0 = -vs[0], vt2 = -vs[2];
    const Real vs2 = vt0 * vt0 + vt2 * vt2;
    Real ivs;
    if constexpr (BF) {
        const Real rvs = fast_rsqrt(vs2);
        ivs = vs2 > 0 ? rvs : zero;
    } else {
        ivs = vs2 > 0 ? fast_rsqrt(vs2) : Real(0);
    }
    const Real vslip = vs2 * ivs;
    const Real vtr = SM.cf_vt[fo], ms = SM.cf_ms[fo], md = SM.cf_md[fo], mv = SM.cf_mv[fo];
    const Real ivtr = fast_rcp(vtr);
    const Real r_ = vslip * ivtr, den = Real(1) + r_ * r_;
    const Real iden = fast_rcp(den);
    const Real ff = fn * (fmin(r_, Real(1)) * (md + Real(2) * (ms - md) * iden) + mv * vslip);
    const bool slip = vslip != 0;
    Real F[3];
    if constexpr (BF) {
        const Real fx = ff * vt0 * ivs, fz = ff * vt2 * ivs;
        F[0] = slip ? fx : zero; F[1] = fn; F[2] = slip ? fz : zero;
    } else {
        F[0] = slip ? ff * vt0 * ivs : Real(0); F[1] = fn; F[2] = slip ? ff * vt2 * ivs : Real(0);
    }
    Real mo[3];
    cross3(P, F, mo);
#pragma unroll
    for (int i = 0; i < 3; ++i) { o.cw[i] = active ? F[i] : Real(0); o.cw[3 + i] = active ? mo[i] : Real(0); }
    o.cw[6] = active ? Real(1) : Real(0);
    const Real kn = Real(1.5) * fH * fast_rcp(dps) * (Real(1) + Real(1.5) * cc * vn);
    /* implicit extra force -h*Kn*v_y (Hertz force at the advanced position) */
#pragma unroll
    for (int i = 0; i < 3; ++i) o.cj[i] = P[i];
    o.cj[3] = F[0];
    o.cj[4] = F[1] - (h > 0 ? h * kn * vs[1] : Real(0));
    o.cj[5] = F[2];
    const Real base = (md + Real(2) * (ms - md) * iden);
    const bool low = r_ < 1;
    Real g_s = low ? base * ivtr + mv : base * ivs + mv;
    Real gp = low ? base * ivtr - Real(4) * (ms - md) * r_ * r_ * (iden * iden * ivtr) + mv
                  : -Real(4) * (ms - md) * r_ * (iden * iden * ivtr) + mv;
    gp = gp < 0 ? Real(0) : gp;
    const Real tx = vslip > 0 ? vt0 * ivs : Real(0), tz = vslip > 0 ? vt2 * ivs : Real(0);
    const Real ctt = h * fn * g_s, cq = h * fn * (gp - g_s);
    const bool imp = h > 0;
    o.cj[6] = imp ? ctt + cq * tx * tx : Real(0);
    o.cj[7] = imp ? cq * tx * tz : Real(0);
    o.cj[8] = imp ? h * Real(1.5) * cc * fH + h * h * kn : Real(0);
    o.cj[9] = imp ? ctt + cq * tz * tz : Real(0);
}
template <class T, typename Real> DEV void contact_store(Real *lds, int s, const ContactOut<Real> &o) {
    using LY = Lay<T, Real>;
    Real *cw = lds + LY::CW + 8 * s, *cj = lds + LY::CJ + LY::CJN * s;
#pragma unroll
    for (int i = 0; i < 7; ++i) cw[i] = o.cw[i];
#pragma unroll
    for (int i = 0; i < 10; ++i) cj[i] = o.cj[i];
}
template <bool BFK, class T, typename Real>
DEV void contact_lane(const SModel<T, Real> &SM, Real *lds, int s, Real h) {
    ContactOut<Real> o;
    contact_compute<BFK, T, Real>(SM, lds, s, h, o);
    contact_store<T, Real>(lds, s, o);
}

/* contact-point Jacobian column of a dof: S.ang x P + S.lin */
template <typename Real> DEV void contact_jac(const Real *Sd, const Real *P, Real *j) {
    cross3(Sd, P, j);
#pragma unroll
    for (int i = 0; i < 3; ++i) j[i] += Sd[3 + i];
}

/* ------------------------------------------------------------ muscles */
template <typename Real> struct MState {
    Real act, lce, vN, vce, Ft, Ff, Fa, dadt, dvdl;
    bool clamped;
};

/* activation rate du/dt = (u - a) / tau, tau = tau_act (0.5 + 1.5 a) or
 * tau_deact / (0.5 + 1.5 a), a the clamped activation (muscle_eval; the
 * cached first substep of CACHE kernels) */
template <bool BF, typename Real> DEV Real act_rate(const SMuscle<Real> &mu, Real a, Real excitation) {
    if constexpr (BF) {
        const Real amin = mu.amin, one = 1;
        Real u = excitation < amin ? amin : (excitation > one ? one : excitation);
        const Real ab = Real(0.5) + Real(1.5) * a;
        const Real da_act = (u - a) * fast_rcp(mu.tau_act * ab), da_deact = (u - a) * ab * fast_rcp(mu.tau_deact);
        return u > a ? da_act : da_deact;
    } else {
        Real u = excitation < mu.amin ? mu.amin : (excitation > Real(1) ? Real(1) : excitation);
        const Real ab = Real(0.5) + Real(1.5) * a;
        return u > a ? (u - a) * fast_rcp(mu.tau_act * ab) : (u - a) * ab * fast_rcp(mu.tau_deact);
    }
}

template <bool BFK, bool BFC, class T, typename Real>
DEV void muscle_eval(const SModel<T, Real> &SM, const SMuscle<Real> &mu, Real a_state, Real l_state, Real excitation,
                     Real L, Real v_warm, MState<Real> &s) {
    STAMP_DECL
    const DCurve<Real> &Cfal = SM.curve[mu.cv[0]], &Cfv = SM.curve[mu.cv[1]], &Cfpe = SM.curve[mu.cv[2]],
                       &Cfse = SM.curve[mu.cv[3]];
    /* ?: arms are plain locals throughout (see below) */
    constexpr bool BF = BFK;
    const Real amin = mu.amin, lmin = mu.lmin, one = 1, zero = 0;
    Real a, lce;
    if constexpr (BF) {
        a = a_state < amin ? amin : (a_state > one ? one : a_state);
        lce = l_state < lmin ? lmin : l_state;
    } else {
        a = a_state < mu.amin ? mu.amin : (a_state > Real(1) ? Real(1) : a_state);
        lce = l_state < mu.lmin ? mu.lmin : l_state;
    }
    Real w = mu.width;
    const Real sq2 = lce * lce - w * w;
    const Real isq = fast_rsqrt(sq2), sq = sq2 * isq;
    const Real icos = lce * isq;          /* 1 / cos(pennation) */
    Real lt = L - sq;
    Real fse, dfse, fal, dfal, fpe, dfpe;
    /* BFC: the three curve chains and the fiber-velocity start and
     * extrapolation in one basic block (every semi-implicit kernel; in the
     * spatial ones only these, the other branch-free forms would spill) */
    curve_eval<BFC>(Cfse, lt * mu.inv_lts, fse, dfse);
    curve_eval<BFC>(Cfal, lce * mu.inv_lopt, fal, dfal);
    curve_eval<BFC>(Cfpe, lce * mu.inv_lopt, fpe, dfpe);
#if BIOIM_SGB == 1
    /* round-5 scheduling experiment: a pipeline that issues
     * the curves' LDS reads in groups ahead of VALU work of this block */
#pragma unroll
    for (int gI = 0; gI < 6; ++gI) {
        __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);   /* DS reads */
        __builtin_amdgcn_sched_group_barrier(0x2, 12, 0);    /* VALU */
    }
#elif BIOIM_SGB == 2
#pragma unroll
    for (int gI = 0; gI < 24; ++gI) {
        __builtin_amdgcn_sched_group_barrier(0x2, 3, 0);     /* VALU */
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   /* DS read */
    }
#endif
    Real rhs = fse * icos - fpe;
    STAMP(16);
    Real vN, fvv, dfv;
    solve_fv<BFC, !T::PLANAR || BIOIM_FV_PE_PLANAR>(Cfv, a * fal, mu.beta, rhs, v_warm, vN, fvv, dfv);
    STAMP(17);
    Real dGdv = a * fal * dfv + mu.beta;
    /* selects over plain locals (a load in a ?: arm or an if body becomes a
     * branch that splits the muscle eval's basic block) */
    bool clamped;
    if constexpr (BF) {
        const Real fv_at0 = Cfv.y_at0;
        clamped = ((l_state <= lmin) & (vN <= 0)) | (l_state < lmin);
        vN = clamped ? zero : vN;
        fvv = clamped ? fv_at0 : fvv;
    } else {
        clamped = (l_state <= mu.lmin && vN <= 0) || l_state < mu.lmin;
        if (clamped) {
            vN = 0;
            fvv = Cfv.y_at0;
        }
    }
    s.act = a;
    s.lce = lce;
    s.vN = vN;
    s.vce = vN * mu.lv;
    s.Ft = mu.fiso * fse;
    s.Fa = mu.fiso * a * fal * fvv;
    s.Ff = mu.fiso * (a * fal * fvv + fpe + mu.beta * vN);
    s.clamped = clamped;
    Real dGdl = (a * dfal * fvv + dfpe) * mu.inv_lopt + dfse * mu.inv_lts * (icos * icos) + fse * w * w * (isq * isq * isq);
    if constexpr (BF) {
        const Real dvdl = -(dGdl * fast_rcp(dGdv)) * mu.lv;
        s.dvdl = clamped ? zero : dvdl;
    } else {
        s.dvdl = clamped ? Real(0) : -(dGdl * fast_rcp(dGdv)) * mu.lv;
    }
    s.dadt = act_rate<BF>(mu, a, excitation);
    STAMP(18);
}

/* static fiber equilibrium at reset (zero fiber velocity) */
template <bool BFK, class T, typename Real>
DEV Real muscle_equilibrium(const SModel<T, Real> &SM, const SMuscle<Real> &mu, Real a_state, Real L) {
    const DCurve<Real> &Cfal = SM.curve[mu.cv[0]], &Cfpe = SM.curve[mu.cv[2]], &Cfse = SM.curve[mu.cv[3]];
    Real a = a_state < mu.amin ? mu.amin : (a_state > Real(1) ? Real(1) : a_state);
    Real w = mu.width, lo = mu.lmin;
    Real hi = sqrt((L - mu.lts) * (L - mu.lts) + w * w);
    if (!(L - mu.lts > sqrt(lo * lo - w * w))) return lo;
    {   /* the fiber out-pulls the tendon even at its minimum length: no root */
        Real sq = sqrt(lo * lo - w * w), fal, dfal, fpe, dfpe, fse, dfse;
        curve_eval<BFK>(Cfal, lo * mu.inv_lopt, fal, dfal);
        curve_eval<BFK>(Cfpe, lo * mu.inv_lopt, fpe, dfpe);
        curve_eval<BFK>(Cfse, (L - sq) * mu.inv_lts, fse, dfse);
        if ((a * fal + fpe) * (sq / lo) - fse >= 0) return lo;
    }
    Real l = sqrt((L - Real(1.01) * mu.lts) * (L - Real(1.01) * mu.lts) + w * w), dprev = 1;
    if (!(l > lo && l < hi)) l = Real(0.5) * (lo + hi);
    for (int it = 0; it < 4 * Eps<Real>::it_max; ++it) {
        Real sq = sqrt(l * l - w * w), cphi = sq / l;
        Real fal, dfal, fpe, dfpe, fse, dfse;
        curve_eval<BFK>(Cfal, l * mu.inv_lopt, fal, dfal);
        curve_eval<BFK>(Cfpe, l * mu.inv_lopt, fpe, dfpe);
        curve_eval<BFK>(Cfse, (L - sq) * mu.inv_lts, fse, dfse);
        Real H = (a * fal + fpe) * cphi - fse;
        Real dH = (a * dfal + dfpe) * mu.inv_lopt * cphi + (a * fal + fpe) * (w * w) / (l * l * sq) + dfse * mu.inv_lts / cphi;
        if (H > 0) hi = l; else lo = l;
        Real ln = l - H / dH;
        const bool newton = ln >= lo && ln <= hi;
        if (!newton) ln = Real(0.5) * (lo + hi);
        /* the residual stop as a zero step (the l_tol exit below), not an
         * exit of its own: the spatial RK kernels have no register to spare */
        ln = fabs(H) < Eps<Real>::h_stop ? l : ln;
        Real dl = fabs(ln - l);
        l = ln;
        if (dl <= Eps<Real>::l_tol || (it >= 1 && dl <= Real(1e3) * Eps<Real>::l_tol && dl >= Real(0.5) * dprev)) break;
        /* a Newton step of at most l_stop leaves an error ~ |H''/2H'| l_stop^2,
         * far below l_tol (as u_stop for the fiber velocity) */
        if (newton && dl <= Eps<Real>::l_stop) break;
        dprev = dl;
    }
    return l;
}

/* path length and dL/dq of one muscle.  Frames from LDS, Plucker columns
 * from registers (loaded once per dynamics call).  Fixed trip count over
 * the topology's maximum point count; only the point indices that can be
 * conditional / moving (compile-time masks) carry that code. */
/* Path length L and the moment arms dL/dq over the muscle's span (dLs[k]
 * for dof mu.span[k], k < mu.nspan): per active point the
 * change of the unit direction g acts at the point, dL/dq_d += S_d . (P x g, g)
 * for the dofs moving the point, plus g . dP/dq for a moving point's own
 * coordinate.  The floating-base dofs are skipped: their sum over a path is
 * zero (sum g = 0, sum P x g = 0).  The span's Plucker columns are read from
 * LDS once per muscle into registers. */
template <bool BFK, class T, typename Real>
DEV void muscle_path(const SModel<T, Real> &SM, const SMuscle<Real> &mu, const Real *lds, Real &L,
                     Real (&dLs)[T::MAXSPAN]) {
    using LY = Lay<T, Real>;
    using PL = Planar<T>;
    constexpr unsigned ZR = PL::ZR, ZW = PL::ZW, ZV = PL::ZV;
    constexpr int NSP = T::MAXSPAN;
    constexpr bool BF = BFK;
    const Real *ldsq = lds + LY::QF;
    L = 0;
    int sd[NSP];
    Real Ss[NSP][6];
#pragma unroll
    for (int k = 0; k < NSP; ++k) {
        dLs[k] = 0;
        /* planar: ?: over plain locals only (an arm with a load becomes a
         * branch); the spatial kernels keep the branches (fewer live values
         * in their two muscle passes) */
        int dk;
        if constexpr (BF) {
            const int spk = mu.span[k], none = -1, zero = 0;
            const bool ink = k < mu.nspan;
            sd[k] = ink ? spk : none;
            dk = ink ? spk : zero;
        } else {
            sd[k] = k < mu.nspan ? mu.span[k] : -1;
            dk = k < mu.nspan ? mu.span[k] : 0;
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) Ss[k][i] = lds[LY::S + 6 * dk + i];
        PL::col(Ss[k]);
    }
    Real Pp[3] = {0, 0, 0}, ep[3] = {0, 0, 0}, dPp[3] = {0, 0, 0};
    uint32_t maskp = 0;
    int mdofp = -1;
    bool have = false;
    auto flush = [&](const Real *g) {
        Real mo[3];
        cross3(Pp, g, mo);
        const Real gd = dot3(g, dPp);
#pragma unroll
        for (int k = 0; k < NSP; ++k) {
            const int d = sd[k];
            const Real on = d >= 0 && ((maskp >> d) & 1u) ? Real(1) : Real(0);
            const Real sm = dot3m<ZW, 0>(Ss[k], mo);
            const Real sg = dot3m<ZV, 0>(Ss[k] + 3, g);
            dLs[k] += on * (sm + sg) + (mdofp == d && d >= 0 ? gd : Real(0));
        }
    };
    const int npt = mu.npt;
    constexpr int MP = T::MAXPT > 0 ? T::MAXPT : 1;
    /* every slot's body and activity first (branch-free, slot 0 for slots
     * past the count), so a point's frame loads wait on one LDS round trip
     * inside its branch, not two */
    int cbj[MP];
    bool onj[MP];
    sfor<0, MP>([&](auto jI) {
        constexpr int j = decltype(jI)::value;
        const DPathPt<Real> &pt = SM.pt[mu.pt_off + (j < npt ? j : 0)];
        cbj[j] = pt.cbody;
        onj[j] = j < npt;
        if constexpr (((T::PT_COND >> j) & 1u) != 0) {
            const bool cnd = pt.type == BIOIM_PT_COND;
            if constexpr (BF) {
                const int ccd = pt.cond_coord, zero = 0;
                const Real qc = ldsq[cnd ? ccd : zero], plo = pt.lo, phi = pt.hi;
                onj[j] = onj[j] & !(cnd & ((qc < plo) | (qc > phi)));   /* no short-circuit branches */
            } else {
                const Real qc = ldsq[cnd ? pt.cond_coord : 0];
                onj[j] = onj[j] && !(cnd && (qc < pt.lo || qc > pt.hi));
            }
        }
    });
    sfor<0, MP>([&](auto jI) {
        constexpr int j = decltype(jI)::value;
        {
            const DPathPt<Real> &pt = SM.pt[mu.pt_off + j];
            if (onj[j]) {
                Real loc[3] = {pt.loc[0], pt.loc[1], pt.loc[2]}, dloc[3] = {0, 0, 0};
                if constexpr (((T::PT_MOVING >> j) & 1u) != 0) {
                    if (pt.type == BIOIM_PT_MOVING) {
                        Real ll[3], dl[3] = {0, 0, 0};
#pragma unroll
                        for (int a = 0; a < 3; ++a) {
                            const int f = pt.mf[a];
                            if constexpr (BF) {
                                const Real l0 = pt.loc[a], fv = lds[LY::MF + 3 * (f < 0 ? 0 : f)],
                                           fd = lds[LY::MF + 3 * (f < 0 ? 0 : f) + 1], zero = 0;
                                ll[a] = f < 0 ? l0 : fv;
                                dl[a] = f < 0 ? zero : fd;
                            } else {
                                ll[a] = f < 0 ? pt.loc[a] : lds[LY::MF + 3 * (f < 0 ? 0 : f)];
                                dl[a] = f < 0 ? Real(0) : lds[LY::MF + 3 * (f < 0 ? 0 : f) + 1];
                            }
                        }
                        mv3(pt.R, ll, loc);
#pragma unroll
                        for (int i = 0; i < 3; ++i) loc[i] += pt.p[i];
                        mv3(pt.R, dl, dloc);
                    }
                }
                const Real *kbp = lds + LY::KB + 18 * cbj[j];
                Real Rb[12];
#pragma unroll
                for (int i = 0; i < 12; ++i) Rb[i] = kbp[i];
                PL::rot(Rb);
                Real P[3], dP[3];
                mv3m<ZR, 0>(Rb, loc, P);
#pragma unroll
                for (int i = 0; i < 3; ++i) P[i] += Rb[9 + i];
                mv3m<ZR, 0>(Rb, dloc, dP);
                Real e[3] = {0, 0, 0};
                if (have) {
                    Real sgm[3] = {P[0] - Pp[0], P[1] - Pp[1], P[2] - Pp[2]};
                    const Real l2 = dot3(sgm, sgm);
                    const Real inv = fast_rsqrt(l2), len = l2 * inv;
                    L += len;
#pragma unroll
                    for (int a = 0; a < 3; ++a) e[a] = sgm[a] * inv;
                    Real g[3] = {ep[0] - e[0], ep[1] - e[1], ep[2] - e[2]};
                    flush(g);
                }
#pragma unroll
                for (int a = 0; a < 3; ++a) { ep[a] = e[a]; Pp[a] = P[a]; dPp[a] = dP[a]; }
                maskp = pt.dofmask;
                mdofp = pt.mdof;
                have = true;
            }
        }
    });
    if (have) flush(ep);
}

/* ------------------------------------------------------------ dynamics */
template <class T, typename Real> struct Dyn {
    static constexpr int MPL = Lay<T, Real>::MPL;
    Real qdd;        /* this lane's dof (lane < ND): generalized acceleration / substep increment */
    MState<Real> ms[MPL]; /* this lane's muscles m = lane + j*G */
    Real act[MPL], lce[MPL]; /* their state used (after a reset equilibrium) */
    Real x0;         /* floating origin used for the published frames */
    bool ok;
};

/* apply_perturbations table (see LaunchArgs) as seen by one env */
template <typename Real> struct PertArgs {
    const double *x;
    const Real *y;   /* [n][N] */
    int n, ob, env, N;
};

/* Force of the env's zero-order-hold table at the call time t0 + k*dt (the
 * slot's base and step, written by lane 0 before the call); the segment
 * cursor [lo, hi) and its value live in the slot, so a binary search over
 * the table runs only when the time leaves the segment. */
template <typename Real>
DEV Real pert_force(const PertArgs<Real> &P, double *sl, int k) {
    const double tc = sl[0] + (double)k * sl[1];
    if (!(tc >= sl[2] && tc < sl[3])) {
        int lo = -1, hi = P.n;               /* x[lo] <= tc < x[hi] */
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (P.x[mid] <= tc) lo = mid; else hi = mid;
        }
        sl[2] = lo >= 0 ? P.x[lo] : -INFINITY;
        sl[3] = hi < P.n ? P.x[hi] : INFINITY;
        sl[4] = (double)GAT(P.y, (size_t)(lo >= 0 ? lo : 0) * P.N + P.env, (size_t)P.n * P.N);
    }
    return (Real)sl[4];
}

/* Forward dynamics at (q, u, this lane's muscle states) with held controls.
 * Lane d < ND owns dof d (qd, ud in, D.qdd out); lane's j-th muscle is
 * m = lane + j*G.  h > 0: increment of the linearly-implicit substep;
 * h == 0: the true accelerations (realize).  Leaves coordinates, frames,
 * contact wrenches, limit forces and q'' (RHS slots) published in LDS.
 * CACHE kernels (CacheLay): CI.make — a realize also forms the implicit
 * system at h = CI.hc and stores it with the fiber-velocity roots into the
 * env's cache row (CI.row()); CI.use — a first substep takes its system and
 * roots from the cache (CI.sys / CI.mus loaded at kernel start in the
 * planar kernels, the row itself in the spatial ones) and only solves: the
 * state is the one the last realize ran at. */
template <class T, typename Real> struct CacheIO {
    static constexpr int PF = CacheLay<T>::PF > 0 ? CacheLay<T>::PF : 1;
    static constexpr int PFA = CacheLay<T>::PREFETCH ? PF : 1, MPA = CacheLay<T>::PREFETCH ? Lay<T, Real>::MPL : 1;
    bool use = false, make = false;
    Real hc = 0;
    /* this env's row, formed at each use from the uniform base and an opaque
     * copy of the env index: a row address kept live through the kernel was
     * split by the register allocator into lane-divergent AGPR copies in the
     * fused C5 kernel (tools/hazard_gate.py) */
    Real *base = nullptr;
    int env = 0, N = 0;
    DEV Real *row() const {
        int e = env;
        asm volatile("" : "+v"(e));
        return base + GIDX((size_t)e * CacheLay<T>::DIM, (size_t)N * CacheLay<T>::DIM);
    }
    Real sys[PFA];     /* PREFETCH: the row's system values k = lane + i G */
    Real mus[MPA][3];  /* PREFETCH: this lane's muscles' root, dv/dl, clamp flag */
};

template <class T, typename Real, bool PERT, bool BF_ROWS, bool IMP, bool CACHE = false>
DEV void dynamics(const DModel<Real> &M, const SModel<T, Real> &SM, Real qd, Real ud,
                  const Real (&act)[Lay<T, Real>::MPL], const Real (&lce)[Lay<T, Real>::MPL],
                  const Real (&control)[Lay<T, Real>::MPL], int lane, Real *lds, Real h, bool equilibrate,
                  const PertArgs<Real> &P, double *pslot, int pk, Dyn<T, Real> &D, const CacheIO<T, Real> &CI) {
    using LY = Lay<T, Real>;
    constexpr int ND = LY::ND, NP = LY::NP, NB = T::NB, G = T::G, MPL = LY::MPL;
    static_assert(!CACHE || (CacheLay<T>::ON && IMP && !PERT), "the realize cache: the default (semi-implicit, no push) step kernels");
    static_assert(NB < G && ND <= G, "lane NB writes the ground slot; one lane per dof");
    /* the semi-implicit planar kernels: the implicit contact / limit terms
     * without a branch on h (the spatial kernels keep it: register budget) */
    constexpr bool IMP_BF = IMP && (T::PLANAR || BIOIM_BF_SPATIAL || ((BIOIM_BF3 & 64) && !PERT));
    /* the branch-free forms (selects over plain locals, blended
     * extrapolations, one basic block per muscle eval) in the planar
     * kernels, except the torque-model RK ones: an RK build of these forms
     * put a lane-divergent copy of a live-in-all-lanes address into an AGPR
     * in the Torque2D RK kernel and faulted; that kernel
     * keeps the GPU-verified code (round 4: the same forms there again give 4
     * flagged copies in tools/hazard_gate.py), and the gate checks the others */
    constexpr bool BFK = (T::PLANAR || BIOIM_BF_SPATIAL) && (IMP || T::NM > 0);
    /* per-piece switches of the branch-free forms in the spatial semi-implicit
     * kernels (BIOIM_BF3 bits: 1 function slots, 2 muscle paths, 4 contact,
     * 8 limits, 16 fiber equilibrium, 32 phase-3 rows, 64 implicit
     * terms without a branch on h, 128 muscle eval) */
    constexpr bool BF3 = !T::PLANAR && (IMP || BIOIM_BF3_RK);
    constexpr bool BFK_FN = BFK || (BF3 && (BIOIM_BF3 & 1)), BFK_PATH = BFK || (BF3 && (BIOIM_BF3 & 2));
    constexpr bool BFK_CON = BFK || (BF3 && (BIOIM_BF3 & 4)), BFK_LIM = BFK || (BF3 && (BIOIM_BF3 & 8));
    constexpr bool BFK_EQ = BFK || (BF3 && (BIOIM_BF3 & 16)), BFK_ROW = BFK || (BF3 && (BIOIM_BF3 & 32));
    constexpr bool BFK_ME = BFK || (BF3 && (BIOIM_BF3 & 128));
    /* the muscle eval's curves and fiber-velocity solve in one block, in
     * every kernel (spatial too: no scratch; same-box 3D -1.6 %,
     * profiles/r03/r03k, r03l) */
    constexpr bool BFC = true;
    STAMP_DECL
    if (CACHE && CI.use) {
        /* the first substep of a launch from the last realize's cache: the
         * implicit system at this h into MP..RHS, the muscles' roots, and the
         * activation rates at this step's excitations */
        using CL = CacheLay<T>;
        Real *const crow = CL::PREFETCH ? nullptr : CI.row();
#pragma unroll
        for (int i = 0; i < CacheIO<T, Real>::PF; ++i)
            if (lane + i * G < CL::SYS) {
                if constexpr (CL::PREFETCH) lds[LY::MP + lane + i * G] = CI.sys[i];
                else lds[LY::MP + lane + i * G] = GAT(crow, lane + i * G, CL::DIM);
            }
        if constexpr (T::NM > 0) {
#pragma unroll
            for (int j = 0; j < MPL; ++j) {
                const int m = mslot<T>(lane + j * G);
                if (m < T::NM) {
                    const SMuscle<Real> &mu = SM.mus[m];
                    const Real amin = mu.amin, one = 1, a_state = act[j];
                    const Real a = a_state < amin ? amin : (a_state > one ? one : a_state);
                    MState<Real> &s = D.ms[j];
                    Real cv[3];
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        if constexpr (CL::PREFETCH) cv[c] = CI.mus[j][c];
                        else cv[c] = GAT(crow, CL::MUS + 3 * m + c, CL::DIM);
                    }
                    s.vN = cv[0];
                    s.vce = s.vN * mu.lv;
                    s.dvdl = cv[1];
                    s.clamped = cv[2] != Real(0);
                    s.dadt = act_rate<BFK_ME>(mu, a, control[j]);
                }
            }
        } else {
            /* this step's actuator torques (as phase 2 stores them), added
             * to the cached right-hand side in phase 3's order */
            if (lane == 0) lds[LY::TAU + LY::TZ] = Real(0);
            sfor<0, MPL>([&](auto jI) {
                constexpr int j = decltype(jI)::value;
                const int m = mslot<T>(lane + j * G);
                if (m < T::NA) lds[LY::TAU + (lane + j * G) * T::MAXSPAN] = control[j] * SM.ca_opt[m];
            });
            wave_sync();
            if (lane < ND) {
                Real r = lds[LY::RHS + lane];
#pragma unroll
                for (int i = 0; i < T::MAXARM; ++i) r += lds[LY::TAU + SM.tau_src[lane][i]];
                lds[LY::RHS + lane] = r;
            }
        }
        wave_sync();
    } else {
    publish_coords<T, Real>(M, SM, lds, lane, qd, ud);
    if (lane < ND) {
#pragma unroll
        for (int i = 0; i < 6; ++i) lds[LY::SL + 6 * lane + i] = 0;
    }
    wave_sync();
    Real x0 = 0;
    if constexpr (T::TX >= 0) {
        if constexpr (T::coord_dof[T::TX] >= 0) x0 = M.float_origin ? lds[LY::QF + T::TX] : Real(0);
    }
    D.x0 = x0;

    /* ---- phase 0b: function slots, one lane each — the moving path points'
     * location functions (read by every muscle that has the point) and the
     * joints' spline axes (read by their body's lane) */
    fn_slots<BFK_FN, T, Real>(SM, lds, lane);
    STAMP(15);

    /* ---- phase 1: lane-parallel kinematics */
    if (lane < NB) kin_local<T, Real>(SM, lds, lane);
    if (lane == NB) kin_ground<T, Real>(lds, x0);
    wave_sync();
    STAMP(0);
    if (lane < NB) kin_chain<T, Real>(SM, lds, lane, x0);
    wave_sync();
    STAMP(1);
    if (lane < ND) kin_column<T, Real>(SM, lds, lane);
    if (lane < NB) {
        body_inertia<T, Real>(SM, M, lds, lane);
        /* apply_perturbations: ground-frame force (fx, 0, 0) at the origin of
         * OpenSim body P.ob (the torso), muscle_walking_imitation_env2D.py:83-100 */
        if (PERT && lane == SM.os_cb[P.ob]) {
            const Real fpx = pert_force<Real>(P, pslot, pk);
            const Real *kb = lds + LY::KB + 18 * lane;
            Real p[3];
            mv3(kb, SM.os_p[P.ob], p);
            Real *wb = lds + LY::WB + 6 * lane;
            wb[1] -= (p[2] + kb[11]) * fpx;
            wb[2] += (p[1] + kb[10]) * fpx;
            wb[3] -= fpx;
        }
    }
    wave_sync();
    STAMP(2);

    /* ---- phase 2: lane-parallel force elements */
    {   /* subtree sums of inertia and wrench, in place (all reads, then all
         * writes).  Planar models: only the components phase 3 reads against
         * planar columns (m, h_x, h_y, J_zz; n_z, f_x, f_y) */
        constexpr unsigned ICU = T::PLANAR ? 0x47u : 0x3FFu, WBU = T::PLANAR ? 0x1Cu : 0x3Fu;
        Real ic[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, wb[6] = {0, 0, 0, 0, 0, 0};
        if (lane < NB) {
            /* planar: every body's record is read and weighted by 0 / 1 (lane
             * an ancestor of d, or d): one basic block, the loads batch */
            sfor<0, NB>([&](auto dI) {
                constexpr int d = decltype(dI)::value;
                const bool mine = (T::anc[d] >> lane) & 1u;
                if (T::PLANAR || mine) {
                    const Real on = !T::PLANAR || mine ? Real(1) : Real(0);
#pragma unroll
                    for (int i = 0; i < 10; ++i)
                        if ((ICU >> i) & 1u) ic[i] = fma(on, lds[LY::IC + 10 * d + i], ic[i]);
#pragma unroll
                    for (int i = 0; i < 6; ++i)
                        if ((WBU >> i) & 1u) wb[i] = fma(on, lds[LY::WB + 6 * d + i], wb[i]);
                }
            });
        }
        wave_sync();
        if (lane < NB) {
#pragma unroll
            for (int i = 0; i < 10; ++i)
                if ((ICU >> i) & 1u) lds[LY::IC + 10 * lane + i] = ic[i];
#pragma unroll
            for (int i = 0; i < 6; ++i)
                if ((WBU >> i) & 1u) lds[LY::WB + 6 * lane + i] = wb[i];
        }
    }
    STAMP(3);
    /* the implicit terms' h: a CACHE realize forms them at the next step's
     * substep length (its explicit q'' below does not use them) */
    const Real hi = (CACHE && CI.make) ? CI.hc : h;
    /* contacts computed by the first muscle pass when every sphere lane
     * holds a muscle there */
    constexpr bool MUSCLE_CONTACT = T::NM >= T::NS && T::NS > 0;
    ContactOut<Real> CO;
    if constexpr (T::NM > 0) {
        /* this lane's muscles' -F_t dL/dq over their spans, stored per muscle
         * slot and span entry (plain stores); the dof lanes gather them in
         * phase 3 through SM.tau_src.  (An LDS read-modify-write of per-lane
         * torque slots at the span's runtime dof indices, combined with the
         * early deque store, produced wrong fp32 3D results on the GPU —
         * DESIGN.md 5.1.) */
        if (lane == 0) lds[LY::TAU + LY::TZ] = Real(0);
        sfor<0, MPL>([&](auto jI) {
            constexpr int j = decltype(jI)::value;
            const int m = mslot<T>(lane + j * G);
            if (m < T::NM) {
                const SMuscle<Real> &mu = SM.mus[m];
                Real L, dLs[T::MAXSPAN];
                muscle_path<BFK_PATH, T, Real>(SM, mu, lds, L, dLs);
                STAMP(4);
                Real a_ = act[j], l_ = lce[j];
                if (equilibrate) /* equilibrateMuscles: static fiber equilibrium at the held activation
                                  * (a reset has set the default activation) */
                    l_ = muscle_equilibrium<BFK_EQ, T, Real>(SM, mu, a_, L);
                D.act[j] = a_;
                D.lce[j] = l_;
                /* the sphere contacts ride in the first muscle pass (every
                 * sphere lane holds a muscle): same block as the curve
                 * evaluations, so their chains interleave */
                if constexpr (j == 0 && MUSCLE_CONTACT) contact_compute<BFK_CON, T, Real>(SM, lds, lane < T::NS ? lane : 0, hi, CO);
                muscle_eval<BFK_ME, BFC, T, Real>(SM, mu, a_, l_, control[j], L, D.ms[j].vN, D.ms[j]);
                const Real nFt = -D.ms[j].Ft;
                Real *ts = lds + LY::TAU + (lane + j * G) * T::MAXSPAN;
#pragma unroll
                for (int k = 0; k < T::MAXSPAN; ++k) ts[k] = nFt * dLs[k];
            }
        });
    } else {
        /* coordinate actuators: one torque per slot, gathered the same way */
        if (lane == 0) lds[LY::TAU + LY::TZ] = Real(0);
        sfor<0, MPL>([&](auto jI) {
            constexpr int j = decltype(jI)::value;
            const int m = mslot<T>(lane + j * G);
            if (m < T::NA) lds[LY::TAU + (lane + j * G) * T::MAXSPAN] = control[j] * SM.ca_opt[m];
        });
    }
    STAMP(5);
    if constexpr (MUSCLE_CONTACT) {
        if (lane < T::NS) contact_store<T, Real>(lds, lane, CO);
    } else {
        if (lane < T::NS) contact_lane<BFK_CON, T, Real>(SM, lds, lane, hi);
    }
    STAMP(6);
    if (lane < T::NL) {
        int cc = SM.lim_coord[lane];
        Real qv = lds[LY::QF + cc], qd = lds[LY::UF + cc];
        Real qup = SM.lim_qup[lane], qlo = SM.lim_qlow[lane], tr = SM.lim_trans[lane], itr = SM.lim_itrans[lane];
        Real up = smooth_step<BFK_LIM>(Real(0), Real(1), qup, qup + tr, itr, qv);
        Real lo = smooth_step<BFK_LIM>(Real(1), Real(0), qlo - tr, qlo, itr, qv);
        Real f = -SM.lim_kup[lane] * up * (qv - qup) + SM.lim_klow[lane] * lo * (qlo - qv) - SM.lim_damp[lane] * (up + lo) * qd;
        Real diag = 0, tadd = f;
        if (IMP_BF || (!IMP_BF && hi > 0)) {   /* IMP_BF: no branch on h (at h = 0 this gives diag = 0, tadd = f) */
            Real dup = smooth_step_d<BFK_LIM>(Real(0), Real(1), qup, qup + tr, itr, qv);
            Real dlo = smooth_step_d<BFK_LIM>(Real(1), Real(0), qlo - tr, qlo, itr, qv);
            Real kq = SM.lim_kup[lane] * (up + dup * (qv - qup)) + SM.lim_klow[lane] * (lo - dlo * (qlo - qv));
            Real cq = SM.lim_damp[lane] * (up + lo);
            diag = hi * cq + hi * hi * kq;
            tadd = f - hi * kq * qd;
        }
        Real *lm = lds + LY::LIM + 4 * lane;
        lm[0] = f; lm[1] = diag; lm[2] = tadd;
    }
    wave_sync();
    STAMP(7);

    /* ---- phase 3 (lane = dof k): right-hand side and row k of the packed
     * lower M, fixed-order sums.
     * rhs_k = -S_k.WB + muscle/actuator torques + contact J_k(s).F_s + limits.
     * Row k holds the entries (k, l) for the dofs l on k's root path (l = k
     * included; the others are structural zeros, never read by ltl_solve):
     * M_kl = S_l . I^c S_k, the composite inertia of k's body times k's
     * column (CRBA).  The implicit contact block of an entry is
     * J_l(s)^T C_s J_k(s) over the spheres s below k; with
     * J_l(s)^T w = S_l . (P_s x w, w) it folds into the same vector:
     * G_k = I^c S_k + sum_s (P_s x w_s, w_s), w_s = C_s J_k(s), and
     * M_kl = S_l . G_k (every l on k's path moves the spheres k moves).  All
     * inputs (S, IC, CJ, LIM) were published before the last sync, so the
     * row needs no exchange between lanes. */
    const bool implicit = hi > 0;
    using PL = Planar<T>;
    constexpr unsigned ZW = PL::ZW, ZV = PL::ZV;
    /* EX: the explicit system of a CACHE realize (h = 0: the contact force
     * without its implicit correction — the CW slot — the limit forces, no
     * implicit blocks), after its implicit one went to the cache; otherwise
     * the system at hi */
    auto phase3 = [&](auto EXc) {
    constexpr bool EX = decltype(EXc)::value;
    if (lane < ND) {
        Real Sd[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) Sd[i] = lds[LY::S + 6 * lane + i];
        PL::col(Sd);
        const Real *wb = lds + LY::WB + 6 * SM.dof_cb[lane];
        Real r = -(dot3m<ZW, 0>(Sd, wb) + dot3m<ZV, 0>(Sd + 3, wb + 3));
        /* torque models with the realize cache: the actuator torques last
         * (the cache keeps the sum before them) */
        constexpr bool TAU_LAST = CACHE && T::NM == 0;
        if constexpr (!TAU_LAST) {
#pragma unroll
            for (int i = 0; i < T::MAXARM; ++i) r += lds[LY::TAU + SM.tau_src[lane][i]];
        }
        Real Gk[6];
        {
            const Real *ic = lds + LY::IC + 10 * SM.dof_cb[lane];
            Real t[3];
            symvm<ZW>(ic + 4, Sd, Gk);
            cross3m<0, ZV>(ic + 1, Sd + 3, t);
#pragma unroll
            for (int i = 0; i < 3; ++i) Gk[i] += t[i];
            cross3m<ZW, 0>(Sd, ic + 1, t);
#pragma unroll
            for (int i = 0; i < 3; ++i) Gk[3 + i] = ic[0] * Sd[3 + i] + t[i];
        }
        sfor<0, T::NS>([&](auto sI) {
            constexpr int sp = decltype(sI)::value;
            constexpr unsigned msk = T::dofmask[T::sphere_cb[sp]];
            const Real *cj = lds + LY::CJ + LY::CJN * sp, *C = cj + 6;
            /* the force: CW (= F where the sphere is active, 0 elsewhere, so
             * on * F alike) for the explicit system */
            const Real *Fs = EX ? lds + LY::CW + 8 * sp : cj + 3;
            Real jd[3];
            cross3m<ZW, 0>(Sd, cj, jd);
#pragma unroll
            for (int i = 0; i < 3; ++i) jd[i] += Sd[3 + i];
            PL::lin(jd);
            /* weighted by on = 0 / 1 (every CJ value is finite: contact_compute
             * is branch-free): a select made the compiler load cj under a
             * branch, two basic blocks per sphere */
            const bool onb = lds[LY::CW + 8 * sp + 6] > 0 && ((msk >> lane) & 1u);
            const Real on = onb ? Real(1) : Real(0);
            if constexpr (BFK_ROW) r = fma(on, dot3m<ZV, 0>(jd, Fs), r);
            else r += onb ? dot3m<ZV, 0>(jd, Fs) : Real(0);
            /* IMP (the semi-implicit kernels): no branch on h — a realize
             * call (h = 0) has C = 0 (contact_compute), adding zeros */
            if (!EX && (IMP_BF || (!IMP_BF && implicit))) {
                Real w[3] = {(ZV & 4u) ? C[0] * jd[0] : C[0] * jd[0] + C[1] * jd[2], C[2] * jd[1],
                             C[1] * jd[0] + C[3] * jd[2]};
                Real pw[3];
                cross3(cj, w, pw);
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    if constexpr (BFK_ROW) {
                        Gk[i] = fma(on, pw[i], Gk[i]);
                        Gk[3 + i] = fma(on, w[i], Gk[3 + i]);
                    } else {
                        Gk[i] += onb ? pw[i] : Real(0);
                        Gk[3 + i] += onb ? w[i] : Real(0);
                    }
                }
            }
        });
        Real dg = 0;
#pragma unroll
        for (int li = 0; li < T::NL; ++li) {   /* selects: no per-limit branch */
            const bool mine = SM.lim_dof[li] == lane;
            r += mine ? lds[LY::LIM + 4 * li + (EX ? 0 : 2)] : Real(0);
            if constexpr (!EX) dg += mine ? lds[LY::LIM + 4 * li + 1] : Real(0);
        }
        if constexpr (TAU_LAST) {
            Real rt = r;
#pragma unroll
            for (int i = 0; i < T::MAXARM; ++i) rt += lds[LY::TAU + SM.tau_src[lane][i]];
            lds[LY::RHS + lane] = (!EX && CI.make) ? r : rt;   /* the cache's rhs: without the controls */
        } else {
            lds[LY::RHS + lane] = r;
        }
        /* Row k's entries (k, l), l <= k.  BF_ROWS: branch-free, every l is
         * computed and stored in row k's own slots (those off k's root path
         * are structural zeros ltl_solve never reads); columns l > k (not in
         * row k) go to slot (k, 0) first, descending l, so the true (k, 0) —
         * dof 0 is every dof's ancestor — is written last.  Same-box 2D
         * 0.329 -> 0.316 ms, 3D 0.581 -> 0.561 (profiles/r03/ab_rows.txt).
         * Otherwise only k's path entries, each under its own branch. */
        static_assert(DofTree<T>::root_common(), "row stores park columns l > k in slot (k, 0)");
        Real *row = lds + LY::MP + (lane * (lane + 1)) / 2;
        unsigned path = 0;   /* dofs on k's root path, k included (compile-time per dof, selected by lane) */
        if constexpr (!BF_ROWS) {
            sfor<0, ND>([&](auto kI) {
                constexpr int k = decltype(kI)::value;
                constexpr unsigned pm = DofTree<T>::path_mask(k);
                path = lane == k ? pm : path;
            });
        }
        sfor<0, ND>([&](auto lI) {
            constexpr int l = ND - 1 - decltype(lI)::value;
            auto entry = [&]() {
                Real Sl[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) Sl[i] = lds[LY::S + 6 * l + i];
                PL::col(Sl);
                Real v = dot3m<ZW, 0>(Sl, Gk) + dot3m<ZV, 0>(Sl + 3, Gk + 3);
                return EX ? v : v + (implicit && l == lane ? dg : Real(0));
            };
            if constexpr (BF_ROWS) row[l <= lane ? l : 0] = entry();
            else if ((path >> l) & 1u) row[l] = entry();
        });
    }
    };
    phase3(std::integral_constant<bool, false>{});
    wave_sync();
    if constexpr (CACHE) {
        if (CI.make) {
            /* the implicit system at hi for the next launch's first substep, then
             * this realize's explicit one over it */
            using CL = CacheLay<T>;
            Real *const crow = CI.row();
            for (int k = lane; k < CL::SYS; k += G) GAT(crow, k, CL::DIM) = lds[LY::MP + k];
            if (lane == 0) GAT(crow, CL::H, CL::DIM) = hi;
#pragma unroll
            for (int j = 0; j < MPL; ++j) {
                const int m = mslot<T>(lane + j * G);
                if (m < T::NM) {
                    GAT(crow, CL::MUS + 3 * m, CL::DIM) = D.ms[j].vN;
                    GAT(crow, CL::MUS + 3 * m + 1, CL::DIM) = D.ms[j].dvdl;
                    GAT(crow, CL::MUS + 3 * m + 2, CL::DIM) = D.ms[j].clamped ? Real(1) : Real(0);
                }
            }
            wave_sync();
            phase3(std::integral_constant<bool, true>{});
            wave_sync();
        }
    }
    }   /* phases 0-3 (not a cached first substep) */
    STAMP(8);

    /* ---- phase 4: tree-sparse LTL solve (ltl_solve), redundant in every
     * lane's registers (the shortest dependency chain for these 9x9 / 14x14
     * systems; a lane-distributed dense factorization with one LDS round trip
     * per column measured 7 % slower per step); lane d keeps q''_d and
     * publishes it for the report */
    Real A[NP], xs[ND];
#pragma unroll
    for (int e = 0; e < NP; ++e) A[e] = lds[LY::MP + e];
#pragma unroll
    for (int d = 0; d < ND; ++d) xs[d] = lds[LY::RHS + d];
    D.ok = ltl_solve<T, ND, Real>(A, xs);
    Real x = 0;
#pragma unroll
    for (int d = 0; d < ND; ++d) x = lane == d ? xs[d] : x;
    D.qdd = x;
    wave_sync();
    if (lane < ND) lds[LY::RHS + lane] = x;   /* q'' of every dof for the report */
    wave_sync();
    STAMP(9);
}

/* Lane-parallel report (lane = OpenSim body b < NOS; lane NOS = system
 * COM): origin position and velocity in absolute ground coordinates, from
 * the published frames, into REP[b] */
template <class T, typename Real>
DEV void report_points(const SModel<T, Real> &SM, Real *lds, int lane, Real x0) {
    using LY = Lay<T, Real>;
    static_assert(T::NOS < T::G, "one lane per reported body plus one for the COM");
    Real pos[3], vel[3], t[3];
    if (lane < T::NOS) {
        const Real *kb = lds + LY::KB + 18 * SM.os_cb[lane];
        mv3(kb, SM.os_p[lane], pos);
#pragma unroll
        for (int i = 0; i < 3; ++i) pos[i] += kb[9 + i];
        cross3(kb + 12, pos, t);
#pragma unroll
        for (int i = 0; i < 3; ++i) vel[i] = kb[15 + i] + t[i];
    } else {
        Real mt = 0, cs[3] = {0, 0, 0}, vs[3] = {0, 0, 0};
#pragma unroll
        for (int c = 0; c < T::NB; ++c) {
            const Real *kb = lds + LY::KB + 18 * c;
            Real cG[3], vc[3];
            mv3(kb, SM.body[c].com, cG);
#pragma unroll
            for (int i = 0; i < 3; ++i) cG[i] += kb[9 + i];
            cross3(kb + 12, cG, t);
#pragma unroll
            for (int i = 0; i < 3; ++i) vc[i] = kb[15 + i] + t[i];
            Real m = SM.body[c].mass;
#pragma unroll
            for (int i = 0; i < 3; ++i) { cs[i] += m * cG[i]; vs[i] += m * vc[i]; }
            mt += m;
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) { pos[i] = cs[i] / mt; vel[i] = vs[i] / mt; }
    }
    pos[0] += x0;
    Real *r = lds + LY::REP + 6 * (lane < T::NOS ? lane : T::NOS);
#pragma unroll
    for (int i = 0; i < 3; ++i) { r[i] = pos[i]; r[3 + i] = vel[i]; }
}

/* REP slot of an OpenSim body index (-1 = COM) */
template <class T> DEV constexpr int rep_slot(int ob) { return ob >= 0 ? ob : T::NOS; }

/* observation offsets (get_state_dict order, muscle_walking_imitation_env2D.py:158-225) */
template <class T> struct ObsLayout {
    static constexpr int NTR = (T::TX >= 0) + (T::TY >= 0) + (T::TZ >= 0);
    static constexpr int NQ = T::NC - NTR;
    static constexpr int QPOS = 1, QVEL = QPOS + NQ, QACC = QVEL + T::NC, TGT = QACC + T::NC;
    static constexpr int body(bool tgt) { return TGT + (tgt ? 2 * (T::NC - 1) : 0); }
};

DEV int clamp_row(int r, int nrows) { return r < 0 ? 0 : (r >= nrows ? nrows - 1 : r); }

/* counter-based RNG (splitmix64) for device-drawn reset indices */
DEV uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
DEV int draw_index(uint64_t seed, int env, int count, int hi) {
    uint64_t r = splitmix64(seed ^ splitmix64(((uint64_t)env << 32) | (uint32_t)count));
    return (int)(r % (uint64_t)(hi + 1));
}


/* ------------------------------------------------- inverse dynamics
 * Batched primitives of the reference's Boost.Python InverseDynamics helper
 * (bioimitation/imitation_envs/inverse_dynamics/inverse_dynamics.cpp:45-205),
 * muscles disabled (:47-52), no controller (actuator controls 0).  One
 * state per G lanes, the env kernel's LDS image and kinematics:
 *   GRAVITY   g(q)            M q'' + c = g + tau           (:127-141)
 *   CORIOLIS  c(q, u)                                       (:143-158)
 *   MULT_M    M(q) v                                        (:160-175)
 *   MULT_MINV M(q)^-1 v                                     (:177-192)
 *   RESIDUAL  M v + c - f_applied(q, u), v = q''            (:63-94)
 *   TOTAL     c - f_applied(q, u)  (M q'' + f = tau)        (:96-125)
 * f_applied = gravity + Hunt-Crossley contact + coordinate limit forces
 * (generalized).  Vectors are [n][ndof] in dof order. */
template <class T, typename Real> struct IdArgs {
    const DModel<Real> *Mg;
    const SModel<T, Real> *Sg;
    int n, op;
    const Real *q, *u, *v;
    Real *out;
};

template <class T, typename Real>
#ifndef BIOIM_ID_NO_WAVES_ATTR
__global__ __launch_bounds__(BIOIM_EPB * T::G) __attribute__((amdgpu_waves_per_eu(1, 1))) void id_kernel(IdArgs<T, Real> a) {
#else   /* the compiler-crash reproducer (profiles/r03/regalloc_crash/): without the occupancy attribute */
__global__ __launch_bounds__(BIOIM_EPB * T::G) void id_kernel(IdArgs<T, Real> a) {
#endif
    using LY = Lay<T, Real>;
    constexpr int G = T::G, ND = LY::ND, NB = T::NB, NP = LY::NP, EPB = BIOIM_EPB;
    constexpr size_t SMB = smodel_bytes<T, Real>();
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(a.Sg);
        uint4 *dst = reinterpret_cast<uint4 *>(smem_raw);
        for (int i = threadIdx.x; i < (int)(SMB / 16); i += BIOIM_EPB * G) dst[i] = src[i];
    }
    __syncthreads();
    const SModel<T, Real> &SM = *reinterpret_cast<const SModel<T, Real> *>(smem_raw);
    const DModel<Real> &M = *a.Mg;
    const int lane = threadIdx.x % G, slot = threadIdx.x / G;
    const int idx = blockIdx.x * EPB + slot;
    if (idx >= a.n) return;
    Real *lds = reinterpret_cast<Real *>(smem_raw + SMB) + slot * LY::SIZE;
    const int op = a.op;
    const bool use_u = op == BIOIM_ID_CORIOLIS || op == BIOIM_ID_RESIDUAL || op == BIOIM_ID_TOTAL;
    const bool applied = op == BIOIM_ID_RESIDUAL || op == BIOIM_ID_TOTAL;
    const bool need_m = op == BIOIM_ID_MULT_M || op == BIOIM_ID_MULT_MINV || op == BIOIM_ID_RESIDUAL;
    Real qd = 0, ud = 0, vd = 0;
    if (lane < ND) {
        qd = GAT(a.q, (size_t)idx * ND + lane, (size_t)a.n * ND);
        ud = use_u ? GAT(a.u, (size_t)idx * ND + lane, (size_t)a.n * ND) : Real(0);
        vd = (need_m || op == BIOIM_ID_MULT_MINV) ? GAT(a.v, (size_t)idx * ND + lane, (size_t)a.n * ND) : Real(0);
    }
    publish_coords<T, Real>(M, SM, lds, lane, qd, ud);
    if (lane < ND) {
#pragma unroll
        for (int i = 0; i < 6; ++i) lds[LY::SL + 6 * lane + i] = 0;
    }
    wave_sync();
    Real x0 = 0;
    if constexpr (T::TX >= 0) {
        if constexpr (T::coord_dof[T::TX] >= 0) x0 = M.float_origin ? lds[LY::QF + T::TX] : Real(0);
    }
    fn_slots<false, T, Real>(SM, lds, lane);
    if (lane < NB) kin_local<T, Real>(SM, lds, lane);
    if (lane == NB) kin_ground<T, Real>(lds, x0);
    wave_sync();
    if (lane < NB) kin_chain<T, Real>(SM, lds, lane, x0);
    wave_sync();
    if (lane < ND) kin_column<T, Real>(SM, lds, lane);
    if (lane < NB) {
        body_inertia<T, Real>(SM, M, lds, lane);
        if (op == BIOIM_ID_CORIOLIS) {   /* velocity terms only: take the gravity wrench back out */
            const Real *kb = lds + LY::KB + 18 * lane;
            Real cG[3], mg[3], t[3];
            mv3(kb, SM.body[lane].com, cG);
#pragma unroll
            for (int i = 0; i < 3; ++i) { cG[i] += kb[9 + i]; mg[i] = SM.body[lane].mass * M.gravity[i]; }
            cross3(cG, mg, t);
            Real *wb = lds + LY::WB + 6 * lane;
#pragma unroll
            for (int i = 0; i < 3; ++i) { wb[i] += t[i]; wb[3 + i] += mg[i]; }
        }
    }
    wave_sync();
    {   /* subtree sums of inertia and wrench (all reads, then all writes) */
        Real ic[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, wb[6] = {0, 0, 0, 0, 0, 0};
        if (lane < NB) {
            sfor<0, NB>([&](auto dI) {
                constexpr int d = decltype(dI)::value;
                if ((T::anc[d] >> lane) & 1u) {
#pragma unroll
                    for (int i = 0; i < 10; ++i) ic[i] += lds[LY::IC + 10 * d + i];
#pragma unroll
                    for (int i = 0; i < 6; ++i) wb[i] += lds[LY::WB + 6 * d + i];
                }
            });
        }
        wave_sync();
        if (lane < NB) {
#pragma unroll
            for (int i = 0; i < 10; ++i) lds[LY::IC + 10 * lane + i] = ic[i];
#pragma unroll
            for (int i = 0; i < 6; ++i) lds[LY::WB + 6 * lane + i] = wb[i];
        }
    }
    if (applied) {
        if (lane < T::NS) contact_lane<false, T, Real>(SM, lds, lane, Real(0));
        if (lane < T::NL) {
            const int cc = SM.lim_coord[lane];
            const Real qv = lds[LY::QF + cc], qdv = lds[LY::UF + cc];
            const Real qup = SM.lim_qup[lane], qlo = SM.lim_qlow[lane], tr = SM.lim_trans[lane];
            const Real itr = SM.lim_itrans[lane];
            const Real up = smooth_step<false>(Real(0), Real(1), qup, qup + tr, itr, qv);
            const Real lo = smooth_step<false>(Real(1), Real(0), qlo - tr, qlo, itr, qv);
            lds[LY::LIM + 4 * lane] = -SM.lim_kup[lane] * up * (qv - qup) + SM.lim_klow[lane] * lo * (qlo - qv) -
                                      SM.lim_damp[lane] * (up + lo) * qdv;
        }
    }
    wave_sync();
    if (need_m && lane < ND) {
        /* row k = lane of the packed lower M, every entry (the structural
         * zeros too: the products below read whole rows): M_kl = S_l . I^c S_k
         * for l on k's root path (as phase 3 of dynamics, without the
         * implicit terms) */
        const Real *Sd = lds + LY::S + 6 * lane, *ic = lds + LY::IC + 10 * SM.dof_cb[lane];
        Real Gk[6], t[3];
        symv(ic + 4, Sd, Gk);
        cross3(ic + 1, Sd + 3, t);
#pragma unroll
        for (int i = 0; i < 3; ++i) Gk[i] += t[i];
        cross3(Sd, ic + 1, t);
#pragma unroll
        for (int i = 0; i < 3; ++i) Gk[3 + i] = ic[0] * Sd[3 + i] + t[i];
        unsigned path = 0;
        sfor<0, ND>([&](auto kI) {
            constexpr int k = decltype(kI)::value;
            constexpr unsigned pm = DofTree<T>::path_mask(k);
            path = lane == k ? pm : path;
        });
        Real *row = lds + LY::MP + (lane * (lane + 1)) / 2;
        sfor<0, ND>([&](auto lI) {
            constexpr int l = decltype(lI)::value;
            if (l <= lane) {
                const Real *Sl = lds + LY::S + 6 * l;
                row[l] = ((path >> l) & 1u) ? dot3(Sl, Gk) + dot3(Sl + 3, Gk + 3) : Real(0);
            }
        });
    }
    if (lane < ND) lds[LY::RHS + lane] = vd;
    wave_sync();
    Real r = 0;
    if (op == BIOIM_ID_MULT_MINV) {
        Real A[NP], xs[ND];
#pragma unroll
        for (int e = 0; e < NP; ++e) A[e] = lds[LY::MP + e];
#pragma unroll
        for (int d = 0; d < ND; ++d) xs[d] = lds[LY::RHS + d];
        ltl_solve<T, ND, Real>(A, xs);
#pragma unroll
        for (int d = 0; d < ND; ++d) r = lane == d ? xs[d] : r;
    } else if (lane < ND) {
        const Real *Sd = lds + LY::S + 6 * lane, *wb = lds + LY::WB + 6 * SM.dof_cb[lane];
        const Real bias = dot3(Sd, wb) + dot3(Sd + 3, wb + 3);   /* c - g (gravity removed for CORIOLIS) */
        Real fa = 0;
        if (applied) {
            sfor<0, T::NS>([&](auto sI) {
                constexpr int sp = decltype(sI)::value;
                constexpr unsigned msk = T::dofmask[T::sphere_cb[sp]];
                const Real *cj = lds + LY::CJ + LY::CJN * sp;
                Real jd[3];
                contact_jac(Sd, cj, jd);
                const Real term = dot3(jd, cj + 3);
                fa += (lds[LY::CW + 8 * sp + 6] > 0 && ((msk >> lane) & 1u)) ? term : Real(0);
            });
#pragma unroll
            for (int li = 0; li < T::NL; ++li)
                if (SM.lim_dof[li] == lane) fa += lds[LY::LIM + 4 * li];
        }
        Real mv = 0;
        if (need_m) {
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                const int hi = lane > k ? lane : k, lo = lane > k ? k : lane;
                mv += lds[LY::MP + hi * (hi + 1) / 2 + lo] * lds[LY::RHS + k];
            }
        }
        if (op == BIOIM_ID_GRAVITY) r = -bias;
        else if (op == BIOIM_ID_CORIOLIS) r = bias;
        else if (op == BIOIM_ID_MULT_M) r = mv;
        else if (op == BIOIM_ID_RESIDUAL) r = mv + bias - fa;
        else r = bias - fa;
    }
    if (lane < ND) GAT(a.out, (size_t)idx * ND + lane, (size_t)a.n * ND) = r;
}

/* ---------------------------------------------------------------- kernel
 * Launch arguments of one env segment (one handle).  mode 0: env step
 * (optionally with in-kernel auto-reset); mode 1: reset the listed envs.
 * I/O rows are strided so several segments (a mixed-topology group) can
 * share padded [N_total][stride] buffers. */
template <class T, typename Real> struct LaunchArgs {
    const DModel<Real> *Mg;
    const SModel<T, Real> *Sg;
    DState<Real> st;
    int N, mode, n_list, auto_reset, env_offset, blocks;
    int act_stride, obs_stride, info_stride;
    const Real *actions;
    Real *obs, *reward, *info;
    Real *final_obs;   /* optional: the step's observation before any auto-reset (row stride obs_stride) */
    Real *force_out;   /* optional: per-force-element values of the realized state, row stride force_dim */
    int force_dim;
    /* optional (RK kernels): the Manager's state storage — a row (t, q, u,
     * activation, fiber length) per accepted integration step of the env step,
     * [N][traj_cap][traj_dim]; traj_n[N] counts them (past traj_cap: counted, not stored) */
    Real *traj;
    int32_t *traj_n;
    int traj_cap, traj_dim;
    uint8_t *done_out;
    const int32_t *env_ids, *ref_index;
    uint64_t seed;
    /* apply_perturbations: zero-order-hold force table x[pert_n] (shared),
     * y[pert_n][N]; force on OpenSim body pert_ob; pert_n == 0: off */
    const double *pert_x;
    const Real *pert_y;
    int pert_n, pert_ob;
    double rk_acc;     /* RK-Merson accuracy (RK kernels) */
    int rk_budget;     /* RK kernels: attempts per env per launch (0: finish every step) */
    uint8_t *ready_out; /* optional [N]: 1 where the env finished its step in this launch */
    const uint8_t *active; /* optional [N] (steps): 0 = no new action, the env is left untouched
                              unless it is finishing a suspended RK step */
    /* mode 2 (OsimModel calls, REP kernels only; bioim_osim): op BIOIM_OSIM_*,
     * optional controls [n_list][nact] actuated first, report rows [N][osim_dim] */
    int osim_op, osim_dim;
    const Real *controls_in;
    Real *osim_out;
    /* optional (default step kernels of muscle models, no push, no force
     * report): the reset table — per reference row r its equilibrium fiber
     * lengths [nmuscle] and reset observation [obs_dim] (row stride
     * reset_tab_dim), computed once per handle by the reset realize itself
     * (build_reset_table); an in-kernel auto-reset reads row r instead of
     * running that realize again */
    const Real *reset_tab;
    int reset_tab_dim;
};

/* Reference integrator (RK kernels): OpenSim's Manager integrates with an
 * adaptive Kutta-Merson 4(5) at accuracy 1e-3 (opensim_wrapper.py:287-301).
 * Stage form, error norm, step control and the attempt cap follow
 * oracle/bioim_oracle.c integrate_rk_merson exactly; per state value the lane
 * keeps y0, K, E (three registers) besides the value itself. */
#define BIOIM_RK_MAX_ATTEMPTS 4096
template <typename Real> DEV void rk_update(int s, Real h, Real f, Real &y, Real &y0, Real &K, Real &E, Real &err) {
    switch (s) {
    case 0: y0 = y; K = f; E = Real(2) * f; y = y0 + h / Real(3) * f; break;
    case 1: y = y0 + h / Real(6) * (K + f); break;
    case 2: E -= Real(9) * f; y = y0 + h / Real(8) * (K + Real(3) * f); break;
    case 3: {
        const Real B = (K + E) / Real(3);
        E += Real(8) * f;
        y = y0 + Real(0.5) * h * (B + Real(4) * f);
        K += Real(4) * f;
        break;
    }
    default: {
        E -= f;
        y = y0 + h / Real(6) * (K + f);
        const Real w = fabs(y0) > Real(1) ? fabs(y0) : Real(1);
        const Real ei = fabs(h / Real(30) * E) / w;
        if (!(ei <= err)) err = ei;
    }
    }
}

/* one muscle's term of calc_cost_of_transport (muscle_walking_imitation_env2D.py:360-403,
 * Umberger-style heat and work rates): mass * (activation + maintenance heat)
 * + shortening + work, from the excitation ex and the realized fiber state */
template <typename Real> DEV Real muscle_cot(const SMuscle<Real> &mu, const MState<Real> &ms, Real ex) {
    Real l = mu.slow, aa = ms.act, hp = Real(0.5 * 3.14159265358979323846);
    Real se, ce, sa, ca;
    sincos_rt(hp * ex, se, ce);
    sincos_rt(hp * aa, sa, ca);
    Real fa = Real(40) * l * se + Real(133) * (Real(1) - l) * (Real(1) - ce);
    Real fm = Real(74) * l * sa + Real(111) * (Real(1) - l) * (Real(1) - ca);
    Real ln = ms.lce * mu.inv_lopt, vv = ms.vce;
    Real g = 0;
    if (ln < Real(0.5)) g = Real(0.5);
    else if (ln < Real(1)) g = ln;
    else if (ln < Real(1.5)) g = Real(-2) * ln + Real(3);
    Real es = fmax(Real(0), Real(0.25) * ms.Ff * -vv);
    Real ew = fmax(Real(0), ms.Fa * -vv);
    return mu.mass * fa + mu.mass * g * fm + es + ew;
}

/* OpenSim's body-fixed XYZ angles of R = Rx(a) Ry(b) Rz(c)
 * (Rotation::convertRotationToBodyFixedXYZ, opensim_wrapper.py:164-167) */
template <typename Real> DEV void body_fixed_xyz(const Real *R, Real *ang) {
    ang[0] = atan2(-R[5], R[8]);
    ang[1] = atan2(R[2], sqrt(R[0] * R[0] + R[1] * R[1]));
    ang[2] = atan2(-R[1], R[0]);
}

/* The realized state as the OsimModel calc_* calls read it (REP kernels,
 * bioim_osim; layout in include/bioim.h, BIOIM_OSIM_REPORT): time, istep;
 * q, u, q'' (CoordinateSet order); per OpenSim body origin position,
 * velocity, acceleration, body-fixed XYZ angles, angular velocity and
 * acceleration (calc_body_kinematics, :137-190), then the system COM
 * position, velocity, acceleration; per muscle activation, fiber length,
 * fiber velocity, fiber force, active fiber force, excitation, tendon force
 * (calc_muscles_info :238-259 and calc_cost_of_transport's getters); the
 * actuation of each actuator; per Hunt-Crossley force the wrench on the feet
 * about the ground origin (calc_forces_info :192-236); the limit forces;
 * calc_cost_of_transport().  Reads the frames, accelerations, columns, q''
 * and force slots the realize left in LDS; lane-parallel. */
template <class T, typename Real>
DEV void osim_report(const DModel<Real> &M, const SModel<T, Real> &SM, const Real *lds, int lane, const Dyn<T, Real> &D,
                     const Real (&control)[Lay<T, Real>::MPL], double t, int istep, Real *out) {
    using LY = Lay<T, Real>;
    constexpr int G = T::G, NC = T::NC, ND = LY::ND, NOS = T::NOS, NM = T::NM, NA = T::NA, MPL = LY::MPL;
    constexpr int CPL = (NC + G - 1) / G;
    constexpr int OB = 2 + 3 * NC, OCOM = OB + 18 * NOS, OMU = OCOM + 9, OACT = OMU + 7 * NM, OCF = OACT + NA;
    constexpr int OLIM = OCF + 6 * T::NF, OCOT = OLIM + T::NL;
    const Real x0 = D.x0;
    if (lane == 0) { out[0] = Real(t); out[1] = Real(istep); }
    /* the muscle rows first: their fiber states then die before the body
     * terms below are live (3D REP kernels: fewer values spilled) */
    Real cot = 0;
#pragma unroll
    for (int j = 0; j < MPL; ++j) {
        const int m = mslot<T>(lane + j * G);
        if constexpr (NM > 0) {
            if (m < NM) {
                const MState<Real> &ms = D.ms[j];
                Real *o = out + OMU + 7 * m;
                o[0] = ms.act; o[1] = ms.lce; o[2] = ms.vce; o[3] = ms.Ff; o[4] = ms.Fa; o[5] = control[j]; o[6] = ms.Ft;
                cot += muscle_cot<Real>(SM.mus[m], ms, control[j]);
            }
        }
        if (m < NA) {
            if constexpr (NM > 0) out[OACT + m] = D.ms[j].Ft;
            else out[OACT + m] = control[j] * SM.ca_opt[m];
        }
    }
    cot = group_sum<G>(cot);
    if (lane == 0) out[OCOT] = NM > 0 ? cot + Real(1.51) * M.total_mass : Real(0);
    /* loops over bodies, spheres and coordinates run rolled (unroll 1): the
     * report is off the stepping path, and unrolled it held every body's terms
     * live at the kernel's peak register pressure — 0.6-2.9 KB/lane of scratch
     * in the REP kernels (profiles/r03/resources.txt).  (Round 4's first cut
     * kept the prosthetic model's loops unrolled: rolled, its non-RK REP
     * kernels then got two lane-divergent AGPR copies of the env offset that
     * tools/hazard_gate.py flags; with the compile-time mode of the REP
     * kernels (env_block) the rolled form is clean there too.) */
    constexpr int UC = 1, UB = 1, US = 1;
#pragma unroll UC
    for (int jc = 0; jc < CPL; ++jc) {
        const int c = lane + jc * G;
        if (c < NC) {
            const int dc = SM.coord_dof[c];
            out[2 + c] = lds[LY::QF + c];
            out[2 + NC + c] = lds[LY::UF + c];
            out[2 + 2 * NC + c] = dc >= 0 ? lds[LY::RHS + dc] : Real(0);
        }
    }
    /* spatial acceleration of composite body cb (at the shifted ground
     * origin): the velocity-product part plus its root path's columns x q'' */
    auto body_acc = [&](int cb, Real *al, Real *aO) {
        const Real *ab = lds + LY::AL + 6 * cb;
        const uint32_t dm = SM.dofmask[cb];
#pragma unroll
        for (int i = 0; i < 3; ++i) { al[i] = ab[i]; aO[i] = ab[3 + i]; }
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            const Real qdd = ((dm >> d) & 1u) ? lds[LY::RHS + d] : Real(0);
            const Real *S = lds + LY::S + 6 * d;
#pragma unroll
            for (int i = 0; i < 3; ++i) { al[i] += S[i] * qdd; aO[i] += S[3 + i] * qdd; }
        }
    };
    if (lane < NOS) {
        /* each term stored as soon as it is computed (fewer values live at once) */
        const int cb = SM.os_cb[lane];
        const Real *kb = lds + LY::KB + 18 * cb;
        Real *o = out + OB + 18 * lane;
        {
            Real Rb[9], ang[3];
            mm3(kb, M.os_R[lane], Rb);
            body_fixed_xyz(Rb, ang);
#pragma unroll
            for (int i = 0; i < 3; ++i) { o[9 + i] = ang[i]; o[12 + i] = kb[12 + i]; }
        }
        Real P[3], v[3], tt[3], al[3], aO[3];
        mv3(kb, SM.os_p[lane], P);
#pragma unroll
        for (int i = 0; i < 3; ++i) P[i] += kb[9 + i];
        cross3(kb + 12, P, tt);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            v[i] = kb[15 + i] + tt[i];
            o[i] = P[i] + (i == 0 ? x0 : Real(0)); o[3 + i] = v[i];
        }
        body_acc(cb, al, aO);
        Real t2[3];
        cross3(al, P, tt);
        cross3(kb + 12, v, t2);
#pragma unroll
        for (int i = 0; i < 3; ++i) { o[6 + i] = aO[i] + tt[i] + t2[i]; o[15 + i] = al[i]; }
    } else if (lane == NOS) {
        Real mt = 0, cs[3] = {0, 0, 0}, vs[3] = {0, 0, 0}, as[3] = {0, 0, 0};
#pragma unroll UB
        for (int c = 0; c < T::NB; ++c) {
            const Real *kb = lds + LY::KB + 18 * c;
            Real cG[3], vc[3], ac[3], tt[3], t2[3], al[3], aO[3];
            mv3(kb, SM.body[c].com, cG);
#pragma unroll
            for (int i = 0; i < 3; ++i) cG[i] += kb[9 + i];
            cross3(kb + 12, cG, tt);
#pragma unroll
            for (int i = 0; i < 3; ++i) vc[i] = kb[15 + i] + tt[i];
            body_acc(c, al, aO);
            cross3(al, cG, tt);
            cross3(kb + 12, vc, t2);
#pragma unroll
            for (int i = 0; i < 3; ++i) ac[i] = aO[i] + tt[i] + t2[i];
            const Real m = SM.body[c].mass;
#pragma unroll
            for (int i = 0; i < 3; ++i) { cs[i] += m * cG[i]; vs[i] += m * vc[i]; as[i] += m * ac[i]; }
            mt += m;
        }
        Real *o = out + OCOM;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            o[i] = cs[i] / mt + (i == 0 ? x0 : Real(0)); o[3 + i] = vs[i] / mt; o[6 + i] = as[i] / mt;
        }
    }
    if (lane < T::NF) {
        Real F[3] = {0, 0, 0}, Mo[3] = {0, 0, 0};
#pragma unroll US
        for (int s2 = 0; s2 < T::NS; ++s2) {
            const Real *cw = lds + LY::CW + 8 * s2;
            const bool mine = SM.sph_force[s2] == lane;
#pragma unroll
            for (int i = 0; i < 3; ++i) { F[i] += mine ? cw[i] : Real(0); Mo[i] += mine ? cw[3 + i] : Real(0); }
        }
        Mo[1] += -x0 * F[2];
        Mo[2] += x0 * F[1];
#pragma unroll
        for (int i = 0; i < 3; ++i) { out[OCF + 6 * lane + i] = F[i]; out[OCF + 6 * lane + 3 + i] = Mo[i]; }
    }
    if (lane < T::NL) out[OLIM + lane] = lds[LY::LIM + 4 * lane];
}

/* One 256-thread workgroup = 256/G envs of segment `a`, block `blk`.
 * RK: the reference integrator (adaptive Kutta-Merson) instead of the
 * fixed semi-implicit substeps. */
template <class T, typename Real, bool PERT, bool RK, bool REP>
DEV void env_block(const LaunchArgs<T, Real> &a, int blk) {
    using LY = Lay<T, Real>;
    constexpr int G = T::G, ND = LY::ND, NA = T::NA, NM = T::NM;
    constexpr int EPB = BIOIM_EPB;
    constexpr size_t SMB = smodel_bytes<T, Real>();
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const DModel<Real> *__restrict__ Mg = a.Mg;
    const DState<Real> &st = a.st;
    /* mode 2 (OsimModel calls) exists in the REP kernels only, and they run
     * nothing else (launch_impl): a compile-time mode there, so the step's
     * reward / termination / auto-reset tail and the RK carry past the report
     * are dead code in them instead of live registers */
    const int N = a.N, mode = REP ? 2 : a.mode;
    const bool osim = REP;
    const Real *__restrict__ actions = a.actions;
    Real *__restrict__ obs = a.obs;
#ifdef BIOIM_STAMPS
    const unsigned long long k_t0 = __builtin_amdgcn_s_memtime();
#endif
    /* stage the shared model image (one copy per workgroup) */
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(a.Sg);
        uint4 *dst = reinterpret_cast<uint4 *>(smem_raw);
        for (int i = threadIdx.x; i < (int)(SMB / 16); i += BIOIM_EPB * G) dst[i] = src[i];
    }
    __syncthreads();
#ifdef BIOIM_STAMPS
    const unsigned long long k_t1 = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[11] += k_t1 - k_t0;
#endif
    const SModel<T, Real> &SM = *reinterpret_cast<const SModel<T, Real> *>(smem_raw);
    const DModel<Real> &M = *Mg;
    const int lane = threadIdx.x % G;
    const int slot = threadIdx.x / G;
    int gidx = blk * EPB + slot;
    Real *lds = reinterpret_cast<Real *>(smem_raw + SMB) + slot * LY::SIZE;
    int env;
    if (mode == 1 || osim) {
        if (gidx >= a.n_list) return;
        env = a.env_ids ? GAT(a.env_ids, gidx, a.n_list) : gidx;
        if (env < 0 || env >= N) return;
    } else {
        if (gidx >= N) return;
        env = gidx;
        if (a.active && !GAT(a.active, env, N) && !(RK && GAT(st.pend, env, (size_t)N) != 0)) return;
    }
    const int H = M.horizon;
    constexpr int MPL = LY::MPL;                  /* muscles / actions per lane: m = lane + j*G */
    constexpr int CPL = (T::NC + G - 1) / G;      /* coordinates per lane (report)              */
    Dyn<T, Real> D;
#pragma unroll
    for (int j = 0; j < MPL; ++j) D.ms[j].vN = 0;
#if BIOIM_FV_PRED
    Real vprev[MPL];
#pragma unroll
    for (int j = 0; j < MPL; ++j) vprev[j] = 0;
#endif
    /* lane d < ND owns dof d (coordinate value qd, speed ud) */
    Real qd = 0, ud = 0;
    if (lane < ND) { qd = GAT(st.q, (size_t)lane * N + env, (size_t)ND * N); ud = GAT(st.u, (size_t)lane * N + env, (size_t)ND * N); }
    double t = GAT(st.t, env, (size_t)N);
    /* has_last, resets, old_px and last[] change only in a step (mode 0) or a
     * reset (mode 1): the REP kernels neither load nor store them, instead of
     * carrying them through the kernel unchanged */
    int istep = GAT(st.istep, env, (size_t)N), has_last = REP ? 0 : GAT(st.has_last, env, (size_t)N),
        resets = REP ? 0 : GAT(st.resets, env, (size_t)N);
    Real old_px = REP ? Real(0) : GAT(st.old_px, env, (size_t)N);
    Real act[MPL], lce[MPL], control[MPL], curr[MPL], last[MPL], hist[MPL][BIOIM_MAX_HORIZON];
#pragma unroll
    for (int j = 0; j < MPL; ++j) {
        const int m = mslot<T>(lane + j * G);
        act[j] = 0; lce[j] = 0; control[j] = 0; curr[j] = 0; last[j] = 0;
        if (NM > 0 && m < NM) { act[j] = GAT(st.act, (size_t)m * N + env, (size_t)(NM > 0 ? NM : 1) * N); lce[j] = GAT(st.lce, (size_t)m * N + env, (size_t)(NM > 0 ? NM : 1) * N); }
#pragma unroll
        for (int hh = 0; hh < BIOIM_MAX_HORIZON; ++hh) hist[j][hh] = 0;
        if (m < NA) {
            if (!REP) last[j] = GAT(st.last, (size_t)m * N + env, (size_t)NA * N);
#pragma unroll
            for (int hh = 0; hh < BIOIM_MAX_HORIZON; ++hh)
                hist[j][hh] = hh < H ? GAT(st.hist, ((size_t)hh * NA + m) * N + env, (size_t)BIOIM_MAX_HORIZON * NA * N) : Real(0);
            /* held controls (OsimModel calls act on the last actuate) */
            if (osim) control[j] = GAT(st.ctl, (size_t)m * N + env, (size_t)NA * N);
        }
    }
    /* the realize cache (CacheLay): a step's first substep takes its system
     * from the last launch's realize when that row is valid for this state
     * and was formed at this step's substep length (checked below); loaded
     * here, ahead of the action pre-processing */
    constexpr bool CACHE = CacheLay<T>::ON && !PERT && !RK && !REP;
    CacheIO<T, Real> CI;
    bool cache_valid = false;
    Real cache_h = 0;
    if constexpr (CACHE) {
        using CL = CacheLay<T>;
        CI.base = st.cache; CI.env = env; CI.N = N;
        Real *const crow = st.cache + GIDX((size_t)env * CL::DIM, (size_t)N * CL::DIM);
        cache_valid = mode == 0 && GAT(st.cache_ok, env, (size_t)N) != 0;
        cache_h = GAT(crow, CL::H, CL::DIM);
        if constexpr (CL::PREFETCH) {
#pragma unroll
            for (int i = 0; i < CacheIO<T, Real>::PF; ++i)
                CI.sys[i] = lane + i * G < CL::SYS ? GAT(crow, lane + i * G, CL::DIM) : Real(0);
#pragma unroll
            for (int j = 0; j < MPL; ++j) {
                const int m = mslot<T>(lane + j * G);
#pragma unroll
                for (int c = 0; c < 3; ++c) CI.mus[j][c] = m < NM ? GAT(crow, CL::MUS + 3 * m + c, CL::DIM) : Real(0);
            }
        }
    }
    int done = 0;
    Real rew = 0, inf[5] = {0, 0, 0, 0, 0};
    bool do_reset = (mode == 1);
    /* budgeted RK: a suspended step resumes (its action row is ignored) */
    const bool budget = RK && !REP && a.rk_budget > 0;   /* make_args: 0 unless mode 0 */
    const bool resume = RK && mode == 0 && GAT(st.pend, env, (size_t)N) != 0;
    bool suspend = false;
    /* RK: dynamics evaluations spent in this launch (the budget is 5 per
     * attempt) and so far (bioim_eval_count).  (Reusing a rejected attempt's
     * first stage for its retry — same start point — saves about a fifth of
     * the rejected attempts' evaluations but measured slower at 4096 envs:
     * the stores of k1 cost every attempt, and the saving rarely removes a
     * launch from a step; profiles/r03/ab_dropped/ab_rk_k1_reuse.txt) */
    int launch_evals = 0;
    /* state-storage rows of this env step so far (a resumed step continues its count) */
    int traj_k = (RK && a.traj && mode == 0 && GAT(st.pend, env, (size_t)N) != 0) ? GAT(a.traj_n, env, N) : 0;
    int reset_row = 0;
    if (mode == 1) reset_row = a.ref_index ? GAT(a.ref_index, gidx, a.n_list) : draw_index(a.seed, a.env_offset + env, resets, M.reset_hi);

    int remaining = 0;
    Real dt = 0;
    /* RK kernels: current step [rk_t, rk_t + rk_h], stage, attempts, next step size */
    double rk_t = 0, rk_tf = 0, rk_h = 0, rk_hnext = RK ? GAT(st.hrk, env, (size_t)N) : 0.0;
    int rk_stage = 0, rk_attempts = 0;
    bool rk_last = false, rk_fail = false;
    Real y0q = 0, y0u = 0, Kq = 0, Ku = 0, Eq = 0, Eu = 0, rk_err = 0;
    Real y0a[MPL], y0l[MPL], Ka[MPL], Kl[MPL], Ea[MPL], El[MPL];
#pragma unroll
    for (int j = 0; j < MPL; ++j) { y0a[j] = y0l[j] = Ka[j] = Kl[j] = Ea[j] = El[j] = 0; }
    const PertArgs<Real> PA{a.pert_x, a.pert_y, a.pert_n, a.pert_ob, env, N};
    double *pslot = reinterpret_cast<double *>(smem_raw + SMB + sizeof(Real) * EPB * LY::SIZE) + PERT_SLOT * slot;
    if (PERT && lane == 0) { pslot[0] = t; pslot[1] = 0; pslot[2] = 0; pslot[3] = -1; pslot[4] = 0; }
    /* OsimModel.integrate (opensim_wrapper.py:299-301): istep += 1, then
     * integrate to the absolute time step_size * istep with the held controls */
    auto begin_integrate = [&]() {
        istep += 1;
        double tf = M.step_size * (double)istep;
        double hstep = tf - t;
        if (hstep > 0) {
            if constexpr (RK) {
                rk_t = t; rk_tf = tf;
                rk_h = rk_hnext > 0 ? rk_hnext : 1e-4;
                remaining = 1;      /* integrating until rk_t reaches rk_tf */
            } else {
                dt = Real(hstep / (double)M.nsub);
                remaining = M.nsub;
                /* substep k starts at t + k * hstep / nsub (the oracle's substep times) */
                if (PERT && lane == 0) { pslot[0] = t; pslot[1] = hstep / (double)M.nsub; }
            }
        }
        t = tf;
    };
    bool eq_only = false;   /* mode 2 EQUILIBRATE: fiber equilibrium at the held state */
    if (osim) {
        if (a.controls_in) {
            /* OsimModel.actuate (opensim_wrapper.py:92-107): NaN -> 0, clip */
            Real raw[MPL];
            bool nan_here = false;
#pragma unroll
            for (int j = 0; j < MPL; ++j) {
                const int m = mslot<T>(lane + j * G);
                raw[j] = m < NA ? GAT(a.controls_in, (size_t)gidx * NA + m, (size_t)a.n_list * NA) : Real(0);
                nan_here = nan_here || (m < NA && isnan(raw[j]));
            }
            const bool anynan = group_any<G>(nan_here);
#pragma unroll
            for (int j = 0; j < MPL; ++j) {
                const int m = mslot<T>(lane + j * G), ms = m < NA ? m : 0;
                const Real lo = NM > 0 ? Real(0) : SM.ca_min[ms];
                const Real hi = NM > 0 ? Real(1) : SM.ca_max[ms];
                const Real v = anynan ? Real(0) : raw[j];
                control[j] = m < NA ? (v < lo ? lo : (v > hi ? hi : v)) : Real(0);
                if (m < NA) GAT(st.ctl, (size_t)m * N + env, (size_t)NA * N) = control[j];
            }
        }
        if (a.osim_op == BIOIM_OSIM_INTEGRATE) begin_integrate();
        if (a.osim_op == BIOIM_OSIM_EQUILIBRATE) {
            eq_only = true;
            rk_hnext = 0;   /* reset_manager: a new Manager / integrator (opensim_wrapper.py:287-291) */
        }
    } else if (resume) {
        /* the state is at the accepted RK point rk_t of the step ending at t.
         * The loads index with an opaque copy of env made inside this
         * lane-divergent branch: with env itself, the allocator split the
         * kernel-long env offsets here and copied them into AGPRs for the
         * resuming lanes only, which the state write-back then used as store
         * addresses in every lane (the r03i fault) */
        int er = env;
        asm volatile("" : "+v"(er));
#pragma unroll
        for (int j = 0; j < MPL; ++j) {
            const int m = mslot<T>(lane + j * G);
            if (m < NA) { control[j] = GAT(st.ctl, (size_t)m * N + er, (size_t)NA * N); curr[j] = GAT(st.cur, (size_t)m * N + er, (size_t)NA * N); }
            if (NM > 0 && m < NM) D.ms[j].vN = GAT(st.vnw, (size_t)m * N + er, (size_t)(NM > 0 ? NM : 1) * N);
        }
        rk_t = GAT(st.rkt, er, (size_t)N); rk_tf = t; rk_h = GAT(st.rkh, er, (size_t)N); rk_attempts = GAT(st.rka, er, (size_t)N);
        remaining = 1;
    } else if (mode == 0) {
        /* ---- action pre-processing (Env.step) */
        Real raw[MPL];
        bool nan_here = false;
#pragma unroll
        for (int j = 0; j < MPL; ++j) {
            const int m = mslot<T>(lane + j * G);
            raw[j] = m < NA ? GAT(actions, (size_t)env * a.act_stride + m, (size_t)N * a.act_stride) : Real(0);
            nan_here = nan_here || (m < NA && isnan(raw[j]));
        }
        const bool anynan = group_any<G>(nan_here);
        Real av[MPL];
#pragma unroll
        for (int j = 0; j < MPL; ++j) av[j] = anynan ? Real(0) : raw[j];
        if constexpr ((T::FLAGS & BIOIM_ENV_PD) != 0) {
            /* PD law on the state at the start of the step (torque_walking_imitation_env2D.py:125-139) */
            publish_coords<T, Real>(M, SM, lds, lane, qd, ud);
            wave_sync();
            if (!anynan) {
#pragma unroll
                for (int j = 0; j < MPL; ++j) {
                    const int m = mslot<T>(lane + j * G);
                    Real xq = 0, xu = 0;
                    sfor<0, NA>([&](auto iI) {
                        constexpr int i = decltype(iI)::value;
                        if (m == i) { xq = lds[LY::QF + T::pd_coord[i]]; xu = lds[LY::UF + T::pd_vcoord[i]]; }
                    });
                    if (m < NA) av[j] = SM.kp[m] * (raw[j] - xq) - SM.kv[m] * xu;
                }
            }
        }
        bool pnan_here = false;
#pragma unroll
        for (int j = 0; j < MPL; ++j) {
            const int m = mslot<T>(lane + j * G);
            if (!has_last) {
                last[j] = av[j];
#pragma unroll
                for (int hh = 0; hh < BIOIM_MAX_HORIZON; ++hh) hist[j][hh] = av[j];
            }
            /* fixed-trip loops keep the history in registers */
#pragma unroll
            for (int hh = 0; hh + 1 < BIOIM_MAX_HORIZON; ++hh)
                if (hh + 1 < H) hist[j][hh] = hist[j][hh + 1];
#pragma unroll
            for (int hh = 0; hh < BIOIM_MAX_HORIZON; ++hh)
                if (hh == H - 1) hist[j][hh] = av[j];
            Real sm = 0;
#pragma unroll
            for (int hh = 0; hh < BIOIM_MAX_HORIZON; ++hh)
                if (hh < H) sm += hist[j][hh];
            curr[j] = sm / Real(H);
            /* the deque is final here: store it now instead of holding it in
             * registers through the substep loop (34 AGPRs in 3D fp64) */
            if (m < NA) {
#pragma unroll
                for (int hh = 0; hh < BIOIM_MAX_HORIZON; ++hh)
                    if (hh < H) GAT(st.hist, ((size_t)hh * NA + m) * N + env, (size_t)BIOIM_MAX_HORIZON * NA * N) = hist[j][hh];
            }
            const Real phys = (M.env_flags & BIOIM_ENV_RAW_ACTION) ? av[j] : curr[j];
            pnan_here = pnan_here || (m < NA && isnan(phys));
            control[j] = phys;
        }
        has_last = 1;
        const bool pnan = group_any<G>(pnan_here);
#pragma unroll
        for (int j = 0; j < MPL; ++j) {
            const int m = mslot<T>(lane + j * G), ms = m < NA ? m : 0;
            const Real lo = NM > 0 ? Real(0) : SM.ca_min[ms];
            const Real hi = NM > 0 ? Real(1) : SM.ca_max[ms];
            const Real v = pnan ? Real(0) : control[j];
            control[j] = m < NA ? (v < lo ? lo : (v > hi ? hi : v)) : Real(0);
            /* the held controls (PrescribedController's Constants): kept through
             * resets, read by resets and OsimModel calls; stored now, so they
             * are not held in registers past the last dynamics call */
            if (m < NA) GAT(st.ctl, (size_t)m * N + env, (size_t)NA * N) = control[j];
        }
        /* ---- integrate to step_size * istep */
        begin_integrate();
    }

    /* One dynamics call site (inlined once): the substeps, then the realize
     * at the end state; a reset (mode 1, or auto-reset after done) loads the
     * reference row and folds the muscle fiber equilibrium into its realize. */
    bool pending_reset = (mode == 1), reported_reset = false;
    for (;;) {
        if constexpr (RK) {
            if (remaining > 0 && rk_stage == 0) {   /* start an RK step, or stop */
                const int cost = 5;
                if (!(rk_tf - rk_t > 1e-14 * (1.0 + fabs(rk_tf)))) remaining = 0;
                else if (budget && launch_evals + cost > 5 * a.rk_budget) { suspend = true; break; }
                else if (++rk_attempts > BIOIM_RK_MAX_ATTEMPTS) { rk_fail = true; remaining = 0; }
                else {
                    launch_evals += cost;
                    rk_last = false;
                    if (rk_h >= rk_tf - rk_t) { rk_h = rk_tf - rk_t; rk_last = true; }
                    rk_err = 0;
                }
            }
        }
        const bool sub = remaining > 0;
        const bool eq = !sub && (pending_reset || eq_only);
        if (!sub && pending_reset) {
                        int r = clamp_row(reset_row, M.nrows);
            if (lane < ND) {
                const int c = SM.dof_coord[lane];
                qd = M.ref_q[r][c];
                ud = M.ref_u[r][c];
            }
            t = M.ref_time[r];
            istep = M.ref_istep[r];
            has_last = 0;
            rk_hnext = 0;   /* reset_manager: a new integrator (opensim_wrapper.py:287-291) */
            /* initializeState: the default activation.  The held controls stay:
             * the PrescribedController's Constant functions keep the last
             * actuate() through OsimModel.reset (opensim_wrapper.py:92-107,
             * :293-297), so a reset realizes with them — reloaded from HBM
             * (stored when the step computed them) rather than kept in
             * registers through the report (+40 VGPRs in 3D fp64) */
#pragma unroll
            for (int j = 0; j < MPL; ++j) {
                const int m = mslot<T>(lane + j * G);
                control[j] = m < NA ? GAT(st.ctl, (size_t)m * N + env, (size_t)NA * N) : Real(0);
                if constexpr (NM > 0)
                    if (m < NM) act[j] = SM.mus[m].default_act;
                /* CACHE: the reset realize's fiber-velocity roots start cold,
                 * as the reset table's do (build_reset_table), so the cache row
                 * it leaves is the table's bit for bit */
                if constexpr (CACHE) D.ms[j].vN = 0;
            }
            resets += 1;
        }
        if constexpr (CACHE) {
            /* the first substep from the cache; a realize (step or reset) forms
             * the cache at the next step's substep length (begin_integrate's
             * arithmetic for istep + 1) */
            CI.use = cache_valid && sub && remaining == M.nsub && cache_h == dt;
            cache_valid = false;
            CI.make = !sub;
            if (!sub) {
                const double tf = M.step_size * (double)(istep + 1);
                const double hstep = tf - t;
                CI.hc = Real(hstep / (double)M.nsub);
            }
        }
        {
            /* opaque per-iteration model pointer: keeps the compiler from
             * hoisting hundreds of loop-invariant constants into registers
             * (they are re-read from the scalar cache instead of spilled) */
            typedef const __attribute__((address_space(4))) DModel<Real> CModel;
            CModel *Mi = (CModel *)Mg;
            asm volatile("" : "+s"(Mi));
            /* realize / reset realize: the call time is t itself */
            if (PERT && !sub && lane == 0) { pslot[0] = t; pslot[1] = 0; }
            if (RK && PERT && sub && lane == 0) {
                const double cs = rk_stage == 0 ? 0.0 : rk_stage <= 2 ? 1.0 / 3.0 : rk_stage == 3 ? 0.5 : 1.0;
                pslot[0] = rk_t + cs * rk_h; pslot[1] = 0;
            }
#if BIOIM_FV_PRED
            if constexpr (!RK && NM > 0) {
#pragma unroll
                for (int j = 0; j < MPL; ++j) {
                    const Real vc = D.ms[j].vN;
                    D.ms[j].vN = vc + (vc - vprev[j]);
                    vprev[j] = vc;
                }
            }
#endif
            /* RK: explicit accelerations (h = 0, the implicit terms compile away) */
            /* branch-free phase-3 row stores, except in the spatial RK kernels
             * (they would take those kernels past the 512-register budget) */
            dynamics<T, Real, PERT, !RK || T::PLANAR, !RK, CACHE>(*(const DModel<Real> *)Mi, SM, qd, ud, act, lce, control, lane, lds,
                                    RK ? Real(0) : (sub ? dt : Real(0)), eq && NM > 0, PA, pslot,
                                    RK ? 0 : M.nsub - remaining, D, CI);
        }
        if (RK && sub) {
            const Real h = Real(rk_h);
            if (lane < ND) {
                const Real fq = ud, fu = D.qdd;
                rk_update<Real>(rk_stage, h, fq, qd, y0q, Kq, Eq, rk_err);
                rk_update<Real>(rk_stage, h, fu, ud, y0u, Ku, Eu, rk_err);
            }
            if constexpr (NM > 0) {
#pragma unroll
                for (int j = 0; j < MPL; ++j) {
                    const int m = mslot<T>(lane + j * G);
                    if (m < NM) {
                        const Real fl = D.ms[j].clamped ? Real(0) : D.ms[j].vce;
                        rk_update<Real>(rk_stage, h, D.ms[j].dadt, act[j], y0a[j], Ka[j], Ea[j], rk_err);
                        rk_update<Real>(rk_stage, h, fl, lce[j], y0l[j], Kl[j], El[j], rk_err);
                    }
                }
            }
            if (rk_stage < 4) {
                ++rk_stage;
                continue;
            }
            rk_stage = 0;
            Real e = isnan(rk_err) ? Real(INFINITY) : rk_err;
            e = group_max<G>(e);
            const double err = (double)e;
            double fac = err > 0 ? 0.9 * sqrt(sqrt(a.rk_acc / err)) : 5.0;
            if (!(fac == fac)) fac = 0.1;
            fac = fac < 0.1 ? 0.1 : (fac > 5.0 ? 5.0 : fac);
            if (err <= a.rk_acc) {
                if constexpr (NM > 0) {
#pragma unroll
                    for (int j = 0; j < MPL; ++j) {
                        const int m = mslot<T>(lane + j * G);
                        if (m < NM && lce[j] < SM.mus[m].lmin) lce[j] = SM.mus[m].lmin;
                    }
                }
                rk_t = rk_last ? rk_tf : rk_t + rk_h;
                if (!rk_last) rk_hnext = rk_h * fac;
                if (a.traj) {   /* the Manager stores every accepted step (opensim_wrapper.py:336) */
                    if (traj_k < a.traj_cap) {
                        Real *row = a.traj + GIDX(((size_t)env * a.traj_cap + traj_k), (size_t)N * a.traj_cap) * a.traj_dim;
                        if (lane == 0) GAT(row, 0, a.traj_dim) = Real(rk_t);
                        if (lane < ND) { GAT(row, 1 + lane, a.traj_dim) = qd; GAT(row, 1 + ND + lane, a.traj_dim) = ud; }
                        if constexpr (NM > 0) {
#pragma unroll
                            for (int j = 0; j < MPL; ++j) {
                                const int m = mslot<T>(lane + j * G);
                                if (m < NM) { GAT(row, 1 + 2 * ND + m, a.traj_dim) = act[j]; GAT(row, 1 + 2 * ND + NM + m, a.traj_dim) = lce[j]; }
                            }
                        }
                    }
                    ++traj_k;
                }
            } else {
                qd = y0q; ud = y0u;
#pragma unroll
                for (int j = 0; j < MPL; ++j) { act[j] = y0a[j]; lce[j] = y0l[j]; }
            }
            rk_h *= fac;
            continue;
        }
        if (!RK && sub) {
            if (lane < ND) { ud += dt * D.qdd; qd += dt * ud; }
            if constexpr (NM > 0) {
#pragma unroll
                for (int j = 0; j < MPL; ++j) {
                    const int m = mslot<T>(lane + j * G);
                    if (m < NM) {
                        act[j] += dt * D.ms[j].dadt;
                        if (!D.ms[j].clamped) {
#if BIOIM_SUBSTEP_RCP
                            /* a refined hardware reciprocal (fast_rcp) instead of the IEEE
                             * division: the divisor 1 - dt dv/dl is a well-scaled positive
                             * quantity; once per muscle and substep */
                            Real ln = lce[j] + dt * D.ms[j].vce * fast_rcp(Real(1) - dt * D.ms[j].dvdl);
#else
                            Real ln = lce[j] + dt * D.ms[j].vce / (Real(1) - dt * D.ms[j].dvdl);
#endif
                            lce[j] = ln < SM.mus[m].lmin ? SM.mus[m].lmin : ln;
                        }
                    }
                }
            }
            --remaining;
            continue;
        }
        if (eq) {
            if constexpr (NM > 0) {
#pragma unroll
                for (int j = 0; j < MPL; ++j)
                    if (lane + j * G < NM) { act[j] = D.act[j]; lce[j] = D.lce[j]; }
            }
            reported_reset = pending_reset;
            pending_reset = false;
            eq_only = false;
        }
                /* ---- realized state: observation (lane-parallel; get_state_dict,
         * muscle_walking_imitation_env2D.py:158-225).  The realize call left
         * the coordinates (QF/UF), frames (KB), contact wrenches (CW) and limit
         * forces (LIM) in LDS; report points first. */
#ifdef BIOIM_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long rp_t0 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
#endif
        using OL = ObsLayout<T>;
        const Real x0 = D.x0;
        Real *ob = lds + LY::OBS;
        const bool tgt = (M.env_flags & BIOIM_ENV_TARGET_OBS) != 0, grf = (M.env_flags & BIOIM_ENV_GRF_OBS) != 0;
        if (lane <= T::NOS) report_points<T, Real>(SM, lds, lane, x0);
        wave_sync();
        const Real px = lds[LY::QF + T::TX], py = lds[LY::QF + T::TY];
        Real pz = 0;
        if constexpr (T::TZ >= 0) pz = lds[LY::QF + T::TZ];
        if (lane == 0) {
            double ph = (double)istep / (double)M.cycle;
            ob[0] = Real(ph - floor(ph));
        }
        const int obody = OL::body(tgt);
#pragma unroll
        for (int jc = 0; jc < CPL; ++jc) {
            const int c = lane + jc * G;
            if (c < T::NC) {
                const bool trans = c == T::TX || c == T::TY || c == T::TZ;
                const int qi = c - (T::TX >= 0 && T::TX < c) - (T::TY >= 0 && T::TY < c) - (T::TZ >= 0 && T::TZ < c);
                if (!trans) ob[OL::QPOS + qi] = lds[LY::QF + c];
                ob[OL::QVEL + c] = lds[LY::UF + c];
                const int dc = SM.coord_dof[c];
                ob[OL::QACC + c] = dc >= 0 ? lds[LY::RHS + dc] : Real(0);
                if (tgt && c != T::TX) {
                    const int r1 = clamp_row(istep + 1, M.nrows), ti = c - (T::TX >= 0 && T::TX < c);
                    ob[OL::TGT + ti] = M.ref_q[r1][c];
                    ob[OL::TGT + (T::NC - 1) + ti] = M.ref_u[r1][c];
                }
            }
        }
        if (lane < T::NOBP) {
            const Real *rp = lds + LY::REP + 6 * SM.obs_slot[lane];
            ob[obody + 3 * lane] = rp[0] - px; ob[obody + 3 * lane + 1] = rp[1] - py; ob[obody + 3 * lane + 2] = rp[2] - pz;
        }
        if (lane < T::NOBV) {
            const Real *rp = lds + LY::REP + 6 * SM.obs_slot[T::NOBP + lane];
#pragma unroll
            for (int i = 0; i < 3; ++i) ob[obody + 3 * T::NOBP + 3 * lane + i] = rp[3 + i];
        }
        const int omus = obody + 3 * T::NOBP + 3 * T::NOBV;
        if constexpr (NM > 0) {
#pragma unroll
            for (int j = 0; j < MPL; ++j) {
                const int m = mslot<T>(lane + j * G);
                if (m < NM) {
                    ob[omus + 3 * m] = D.ms[j].act;
                    ob[omus + 3 * m + 1] = D.ms[j].lce;
                    ob[omus + 3 * m + 2] = D.ms[j].vce;
                }
            }
        }
        if (grf && lane < T::NF) {
            Real F[3] = {0, 0, 0}, Mo[3] = {0, 0, 0};
#pragma unroll
            for (int s2 = 0; s2 < T::NS; ++s2) {
                const Real *cw = lds + LY::CW + 8 * s2;
                const bool mine = SM.sph_force[s2] == lane;
#pragma unroll
                for (int i = 0; i < 3; ++i) { F[i] += mine ? cw[i] : Real(0); Mo[i] += mine ? cw[3 + i] : Real(0); }
            }
            /* moments about the absolute ground origin: (x0,0,0) x F */
            Mo[1] += -x0 * F[2];
            Mo[2] += x0 * F[1];
            const int og = omus + 3 * NM + 6 * lane;
#pragma unroll
            for (int i = 0; i < 3; ++i) { ob[og + i] = F[i] / M.weight; ob[og + 3 + i] = Mo[i] / M.moment; }
        }
        if (a.force_out) {
            /* ForceReporter values (opensim_wrapper.py:10-15): actuation of each
             * muscle (tendon force) or coordinate actuator, the wrench on the feet
             * of each contact force about the ground origin, each limit force */
            Real *fo = a.force_out + GIDX((size_t)env, (size_t)N) * a.force_dim;
#pragma unroll
            for (int j = 0; j < MPL; ++j) {
                const int m = mslot<T>(lane + j * G);
                if (m < NA) {
                    if constexpr (NM > 0) GAT(fo, m, a.force_dim) = D.ms[j].Ft;
                    else GAT(fo, m, a.force_dim) = control[j] * SM.ca_opt[m];
                }
            }
            if (lane < T::NF) {
                Real F[3] = {0, 0, 0}, Mo[3] = {0, 0, 0};
#pragma unroll
                for (int s2 = 0; s2 < T::NS; ++s2) {
                    const Real *cw = lds + LY::CW + 8 * s2;
                    const bool mine = SM.sph_force[s2] == lane;
#pragma unroll
                    for (int i = 0; i < 3; ++i) { F[i] += mine ? cw[i] : Real(0); Mo[i] += mine ? cw[3 + i] : Real(0); }
                }
                Mo[1] += -x0 * F[2];
                Mo[2] += x0 * F[1];
#pragma unroll
                for (int i = 0; i < 3; ++i) { GAT(fo, NA + 6 * lane + i, a.force_dim) = F[i]; GAT(fo, NA + 6 * lane + 3 + i, a.force_dim) = Mo[i]; }
            }
            if (lane < T::NL) GAT(fo, NA + 6 * T::NF + lane, a.force_dim) = lds[LY::LIM + 4 * lane];
            /* the contact record's foot-side entries: per sphere its force on
             * its OpenSim body and the moment about that body's origin (the
             * HuntCrossleyForce record sums these per body, in ground) */
            if (lane < T::NS) {
                const Real *cw = lds + LY::CW + 8 * lane;
                const Real *rp = lds + LY::REP + 6 * SM.sph_ob[lane];   /* body origin, absolute x */
                const Real O[3] = {rp[0] - x0, rp[1], rp[2]}, F[3] = {cw[0], cw[1], cw[2]};
                Real oxf[3];
                cross3(O, F, oxf);
                Real *fs = fo + NA + 6 * T::NF + T::NL + 6 * lane;
#pragma unroll
                for (int i = 0; i < 3; ++i) { fs[i] = F[i]; fs[3 + i] = cw[3 + i] - oxf[i]; }
            }
        }
        if constexpr (REP) {
            /* the observation rows first, so the report runs with ob's
             * addresses dead (the spatial push + RK report kernel is at 512) */
            wave_sync();
            if (obs)
                for (int k = lane; k < M.obs_dim; k += G) GAT(obs, (size_t)env * a.obs_stride + k, (size_t)N * a.obs_stride) = ob[k];
            wave_sync();
            if (a.osim_out)
                osim_report<T, Real>(M, SM, lds, lane, D, control, t, istep, a.osim_out + GIDX((size_t)env, (size_t)N) * a.osim_dim);
            break;
        }
        wave_sync();
        if (obs)
            for (int k = lane; k < M.obs_dim; k += G) GAT(obs, (size_t)env * a.obs_stride + k, (size_t)N * a.obs_stride) = ob[k];
        if (a.final_obs && !reported_reset)
            for (int k = lane; k < M.obs_dim; k += G) GAT(a.final_obs, (size_t)env * a.obs_stride + k, (size_t)N * a.obs_stride) = ob[k];
        wave_sync();
        if (reported_reset || osim) break;

#ifdef BIOIM_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long rp_t1 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
#endif
        /* ---- reward (get_reward) and termination (is_done); group sums are
         * xor butterflies, so every lane holds bitwise-identical totals */
        {
            const int r = clamp_row(istep, M.nrows);
            Real e2 = 0;
#pragma unroll
            for (int jc = 0; jc < CPL; ++jc) {
                const int c = lane + jc * G;
                if (c < T::NC) {
                    Real e = lds[LY::QF + c] - M.ref_q[r][c];
                    e2 += e * e;
                }
            }
            const Real qerr = group_sum<G>(e2) / Real(T::NC);
            Real eb = 0;
            if (lane < BIOIM_NREFBODY) {
                const Real *rp = lds + LY::REP + 6 * SM.rw_slot[lane];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    Real e = rp[i] - M.ref_x[r][lane][i];
                    eb += e * e;
                }
                eb /= Real(3);
            }
            /* rw bodies: 0 COM, 1/2 femur r/l, 3/4 tibia, 5/6 talus, 7/8 calcn */
            const bool odd = (lane & 1) != 0 && lane < BIOIM_NREFBODY, even = (lane & 1) == 0 && lane > 0 && lane < BIOIM_NREFBODY;
            const Real err_com = group_sum<G>(lane == 0 ? eb : Real(0));
            const Real err_r = group_sum<G>(odd ? eb : Real(0));
            const Real err_l = group_sum<G>(even ? eb : Real(0));
            Real position_r = exp(Real(-30) * qerr);
            Real com_r = exp(Real(-20) * err_com);
            Real foot_r = Real(0.5) * exp(Real(-20) * err_r);
            Real foot_l = Real(0.5) * exp(Real(-20) * err_l);
            Real pelvis_x = px;
            Real da2 = 0;
#pragma unroll
            for (int j = 0; j < MPL; ++j) {
                const Real da = lane + j * G < NA ? curr[j] - last[j] : Real(0);
                da2 += da * da;
            }
            Real action_r = exp(-M.action_r_scale * sqrt(group_sum<G>(da2)));
            Real effort, a_error = 0;
            if constexpr (NM > 0) {
                Real an = 0, cot = 0;
#pragma unroll
                for (int j = 0; j < MPL; ++j) {
                    const int m = mslot<T>(lane + j * G);
                    if (m < NM) {
                        an += D.ms[j].act * D.ms[j].act;
                        cot += muscle_cot<Real>(SM.mus[m], D.ms[j], control[j]);
                    }
                }
                a_error = exp(Real(-2) * sqrt(group_sum<G>(an)));
                cot = group_sum<G>(cot) + Real(1.51) * M.total_mass;
                effort = cot / (Real(20) * Real(NM * NM));
            } else {
                Real cn = 0;
#pragma unroll
                for (int j = 0; j < MPL; ++j) cn += lane + j * G < NA ? curr[j] * curr[j] : Real(0);
                effort = sqrt(group_sum<G>(cn)) / (M.max_actuation * Real(NA * NA));
            }
            Real effort_r = exp(-effort / fmax(pelvis_x - old_px + Real(1), Real(1)));
            Real imit = position_r * com_r;
            if constexpr ((T::FLAGS & BIOIM_ENV_REWARD_FEET) != 0) imit *= (foot_l + foot_r);
            rew = (Real(0.5) + M.w_imitate) * imit + M.w_effort * effort_r + M.w_action * action_r;
            inf[0] = position_r; inf[1] = com_r; inf[2] = foot_l; inf[3] = foot_r; inf[4] = a_error;
#pragma unroll
            for (int j = 0; j < MPL; ++j) last[j] = curr[j];
            old_px = pelvis_x;
            /* is_done (muscle_walking_imitation_env2D.py:237-265) */
            const Real torso_y = lds[LY::REP + 6 * T::TORSO + 1];
            Real lmax = 0, amax = 0;
#pragma unroll
            for (int li = 0; li < T::NL; ++li) lmax = fmax(lmax, fabs(lds[LY::LIM + 4 * li]));
            amax = group_max<G>(lane < ND ? fabs(D.qdd) : Real(0));
            int d_ = 0;
            if (torso_y < M.torso_y_min) d_ = 1;
            else if (lmax > M.limit_force_max) d_ = 1;
            else if (amax > M.acc_max) d_ = 1;
            else if (istep >= M.n_episode) d_ = 1;
            else if constexpr ((T::FLAGS & BIOIM_ENV_DONE_CROSS) != 0) {
                if (lds[LY::REP + 6 * T::CALCN_R + 2] - lds[LY::REP + 6 * T::CALCN_L + 2] < 0) d_ = 1;
            }
            if (group_any<G>(lane < ND && (!isfinite(qd) || !isfinite(ud)))) d_ = 1;
            if (!D.ok || rk_fail) d_ = 1;
            done = d_;
        }
        if (lane == 0) {
            if (a.reward) GAT(a.reward, env, N) = rew;
            GAT(a.done_out, env, N) = (uint8_t)done;
        }
        if (a.info && lane < M.info_dim) {
            Real iv = inf[0];
#pragma unroll
            for (int i = 1; i < 5; ++i) iv = lane == i ? inf[i] : iv;
            GAT(a.info, (size_t)env * a.info_stride + lane, (size_t)N * a.info_stride) = iv;
        }
        wave_sync();
#ifdef BIOIM_STAMPS
        {   /* the report of the first env of workgroup 0: observation part, reward + done part, reports */
            __builtin_amdgcn_sched_barrier(0);
            const unsigned long long rp_t2 = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_s_waitcnt(0xC07F);
            if (blockIdx.x == 0 && threadIdx.x == 0) { g_stamps[19] += rp_t1 - rp_t0; g_stamps[20] += rp_t2 - rp_t1; g_stamps[21] += 1; }
            __builtin_amdgcn_sched_barrier(0);
        }
#endif
        if (done && a.auto_reset) {
            pending_reset = true;
            do_reset = true;
            reset_row = draw_index(a.seed, a.env_offset + env, resets, M.reset_hi);
            if constexpr ((!RK || (BIOIM_RESET_TAB_RK && (T::PLANAR || BIOIM_RESET_TAB_RK_SPATIAL))) && !PERT && !REP) {
                /* the reset table (LaunchArgs::reset_tab): the state the reset
                 * realize would leave (reference row, default activation,
                 * equilibrium fiber lengths) and its observation, without a
                 * dynamics call and fiber equilibrium in this wave — they made
                 * the launch wait for its slowest wave.  Torque
                 * models: the observation's q'' holds the held torques, so the
                 * row carries M^-1 too and q''_d = q''_d(0) + (M^-1 tau)_d */
                if (a.reset_tab) {
                    const int r = clamp_row(reset_row, M.nrows);
                    const Real *tr = a.reset_tab + (size_t)r * a.reset_tab_dim;
                    if (lane < ND) {
                        const int c = SM.dof_coord[lane];
                        qd = M.ref_q[r][c];
                        ud = M.ref_u[r][c];
                    }
                    t = M.ref_time[r];
                    istep = M.ref_istep[r];
                    has_last = 0;
                    rk_hnext = 0;   /* reset_manager: a new integrator (opensim_wrapper.py:287-291) */
                    resets += 1;
                    if constexpr (RK) launch_evals -= 1;   /* no reset realize ran: not an evaluation */
                    if constexpr (NM > 0) {
#pragma unroll
                        for (int j = 0; j < MPL; ++j) {
                            const int m = mslot<T>(lane + j * G);
                            if (m < NM) { act[j] = SM.mus[m].default_act; lce[j] = tr[m]; }
                        }
                        if (obs)
                            for (int k = lane; k < M.obs_dim; k += G)
                                GAT(obs, (size_t)env * a.obs_stride + k, (size_t)N * a.obs_stride) = tr[NM + k];
                        if constexpr (CACHE) {   /* the row's realize cache (after its observation) */
                            using CL = CacheLay<T>;
                            const Real *tc = tr + NM + M.obs_dim;
                            Real *const crow = CI.row();
                            for (int k = lane; k < CL::DIM; k += G) GAT(crow, k, CL::DIM) = tc[k];
                        }
                    } else {
                        /* the held torques per dof, gathered as in the dynamics
                         * call (TAU slots, SM.tau_src), then q'' per dof lane */
                        constexpr int NI = ND * ND;
                        if (lane == 0) lds[LY::TAU + LY::TZ] = Real(0);
#pragma unroll
                        for (int j = 0; j < MPL; ++j) {
                            const int m = mslot<T>(lane + j * G);
                            if (m < NA) lds[LY::TAU + (lane + j * G) * T::MAXSPAN] = control[j] * SM.ca_opt[m];
                        }
                        wave_sync();
                        if (lane < ND) {
                            Real tau = 0;
#pragma unroll
                            for (int i = 0; i < T::MAXARM; ++i) tau += lds[LY::TAU + SM.tau_src[lane][i]];
                            lds[LY::RHS + lane] = tau;
                        }
                        wave_sync();
                        Real *ob = lds + LY::OBS;
                        for (int k = lane; k < M.obs_dim; k += G) ob[k] = tr[NI + k];
                        wave_sync();
                        if (lane < ND) {
                            using OL = ObsLayout<T>;
                            const int c = SM.dof_coord[lane];
                            Real x = ob[OL::QACC + c];
#pragma unroll
                            for (int k = 0; k < ND; ++k) x = fma(tr[lane * ND + k], lds[LY::RHS + k], x);
                            ob[OL::QACC + c] = x;
                        }
                        wave_sync();
                        if (obs)
                            for (int k = lane; k < M.obs_dim; k += G)
                                GAT(obs, (size_t)env * a.obs_stride + k, (size_t)N * a.obs_stride) = ob[k];
                        if constexpr (CACHE) {   /* the row's realize cache (after its observation) */
                            using CL = CacheLay<T>;
                            const Real *tc = tr + NI + M.obs_dim;
                            Real *const crow = CI.row();
                            for (int k = lane; k < CL::DIM; k += G) GAT(crow, k, CL::DIM) = tc[k];
                        }
                    }
                    break;
                }
            }
            continue;
        }
        break;
    }

#ifdef BIOIM_STAMPS
    if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[10] += __builtin_amdgcn_s_memtime() - k_t1;
#endif
    /* ---- store state */
        if (lane == 0) {
        GAT(st.t, env, (size_t)N) = t;
        GAT(st.istep, env, (size_t)N) = istep;
        if (!REP) {
            GAT(st.has_last, env, (size_t)N) = has_last;
            GAT(st.old_px, env, (size_t)N) = old_px;
            GAT(st.done, env, (size_t)N) = (mode == 0 && !do_reset && !suspend) ? done : 0;
            GAT(st.resets, env, (size_t)N) = resets;
        }
        if (RK || mode == 1 || (osim && a.osim_op == BIOIM_OSIM_EQUILIBRATE)) GAT(st.hrk, env, (size_t)N) = rk_hnext;
        /* the realize cache: every step or reset of a CACHE kernel ends with a
         * realize (or a reset-table row) that formed this env's row.  The other
         * kernels of such a topology (push, RK, OsimModel calls) change the
         * state without it: the host clears the flags before launching them
         * (launch_impl; a store here cost the spatial push + RK kernel its
         * last registers) */
        if constexpr (CACHE) GAT(st.cache_ok, env, (size_t)N) = 1;
        if constexpr (RK) {
            GAT(st.pend, env, (size_t)N) = suspend ? 1 : 0;
            /* evaluations (low 32 bits): the attempts', plus one realize per
             * finished step and per reset that ran one (a reset-table reset
             * took one back, see above); finished steps (high 32 bits).  Two
             * independent wrapping halves: no carry from one into the other */
            const uint64_t ev0 = GAT(st.rkev, env, (size_t)N);
            const uint32_t ev_lo = (uint32_t)ev0 + (uint32_t)(launch_evals + (suspend ? 0 : 1) + (do_reset && mode == 0 ? 1 : 0));
            const uint32_t ev_hi = (uint32_t)(ev0 >> 32) + (uint32_t)(mode == 0 && !suspend);
            GAT(st.rkev, env, (size_t)N) = ((uint64_t)ev_hi << 32) | ev_lo;
            if (a.traj && (mode == 0 || (osim && a.osim_op == BIOIM_OSIM_INTEGRATE))) GAT(a.traj_n, env, N) = traj_k;
            if (suspend) {
                GAT(st.rkt, env, (size_t)N) = rk_t; GAT(st.rkh, env, (size_t)N) = rk_h; GAT(st.rka, env, (size_t)N) = rk_attempts;
                GAT(a.done_out, env, N) = 0;
            }
            if (mode == 0 && a.ready_out) GAT(a.ready_out, env, N) = suspend ? 0 : 1;
        }
    }
    if (RK && suspend) {
#pragma unroll
        for (int j = 0; j < MPL; ++j) {
            const int m = mslot<T>(lane + j * G);
            if (m < NA) GAT(st.cur, (size_t)m * N + env, (size_t)NA * N) = curr[j];
            if (NM > 0 && m < NM) GAT(st.vnw, (size_t)m * N + env, (size_t)(NM > 0 ? NM : 1) * N) = D.ms[j].vN;
        }
    }
    if (lane < ND) {
        GAT(st.q, (size_t)lane * N + env, (size_t)ND * N) = qd;
        GAT(st.u, (size_t)lane * N + env, (size_t)ND * N) = ud;
    }
#pragma unroll
    for (int j = 0; j < MPL; ++j) {
        const int m = mslot<T>(lane + j * G);
        if (NM > 0 && m < NM) { GAT(st.act, (size_t)m * N + env, (size_t)(NM > 0 ? NM : 1) * N) = act[j]; GAT(st.lce, (size_t)m * N + env, (size_t)(NM > 0 ? NM : 1) * N) = lce[j]; }
        if (!REP && m < NA) GAT(st.last, (size_t)m * N + env, (size_t)NA * N) = last[j];
    }
}

/* REP: the OsimModel-call kernels (mode 2, bioim_osim): the same code plus
 * the full realize report; separate instantiations, so the step kernels are
 * untouched by it */
template <class T, typename Real, bool PERT, bool RK, bool REP = false>
__global__ __launch_bounds__(BIOIM_EPB * T::G) __attribute__((amdgpu_waves_per_eu(1, 1))) void env_kernel(LaunchArgs<T, Real> a) {
#ifdef BIOIM_WAVETIME
    const unsigned long long w0 = __builtin_amdgcn_s_memtime();
    if (diag_tid() < BIOIM_WAVETIME_N * 4) { g_fvit[diag_tid()] = 0; g_fvmax[diag_tid()] = 0; g_fvbis[diag_tid()] = 0; }
#endif
    env_block<T, Real, PERT, RK, REP>(a, blockIdx.x);
#ifdef BIOIM_WAVETIME
    const unsigned w = blockIdx.x * (BIOIM_EPB * T::G / 64) + threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0 && w < BIOIM_WAVETIME_N) g_wavetime[w] = __builtin_amdgcn_s_memtime() - w0;
#endif
}


/* Fused two-topology step (a mixed batch, config C5, in ONE launch):
 * workgroups [0, a0.blocks) step segment 0 with topology T0, the rest segment
 * 1 with T1.  Both segments are the default step kernels' code (no push
 * table, semi-implicit); the two bodies sit in one kernel, so its registers
 * are the larger of the two (the 3D pair: 462, no scratch, hazard gate clean).
 * Instantiated for the pairs in BIOIM_FUSED_PAIRS, in the library's fused
 * unit (-DBIOIM_FUSED_ONLY). */
template <class T0, class T1, typename Real>
__global__ __launch_bounds__(BIOIM_EPB * T0::G) __attribute__((amdgpu_waves_per_eu(1, 1))) void env_kernel2(
    LaunchArgs<T0, Real> a0, LaunchArgs<T1, Real> a1) {
    static_assert(T0::G == T1::G, "a fused launch needs one workgroup shape");
    if ((int)blockIdx.x < a0.blocks) env_block<T0, Real, false, false, false>(a0, blockIdx.x);
    else env_block<T1, Real, false, false, false>(a1, blockIdx.x - a0.blocks);
}

#define BIOIM_FUSED_PAIRS(X)                                                         \
    X(Topo_MuscleLockedKneeImitation3D_v0, Topo_MuscleWalkingImitation3D_v0)          \
    X(Topo_MuscleWalkingImitation3D_v0, Topo_MuscleLockedKneeImitation3D_v0)

/* =================================================================== host
 * Build modes (the library links 8 objects compiled in parallel):
 *   BIOIM_TOPO_ONLY=k  the kernels and host launchers of topology k only
 *                      (bioim_pick_k);
 *   BIOIM_ABI_ONLY     the C-ABI, no kernels;
 *   BIOIM_FUSED_ONLY   the fused two-topology kernels (BIOIM_FUSED_PAIRS) and their launcher;
 *   neither            everything in one translation unit (diagnostic builds). */
#if defined(BIOIM_TOPO_ONLY) + defined(BIOIM_ABI_ONLY) + defined(BIOIM_FUSED_ONLY) > 1
#error "BIOIM_TOPO_ONLY, BIOIM_ABI_ONLY and BIOIM_FUSED_ONLY are exclusive"
#endif
extern thread_local std::string g_err;   /* bioim_last_error(); defined with the C-ABI */

namespace {

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                       \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) return fail(BIOIM_E_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

double host_bez5(const double *p, double u) {
    double v = 1.0 - u;
    return p[0] * v * v * v * v * v + 5 * p[1] * u * v * v * v * v + 10 * p[2] * u * u * v * v * v +
           10 * p[3] * u * u * u * v * v + 5 * p[4] * u * u * u * u * v + p[5] * u * u * u * u * u;
}

double host_dbez5(const double *p, double u) {
    double v = 1.0 - u;
    return 5 * ((p[1] - p[0]) * v * v * v * v + 4 * (p[2] - p[1]) * u * v * v * v +
                6 * (p[3] - p[2]) * u * u * v * v + 4 * (p[4] - p[3]) * u * u * u * v + (p[5] - p[4]) * u * u * u * u);
}

/* exact inverse of the monotone quintic x(u) by bisection (host, table build) */
double host_invert(const double *px, double x) {
    double lo = 0.0, hi = 1.0;
    for (int it = 0; it < 200; ++it) {
        double m = 0.5 * (lo + hi);
        if (host_bez5(px, m) > x) hi = m; else lo = m;
    }
    return 0.5 * (lo + hi);
}

/* y(x) of a pack curve, to machine precision (the device's curve_eval
 * semantics: linear extrapolation outside [x0, x1]) */
double host_curve_y(const bioim_curve_t &s, double x) {
    if (x < s.x0) return s.y0 + s.dydx0 * (x - s.x0);
    if (x > s.x1) return s.y1 + s.dydx1 * (x - s.x1);
    int k = 0;
    while (k < s.nseg - 1 && x > s.x[k][5]) ++k;
    return host_bez5(s.y[k], host_invert(s.x[k], x));
}

/* Bernstein control points of a quintic -> power-basis coefficients:
 * c_j = C(5, j) sum_{k <= j} C(j, k) (-1)^(j-k) p_k */
void bernstein_to_power(const double *p, double *c) {
    static const double B5[6] = {1, 5, 10, 10, 5, 1};
    for (int j = 0; j < 6; ++j) {
        double s = 0, bjk = 1;   /* C(j, k) */
        for (int k = 0; k <= j; ++k) {
            s += bjk * (((j - k) & 1) ? -p[k] : p[k]);
            bjk = bjk * (j - k) / (k + 1);
        }
        c[j] = B5[j] * s;
    }
}

template <typename Real> void convert_curve(const bioim_curve_t &s, DCurve<Real> &d) {
    for (int i = 0; i < BIOIM_MAX_CURVESEG; ++i) {
        double cx[6], cy[6];
        bernstein_to_power(s.x[i], cx);
        bernstein_to_power(s.y[i], cy);
        for (int j = 0; j < 6; ++j) { d.cx[i][j] = (Real)cx[j]; d.cy[i][j] = (Real)cy[j]; }
        d.xa[i] = i < s.nseg ? (Real)s.x[i][0] : (Real)INFINITY; d.xb[i] = (Real)s.x[i][5];
        d.ya[i] = i < s.nseg ? (Real)s.y[i][0] : Real(0); d.yb[i] = (Real)s.y[i][5];
        d.xsep[i] = i < s.nseg - 1 ? (Real)s.x[i][5] : (Real)INFINITY;
    }
    for (int k = 0; k < BIOIM_MAX_CURVESEG; ++k) {
        if (k >= s.nseg) {
            d.inv_h[k] = 0;
            for (int i = 0; i <= BIOIM_UTAB; ++i) d.ut[k][i] = d.mt[k][i] = 0;
            continue;
        }
        double a = s.x[k][0], b = s.x[k][5];
        d.inv_h[k] = (Real)(BIOIM_UTAB / (b - a));
        for (int i = 0; i <= BIOIM_UTAB; ++i) {
            double u = host_invert(s.x[k], a + (b - a) * i / BIOIM_UTAB);
            d.ut[k][i] = (float)u;
            /* du/dt = (dx/dt) / (dx/du), dx/dt = (b - a) / BIOIM_UTAB */
            d.mt[k][i] = (float)((b - a) / BIOIM_UTAB / host_dbez5(s.x[k], u));
        }
    }
    d.x0 = (Real)s.x0; d.y0 = (Real)s.y0; d.dydx0 = (Real)s.dydx0;
    d.x1 = (Real)s.x1; d.y1 = (Real)s.y1; d.dydx1 = (Real)s.dydx1;
    d.y_at0 = s.nseg > 0 ? (Real)host_curve_y(s, 0.0) : Real(0);
    d.nseg = s.nseg;
}

template <typename Real> void convert_model(const bioim_modelpack_t &p, DModel<Real> &m) {
    memset(&m, 0, sizeof(m));
    for (int c = 0; c < p.ncbody; ++c) {
        for (int i = 0; i < 3; ++i) m.com[c][i] = (Real)p.cbody[c].com[i];
        m.mass[c] = (Real)p.cbody[c].mass;
    }
    for (int c = 0; c < p.ncoord; ++c) { m.coord_default[c] = (Real)p.coord[c].default_value; m.coord_dof[c] = p.coord[c].dof; }
    for (int b = 0; b < p.nosbody; ++b) {
        for (int i = 0; i < 9; ++i) m.os_R[b][i] = (Real)p.osbody[b].R[i];
        for (int i = 0; i < 3; ++i) m.os_p[b][i] = (Real)p.osbody[b].p[i];
    }
    m.w_imitate = (Real)p.w_imitate; m.w_effort = (Real)p.w_effort; m.w_action = (Real)p.w_action;
    m.action_r_scale = (Real)p.action_r_scale; m.max_actuation = (Real)p.max_actuation;
    m.total_mass = (Real)p.total_mass;
    double wgt = fabs(p.total_mass * p.gravity[1]);
    m.weight = (Real)wgt;
    m.moment = (Real)(wgt * p.height);
    m.torso_y_min = (Real)p.torso_y_min; m.limit_force_max = (Real)p.limit_force_max; m.acc_max = (Real)p.acc_max;
    for (int i = 0; i < 3; ++i) m.gravity[i] = (Real)p.gravity[i];
    m.float_origin = 1;
    m.horizon = p.horizon; m.cycle = p.cycle; m.n_episode = p.n_episode; m.reset_hi = p.reset_hi;
    m.nsub = p.nsub; m.nrows = p.nrows; m.obs_dim = p.obs_dim; m.info_dim = p.info_dim; m.env_flags = p.env_flags;
    m.step_size = p.step_size;
    for (int r = 0; r < p.nrows; ++r) {
        m.ref_time[r] = p.ref_time[r];
        m.ref_istep[r] = p.ref_istep[r];
        for (int c = 0; c < p.ncoord; ++c) { m.ref_q[r][c] = (Real)p.ref_q[r][c]; m.ref_u[r][c] = (Real)p.ref_u[r][c]; }
        for (int b = 0; b < BIOIM_NREFBODY; ++b)
            for (int i = 0; i < 3; ++i) m.ref_x[r][b][i] = (Real)p.ref_x[r][b][i];
    }
}

/* distinct muscle curves in first-appearance order over (fal, fv, fpe, fse)
 * of each muscle (tools/build_packs.py: unique_curves) */
static std::vector<const bioim_curve_t *> unique_curves(const bioim_modelpack_t &p, std::vector<int> *index) {
    std::vector<const bioim_curve_t *> u;
    for (int i = 0; i < p.nmuscle; ++i) {
        const bioim_curve_t *cs[4] = {&p.muscle[i].fal, &p.muscle[i].fv, &p.muscle[i].fpe, &p.muscle[i].fse};
        for (const bioim_curve_t *c : cs) {
            int k = 0;
            while (k < (int)u.size() && memcmp(u[k], c, sizeof(bioim_curve_t)) != 0) ++k;
            if (k == (int)u.size()) u.push_back(c);
            if (index) index->push_back(k);
        }
    }
    return u;
}

/* the LDS model image of a pack (layout: bioim_device.h, SModel) */
template <class T, typename Real> void build_smodel(const bioim_modelpack_t &p, SModel<T, Real> &m) {
    memset(&m, 0, sizeof(m));
    std::vector<int> cidx;
    std::vector<const bioim_curve_t *> cu = unique_curves(p, &cidx);
    for (size_t k = 0; k < cu.size(); ++k) convert_curve(*cu[k], m.curve[k]);
    for (int i = 0; i < p.nmuscle; ++i) {
        const bioim_muscle_t &s = p.muscle[i];
        SMuscle<Real> &d = m.mus[i];
        d.fiso = (Real)s.fiso; d.lopt = (Real)s.lopt; d.inv_lopt = (Real)(1.0 / s.lopt);
        d.lts = (Real)s.lts; d.inv_lts = (Real)(1.0 / s.lts); d.lv = (Real)(s.lopt * s.vmax);
        d.tau_act = (Real)s.tau_act; d.tau_deact = (Real)s.tau_deact; d.amin = (Real)s.amin; d.beta = (Real)s.damping;
        d.width = (Real)s.width; d.lmin = (Real)s.lmin; d.slow = (Real)s.slow_twitch; d.mass = (Real)s.mass;
        d.default_act = (Real)s.default_act; d.pt_off = s.pt_off; d.npt = s.npt;
        for (int k = 0; k < 4; ++k) d.cv[k] = cidx[4 * i + k];
        uint32_t root = ~0u, u = 0;
        for (int c = 0; c < T::NB; ++c) root &= T::dofmask[c];
        for (int j = 0; j < s.npt; ++j) u |= T::dofmask[p.pathpt[s.pt_off + j].cbody];
        u &= ~root;
        d.nspan = 0;
        for (int dd = 0; dd < T::ND; ++dd)
            if ((u >> dd) & 1u) d.span[d.nspan++] = dd;
        for (int k = d.nspan; k < BIOIM_MAX_SPAN; ++k) d.span[k] = d.nspan ? d.span[0] : 0;
    }
    {   /* muscle torque gather lists (Lay::TZ: the zero slot) */
        using LY = Lay<T, Real>;
        static_assert(LY::TZ < 256, "TAU slot indices are bytes");
        for (int d = 0; d < SDim<T>::NDD; ++d)
            for (int i = 0; i < T::MAXARM; ++i) m.tau_src[d][i] = (uint8_t)LY::TZ;
        int cnt[SDim<T>::NDD] = {};
        auto add = [&](int d, int slot) {
            if (d >= 0 && d < T::ND && cnt[d] < T::MAXARM) m.tau_src[d][cnt[d]++] = (uint8_t)slot;
        };
        for (int sl = 0; sl < LY::MPL * T::G; ++sl) {
            const int mi = (T::NM > T::G && sl < T::NM) ? T::mperm[sl] : sl;
            if constexpr (T::NM > 0) {
                if (mi < p.nmuscle)
                    for (int k = 0; k < m.mus[mi].nspan; ++k) add(m.mus[mi].span[k], sl * T::MAXSPAN + k);
            } else {
                if (mi < T::NA) add(T::act_dof[mi], sl * T::MAXSPAN);
            }
        }
    }
    std::vector<uint32_t> dofmask(T::NB, 0);
    for (int c = 0; c < T::NB; ++c) dofmask[c] = T::dofmask[c];
    int nmf = 0;
    for (int j = 0; j < p.npathpt; ++j) {
        const bioim_pathpt_t &s = p.pathpt[j];
        DPathPt<Real> &d = m.pt[j];
        d.type = s.type; d.cbody = s.cbody; d.cond_coord = s.cond_coord;
        d.mcoord = -1; d.mdof = -1;
        for (int a = 0; a < 3; ++a) {
            d.mf[a] = -1;
            if (s.type == BIOIM_PT_MOVING && s.fn[a] >= 0) {
                d.mcoord = p.fn[s.fn[a]].coord;
                d.mdof = d.mcoord >= 0 ? p.coord[d.mcoord].dof : -1;
                if (nmf < T::NMF) {
                    m.mf_fn[nmf] = s.fn[a];
                    m.mf_coord[nmf] = p.fn[s.fn[a]].coord;
                    d.mf[a] = nmf;
                }
                ++nmf;
            }
        }
        d.dofmask = dofmask[s.cbody];
        for (int i = 0; i < 3; ++i) { d.loc[i] = (Real)s.loc[i]; d.p[i] = (Real)s.p[i]; }
        for (int i = 0; i < 9; ++i) d.R[i] = (Real)s.R[i];
        d.lo = (Real)s.range_lo; d.hi = (Real)s.range_hi;
    }
    int jslot = T::NMF;   /* joint spline slots follow the moving-point ones */
    for (int c = 0; c < p.ncbody; ++c) {
        const bioim_cbody_t &b = p.cbody[c];
        SBody<Real> &d = m.body[c];
        for (int a = 0; a < 6; ++a) {
            const int fi = p.cbody[c].fn[a];
            if (fi >= 0 && p.fn[fi].type == BIOIM_FN_SPLINE && jslot < TopoInfo<T>::nslot()) {
                m.mf_fn[jslot] = fi;   /* slot TopoInfo<T>::jslot(c, a) */
                m.mf_coord[jslot] = p.fn[fi].coord;
                ++jslot;
            }
        }
        for (int i = 0; i < 9; ++i) { d.R_pf[i] = (Real)b.R_pf[i]; d.R_mb[i] = (Real)b.R_mb[i]; }
        for (int i = 0; i < 3; ++i) { d.p_pf[i] = (Real)b.p_pf[i]; d.p_mb[i] = (Real)b.p_mb[i]; d.com[i] = (Real)b.com[i]; }
        for (int a = 0; a < 6; ++a) {
            for (int i = 0; i < 3; ++i) d.axis[a][i] = (Real)b.axis[a][i];
            d.fa[a] = b.fn[a] >= 0 ? (Real)p.fn[b.fn[a]].a : Real(0);
            d.fb[a] = b.fn[a] >= 0 ? (Real)p.fn[b.fn[a]].b : Real(0);
        }
        d.mass = (Real)b.mass;
        for (int i = 0; i < 6; ++i) d.inertia[i] = (Real)b.inertia[i];
        d.pslot = b.parent >= 0 ? b.parent : T::NB;
        d.pad = 0;
        constexpr int DEP = TopoInfo<T>::depth();
        int path[DEP], n = 0;
        for (int q = c; q >= 0 && n < DEP; q = p.cbody[q].parent) path[n++] = q;
        for (int l = 0; l < DEP; ++l) m.chain[c][l] = l < DEP - n ? T::NB : path[DEP - 1 - l];
    }
    for (int f = 0; f < p.nfn; ++f) {
        m.fn[f].type = p.fn[f].type; m.fn[f].coord = p.fn[f].coord; m.fn[f].off = p.fn[f].knot_off;
        m.fn[f].n = p.fn[f].nknots; m.fn[f].a = (Real)p.fn[f].a; m.fn[f].b = (Real)p.fn[f].b;
    }
    for (int k = 0; k < p.nknots; ++k) {
        m.kx[k] = (Real)p.knot_x[k]; m.ky[k] = (Real)p.knot_y[k]; m.kb[k] = (Real)p.knot_b[k];
        m.kc[k] = (Real)p.knot_c[k]; m.kd[k] = (Real)p.knot_d[k];
    }
    for (int s = 0; s < p.nsphere; ++s) {
        for (int i = 0; i < 3; ++i) m.sph_loc[s][i] = (Real)p.sphere[s].loc[i];
        m.sph_r[s] = (Real)p.sphere[s].radius;
        m.sph_cb[s] = p.sphere[s].cbody; m.sph_force[s] = p.sphere[s].force; m.sph_ob[s] = p.sphere[s].obody;
    }
    for (int f = 0; f < p.ncforce; ++f) {
        const bioim_cforce_t &c = p.cforce[f];
        m.cf_kk[f] = (Real)(0.5 * pow(c.stiffness, 2.0 / 3.0));
        m.cf_c[f] = (Real)c.dissipation; m.cf_ms[f] = (Real)c.static_friction; m.cf_md[f] = (Real)c.dynamic_friction;
        m.cf_mv[f] = (Real)c.viscous_friction; m.cf_vt[f] = (Real)c.transition_velocity;
    }
    for (int l = 0; l < p.nlimit; ++l) {
        const bioim_limit_t &s = p.limit[l];
        m.lim_qup[l] = (Real)s.qup; m.lim_qlow[l] = (Real)s.qlow; m.lim_kup[l] = (Real)s.kup;
        m.lim_klow[l] = (Real)s.klow; m.lim_damp[l] = (Real)s.damping; m.lim_trans[l] = (Real)s.trans;
        m.lim_itrans[l] = (Real)(1.0 / s.trans);
        m.lim_coord[l] = s.coord; m.lim_dof[l] = s.dof;
    }
    for (int a = 0; a < p.ncoordact; ++a) {
        m.ca_opt[a] = (Real)p.coordact[a].optimal_force;
        m.ca_min[a] = (Real)p.coordact[a].min_control;
        m.ca_max[a] = (Real)p.coordact[a].max_control;
        m.act_dof[a] = p.coordact[a].dof;
    }
    for (int a = 0; a < p.nact && a < SDim<T>::NAD; ++a) { m.kp[a] = (Real)p.kp[a]; m.kv[a] = (Real)p.kv[a]; }
    for (int c = 0; c < p.ncoord; ++c) m.coord_dof[c] = p.coord[c].dof;
    for (int c = 0; c < p.ncoord; ++c)
        if (p.coord[c].dof >= 0) { m.dof_cb[p.coord[c].dof] = p.coord[c].cbody; m.dof_coord[p.coord[c].dof] = c; }
    for (int c = 0; c < T::NB; ++c) m.dofmask[c] = T::dofmask[c];
    for (int b = 0; b < T::NOBP; ++b) m.obs_slot[b] = T::obs_bpos[b] >= 0 ? T::obs_bpos[b] : T::NOS;
    for (int b = 0; b < T::NOBV; ++b) m.obs_slot[T::NOBP + b] = T::obs_bvel[b] >= 0 ? T::obs_bvel[b] : T::NOS;
    for (int b = 0; b < BIOIM_NREFBODY; ++b) m.rw_slot[b] = T::rw_body[b] >= 0 ? T::rw_body[b] : T::NOS;
    for (int b = 0; b < T::NOS; ++b) {
        m.os_cb[b] = p.osbody[b].cbody;
        for (int i = 0; i < 3; ++i) m.os_p[b][i] = (Real)p.osbody[b].p[i];
    }
}

/* structural match of a pack against a compiled topology */
/* the pack keeps every motion in the x-y plane (tools/build_packs.py:
 * is_planar; the PLANAR kernels carry planar frames' zeros as constants) */
static bool pack_is_planar(const bioim_modelpack_t &p) {
    auto zrot = [](const double *R) { return R[2] == 0 && R[5] == 0 && R[6] == 0 && R[7] == 0 && R[8] == 1; };
    for (int c = 0; c < p.ncbody; ++c) {
        const bioim_cbody_t &b = p.cbody[c];
        if (!zrot(b.R_pf) || !zrot(b.R_mb)) return false;
        for (int a = 0; a < 6; ++a) {
            const int fi = b.fn[a];
            if (fi < 0) continue;
            if (a < 3 && !(b.axis[a][0] == 0 && b.axis[a][1] == 0)) return false;
            if (a >= 3 && p.fn[fi].type != BIOIM_FN_CONST && b.axis[a][2] != 0) return false;
        }
    }
    return p.gravity[2] == 0;
}

template <class T> bool topology_matches(const bioim_modelpack_t &p) {
    if (T::PLANAR && !pack_is_planar(p)) return false;
    if (p.ncbody != T::NB || p.ndof != T::ND || p.ncoord != T::NC || p.nmuscle != T::NM || p.nact != T::NA ||
        p.nsphere != T::NS || p.ncforce != T::NF || p.nlimit != T::NL || p.nosbody != T::NOS ||
        p.n_obs_bpos != T::NOBP || p.n_obs_bvel != T::NOBV)
        return false;
    if (p.coord_tx != T::TX || p.coord_ty != T::TY || p.coord_tz != T::TZ) return false;
    for (int s = 0; s < p.nsphere; ++s)   /* the report slot a sphere's foot-side record reads */
        if (p.sphere[s].obody < 0 || p.sphere[s].obody >= p.nosbody || T::os_cb[p.sphere[s].obody] != p.sphere[s].cbody)
            return false;
    if (p.npathpt != T::NPT || p.nfn != T::NFN || p.nknots != T::NKNOT) return false;
    {   /* moving-point function slots and muscle spans fit the compiled sizes */
        int nmf = 0;
        for (int j = 0; j < p.npathpt; ++j)
            for (int a = 0; a < 3; ++a) nmf += (p.pathpt[j].type == BIOIM_PT_MOVING && p.pathpt[j].fn[a] >= 0) ? 1 : 0;
        if (nmf != T::NMF) return false;
        uint32_t root = ~0u;
        for (int c = 0; c < T::NB; ++c) root &= T::dofmask[c];
        int arms[32] = {};
        for (int i = 0; i < p.nmuscle; ++i) {
            uint32_t u = 0;
            for (int j = 0; j < p.muscle[i].npt; ++j) u |= T::dofmask[p.pathpt[p.muscle[i].pt_off + j].cbody];
            if (__builtin_popcount(u & ~root) > T::MAXSPAN || T::MAXSPAN > BIOIM_MAX_SPAN) return false;
            for (int d = 0; d < T::ND; ++d) arms[d] += ((u & ~root) >> d) & 1u;
        }
        for (int d = 0; d < T::ND; ++d)
            if (arms[d] > T::MAXARM) return false;
    }
    for (int f = 0; f < p.nfn; ++f)
        if (p.fn[f].nknots > T::NKMAX) return false;
    if ((int)unique_curves(p, nullptr).size() != T::NCURVE) return false;
    if (p.nmuscle == 0 && p.nact > SDim<T>::NAD) return false;
    if (p.torso_body != T::TORSO || p.calcn_r_body != T::CALCN_R || p.calcn_l_body != T::CALCN_L) return false;
    if ((p.env_flags & BIOIM_STRUCT_FLAGS) != T::FLAGS) return false;
    for (int c = 0; c < T::NB; ++c) {
        if (p.cbody[c].parent != T::parent[c]) return false;
        uint32_t m = 1u << c;
        for (int q = p.cbody[c].parent; q >= 0; q = p.cbody[q].parent) m |= 1u << q;
        if (m != T::anc[c]) return false;
        for (int a = 0; a < 6; ++a) {
            int fi = p.cbody[c].fn[a];
            int kind = fi < 0 ? -1 : p.fn[fi].type, cc = fi < 0 ? -1 : p.fn[fi].coord;
            if (kind != T::axis_kind[c * 6 + a] || cc != T::axis_coord[c * 6 + a]) return false;
        }
    }
    for (int c = 0; c < T::NC; ++c)
        if (p.coord[c].dof != T::coord_dof[c]) return false;
    for (int c = 0; c < T::NC; ++c) {
        int d = p.coord[c].dof;
        if (d >= 0 && (p.coord[c].cbody != T::dof_cb[d] || T::dof_coord[d] != c)) return false;
    }
    for (int s = 0; s < T::NS; ++s)
        if (p.sphere[s].cbody != T::sphere_cb[s] || p.sphere[s].force != T::sphere_force[s]) return false;
    for (int b = 0; b < T::NOS; ++b)
        if (p.osbody[b].cbody != T::os_cb[b]) return false;
    for (int l = 0; l < T::NL; ++l)
        if (p.limit[l].dof != T::limit_dof[l] || p.limit[l].coord != T::limit_coord[l]) return false;
    if (p.nmuscle == 0) {
        int arms[32] = {};
        for (int a = 0; a < T::NA; ++a) {
            if (p.coordact[a].dof != T::act_dof[a] || p.pd_coord[a] != T::pd_coord[a] || p.pd_vcoord[a] != T::pd_vcoord[a])
                return false;
            if (T::act_dof[a] >= 0 && ++arms[T::act_dof[a]] > T::MAXARM) return false;
        }
    }
    for (int b = 0; b < T::NOBP; ++b)
        if (p.obs_bpos[b] != T::obs_bpos[b]) return false;
    for (int b = 0; b < T::NOBV; ++b)
        if (p.obs_bvel[b] != T::obs_bvel[b]) return false;
    for (int b = 0; b < BIOIM_NREFBODY; ++b)
        if (p.rw_body[b] != T::rw_body[b]) return false;
    return true;
}

}  // namespace

struct OsimCall {   /* mode 2 launch arguments (bioim_osim) */
    int op;
    const void *controls;
    void *report;
};

struct Ops {
    const char *topo;   /* the topology struct's name (fused-pair lookup) */
    int lanes;
    size_t lds_bytes;   /* per workgroup: model image + BIOIM_EPB env regions */
    int cache_dim;      /* reals per env of the realize cache (CacheLay<T>::DIM; 0: none) */
    int (*upload)(bioim_handle_t *);
    void (*launch)(bioim_handle_t *, int mode, const void *actions, void *obs, void *reward, uint8_t *done, void *info,
                   const int32_t *env_ids, const int32_t *ref_index, int n_list, const OsimCall *oc);
    void (*id_launch)(bioim_handle_t *, int op, int n, const void *q, const void *u, const void *v, void *out);
};

struct bioim_handle {
    int n, device, precision, ndof, nmuscle, nact, horizon, obs_dim, info_dim, nsub, auto_reset, env_offset;
    int act_stride, obs_stride, info_stride; /* I/O row strides (default nact, obs_dim, info_dim) */
    uint64_t seed;
    hipStream_t stream;
    bool own_stream;
    hipStream_t side;     /* private stream: this handle's segment of a concurrent group step */
    hipEvent_t ev_fork, ev_join;
    void *model;        /* DModel<Real> on device */
    void *smodel;       /* SModel<T, Real> on device (staged into LDS per workgroup) */
    void *state_buf;    /* one allocation for every SoA array */
    size_t state_bytes;
    void *dstate;       /* DState<Real> (host copy of pointers) */
    void *pert_x, *pert_y; /* apply_perturbations table: double [pert_n], Real [pert_n][n] */
    int pert_n, pert_ob;
    void *final_obs;    /* caller's device buffer [n][obs_stride] or null (bioim_set_final_obs) */
    void *force_out;    /* caller's device buffer [n][force_dim] or null (bioim_set_force_report) */
    void *traj;         /* caller's device buffers (bioim_set_state_storage) or null */
    int32_t *traj_n;
    int traj_cap;
    int rk;             /* integrator: 0 semi-implicit substeps (pack nsub), 1 RK-Merson (bioim_set_integrator) */
    double rk_acc;
    int rk_budget;      /* RK attempts per env per launch, 0: unbudgeted (bioim_set_rk_budget) */
    uint8_t *ready_out; /* caller's device buffer [n] or null */
    const uint8_t *active; /* caller's device buffer [n] or null (bioim_set_active_mask) */
    int last_group_fused; /* the last bioim_step_group with this handle first ran one fused launch */
    void *reset_tab;      /* Real [pack.nrows][reset_table_dim] or null (build_reset_table) */
    int planar;           /* the pack's topology is planar (pack_is_planar) */
    int reset_tab_on;     /* bioim_set_reset_table (default 1) */
    int cache_live;       /* a default step kernel ran since the realize-cache flags were last cleared */
    Ops ops;
    bioim_modelpack_t pack;
};

/* the launches that read the reset table: steps of a muscle model with the
 * default kernels (no push table, semi-implicit) and no force report or
 * state storage (their rows come from the reset realize itself) */
static inline bool reset_table_wanted(const bioim_handle_t *h) {
    return h->reset_tab_on && h->auto_reset && h->pert_n == 0 && (!h->rk || (BIOIM_RESET_TAB_RK && (h->planar || BIOIM_RESET_TAB_RK_SPATIAL))) &&
           !h->force_out && !h->traj;
}
static inline bool reset_table_eligible(const bioim_handle_t *h) { return h->reset_tab && reset_table_wanted(h); }
/* reals per env of the realize cache (CacheLay) */
static inline int cache_dim(const bioim_handle_t *h) { return h->ops.cache_dim; }
/* reals per table row: muscle models [nmuscle fiber lengths][obs]; torque
 * models [ndof x ndof M^-1, row-major][obs at zero held torques]; then the
 * reset realize's cache row (CacheLay; torque models: without the controls) */
static inline int reset_table_dim(const bioim_handle_t *h) {
    return (h->nmuscle > 0 ? h->nmuscle : h->ndof * h->ndof) + h->obs_dim + cache_dim(h);
}

namespace {

template <class T, typename Real, bool PERT = false> constexpr size_t lds_bytes() {
    return smodel_bytes<T, Real>() + (size_t)BIOIM_EPB * Lay<T, Real>::SIZE * sizeof(Real) +
           (PERT ? (size_t)BIOIM_EPB * PERT_SLOT * sizeof(double) : 0);
}

/* bioim_osim_report_dim (include/bioim.h layout) */
int osim_report_dim(const bioim_modelpack_t &p) {
    return 2 + 3 * p.ncoord + 18 * p.nosbody + 9 + 7 * p.nmuscle + p.nact + 6 * p.ncforce + p.nlimit + 1;
}

template <class T, typename Real>
LaunchArgs<T, Real> make_args(bioim_handle_t *h, int mode, const void *actions, void *obs, void *reward, uint8_t *done,
                              void *info, const int32_t *env_ids, const int32_t *ref_index, int n_list,
                              const OsimCall *oc) {
    constexpr int EPB = BIOIM_EPB;
    LaunchArgs<T, Real> a;
    const int count = mode != 0 ? n_list : h->n;
    a.Mg = reinterpret_cast<const DModel<Real> *>(h->model);
    a.Sg = reinterpret_cast<const SModel<T, Real> *>(h->smodel);
    a.st = *reinterpret_cast<DState<Real> *>(h->dstate);
    a.N = h->n; a.mode = mode; a.n_list = n_list; a.auto_reset = h->auto_reset; a.env_offset = h->env_offset;
    a.blocks = (count + EPB - 1) / EPB;
    a.act_stride = h->act_stride; a.obs_stride = h->obs_stride; a.info_stride = h->info_stride;
    a.actions = reinterpret_cast<const Real *>(actions);
    a.obs = reinterpret_cast<Real *>(obs);
    a.final_obs = mode == 0 ? reinterpret_cast<Real *>(h->final_obs) : nullptr;
    a.force_out = reinterpret_cast<Real *>(h->force_out);
    a.force_dim = h->nact + 6 * h->pack.ncforce + h->pack.nlimit + 6 * h->pack.nsphere;   /* bioim_force_report_dim */
    const bool integrates = mode == 0 || (oc && oc->op == BIOIM_OSIM_INTEGRATE);
    a.traj = integrates ? reinterpret_cast<Real *>(h->traj) : nullptr;
    a.traj_n = h->traj_n;
    a.traj_cap = h->traj_cap;
    a.traj_dim = 1 + 2 * h->ndof + 2 * h->nmuscle;
    a.reward = reinterpret_cast<Real *>(reward);
    a.info = reinterpret_cast<Real *>(info);
    a.done_out = done;
    a.env_ids = env_ids; a.ref_index = ref_index;
    a.seed = h->seed;
    a.pert_x = reinterpret_cast<const double *>(h->pert_x);
    a.pert_y = reinterpret_cast<const Real *>(h->pert_y);
    a.pert_n = h->pert_n; a.pert_ob = h->pert_ob;
    a.rk_acc = h->rk_acc;
    a.rk_budget = h->rk && mode == 0 ? h->rk_budget : 0;   /* an OsimModel integrate finishes its step */
    a.ready_out = mode == 0 ? h->ready_out : nullptr;
    a.active = mode == 0 ? h->active : nullptr;
    a.osim_op = oc ? oc->op : 0;
    a.osim_dim = osim_report_dim(h->pack);
    a.controls_in = oc ? reinterpret_cast<const Real *>(oc->controls) : nullptr;
    a.osim_out = oc ? reinterpret_cast<Real *>(oc->report) : nullptr;
    a.reset_tab = mode == 0 && reset_table_eligible(h) ? reinterpret_cast<const Real *>(h->reset_tab) : nullptr;
    a.reset_tab_dim = reset_table_dim(h);
    return a;
}

template <class T, typename Real>
void launch_impl(bioim_handle_t *h, int mode, const void *actions, void *obs, void *reward, uint8_t *done, void *info,
                 const int32_t *env_ids, const int32_t *ref_index, int n_list, const OsimCall *oc) {
    LaunchArgs<T, Real> a = make_args<T, Real>(h, mode, actions, obs, reward, done, info, env_ids, ref_index, n_list, oc);
    if (a.blocks <= 0) return;
    /* the perturbation kernels are separate instantiations, so the default
     * kernels' code is untouched by the (rarely used) push */
    constexpr size_t lds0 = lds_bytes<T, Real, false>(), lds1 = lds_bytes<T, Real, true>();
    const dim3 g(a.blocks), b(BIOIM_EPB * T::G);
    /* the realize cache (CacheLay): only the default step kernels form and
     * read it; before any other kernel changes the state, every env's row is
     * marked stale (once per switch: cache_live says a default launch may
     * have set flags since) */
    const bool default_kernel = mode != 2 && a.pert_n == 0 && !h->rk;
    if constexpr (CacheLay<T>::ON) {
        if (!default_kernel && h->cache_live) {
            hipMemsetAsync(a.st.cache_ok, 0, sizeof(int32_t) * (size_t)h->n, h->stream);
            h->cache_live = 0;
        }
        if (default_kernel) h->cache_live = 1;
    }
    if (mode == 2) {   /* OsimModel calls: the REP kernels */
        if (a.pert_n > 0 && h->rk) hipLaunchKernelGGL((env_kernel<T, Real, true, true, true>), g, b, lds1, h->stream, a);
        else if (a.pert_n > 0) hipLaunchKernelGGL((env_kernel<T, Real, true, false, true>), g, b, lds1, h->stream, a);
        else if (h->rk) hipLaunchKernelGGL((env_kernel<T, Real, false, true, true>), g, b, lds0, h->stream, a);
        else hipLaunchKernelGGL((env_kernel<T, Real, false, false, true>), g, b, lds0, h->stream, a);
        return;
    }
    if (a.pert_n > 0 && h->rk) hipLaunchKernelGGL((env_kernel<T, Real, true, true>), g, b, lds1, h->stream, a);
    else if (a.pert_n > 0) hipLaunchKernelGGL((env_kernel<T, Real, true, false>), g, b, lds1, h->stream, a);
    else if (h->rk) hipLaunchKernelGGL((env_kernel<T, Real, false, true>), g, b, lds0, h->stream, a);
    else hipLaunchKernelGGL((env_kernel<T, Real, false, false>), g, b, lds0, h->stream, a);
}

/* one launch of env_kernel2 for the segments h0 (rows [0, n0)) and h1 (the
 * rows after them) of a group step; on h0's stream */
template <class T0, class T1, typename Real>
int fused_launch_impl(bioim_handle_t *h0, bioim_handle_t *h1, const void *actions, void *obs, void *reward,
                      uint8_t *done, void *info) {
    constexpr size_t R = sizeof(Real);
    const size_t n0 = (size_t)h0->n;
    LaunchArgs<T0, Real> a0 = make_args<T0, Real>(h0, 0, actions, obs, reward, done, info, nullptr, nullptr, 0, nullptr);
    LaunchArgs<T1, Real> a1 = make_args<T1, Real>(
        h1, 0, (const char *)actions + n0 * h1->act_stride * R, obs ? (char *)obs + n0 * h1->obs_stride * R : nullptr,
        reward ? (char *)reward + n0 * R : nullptr, done + n0, info ? (char *)info + n0 * h1->info_stride * R : nullptr,
        nullptr, nullptr, 0, nullptr);
    constexpr size_t l0 = lds_bytes<T0, Real, false>(), l1 = lds_bytes<T1, Real, false>();
    constexpr size_t lds = l0 > l1 ? l0 : l1;
    static_assert(lds <= 163840, "LDS image + env regions exceed 160 KiB");
    /* the dynamic-LDS attribute is per device: set it once on each (the
     * per-topology kernels set theirs at handle creation, upload_smodel) */
    static bool attr[64] = {};
    const int dev = h0->device;
    if (dev < 0 || dev >= 64 || !attr[dev]) {
        HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&env_kernel2<T0, T1, Real>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        if (dev >= 0 && dev < 64) attr[dev] = true;
    }
    if (a0.blocks + a1.blocks <= 0) return 0;
    h0->cache_live = 1; h1->cache_live = 1;   /* default step kernels: they form the realize cache */
    hipLaunchKernelGGL((env_kernel2<T0, T1, Real>), dim3(a0.blocks + a1.blocks), dim3(BIOIM_EPB * T0::G), lds,
                       h0->stream, a0, a1);
    return 0;
}

template <class T, typename Real>
void id_launch_impl(bioim_handle_t *h, int op, int n, const void *q, const void *u, const void *v, void *out) {
    constexpr int EPB = BIOIM_EPB;
    IdArgs<T, Real> a;
    a.Mg = reinterpret_cast<const DModel<Real> *>(h->model);
    a.Sg = reinterpret_cast<const SModel<T, Real> *>(h->smodel);
    a.n = n; a.op = op;
    a.q = reinterpret_cast<const Real *>(q); a.u = reinterpret_cast<const Real *>(u);
    a.v = reinterpret_cast<const Real *>(v); a.out = reinterpret_cast<Real *>(out);
    constexpr size_t lds = lds_bytes<T, Real, false>();
    hipLaunchKernelGGL((id_kernel<T, Real>), dim3((n + EPB - 1) / EPB), dim3(BIOIM_EPB * T::G), lds, h->stream, a);
}

template <class T, typename Real> int upload_smodel(bioim_handle_t *h) {
    static_assert(lds_bytes<T, Real, true>() <= 163840, "LDS image + env regions exceed 160 KiB");
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&env_kernel<T, Real, false, false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, Real, false>()));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&env_kernel<T, Real, true, false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, Real, true>()));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&env_kernel<T, Real, false, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, Real, false>()));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&env_kernel<T, Real, true, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, Real, true>()));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&env_kernel<T, Real, false, false, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, Real, false>()));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&env_kernel<T, Real, true, false, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, Real, true>()));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&env_kernel<T, Real, false, true, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, Real, false>()));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&env_kernel<T, Real, true, true, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, Real, true>()));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&id_kernel<T, Real>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, Real, false>()));
    constexpr size_t B = smodel_bytes<T, Real>();
    std::vector<unsigned char> img(B, 0);
    build_smodel<T, Real>(h->pack, *reinterpret_cast<SModel<T, Real> *>(img.data()));
    HIPCHK(hipMalloc(&h->smodel, B));
    HIPCHK(hipMemcpyAsync(h->smodel, img.data(), B, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return 0;
}

template <class T> bool pick(const bioim_modelpack_t &p, int precision, Ops &ops, const char *name) {
    if (!topology_matches<T>(p)) return false;
    if (p.obs_dim > Lay<T, double>::OBSMAX) return false;
    ops.topo = name;
    ops.lanes = T::G;
    ops.cache_dim = CacheLay<T>::DIM;
    if (precision == 64) {
        ops.launch = &launch_impl<T, double>;
        ops.id_launch = &id_launch_impl<T, double>;
        ops.upload = &upload_smodel<T, double>;
        ops.lds_bytes = lds_bytes<T, double>();
    } else {
        ops.launch = &launch_impl<T, float>;
        ops.id_launch = &id_launch_impl<T, float>;
        ops.upload = &upload_smodel<T, float>;
        ops.lds_bytes = lds_bytes<T, float>();
    }
    return true;
}

template <typename Real> size_t state_layout(bioim_handle_t *h, char *base, DState<Real> *st) {
    size_t n = h->n, off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    size_t oq = take(sizeof(Real) * h->ndof * n), ou = take(sizeof(Real) * h->ndof * n);
    size_t oa = take(sizeof(Real) * (h->nmuscle ? h->nmuscle : 1) * n), ol = take(sizeof(Real) * (h->nmuscle ? h->nmuscle : 1) * n);
    size_t oh = take(sizeof(Real) * BIOIM_MAX_HORIZON * h->nact * n), olast = take(sizeof(Real) * h->nact * n);
    size_t opx = take(sizeof(Real) * n), ot = take(sizeof(double) * n);
    size_t oi = take(sizeof(int32_t) * n), ohl = take(sizeof(int32_t) * n), od = take(sizeof(int32_t) * n),
           orr = take(sizeof(int32_t) * n), ohr = take(sizeof(double) * n);
    const size_t na1 = h->nact ? h->nact : 1, nm1 = h->nmuscle ? h->nmuscle : 1;
    size_t opd = take(sizeof(int32_t) * n), ork = take(sizeof(double) * n), orh = take(sizeof(double) * n),
           ora = take(sizeof(int32_t) * n), octl = take(sizeof(Real) * na1 * n), ocur = take(sizeof(Real) * na1 * n),
           ovn = take(sizeof(Real) * nm1 * n);
    size_t oev = take(sizeof(uint64_t) * n);
    size_t occ = take(sizeof(Real) * (size_t)cache_dim(h) * n), ocv = take(sizeof(int32_t) * n);
    if (st) {
        st->q = (Real *)(base + oq); st->u = (Real *)(base + ou); st->act = (Real *)(base + oa);
        st->lce = (Real *)(base + ol); st->hist = (Real *)(base + oh); st->last = (Real *)(base + olast);
        st->old_px = (Real *)(base + opx); st->t = (double *)(base + ot); st->istep = (int32_t *)(base + oi);
        st->has_last = (int32_t *)(base + ohl); st->done = (int32_t *)(base + od); st->resets = (int32_t *)(base + orr);
        st->hrk = (double *)(base + ohr);
        st->pend = (int32_t *)(base + opd); st->rkt = (double *)(base + ork); st->rkh = (double *)(base + orh);
        st->rka = (int32_t *)(base + ora); st->ctl = (Real *)(base + octl); st->cur = (Real *)(base + ocur);
        st->vnw = (Real *)(base + ovn);
        st->rkev = (uint64_t *)(base + oev);
        st->cache = (Real *)(base + occ); st->cache_ok = (int32_t *)(base + ocv);
    }
    return off;
}

template <typename Real> int alloc_state(bioim_handle_t *h) {
    size_t bytes = state_layout<Real>(h, nullptr, nullptr);
    HIPCHK(hipMalloc(&h->state_buf, bytes));
    HIPCHK(hipMemsetAsync(h->state_buf, 0, bytes, h->stream));
    h->state_bytes = bytes;
    DState<Real> *st = new DState<Real>();
    state_layout<Real>(h, (char *)h->state_buf, st);
    h->dstate = st;
    DModel<Real> *hm = new DModel<Real>();
    convert_model<Real>(h->pack, *hm);
    HIPCHK(hipMalloc(&h->model, sizeof(DModel<Real>)));
    HIPCHK(hipMemcpyAsync(h->model, hm, sizeof(DModel<Real>), hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    delete hm;
    return h->ops.upload(h);
}

template <typename Real> int xfer_state(bioim_handle_t *h, double *host, const double *in) {
    DState<Real> &st = *reinterpret_cast<DState<Real> *>(h->dstate);
    size_t n = h->n;
    int nd = h->ndof, nm = h->nmuscle, na = h->nact, H = h->horizon;
    std::vector<char> buf(h->state_bytes);
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipStreamSynchronize(h->side));
    HIPCHK(hipMemcpy(buf.data(), h->state_buf, h->state_bytes, hipMemcpyDeviceToHost));
    DState<Real> hs;
    state_layout<Real>(h, buf.data(), &hs);
    int dim = bioim_state_dim(h);
    if (host)
        for (size_t e = 0; e < n; ++e)
            if (hs.pend[e])   /* mid-step: t is the step's end time but q/u/act/lce an accepted RK point */
                return fail(BIOIM_E_ARG, "bioim_get_state: envs are suspended mid-step by the RK budget "
                                         "(step until bioim_pending_count() is 0)");
    for (size_t e = 0; e < n; ++e) {
        if (host) {
            double *s = host + e * dim;
            int k = 0;
            s[k++] = hs.t[e]; s[k++] = hs.istep[e]; s[k++] = hs.has_last[e]; s[k++] = hs.old_px[e]; s[k++] = hs.done[e];
            for (int i = 0; i < nd; ++i) s[k++] = hs.q[i * n + e];
            for (int i = 0; i < nd; ++i) s[k++] = hs.u[i * n + e];
            for (int i = 0; i < nm; ++i) s[k++] = hs.act[i * n + e];
            for (int i = 0; i < nm; ++i) s[k++] = hs.lce[i * n + e];
            for (int hh = 0; hh < H; ++hh)
                for (int i = 0; i < na; ++i) s[k++] = hs.hist[(hh * na + i) * n + e];
            for (int i = 0; i < na; ++i) s[k++] = hs.last[i * n + e];
            s[k++] = hs.hrk[e];
            for (int i = 0; i < na; ++i) s[k++] = hs.ctl[i * n + e];
        } else {
            const double *s = in + e * dim;
            int k = 0;
            hs.t[e] = s[k++]; hs.istep[e] = (int32_t)s[k++]; hs.has_last[e] = (int32_t)s[k++];
            hs.old_px[e] = (Real)s[k++]; hs.done[e] = (int32_t)s[k++];
            for (int i = 0; i < nd; ++i) hs.q[i * n + e] = (Real)s[k++];
            for (int i = 0; i < nd; ++i) hs.u[i * n + e] = (Real)s[k++];
            for (int i = 0; i < nm; ++i) hs.act[i * n + e] = (Real)s[k++];
            for (int i = 0; i < nm; ++i) hs.lce[i * n + e] = (Real)s[k++];
            for (int hh = 0; hh < H; ++hh)
                for (int i = 0; i < na; ++i) hs.hist[(hh * na + i) * n + e] = (Real)s[k++];
            for (int i = 0; i < na; ++i) hs.last[i * n + e] = (Real)s[k++];
            hs.hrk[e] = s[k++];
            for (int i = 0; i < na; ++i) hs.ctl[i * n + e] = (Real)s[k++];
            hs.pend[e] = 0;   /* a state set from outside is at a step boundary */
            hs.cache_ok[e] = 0;   /* the realize cache belongs to the state it was formed at */
        }
    }
    if (in) HIPCHK(hipMemcpy(h->state_buf, buf.data(), h->state_bytes, hipMemcpyHostToDevice));
    return 0;
}

}  // namespace

/* topology k's kernel table (one object per topology, or all in this TU) */
#define BIOIM_PICK_DECL(S, NAME) bool bioim_pick_##S(const bioim_modelpack_t &p, int precision, Ops &ops);
BIOIM_FOR_EACH_TOPOLOGY(BIOIM_PICK_DECL)
#undef BIOIM_PICK_DECL
/* the fused two-topology launches (the fused unit, or all in this TU):
 * 1 if (h0, h1) is a pair of BIOIM_FUSED_PAIRS and was launched, 0 if not */
int bioim_fused_launch(bioim_handle_t *h0, bioim_handle_t *h1, const void *actions, void *obs, void *reward,
                       uint8_t *done, void *info);
#if defined(BIOIM_FUSED_ONLY) || (!defined(BIOIM_TOPO_ONLY) && !defined(BIOIM_ABI_ONLY))
int bioim_fused_launch(bioim_handle_t *h0, bioim_handle_t *h1, const void *actions, void *obs, void *reward,
                       uint8_t *done, void *info) {
    /* fp64 only: the fp32 fused kernel of the 3D pair spills 68 B/lane; fp32
     * batches keep the concurrent per-segment launches */
    if (h0->precision != 64) return 0;
#define BIOIM_TRY_PAIR(S0, S1)                                                                      \
    if (!strcmp(h0->ops.topo, #S0) && !strcmp(h1->ops.topo, #S1)) {                                  \
        const int rc = fused_launch_impl<S0, S1, double>(h0, h1, actions, obs, reward, done, info);  \
        return rc ? rc : 1;                                                                          \
    }
    BIOIM_FUSED_PAIRS(BIOIM_TRY_PAIR)
#undef BIOIM_TRY_PAIR
    return 0;
}
#endif
#if !defined(BIOIM_ABI_ONLY) && !defined(BIOIM_FUSED_ONLY)
#define BIOIM_PICK_DEF(S, NAME)                                                      \
    bool bioim_pick_##S(const bioim_modelpack_t &p, int precision, Ops &ops) { return pick<S>(p, precision, ops, #S); }
#ifdef BIOIM_TOPO_ONLY
#define BIOIM_PICK_ONE(S, NAME) BIOIM_PICK_DEF(S, NAME)
BIOIM_TOPOLOGY_AT(BIOIM_TOPO_ONLY, BIOIM_PICK_ONE)
#undef BIOIM_PICK_ONE
#else
BIOIM_FOR_EACH_TOPOLOGY(BIOIM_PICK_DEF)
#endif
#undef BIOIM_PICK_DEF
#endif

#if !defined(BIOIM_TOPO_ONLY) && !defined(BIOIM_FUSED_ONLY)
thread_local std::string g_err;

/* ================================================================ C-ABI */
extern "C" {

const char *bioim_last_error(void) { return g_err.c_str(); }
#ifndef BIOIM_BUILD_ID
#define BIOIM_BUILD_ID "unstamped"
#endif
/* sha256 of the kernel sources + hipcc flags (bioimitation/_buildinfo.py) */
const char *bioim_build_id(void) { return BIOIM_BUILD_ID; }
uint64_t bioim_modelpack_size(void) { return sizeof(bioim_modelpack_t); }

int bioim_create(const bioim_modelpack_t *pack, int n_envs, int device, int precision, uint64_t seed,
                 bioim_handle_t **out) {
    if (!pack || !out || n_envs <= 0) return fail(BIOIM_E_ARG, "bioim_create: bad arguments");
    if (precision != 32 && precision != 64) return fail(BIOIM_E_ARG, "bioim_create: precision must be 32 or 64");
    if (pack->magic != BIOIM_PACK_MAGIC || pack->version != BIOIM_PACK_VERSION)
        return fail(BIOIM_E_PACK, "bioim_create: bad ModelPack magic/version");
    if (pack->horizon < 1 || pack->horizon > BIOIM_MAX_HORIZON || pack->nsub < 1 || pack->obs_dim > BIOIM_OBS_MAX ||
        pack->nrows < 2)
        return fail(BIOIM_E_PACK, "bioim_create: ModelPack env fields out of range");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(BIOIM_E_DEVICE, "bioim_create: no HIP device");
    if (device < 0 || device >= ndev) return fail(BIOIM_E_DEVICE, "bioim_create: bad device index");
    HIPCHK(hipSetDevice(device));
    Ops ops{};
    bool found = false;
#define BIOIM_TRY(S, NAME) \
    if (!found) found = bioim_pick_##S(*pack, precision, ops);
    BIOIM_FOR_EACH_TOPOLOGY(BIOIM_TRY)
#undef BIOIM_TRY
    if (!found) return fail(BIOIM_E_NOKERNEL, std::string("bioim_create: no compiled kernel for the topology of ") + pack->env_id);
    bioim_handle_t *h = new bioim_handle();
    h->n = n_envs; h->device = device; h->precision = precision; h->seed = seed;
    h->ndof = pack->ndof; h->nmuscle = pack->nmuscle; h->nact = pack->nact; h->horizon = pack->horizon;
    h->obs_dim = pack->obs_dim; h->info_dim = pack->info_dim; h->nsub = pack->nsub; h->auto_reset = 0;
    h->env_offset = 0;
    h->pert_n = 0; h->pert_ob = -1;
    h->reset_tab = nullptr; h->reset_tab_on = 1; h->cache_live = 0;
    h->planar = pack_is_planar(*pack) ? 1 : 0;
    h->act_stride = pack->nact; h->obs_stride = pack->obs_dim; h->info_stride = pack->info_dim;
    h->ops = ops;
    memcpy(&h->pack, pack, sizeof(bioim_modelpack_t));
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return fail(BIOIM_E_DEVICE, "bioim_create: stream creation failed");
    }
    h->own_stream = true;
    if (hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess) {
        bioim_destroy(h);
        return fail(BIOIM_E_DEVICE, "bioim_create: stream/event creation failed");
    }
    int rc = precision == 64 ? alloc_state<double>(h) : alloc_state<float>(h);
    if (rc) { bioim_destroy(h); return rc; }
    *out = h;
    return 0;
}

int bioim_destroy(bioim_handle_t *h) {
    if (!h) return 0;
    if (h->stream) hipStreamSynchronize(h->stream);
    if (h->state_buf) hipFree(h->state_buf);
    if (h->model) hipFree(h->model);
    if (h->smodel) hipFree(h->smodel);
    if (h->pert_x) hipFree(h->pert_x);
    if (h->pert_y) hipFree(h->pert_y);
    if (h->reset_tab) hipFree(h->reset_tab);
    if (h->dstate) {
        if (h->precision == 64) delete reinterpret_cast<DState<double> *>(h->dstate);
        else delete reinterpret_cast<DState<float> *>(h->dstate);
    }
    if (h->side) { hipStreamSynchronize(h->side); hipStreamDestroy(h->side); }
    if (h->ev_fork) hipEventDestroy(h->ev_fork);
    if (h->ev_join) hipEventDestroy(h->ev_join);
    if (h->own_stream && h->stream) hipStreamDestroy(h->stream);
    delete h;
    return 0;
}

int bioim_reset(bioim_handle_t *h, const int32_t *env_ids, const int32_t *ref_index, int n, void *obs) {
    if (!h) return fail(BIOIM_E_ARG, "bioim_reset: null handle");
    int count = env_ids ? n : h->n;
    if (count <= 0) return 0;
    HIPCHK(hipSetDevice(h->device));
    h->ops.launch(h, 1, nullptr, obs, nullptr, nullptr, nullptr, env_ids, ref_index, count, nullptr);
    HIPCHK(hipGetLastError());
    return 0;
}

/* The reset table of a handle (LaunchArgs::reset_tab), built once, on the
 * first step that can use it: a scratch handle of the same pack and precision
 * with one env per reference row is reset to row r (mode 1 — the very reset
 * realize, with fiber equilibrium, an auto-reset runs) and its observations
 * are kept.  Muscle models: with the equilibrium fiber lengths; the reset
 * realize depends on the row alone (the held excitations enter only the
 * activation rate, which the observation does not hold; the fiber-velocity
 * root differs from a warm-started one at the rounding level: its start is
 * cold).  Torque models: the held torques enter the observation's q'' only,
 * linearly (q'' = M^-1 (f + tau)), so the row keeps q'' at zero torque (the
 * scratch handle's held controls are 0) and M^-1 at the row's coordinates. */
static int build_reset_table(bioim_handle_t *h) {
    const int nr = h->pack.nrows, nm = h->nmuscle, od = h->obs_dim, nd = h->ndof;
    const size_t R = h->precision == 64 ? 8 : 4, head = nm > 0 ? (size_t)nm : (size_t)nd * nd;
    const int cdim = cache_dim(h);
    const size_t dim = head + od + cdim;   /* = reset_table_dim(h) */
    bioim_handle_t *tmp = nullptr;
    int rc = bioim_create(&h->pack, nr, h->device, h->precision, h->seed, &tmp);
    if (rc) return rc;
    int32_t *d_idx = nullptr;
    void *d_obs = nullptr, *d_tab = nullptr, *d_q = nullptr, *d_v = nullptr, *d_out = nullptr;
    std::vector<int32_t> idx(nr);
    for (int r = 0; r < nr; ++r) idx[r] = r;
    const int sdim = bioim_state_dim(tmp);
    std::vector<double> st((size_t)nr * sdim);
    std::vector<unsigned char> obs((size_t)nr * od * R), tab((size_t)nr * dim * R);
    auto put = [&](unsigned char *dst, double x) {
        if (R == 8) memcpy(dst, &x, 8);
        else { const float f = (float)x; memcpy(dst, &f, 4); }
    };
    auto done = [&](int code) {
        for (void *p : {(void *)d_idx, d_obs, d_q, d_v, d_out})
            if (p) hipFree(p);
        if (code && d_tab) hipFree(d_tab);
        bioim_destroy(tmp);
        return code;
    };
    if (hipMalloc(&d_idx, sizeof(int32_t) * nr) != hipSuccess || hipMalloc(&d_obs, (size_t)nr * od * R) != hipSuccess ||
        hipMalloc(&d_tab, (size_t)nr * dim * R) != hipSuccess ||
        hipMemcpy(d_idx, idx.data(), sizeof(int32_t) * nr, hipMemcpyHostToDevice) != hipSuccess)
        return done(fail(BIOIM_E_DEVICE, "build_reset_table: allocation failed"));
    if ((rc = bioim_reset(tmp, nullptr, d_idx, nr, d_obs)) != 0) return done(rc);
    if (hipStreamSynchronize(tmp->stream) != hipSuccess ||
        hipMemcpy(obs.data(), d_obs, obs.size(), hipMemcpyDeviceToHost) != hipSuccess)
        return done(fail(BIOIM_E_DEVICE, "build_reset_table: reset realize failed"));
    if ((rc = bioim_get_state(tmp, st.data())) != 0) return done(rc);
    if (nm > 0) {
        for (int r = 0; r < nr; ++r)
            for (int m = 0; m < nm; ++m)   /* fiber_length[m] */
                put(tab.data() + ((size_t)r * dim + m) * R, st[(size_t)r * sdim + 5 + 2 * nd + nm + m]);
    } else {
        /* torque models: M^-1 at each row's coordinates, column k = M^-1 e_k
         * (the inverse-dynamics kernel, BIOIM_ID_MULT_MINV: the realize's
         * mass matrix — at h = 0 no implicit contact or limit terms) */
        const size_t n = (size_t)nr * nd;
        std::vector<unsigned char> q(n * nd * R), v(n * nd * R, 0), out(n * nd * R);
        for (int r = 0; r < nr; ++r)
            for (int k = 0; k < nd; ++k) {
                const size_t s_ = (size_t)r * nd + k;   /* state: row r, unit vector e_k */
                for (int d = 0; d < nd; ++d) put(q.data() + (s_ * nd + d) * R, st[(size_t)r * sdim + 5 + d]);
                put(v.data() + (s_ * nd + k) * R, 1.0);
            }
        if (hipMalloc(&d_q, q.size()) != hipSuccess || hipMalloc(&d_v, v.size()) != hipSuccess ||
            hipMalloc(&d_out, out.size()) != hipSuccess ||
            hipMemcpy(d_q, q.data(), q.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(d_v, v.data(), v.size(), hipMemcpyHostToDevice) != hipSuccess)
            return done(fail(BIOIM_E_DEVICE, "build_reset_table: allocation failed"));
        if ((rc = bioim_id_eval(tmp, BIOIM_ID_MULT_MINV, (int)n, d_q, d_q, d_v, d_out)) != 0) return done(rc);
        if (hipStreamSynchronize(tmp->stream) != hipSuccess ||
            hipMemcpy(out.data(), d_out, out.size(), hipMemcpyDeviceToHost) != hipSuccess)
            return done(fail(BIOIM_E_DEVICE, "build_reset_table: M^-1 columns failed"));
        for (int r = 0; r < nr; ++r)
            for (int k = 0; k < nd; ++k)
                for (int d = 0; d < nd; ++d)   /* M^-1[d][k] = (M^-1 e_k)_d, row-major */
                    memcpy(tab.data() + ((size_t)r * dim + (size_t)d * nd + k) * R,
                           out.data() + (((size_t)r * nd + k) * nd + d) * R, R);
    }
    for (int r = 0; r < nr; ++r)
        memcpy(tab.data() + ((size_t)r * dim + head) * R, obs.data() + (size_t)r * od * R, (size_t)od * R);
    if (cdim > 0) {   /* the reset realize's cache rows (DState::cache, [nr][cdim]) */
        const DState<double> &ts = *reinterpret_cast<const DState<double> *>(tmp->dstate);
        const size_t cb = (size_t)nr * cdim * R;
        std::vector<unsigned char> crow(cb);
        if (hipMemcpy(crow.data(), ts.cache, cb, hipMemcpyDeviceToHost) != hipSuccess)
            return done(fail(BIOIM_E_DEVICE, "build_reset_table: cache rows failed"));
        for (int r = 0; r < nr; ++r)
            memcpy(tab.data() + ((size_t)r * dim + head + od) * R, crow.data() + (size_t)r * cdim * R, (size_t)cdim * R);
    }
    if (hipMemcpy(d_tab, tab.data(), tab.size(), hipMemcpyHostToDevice) != hipSuccess)
        return done(fail(BIOIM_E_DEVICE, "build_reset_table: upload failed"));
    h->reset_tab = d_tab;
    return done(0);
}
static int ensure_reset_table(bioim_handle_t *h) {
    if (h->reset_tab || !reset_table_wanted(h)) return 0;
    return build_reset_table(h);
}

int bioim_set_reset_table(bioim_handle_t *h, int on) {
    if (!h) return fail(BIOIM_E_ARG, "bioim_set_reset_table: null handle");
    h->reset_tab_on = on ? 1 : 0;
    return 0;
}

int bioim_reset_table_rows(const bioim_handle_t *h) {
    if (!h) return fail(BIOIM_E_ARG, "bioim_reset_table_rows: null handle");
    return h->reset_tab ? h->pack.nrows : 0;
}

int bioim_step(bioim_handle_t *h, const void *actions, void *obs, void *reward, uint8_t *done, void *info) {
    if (!h || !actions || !done) return fail(BIOIM_E_ARG, "bioim_step: null handle/actions/done");
    HIPCHK(hipSetDevice(h->device));
    if (const int rc = ensure_reset_table(h)) return rc;
    h->ops.launch(h, 0, actions, obs, reward, done, info, nullptr, nullptr, 0, nullptr);
    HIPCHK(hipGetLastError());
    return 0;
}

int bioim_set_auto_reset(bioim_handle_t *h, int on) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    h->auto_reset = on ? 1 : 0;
    return 0;
}

int bioim_set_integrator(bioim_handle_t *h, int kind, double accuracy) {
    if (!h || kind < 0 || kind > 1 || (kind == 1 && !(accuracy > 0)))
        return fail(BIOIM_E_ARG, "bioim_set_integrator: kind 0 (semi-implicit) or 1 (RK-Merson, accuracy > 0)");
    if (kind != h->rk) {
        const int np = bioim_pending_count(h);
        if (np < 0) return np;
        if (np > 0) return fail(BIOIM_E_ARG, "bioim_set_integrator: envs are suspended mid-step (bioim_set_rk_budget)");
    }
    h->rk = kind;
    h->rk_acc = kind == 1 ? accuracy : 0.0;
    return 0;
}

int bioim_set_rk_budget(bioim_handle_t *h, int attempts, uint8_t *ready_out) {
    if (!h || attempts < 0) return fail(BIOIM_E_ARG, "bioim_set_rk_budget: null handle or negative budget");
    h->rk_budget = attempts;
    h->ready_out = ready_out;
    return 0;
}

int bioim_set_active_mask(bioim_handle_t *h, const uint8_t *active) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    if (active) {
        /* the step kernel reads active[env] for every env: refuse host memory
         * and memory of another device (a GPU fault otherwise); the length
         * (n bytes) is the caller's contract, checked by VectorEnv */
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, active) != hipSuccess) {
            (void)hipGetLastError();
            return fail(BIOIM_E_ARG, "bioim_set_active_mask: not a device pointer");
        }
        if (at.type != hipMemoryTypeDevice || at.device != h->device)
            return fail(BIOIM_E_ARG, "bioim_set_active_mask: mask must be device memory on the handle's device");
    }
    h->active = active;
    return 0;
}

int bioim_pending_count(bioim_handle_t *h) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipStreamSynchronize(h->side));   /* a group step may have run this handle on its side stream */
    std::vector<int32_t> p(h->n);
    const int32_t *dp = h->precision == 64 ? reinterpret_cast<DState<double> *>(h->dstate)->pend
                                           : reinterpret_cast<DState<float> *>(h->dstate)->pend;
    HIPCHK(hipMemcpy(p.data(), dp, sizeof(int32_t) * h->n, hipMemcpyDeviceToHost));
    int c = 0;
    for (int32_t v : p) c += v != 0;
    return c;
}

int bioim_force_report_dim(const bioim_handle_t *h) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    return h->nact + 6 * h->pack.ncforce + h->pack.nlimit + 6 * h->pack.nsphere;
}

int bioim_set_state_storage(bioim_handle_t *h, void *rows, int capacity, int32_t *count) {
    if (!h || (rows && (capacity <= 0 || !count))) return fail(BIOIM_E_ARG, "bioim_set_state_storage: bad arguments");
    h->traj = rows;
    h->traj_n = rows ? count : nullptr;
    h->traj_cap = rows ? capacity : 0;
    return 0;
}

int bioim_set_force_report(bioim_handle_t *h, void *force_out) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    h->force_out = force_out;
    return 0;
}

int bioim_set_final_obs(bioim_handle_t *h, void *final_obs) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    h->final_obs = final_obs;
    return 0;
}

int bioim_set_io_strides(bioim_handle_t *h, int act_stride, int obs_stride, int info_stride) {
    if (!h || act_stride < h->nact || obs_stride < h->obs_dim || info_stride < h->info_dim)
        return fail(BIOIM_E_ARG, "bioim_set_io_strides: a stride is smaller than the row it holds");
    h->act_stride = act_stride; h->obs_stride = obs_stride; h->info_stride = info_stride;
    return 0;
}

static int g_group_fusion = 1;

int bioim_set_group_fusion(int on) {
    g_group_fusion = on ? 1 : 0;
    return 0;
}

int bioim_group_fused(const bioim_handle_t *h) {
    if (!h) return fail(BIOIM_E_ARG, "bioim_group_fused: null handle");
    return h->last_group_fused ? 1 : 0;
}

int bioim_step_group(bioim_handle_t **hs, int nh, const void *actions, void *obs, void *reward, uint8_t *done,
                     void *info) {
    if (!hs || nh <= 0 || !actions || !done) return fail(BIOIM_E_ARG, "bioim_step_group: bad arguments");
    for (int i = 0; i < nh; ++i) {
        if (!hs[i]) return fail(BIOIM_E_ARG, "bioim_step_group: null handle");
        if (hs[i]->device != hs[0]->device || hs[i]->precision != hs[0]->precision ||
            hs[i]->act_stride != hs[0]->act_stride || hs[i]->obs_stride != hs[0]->obs_stride ||
            hs[i]->info_stride != hs[0]->info_stride)
            return fail(BIOIM_E_ARG, "bioim_step_group: handles differ in device, precision or I/O strides");
    }
    HIPCHK(hipSetDevice(hs[0]->device));
    for (int i = 0; i < nh; ++i)
        if (const int rc = ensure_reset_table(hs[i])) return rc;
    const size_t R = hs[0]->precision == 64 ? 8 : 4;
    hipStream_t stream = hs[0]->stream;
    /* two segments whose topology pair has a fused kernel (BIOIM_FUSED_PAIRS)
     * and that run the default step kernels (no push table, semi-implicit):
     * one launch, workgroups [0, B0) segment 0, the rest segment 1 */
    hs[0]->last_group_fused = 0;
    if (nh == 2 && g_group_fusion && hs[0]->pert_n == 0 && hs[1]->pert_n == 0 && !hs[0]->rk && !hs[1]->rk) {
        const int rc = bioim_fused_launch(hs[0], hs[1], actions, obs, reward, done, info);
        if (rc < 0) return rc;
        if (rc == 1) {
            HIPCHK(hipGetLastError());
            hs[0]->last_group_fused = 1;
            return 0;
        }
    }
    /* Otherwise one launch per segment, concurrently: segment 0 on the
     * caller's stream (hs[0]), segment i > 0 on handle i's private stream,
     * forked from and joined back into the caller's stream with events.  At
     * 4096 envs per GPU a mixed 50/50 batch gives each segment half the CUs
     * (one 16-env workgroup per CU); in order on one stream the halves would
     * run one after the other. */
    size_t off = 0;
    if (nh > 1) HIPCHK(hipEventRecord(hs[0]->ev_fork, stream));
    for (int i = 0; i < nh; ++i) {
        bioim_handle_t *h = hs[i];
        hipStream_t own = h->stream;
        h->stream = i == 0 ? stream : h->side;
        if (i > 0) HIPCHK(hipStreamWaitEvent(h->side, hs[0]->ev_fork, 0));
        h->ops.launch(h, 0, (const char *)actions + off * h->act_stride * R,
                      obs ? (char *)obs + off * h->obs_stride * R : nullptr,
                      reward ? (char *)reward + off * R : nullptr, done + off,
                      info ? (char *)info + off * h->info_stride * R : nullptr, nullptr, nullptr, 0, nullptr);
        h->stream = own;
        if (i > 0) {
            HIPCHK(hipEventRecord(h->ev_join, h->side));
            HIPCHK(hipStreamWaitEvent(stream, h->ev_join, 0));
        }
        off += (size_t)h->n;
    }
    HIPCHK(hipGetLastError());
    return 0;
}

int bioim_set_perturbation(bioim_handle_t *h, int os_body, int npts, const double *x, const double *y) {
    if (!h || npts < 0 || (npts > 0 && (!x || !y || os_body < 0 || os_body >= h->pack.nosbody)))
        return fail(BIOIM_E_ARG, "bioim_set_perturbation: bad arguments");
    for (int k = 0; k + 1 < npts; ++k)
        if (!(x[k] < x[k + 1])) return fail(BIOIM_E_ARG, "bioim_set_perturbation: breakpoints must increase");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipStreamSynchronize(h->side));
    if (h->pert_x) { HIPCHK(hipFree(h->pert_x)); h->pert_x = nullptr; }
    if (h->pert_y) { HIPCHK(hipFree(h->pert_y)); h->pert_y = nullptr; }
    h->pert_n = 0;
    h->pert_ob = -1;
    if (npts == 0) return 0;
    const size_t n = h->n, R = h->precision == 64 ? 8 : 4;
    std::vector<unsigned char> yt(R * n * npts);   /* [npts][n], env index fastest */
    for (size_t e = 0; e < n; ++e)
        for (int k = 0; k < npts; ++k) {
            const double v = y[e * npts + k];
            if (R == 8) reinterpret_cast<double *>(yt.data())[k * n + e] = v;
            else reinterpret_cast<float *>(yt.data())[k * n + e] = (float)v;
        }
    HIPCHK(hipMalloc(&h->pert_x, sizeof(double) * npts));
    HIPCHK(hipMalloc(&h->pert_y, yt.size()));
    HIPCHK(hipMemcpy(h->pert_x, x, sizeof(double) * npts, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->pert_y, yt.data(), yt.size(), hipMemcpyHostToDevice));
    h->pert_n = npts;
    h->pert_ob = os_body;
    return 0;
}

int bioim_id_eval(bioim_handle_t *h, int op, int n, const void *q, const void *u, const void *v, void *out) {
    if (!h || n < 0 || op < BIOIM_ID_GRAVITY || op > BIOIM_ID_TOTAL || (n > 0 && (!q || !out)))
        return fail(BIOIM_E_ARG, "bioim_id_eval: bad arguments");
    const bool use_u = op == BIOIM_ID_CORIOLIS || op == BIOIM_ID_RESIDUAL || op == BIOIM_ID_TOTAL;
    const bool use_v = op == BIOIM_ID_MULT_M || op == BIOIM_ID_MULT_MINV || op == BIOIM_ID_RESIDUAL;
    if (n > 0 && ((use_u && !u) || (use_v && !v))) return fail(BIOIM_E_ARG, "bioim_id_eval: missing u or v");
    if (n == 0) return 0;
    HIPCHK(hipSetDevice(h->device));
    h->ops.id_launch(h, op, n, q, u, v, out);
    HIPCHK(hipGetLastError());
    return 0;
}

int bioim_osim_report_dim(const bioim_handle_t *h) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    return osim_report_dim(h->pack);
}

int bioim_osim(bioim_handle_t *h, int op, const int32_t *env_ids, int n, const void *controls, void *obs, void *report) {
    if (!h || op < BIOIM_OSIM_REALIZE || op > BIOIM_OSIM_INTEGRATE || n < 0 || (n > 0 && !env_ids))
        return fail(BIOIM_E_ARG, "bioim_osim: bad arguments");
    if (n == 0) return 0;
    const int np = bioim_pending_count(h);
    if (np < 0) return np;
    if (np > 0) return fail(BIOIM_E_ARG, "bioim_osim: envs are suspended mid-step (bioim_set_rk_budget)");
    HIPCHK(hipSetDevice(h->device));
    const OsimCall oc{op, controls, report};
    h->ops.launch(h, 2, nullptr, obs, nullptr, nullptr, nullptr, env_ids, nullptr, n, &oc);
    HIPCHK(hipGetLastError());
    return 0;
}

int bioim_set_env_offset(bioim_handle_t *h, int offset) {
    if (!h || offset < 0) return fail(BIOIM_E_ARG, "bioim_set_env_offset: bad arguments");
    h->env_offset = offset;
    return 0;
}

int bioim_state_dim(const bioim_handle_t *h) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    return 5 + 2 * h->ndof + 2 * h->nmuscle + h->horizon * h->nact + h->nact + 1 + h->nact;
}

int bioim_get_state(bioim_handle_t *h, double *host_state) {
    if (!h || !host_state) return fail(BIOIM_E_ARG, "bioim_get_state: bad arguments");
    HIPCHK(hipSetDevice(h->device));
    return h->precision == 64 ? xfer_state<double>(h, host_state, nullptr) : xfer_state<float>(h, host_state, nullptr);
}

/* bioim_copy_state: the flat state rows (bioim_get_state's layout) gathered
 * on the device, one thread per value, on the handle's stream — no
 * synchronization, so a caller can fold them into the copy of a step's
 * outputs (the single-env recorder, envs.py) */
extern "C++" {
template <typename Real>
__global__ void state_rows_kernel(DState<Real> st, int n, int nd, int nm, int na, int H, int dim, double *out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)n * dim) return;
    const int e = (int)(i / dim);
    int k = (int)(i % dim);
    const size_t N = (size_t)n;
    double v = 0;
    if (k < 5) {
        v = k == 0 ? st.t[e] : k == 1 ? (double)st.istep[e] : k == 2 ? (double)st.has_last[e]
          : k == 3 ? (double)st.old_px[e] : (double)st.done[e];
    } else if ((k -= 5) < nd) v = st.q[k * N + e];
    else if ((k -= nd) < nd) v = st.u[k * N + e];
    else if ((k -= nd) < nm) v = st.act[k * N + e];
    else if ((k -= nm) < nm) v = st.lce[k * N + e];
    else if ((k -= nm) < H * na) v = st.hist[k * N + e];   /* [hh][a] = hh * na + a */
    else if ((k -= H * na) < na) v = st.last[k * N + e];
    else if ((k -= na) == 0) v = st.hrk[e];
    else v = st.ctl[(k - 1) * N + e];
    out[i] = v;
}
}  // extern "C++"

int bioim_copy_state(bioim_handle_t *h, void *device_out) {
    if (!h || !device_out) return fail(BIOIM_E_ARG, "bioim_copy_state: bad arguments");
    HIPCHK(hipSetDevice(h->device));
    const int dim = bioim_state_dim(h), n = h->n;
    const size_t total = (size_t)n * dim;
    const int bs = 256;
    const dim3 g((unsigned)((total + bs - 1) / bs)), b(bs);
    if (h->precision == 64)
        hipLaunchKernelGGL(state_rows_kernel<double>, g, b, 0, h->stream, *reinterpret_cast<DState<double> *>(h->dstate), n,
                           h->ndof, h->nmuscle, h->nact, h->horizon, dim, reinterpret_cast<double *>(device_out));
    else
        hipLaunchKernelGGL(state_rows_kernel<float>, g, b, 0, h->stream, *reinterpret_cast<DState<float> *>(h->dstate), n,
                           h->ndof, h->nmuscle, h->nact, h->horizon, dim, reinterpret_cast<double *>(device_out));
    HIPCHK(hipGetLastError());
    return 0;
}

int bioim_set_state(bioim_handle_t *h, const double *host_state) {
    if (!h || !host_state) return fail(BIOIM_E_ARG, "bioim_set_state: bad arguments");
    HIPCHK(hipSetDevice(h->device));
    return h->precision == 64 ? xfer_state<double>(h, nullptr, host_state) : xfer_state<float>(h, nullptr, host_state);
}

/* one per-env plane of the device state (a DState member; the pointer
 * layout is the same for both precisions), copied to the host — the
 * counters read that plane alone, not the whole state (round 6: with the
 * realize cache the state is ~10 MB at 4096 envs) */
extern "C++" template <typename V> static int read_plane(bioim_handle_t *h, V *DState<double>::*member, std::vector<V> &out) {
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipStreamSynchronize(h->side));
    const DState<double> &st = *reinterpret_cast<const DState<double> *>(h->dstate);
    out.resize((size_t)h->n);
    HIPCHK(hipMemcpy(out.data(), st.*member, sizeof(V) * (size_t)h->n, hipMemcpyDeviceToHost));
    return 0;
}

/* total resets (explicit + in-kernel auto-resets) over the handle's envs */
int bioim_reset_count(bioim_handle_t *h, uint64_t *total) {
    if (!h || !total) return fail(BIOIM_E_ARG, "bioim_reset_count: bad arguments");
    std::vector<int32_t> r;
    if (const int rc = read_plane<int32_t>(h, &DState<double>::resets, r)) return rc;
    uint64_t sum = 0;
    for (int e = 0; e < h->n; ++e) sum += (uint32_t)r[e];
    *total = sum;
    return 0;
}

/* one of the per-env RK counters of the state (DState::rkev) summed over the envs */
static int rk_counter(bioim_handle_t *h, uint64_t *total, bool fin, const char *who) {
    if (!h || !total) return fail(BIOIM_E_ARG, std::string(who) + ": bad arguments");
    std::vector<uint64_t> r;
    if (const int rc = read_plane<uint64_t>(h, &DState<double>::rkev, r)) return rc;
    uint64_t sum = 0;
    for (int e = 0; e < h->n; ++e) sum += (uint32_t)(fin ? r[e] >> 32 : r[e]);
    *total = sum;
    return 0;
}

/* dynamics evaluations of the RK integrator so far, summed over the envs */
int bioim_eval_count(bioim_handle_t *h, uint64_t *total) { return rk_counter(h, total, false, "bioim_eval_count"); }

/* env steps the RK integrator finished so far (bioim_step launches whose
 * ready[env] was 1), summed over the envs */
int bioim_finished_count(bioim_handle_t *h, uint64_t *total) {
    return rk_counter(h, total, true, "bioim_finished_count");
}

int bioim_set_rk_counters(bioim_handle_t *h, uint32_t evals, uint32_t finished) {
    if (!h) return fail(BIOIM_E_ARG, "bioim_set_rk_counters: null handle");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipStreamSynchronize(h->side));
    std::vector<char> buf(h->state_bytes);
    HIPCHK(hipMemcpy(buf.data(), h->state_buf, h->state_bytes, hipMemcpyDeviceToHost));
    const uint64_t v = ((uint64_t)finished << 32) | evals;
    if (h->precision == 64) {
        DState<double> hs;
        state_layout<double>(h, buf.data(), &hs);
        for (int e = 0; e < h->n; ++e) hs.rkev[e] = v;
    } else {
        DState<float> hs;
        state_layout<float>(h, buf.data(), &hs);
        for (int e = 0; e < h->n; ++e) hs.rkev[e] = v;
    }
    HIPCHK(hipMemcpy(h->state_buf, buf.data(), h->state_bytes, hipMemcpyHostToDevice));
    return 0;
}

int bioim_query(const bioim_handle_t *h, int32_t *out) {
    if (!h || !out) return fail(BIOIM_E_ARG, "bioim_query: bad arguments");
    out[0] = h->n; out[1] = h->obs_dim; out[2] = h->nact; out[3] = h->info_dim;
    out[4] = h->precision; out[5] = h->ops.lanes; out[6] = h->nsub; out[7] = bioim_state_dim(h);
    return 0;
}

int bioim_query_launch(const bioim_handle_t *h, int32_t *out) {
    if (!h || !out) return fail(BIOIM_E_ARG, "bioim_query_launch: bad arguments");
    const int epb = BIOIM_EPB;
    out[0] = h->ops.lanes; out[1] = BIOIM_EPB * h->ops.lanes; out[2] = epb; out[3] = (int32_t)h->ops.lds_bytes;
    out[4] = (h->n + epb - 1) / epb;
    return 0;
}

void *bioim_stream(bioim_handle_t *h) { return h ? (void *)h->stream : nullptr; }

int bioim_set_stream(bioim_handle_t *h, void *s) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    if (h->own_stream && h->stream) {
        hipStreamSynchronize(h->stream);
        hipStreamDestroy(h->stream);
    }
    h->stream = (hipStream_t)s;
    h->own_stream = false;
    return 0;
}

#ifdef BIOIM_WAVETIME
int bioim_debug_wavetime(unsigned long long *out, int n) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wavetime), sizeof(unsigned long long) * (n < BIOIM_WAVETIME_N ? n : BIOIM_WAVETIME_N)));
    return 0;
}
/* per thread: [0, n) Newton iterations, [n, 2n) most in one solve, [2n, 3n) bisections */
int bioim_debug_fviter(unsigned *out, int n) {
    HIPCHK(hipDeviceSynchronize());
    const int m = n < BIOIM_WAVETIME_N * 4 ? n : BIOIM_WAVETIME_N * 4;
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fvit), sizeof(unsigned) * m));
    HIPCHK(hipMemcpyFromSymbol(out + n, HIP_SYMBOL(g_fvmax), sizeof(unsigned) * m));
    HIPCHK(hipMemcpyFromSymbol(out + 2 * n, HIP_SYMBOL(g_fvbis), sizeof(unsigned) * m));
    return 0;
}
#endif
#ifdef BIOIM_STAMPS
int bioim_debug_stamps(unsigned long long *out, int reset) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 24));
    if (reset) {
        unsigned long long z[24] = {0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)));
    }
    return 0;
}
#endif

int bioim_sync(bioim_handle_t *h) {
    if (!h) return fail(BIOIM_E_ARG, "null handle");
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipStreamSynchronize(h->side));
    return 0;
}

}  // extern "C"
#endif  // BIOIM_TOPO_ONLY
