// Per-instruction issue cost and dependent latency, one wave (64 lanes)
// alone on its SIMD — the step kernel's situation (one wave per SIMD).
// Each test is an unrolled straight-line run of one instruction (inline asm,
// so the compiler cannot reorder or fold it) inside a clock64() bracket:
//   dep   — every instruction reads the previous one's result;
//   ind8  — eight independent registers in rotation.
// Prints shader-clock cycles per instruction.
//   hipcc --offload-arch=gfx950 -O3 -o lat2 lat2.hip && ./lat2
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256   /* instructions per timed block (x 8 for ind8 tests in the macro) */

#define R8(...) __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__
#define R32(...) R8(__VA_ARGS__) R8(__VA_ARGS__) R8(__VA_ARGS__) R8(__VA_ARGS__)
#define R256(...) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__)

#define START long long t0 = clock64();
#define STOP(sink) long long t1 = clock64(); out[threadIdx.x] = (sink); if (threadIdx.x == 0) cyc[0] = t1 - t0;
#define KHEAD(name) __global__ void name(double *out, long long *cyc, double a)

/* fp64 FMA */
KHEAD(k_fma64_dep) {
    double x = threadIdx.x, c = a;
    START
    R256(asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x) : "v"(c));)
    STOP(x)
}

KHEAD(k_fma64_ind) {
    double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7; double c = a;
    START
    R32(asm volatile("v_fma_f64 %0, %0, %8, %8\n v_fma_f64 %1, %1, %8, %8\n v_fma_f64 %2, %2, %8, %8\n v_fma_f64 %3, %3, %8, %8\n v_fma_f64 %4, %4, %8, %8\n v_fma_f64 %5, %5, %8, %8\n v_fma_f64 %6, %6, %8, %8\n v_fma_f64 %7, %7, %8, %8" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(c));)
    STOP(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7)
}

/* fp64 add */
KHEAD(k_add64_dep) {
    double x = threadIdx.x, c = a;
    START
    R256(asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(c));)
    STOP(x)
}

/* fp32 FMA */
KHEAD(k_fma32_dep) {
    float x = threadIdx.x, c = (float)a;
    START
    R256(asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(c));)
    STOP(x)
}

KHEAD(k_fma32_ind) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7; float c = (float)a;
    START
    R32(asm volatile("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n v_fma_f32 %3, %3, %8, %8\n v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(c));)
    STOP(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7)
}

/* integer add */
KHEAD(k_add32_dep) {
    unsigned x = threadIdx.x, c = (unsigned)a;
    START
    R256(asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(c));)
    STOP((double)x)
}

/* v_mov_b32 (self-copies, independent) */
KHEAD(k_mov32_ind) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    START
    R32(asm volatile("v_mov_b32 %0, %0\n v_mov_b32 %1, %1\n v_mov_b32 %2, %2\n v_mov_b32 %3, %3\n v_mov_b32 %4, %4\n v_mov_b32 %5, %5\n v_mov_b32 %6, %6\n v_mov_b32 %7, %7" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));)
    STOP(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7)
}

/* v_cndmask_b32 with vcc from a compare before the bracket */
KHEAD(k_cnd_dep) {
    float x = threadIdx.x, c = (float)a; asm volatile("v_cmp_gt_f32 vcc, %0, %1" :: "v"(x), "v"(c) : "vcc");
    START
    R256(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(c) : "vcc");)
    STOP(x)
}

KHEAD(k_cnd_ind) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7; float c = (float)a; asm volatile("v_cmp_gt_f32 vcc, %0, %1" :: "v"(x0), "v"(c) : "vcc");
    START
    R32(asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(c) : "vcc");)
    STOP(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7)
}

/* compare into vcc then two selects reading it (the shape of a double select), dependent */
KHEAD(k_cmpsel_dep) {
    float x = threadIdx.x, y = x + 1, c = (float)a;
    START
    R256(asm volatile("v_cmp_gt_f32 vcc, %0, %2\n v_cndmask_b32 %0, %0, %2, vcc\n v_cndmask_b32 %1, %1, %2, vcc" : "+v"(x), "+v"(y) : "v"(c) : "vcc");)
    STOP(x + y)
}

/* fp64 compares into SGPR pairs, independent */
KHEAD(k_cmp64_ind) {
    double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7; double c = a;
    START
    R32(asm volatile("v_cmp_gt_f64 s[0:1], %0, %8\n v_cmp_gt_f64 s[2:3], %1, %8\n v_cmp_gt_f64 s[4:5], %2, %8\n v_cmp_gt_f64 s[6:7], %3, %8\n v_cmp_gt_f64 s[8:9], %4, %8\n v_cmp_gt_f64 s[10:11], %5, %8\n v_cmp_gt_f64 s[12:13], %6, %8\n v_cmp_gt_f64 s[14:15], %7, %8" :: "v"(x0), "v"(x1), "v"(x2), "v"(x3), "v"(x4), "v"(x5), "v"(x6), "v"(x7), "v"(c) : "s0","s1","s2","s3","s4","s5","s6","s7","s8","s9","s10","s11","s12","s13","s14","s15");)
    STOP(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7)
}

/* AGPR write then read back (dependent pair) */
KHEAD(k_agpr_dep) {
    float x = threadIdx.x;
    START
    R256(asm volatile("v_accvgpr_write_b32 a0, %0\n v_accvgpr_read_b32 %0, a0" : "+v"(x) :: "a0");)
    STOP(x)
}

/* AGPR writes, independent */
KHEAD(k_agprw_ind) {
    float x0 = threadIdx.x;
    START
    R32(asm volatile("v_accvgpr_write_b32 a0, %0\n v_accvgpr_write_b32 a1, %0\n v_accvgpr_write_b32 a2, %0\n v_accvgpr_write_b32 a3, %0\n v_accvgpr_write_b32 a4, %0\n v_accvgpr_write_b32 a5, %0\n v_accvgpr_write_b32 a6, %0\n v_accvgpr_write_b32 a7, %0" :: "v"(x0) : "a0","a1","a2","a3","a4","a5","a6","a7");)
    STOP(x0)
}

/* fp64 reciprocal */
KHEAD(k_rcp64_dep) {
    double x = threadIdx.x + 1.5;
    START
    R256(asm volatile("v_rcp_f64 %0, %0" : "+v"(x));)
    STOP(x)
}

KHEAD(k_rcp64_ind) {
    double x0 = threadIdx.x + 1.5, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    START
    R32(asm volatile("v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n v_rcp_f64 %4, %4\n v_rcp_f64 %5, %5\n v_rcp_f64 %6, %6\n v_rcp_f64 %7, %7" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));)
    STOP(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7)
}

/* dependent fp64 FMAs with an independent 32-bit move between each pair */
KHEAD(k_fma64_mov) {
    double x = threadIdx.x, c = a; float m0 = 0, m1 = 1;
    START
    R256(asm volatile("v_fma_f64 %0, %0, %3, %3\n v_mov_b32 %1, %2" : "+v"(x), "=v"(m0) : "v"(m1), "v"(c));)
    STOP(x + m0)
}

/* two interleaved dependent fp64 FMA chains */
KHEAD(k_fma64_dual) {
    double x = threadIdx.x, y = x + 1, c = a;
    START
    R256(asm volatile("v_fma_f64 %0, %0, %2, %2\n v_fma_f64 %1, %1, %2, %2" : "+v"(x), "+v"(y) : "v"(c));)
    STOP(x + y)
}

/* s_nop 0 */
KHEAD(k_snop) {
    float x = threadIdx.x;
    START
    R256(asm volatile("s_nop 0");)
    STOP(x)
}
/* ds_read_b64, independent (same address per lane, 8 in flight), then one wait */
__global__ void k_dsread_ind(double *out, long long *cyc, double a) {
    __shared__ double sh[512];
    for (int i = threadIdx.x; i < 512; i += 64) sh[i] = i;
    __syncthreads();
    unsigned addr = threadIdx.x * 8;
    double x0, x1, x2, x3, x4, x5, x6, x7, s = 0;
    long long t0 = clock64();
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        asm volatile("ds_read_b64 %0, %8\n ds_read_b64 %1, %8 offset:512\n ds_read_b64 %2, %8 offset:1024\n ds_read_b64 %3, %8 offset:1536\n"
                     "ds_read_b64 %4, %8 offset:2048\n ds_read_b64 %5, %8 offset:2560\n ds_read_b64 %6, %8 offset:3072\n ds_read_b64 %7, %8 offset:3584\n"
                     "s_waitcnt lgkmcnt(0)"
                     : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3), "=v"(x4), "=v"(x5), "=v"(x6), "=v"(x7) : "v"(addr));
    }
    long long t1 = clock64();
    s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
/* ds_read_b64 dependent: address from the previous load */
__global__ void k_dsread_dep(double *out, long long *cyc, double a) {
    __shared__ unsigned sh[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) sh[i] = ((i + 1) & 511) * 4;
    __syncthreads();
    unsigned addr = threadIdx.x * 4;
    long long t0 = clock64();
    R256(asm volatile("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)" : "+v"(addr));)
    long long t1 = clock64();
    out[threadIdx.x] = addr;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

typedef void (*kfn)(double *, long long *, double);

static void run(const char *name, kfn f, int ops, double *d_out, long long *d_cyc) {
    long long best = -1;
    for (int r = 0; r < 7; ++r) {
        hipLaunchKernelGGL(f, dim3(1), dim3(64), 0, 0, d_out, d_cyc, 1.0000001);
        (void)hipDeviceSynchronize();
        long long c;
        (void)hipMemcpy(&c, d_cyc, sizeof(c), hipMemcpyDeviceToHost);
        if (best < 0 || c < best) best = c;
    }
    printf("%-14s cycles/instr %6.2f   (%d instr, delta %lld)\n", name, (double)best / ops, ops, best);
}

int main() {
    double *d_out;
    long long *d_cyc;
    (void)hipMalloc(&d_out, 64 * sizeof(double));
    (void)hipMalloc(&d_cyc, sizeof(long long));
    run("fma64 dep", k_fma64_dep, 256, d_out, d_cyc);
    run("fma64 ind8", k_fma64_ind, 256, d_out, d_cyc);
    run("add64 dep", k_add64_dep, 256, d_out, d_cyc);
    run("fma32 dep", k_fma32_dep, 256, d_out, d_cyc);
    run("fma32 ind8", k_fma32_ind, 256, d_out, d_cyc);
    run("add32 dep", k_add32_dep, 256, d_out, d_cyc);
    run("mov32 ind8", k_mov32_ind, 256, d_out, d_cyc);
    run("cndmask dep", k_cnd_dep, 256, d_out, d_cyc);
    run("cndmask ind8", k_cnd_ind, 256, d_out, d_cyc);
    run("cmp+2cnd dep", k_cmpsel_dep, 768, d_out, d_cyc);
    run("cmp64 ind8", k_cmp64_ind, 256, d_out, d_cyc);
    run("agpr w+r dep", k_agpr_dep, 512, d_out, d_cyc);
    run("agpr w ind8", k_agprw_ind, 256, d_out, d_cyc);
    run("rcp64 dep", k_rcp64_dep, 256, d_out, d_cyc);
    run("rcp64 ind8", k_rcp64_ind, 256, d_out, d_cyc);
    run("fma64+mov32", k_fma64_mov, 512, d_out, d_cyc);
    run("fma64 2 chains", k_fma64_dual, 512, d_out, d_cyc);
    run("s_nop 0", k_snop, 256, d_out, d_cyc);
    run("ds_read_b64 ind8", k_dsread_ind, 256, d_out, d_cyc);
    run("ds_read_b32 dep", k_dsread_dep, 256, d_out, d_cyc);
    return 0;
}
