// Dependent-latency curve: K interleaved dependency chains (distance K
// between producer and consumer), operand-bank and mixed-pipe cases, one
// wave alone on its SIMD (round 5; complements lat3.hip).
// Each test is an unrolled straight-line run of one instruction (inline asm,
// so the compiler cannot reorder or fold it) inside a clock64() bracket:
//   dep   — every instruction reads the previous one's result;
//   ind8  — eight independent registers in rotation.
// Prints shader-clock cycles per instruction.
//   hipcc --offload-arch=gfx950 -O3 -o lat3 lat3.hip && ./lat3
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256   /* instructions per timed block (x 8 for ind8 tests in the macro) */

#define R8(...) __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__ __VA_ARGS__
#define R32(...) R8(__VA_ARGS__) R8(__VA_ARGS__) R8(__VA_ARGS__) R8(__VA_ARGS__)
#define R256(...) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__) R32(__VA_ARGS__)

#define START long long t0 = clock64();
#define STOP(sink) long long t1 = clock64(); out[threadIdx.x] = (sink); if (threadIdx.x == 0) cyc[0] = t1 - t0;
#define KHEAD(name) __global__ void name(double *out, long long *cyc, double a)

KHEAD(k_fma64_c1) {
    double x0 = threadIdx.x + 0; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 256; ++r) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x0) : "v"(c));
    STOP(x0)
}

KHEAD(k_fma64_c2) {
    double x0 = threadIdx.x + 0, x1 = threadIdx.x + 1; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 128; ++r) asm volatile("v_fma_f64 %0, %0, %2, %2\n v_fma_f64 %1, %1, %2, %2" : "+v"(x0), "+v"(x1) : "v"(c));
    STOP(x0 + x1)
}

KHEAD(k_fma64_c3) {
    double x0 = threadIdx.x + 0, x1 = threadIdx.x + 1, x2 = threadIdx.x + 2; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 85; ++r) asm volatile("v_fma_f64 %0, %0, %3, %3\n v_fma_f64 %1, %1, %3, %3\n v_fma_f64 %2, %2, %3, %3" : "+v"(x0), "+v"(x1), "+v"(x2) : "v"(c));
    STOP(x0 + x1 + x2)
}

KHEAD(k_fma64_c4) {
    double x0 = threadIdx.x + 0, x1 = threadIdx.x + 1, x2 = threadIdx.x + 2, x3 = threadIdx.x + 3; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 64; ++r) asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(c));
    STOP(x0 + x1 + x2 + x3)
}

KHEAD(k_fma64_c5) {
    double x0 = threadIdx.x + 0, x1 = threadIdx.x + 1, x2 = threadIdx.x + 2, x3 = threadIdx.x + 3, x4 = threadIdx.x + 4; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 51; ++r) asm volatile("v_fma_f64 %0, %0, %5, %5\n v_fma_f64 %1, %1, %5, %5\n v_fma_f64 %2, %2, %5, %5\n v_fma_f64 %3, %3, %5, %5\n v_fma_f64 %4, %4, %5, %5" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4) : "v"(c));
    STOP(x0 + x1 + x2 + x3 + x4)
}

KHEAD(k_fma64_c6) {
    double x0 = threadIdx.x + 0, x1 = threadIdx.x + 1, x2 = threadIdx.x + 2, x3 = threadIdx.x + 3, x4 = threadIdx.x + 4, x5 = threadIdx.x + 5; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 42; ++r) asm volatile("v_fma_f64 %0, %0, %6, %6\n v_fma_f64 %1, %1, %6, %6\n v_fma_f64 %2, %2, %6, %6\n v_fma_f64 %3, %3, %6, %6\n v_fma_f64 %4, %4, %6, %6\n v_fma_f64 %5, %5, %6, %6" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5) : "v"(c));
    STOP(x0 + x1 + x2 + x3 + x4 + x5)
}

KHEAD(k_fma64_c8) {
    double x0 = threadIdx.x + 0, x1 = threadIdx.x + 1, x2 = threadIdx.x + 2, x3 = threadIdx.x + 3, x4 = threadIdx.x + 4, x5 = threadIdx.x + 5, x6 = threadIdx.x + 6, x7 = threadIdx.x + 7; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 32; ++r) asm volatile("v_fma_f64 %0, %0, %8, %8\n v_fma_f64 %1, %1, %8, %8\n v_fma_f64 %2, %2, %8, %8\n v_fma_f64 %3, %3, %8, %8\n v_fma_f64 %4, %4, %8, %8\n v_fma_f64 %5, %5, %8, %8\n v_fma_f64 %6, %6, %8, %8\n v_fma_f64 %7, %7, %8, %8" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(c));
    STOP(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7)
}

KHEAD(k_fma32_c1) {
    float x0 = threadIdx.x + 0; float c = (float)a;
    START
#pragma unroll
    for (int r = 0; r < 256; ++r) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x0) : "v"(c));
    STOP(x0)
}

KHEAD(k_fma32_c2) {
    float x0 = threadIdx.x + 0, x1 = threadIdx.x + 1; float c = (float)a;
    START
#pragma unroll
    for (int r = 0; r < 128; ++r) asm volatile("v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2" : "+v"(x0), "+v"(x1) : "v"(c));
    STOP(x0 + x1)
}

KHEAD(k_fma32_c3) {
    float x0 = threadIdx.x + 0, x1 = threadIdx.x + 1, x2 = threadIdx.x + 2; float c = (float)a;
    START
#pragma unroll
    for (int r = 0; r < 85; ++r) asm volatile("v_fma_f32 %0, %0, %3, %3\n v_fma_f32 %1, %1, %3, %3\n v_fma_f32 %2, %2, %3, %3" : "+v"(x0), "+v"(x1), "+v"(x2) : "v"(c));
    STOP(x0 + x1 + x2)
}

KHEAD(k_fma32_c4) {
    float x0 = threadIdx.x + 0, x1 = threadIdx.x + 1, x2 = threadIdx.x + 2, x3 = threadIdx.x + 3; float c = (float)a;
    START
#pragma unroll
    for (int r = 0; r < 64; ++r) asm volatile("v_fma_f32 %0, %0, %4, %4\n v_fma_f32 %1, %1, %4, %4\n v_fma_f32 %2, %2, %4, %4\n v_fma_f32 %3, %3, %4, %4" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(c));
    STOP(x0 + x1 + x2 + x3)
}

KHEAD(k_mul64_c1) {
    double x0 = threadIdx.x + 0; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 256; ++r) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x0) : "v"(c));
    STOP(x0)
}

KHEAD(k_mul64_c2) {
    double x0 = threadIdx.x + 0, x1 = threadIdx.x + 1; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 128; ++r) asm volatile("v_mul_f64 %0, %0, %2\n v_mul_f64 %1, %1, %2" : "+v"(x0), "+v"(x1) : "v"(c));
    STOP(x0 + x1)
}

KHEAD(k_mul64_c3) {
    double x0 = threadIdx.x + 0, x1 = threadIdx.x + 1, x2 = threadIdx.x + 2; double c = (double)a;
    START
#pragma unroll
    for (int r = 0; r < 85; ++r) asm volatile("v_mul_f64 %0, %0, %3\n v_mul_f64 %1, %1, %3\n v_mul_f64 %2, %2, %3" : "+v"(x0), "+v"(x1), "+v"(x2) : "v"(c));
    STOP(x0 + x1 + x2)
}

KHEAD(k_fma64_3src) {
    double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y0 = a, y1 = a + 1, y2 = a + 2, y3 = a + 3, z0 = 1, z1 = 2, z2 = 3, z3 = 4;
    START
#pragma unroll
    for (int r = 0; r < 64; ++r)
        asm volatile("v_fma_f64 %0, %4, %8, %0\n v_fma_f64 %1, %5, %9, %1\n v_fma_f64 %2, %6, %10, %2\n v_fma_f64 %3, %7, %11, %3"
                     : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(y0), "v"(y1), "v"(y2), "v"(y3), "v"(z0), "v"(z1), "v"(z2), "v"(z3));
    STOP(x0 + x1 + x2 + x3)
}

KHEAD(k_sel_fma) {
    double x = threadIdx.x, c = a;
    asm volatile("v_mov_b64 v[12:13], %0\n v_mov_b64 v[10:11], %1\n v_cmp_gt_f64 vcc, %1, %0" :: "v"(c), "v"(x) : "v10", "v11", "v12", "v13", "vcc");
    START
#pragma unroll
    for (int r = 0; r < 128; ++r)
        asm volatile("v_cndmask_b32 v10, v10, v12, vcc\n v_cndmask_b32 v11, v11, v13, vcc\n v_fma_f64 v[10:11], v[10:11], v[12:13], v[12:13]" ::: "v10", "v11", "vcc");
    asm volatile("v_mov_b64 %0, v[10:11]" : "=v"(x));
    STOP(x)
}

KHEAD(k_lds_use) {
    __shared__ double sh[512];
    for (int i = threadIdx.x; i < 512; i += 64) sh[i] = 0.0;
    __syncthreads();
    double x = threadIdx.x * 8.0, c = 1.0;
    START
#pragma unroll
    for (int r = 0; r < 64; ++r) {
        unsigned ad;
        asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(ad) : "v"(x));
        asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)\n v_add_f64 %0, %0, %2" : "=v"(x) : "v"(ad), "v"(c));
    }
    STOP(x)
}

KHEAD(k_vbranch) {
    double x = threadIdx.x, c = -1e30;
    START
#pragma unroll
    for (int r = 0; r < 64; ++r)
        asm volatile("v_cmp_gt_f64 vcc, %0, %1\n s_cbranch_vccz 1f\n v_add_f64 %0, %0, %1\n 1:" : "+v"(x) : "v"(c) : "vcc");
    STOP(x)
}

KHEAD(k_execmask) {
    double x = threadIdx.x, c = a;
    START
#pragma unroll
    for (int r = 0; r < 64; ++r)
        asm volatile("v_cmp_gt_f64 vcc, %0, %1\n s_and_saveexec_b64 s[20:21], vcc\n v_fma_f64 %0, %0, %1, %1\n s_or_b64 exec, exec, s[20:21]" : "+v"(x) : "v"(c) : "vcc", "s20", "s21");
    STOP(x)
}

KHEAD(k_halfexec) {
    double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7, c = a;
    long long t0 = 0, t1 = 0;
    if (threadIdx.x < 32) {
        t0 = clock64();
#pragma unroll
        for (int r = 0; r < 32; ++r)
            asm volatile("v_fma_f64 %0, %0, %8, %8\n v_fma_f64 %1, %1, %8, %8\n v_fma_f64 %2, %2, %8, %8\n v_fma_f64 %3, %3, %8, %8\n v_fma_f64 %4, %4, %8, %8\n v_fma_f64 %5, %5, %8, %8\n v_fma_f64 %6, %6, %8, %8\n v_fma_f64 %7, %7, %8, %8"
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(c));
        t1 = clock64();
    }
    out[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
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
    run("fma64 dist 1", k_fma64_c1, 256, d_out, d_cyc);
    run("fma64 dist 2", k_fma64_c2, 256, d_out, d_cyc);
    run("fma64 dist 3", k_fma64_c3, 255, d_out, d_cyc);
    run("fma64 dist 4", k_fma64_c4, 256, d_out, d_cyc);
    run("fma64 dist 5", k_fma64_c5, 255, d_out, d_cyc);
    run("fma64 dist 6", k_fma64_c6, 252, d_out, d_cyc);
    run("fma64 dist 8", k_fma64_c8, 256, d_out, d_cyc);
    run("fma32 dist 1", k_fma32_c1, 256, d_out, d_cyc);
    run("fma32 dist 2", k_fma32_c2, 256, d_out, d_cyc);
    run("fma32 dist 3", k_fma32_c3, 255, d_out, d_cyc);
    run("fma32 dist 4", k_fma32_c4, 256, d_out, d_cyc);
    run("mul64 dist 1", k_mul64_c1, 256, d_out, d_cyc);
    run("mul64 dist 2", k_mul64_c2, 256, d_out, d_cyc);
    run("mul64 dist 3", k_mul64_c3, 255, d_out, d_cyc);
    run("fma64 4ch 3src", k_fma64_3src, 256, d_out, d_cyc);
    run("2cnd+fma64 dep", k_sel_fma, 384, d_out, d_cyc);
    run("cvt+ds_read64+add64 dep", k_lds_use, 192, d_out, d_cyc);
    run("cmp64+cbranch+add64", k_vbranch, 192, d_out, d_cyc);
    run("cmp/saveexec/fma/restore", k_execmask, 256, d_out, d_cyc);
    run("fma64 ind8 32 lanes", k_halfexec, 256, d_out, d_cyc);
    return 0;
}
