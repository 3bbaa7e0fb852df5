// Dependent-chain latency and issue cost of the instruction classes the step
// kernel's dynamics call is made of, one wave alone on its SIMD (the step
// kernel's situation: 4096 envs x 16 lanes = one wave per SIMD).
// Each test runs a chain of N dependent (or K interleaved independent)
// operations inside a clock64() bracket; cycles per op = delta / ops.
//   hipcc --offload-arch=gfx950 -O3 -o lat lat.hip && ./lat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define N 4096

template <int K>
__global__ void fma64(double *out, long long *cyc, double a, double b) {
    double x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = threadIdx.x + k;
    __syncthreads();
    long long t0 = clock64();
    for (int i = 0; i < N / K; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = fma(x[k], a, b);
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int K>
__global__ void mul64(double *out, long long *cyc, double a, double b) {
    double x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = threadIdx.x + k + b;
    long long t0 = clock64();
    for (int i = 0; i < N / K; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = x[k] * a;
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

/* fp64 select chain: x = (x > c) ? x*a : x  -> v_cmp + 2 v_cndmask + mul */
template <int K>
__global__ void sel64(double *out, long long *cyc, double a, double b) {
    double x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = threadIdx.x + k + b;
    long long t0 = clock64();
    for (int i = 0; i < N / K; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double y = x[k] * a;
            x[k] = (x[k] > b) ? y : x[k];
        }
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int K>
__global__ void rcp64(double *out, long long *cyc, double a, double b) {
    double x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = threadIdx.x + k + 1.5;
    long long t0 = clock64();
    for (int i = 0; i < N / K; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = __builtin_amdgcn_rcp(x[k]);
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

/* 16-lane xor butterfly step on a double (the kernel's group sums) */
template <int K>
__global__ void shfl64(double *out, long long *cyc, double a, double b) {
    double x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = threadIdx.x + k;
    long long t0 = clock64();
    for (int i = 0; i < N / 16 / K; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = x[k] * a + __shfl_xor(x[k], 1 + (k & 7), 16);
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

/* dependent LDS round trip: store a double, read it back at a lane-dependent address */
template <int K>
__global__ void lds64(double *out, long long *cyc, double a, double b) {
    __shared__ double sh[64 * K];
    double x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = threadIdx.x + k;
    long long t0 = clock64();
    for (int i = 0; i < N / 16 / K; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            sh[k * 64 + threadIdx.x] = x[k];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            x[k] = sh[k * 64 + (threadIdx.x ^ 1)] * a;
        }
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

/* LDS loads only (read-only table, dependent index) */
template <int K>
__global__ void ldsld(double *out, long long *cyc, double a, double b) {
    __shared__ double sh[256];
    sh[threadIdx.x] = threadIdx.x * 0.5;
    sh[threadIdx.x + 64] = threadIdx.x * 0.25;
    sh[threadIdx.x + 128] = threadIdx.x;
    sh[threadIdx.x + 192] = 3.0;
    __syncthreads();
    int idx[K];
#pragma unroll
    for (int k = 0; k < K; ++k) idx[k] = (threadIdx.x + k) & 63;
    double acc = 0;
    long long t0 = clock64();
    for (int i = 0; i < N / 16 / K; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double v = sh[idx[k]];
            idx[k] = ((int)v + k) & 255;
        }
    }
    long long t1 = clock64();
#pragma unroll
    for (int k = 0; k < K; ++k) acc += idx[k];
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

typedef void (*kfn)(double *, long long *, double, double);

static void run(const char *name, kfn f, int ops, int k, double *d_out, long long *d_cyc) {
    long long best = -1;
    for (int r = 0; r < 5; ++r) {
        hipLaunchKernelGGL(f, dim3(1), dim3(64), 0, 0, d_out, d_cyc, 1.0000001, 0.5);
        hipDeviceSynchronize();
        long long c;
        hipMemcpy(&c, d_cyc, sizeof(c), hipMemcpyDeviceToHost);
        if (best < 0 || c < best) best = c;
    }
    printf("%-8s K=%d  cycles/op %.2f  (ops %d, clock64 delta %lld)\n", name, k, (double)best / ops, ops, best);
}

int main() {
    double *d_out;
    long long *d_cyc;
    hipMalloc(&d_out, 64 * sizeof(double));
    hipMalloc(&d_cyc, sizeof(long long));
    run("fma64", fma64<1>, N, 1, d_out, d_cyc);
    run("fma64", fma64<2>, N, 2, d_out, d_cyc);
    run("fma64", fma64<4>, N, 4, d_out, d_cyc);
    run("fma64", fma64<8>, N, 8, d_out, d_cyc);
    run("mul64", mul64<1>, N, 1, d_out, d_cyc);
    run("mul64", mul64<4>, N, 4, d_out, d_cyc);
    run("sel64", sel64<1>, N, 1, d_out, d_cyc);
    run("sel64", sel64<4>, N, 4, d_out, d_cyc);
    run("rcp64", rcp64<1>, N, 1, d_out, d_cyc);
    run("rcp64", rcp64<4>, N, 4, d_out, d_cyc);
    run("shfl64", shfl64<1>, N / 16, 1, d_out, d_cyc);
    run("shfl64", shfl64<4>, N / 16, 4, d_out, d_cyc);
    run("lds64", lds64<1>, N / 16, 1, d_out, d_cyc);
    run("lds64", lds64<4>, N / 16, 4, d_out, d_cyc);
    run("ldsld", ldsld<1>, N / 16, 1, d_out, d_cyc);
    run("ldsld", ldsld<4>, N / 16, 4, d_out, d_cyc);
    return 0;
}
