// Micro: do a wave running fp64 FMA chains and a wave running 32-bit integer VALU chains share one SIMD's issue
// (time = sum) or overlap (time = max)?  Work-groups of 8 waves (two per SIMD): waves 0-3 run workload A, waves 4-7
// workload B.  Modes: 0 = fp64 + fp64, 1 = int + int, 2 = fp64 + int.  Prints ms per mode.
// build: hipcc --offload-arch=gfx950 -O3 -o coissue coissue.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ double fp64_work(int n, double seed) {
    double acc[9], x[9];
    for (int l = 0; l < 9; l++) acc[l] = 0.0, x[l] = seed + l;
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int l = 0; l < 9; l++) acc[l] = fma(x[l], x[(l + 3) % 9], acc[l]);
#pragma unroll
        for (int l = 0; l < 9; l++) asm volatile("" : "+v"(x[l]));
    }
    double s = 0;
    for (int l = 0; l < 9; l++) s += acc[l];
    return s;
}

__device__ unsigned int_work(int n, unsigned seed) {
    unsigned a[9];
    for (int l = 0; l < 9; l++) a[l] = seed * (l + 1);
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int l = 0; l < 9; l++) {
            unsigned d;
            asm volatile("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a[l]), "v"(a[(l + 1) % 9]), "v"(a[l]));
            a[l] = (d ^ 0x80000000u) + 7u;  // 3 VALU per element: sad, xor, add
        }
    }
    unsigned s = 0;
    for (int l = 0; l < 9; l++) s += a[l];
    return s;
}

__global__ void __launch_bounds__(512) k_mix(int mode, int n, double *out) {
    const int wave = threadIdx.x >> 6;
    const bool second = wave >= 4;
    double r;
    // fp64: 9 FMAs per iteration; int: 27 VALU per iteration -- iteration counts scaled so each alone is comparable
    const bool fp = mode == 0 || (mode == 2 && !second);
    if (fp) r = fp64_work(n, threadIdx.x);
    else r = (double)int_work(n * 2, threadIdx.x);
    out[blockIdx.x * 512 + threadIdx.x] = r;
}

int main() {
    double *out;
    const int blocks = 256;  // one 8-wave work-group per CU: two waves per SIMD
    hipMalloc(&out, sizeof(double) * blocks * 512);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int n = 8192;
    for (int rep = 0; rep < 2; rep++)
        for (int mode : {0, 1, 2}) {
            k_mix<<<blocks, 512>>>(mode, n, out);
            hipEventRecord(a);
            k_mix<<<blocks, 512>>>(mode, n, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("mode %d (%s): %.3f ms\n", mode, mode == 0 ? "fp64+fp64" : mode == 1 ? "int+int" : "fp64+int", ms);
        }
    return 0;
}
