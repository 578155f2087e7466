// Micro: sustained v_fmac_f64 rate in the autocorrelation pattern (9 accumulators, each updated once per sample,
// operands from a 16-register window), vs waves per SIMD.  Prints cycles per wave64 FMA per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 -o fma64_rate fma64_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int LAGS>
__global__ void __launch_bounds__(256) k_autoc(const float *in, double *out, int n) {
    double acc[LAGS], prev[8];
    for (int l = 0; l < LAGS; l++) acc[l] = 0.0;
    for (int j = 0; j < 8; j++) prev[j] = (double)in[(threadIdx.x + j) & 255];
    float x = in[threadIdx.x];
    for (int i = 0; i < n; i += 8) {
        double cur[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            x = x * 1.0001f + 0.5f;
            cur[j] = (double)x;
        }
#pragma unroll
        for (int j = 0; j < 8; j++)
#pragma unroll
            for (int l = 0; l < LAGS; l++) acc[l] = fma(cur[j], (j - l >= 0) ? cur[j - l] : prev[8 + j - l], acc[l]);
#pragma unroll
        for (int j = 0; j < 8; j++) prev[j] = cur[j];
    }
    double s = 0;
    for (int l = 0; l < LAGS; l++) s += acc[l];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    float *in;
    double *out;
    hipMalloc(&in, 1024);
    hipMemset(in, 0, 1024);
    const int n = 4096;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int wps : {1, 2, 3, 4, 6, 8}) {
        const int blocks = 256 * wps;  // 4 waves per block, 4 SIMDs per CU
        hipMalloc(&out, sizeof(double) * blocks * 256);
        k_autoc<9><<<blocks, 256>>>(in, out, n);
        hipEventRecord(a);
        k_autoc<9><<<blocks, 256>>>(in, out, n);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double fmas = (double)blocks * 4 * n * 9;  // wave64 FMAs
        const double per_simd = fmas / 1024.0;
        printf("waves/SIMD %d: %.3f ms, %.2f ns per wave-FMA per SIMD (%.2f cycles @2.4GHz)\n", wps, ms,
               ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
        hipFree(out);
    }
    return 0;
}
