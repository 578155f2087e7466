// Micro: issue rate and dependent latency of single VALU ops for ONE wave alone on its SIMD (the C5 consumer wave's
// situation): cycles per instruction from s_memtime around 8 x 1024 instructions, either as 8 independent chains
// (throughput) or one dependent chain (latency).  Ops: v_add_u32, v_mad_i32_i24, v_dot2_i32_i16, v_perm_b32,
// v_ashrrev_i32, v_mad_u32_u24, v_alignbit_b32.
// build: hipcc --offload-arch=gfx950 -O3 -o valu_rates valu_rates.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define OP_ADD(d, a, b) asm volatile("v_add_u32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b))
#define OP_MAD24(d, a, b) asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b))
#define OP_DOT2(d, a, b) asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b))
#define OP_PERM(d, a, b) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b))
#define OP_ASHR(d, a, b) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(d) : "v"(a))
#define OP_MADU24(d, a, b) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b))
#define OP_ALIGN(d, a, b) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(d) : "v"(a), "v"(b))

template <int OP, bool DEP>
__global__ void __launch_bounds__(64) k_rate(uint32_t a0, uint32_t b0, uint32_t *out, uint64_t *cyc) {
    uint32_t a = a0 + threadIdx.x, b = b0;
    uint32_t d[8];
#pragma unroll
    for (int k = 0; k < 8; k++) d[k] = threadIdx.x * (k + 1);
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int it = 0; it < 1024; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint32_t &x = DEP ? d[0] : d[k];
            if constexpr (OP == 0) { uint32_t y; OP_ADD(y, x, a); x = y; }
            if constexpr (OP == 1) OP_MAD24(x, a, b);
            if constexpr (OP == 2) OP_DOT2(x, a, b);
            if constexpr (OP == 3) OP_PERM(x, a, b);
            if constexpr (OP == 4) OP_ASHR(x, b, a);
            if constexpr (OP == 5) OP_MADU24(x, a, b);
            if constexpr (OP == 6) OP_ALIGN(x, a, b);
        }
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += d[k];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int OP, bool DEP>
double run(uint32_t *out, uint64_t *cyc) {
    uint64_t best = ~0ull;
    for (int r = 0; r < 5; r++) {
        k_rate<OP, DEP><<<1, 64>>>(3u, 0x00050007u, out, cyc);
        uint64_t c;
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        if (c < best) best = c;
    }
    return (double)best / (8.0 * 1024.0);
}

int main() {
    uint32_t *out;
    uint64_t *cyc;
    (void)hipMalloc(&out, 4096);
    (void)hipMalloc(&cyc, 8);
    const char *names[] = {"v_add_u32", "v_mad_i32_i24", "v_dot2_i32_i16", "v_perm_b32", "v_ashrrev_i32", "v_mad_u32_u24",
                           "v_alignbit_b32"};
    double tp[7], lat[7];
    tp[0] = run<0, false>(out, cyc), lat[0] = run<0, true>(out, cyc);
    tp[1] = run<1, false>(out, cyc), lat[1] = run<1, true>(out, cyc);
    tp[2] = run<2, false>(out, cyc), lat[2] = run<2, true>(out, cyc);
    tp[3] = run<3, false>(out, cyc), lat[3] = run<3, true>(out, cyc);
    tp[4] = run<4, false>(out, cyc), lat[4] = run<4, true>(out, cyc);
    tp[5] = run<5, false>(out, cyc), lat[5] = run<5, true>(out, cyc);
    tp[6] = run<6, false>(out, cyc), lat[6] = run<6, true>(out, cyc);
    for (int i = 0; i < 7; i++)
        printf("%-16s independent %.2f  dependent %.2f  (counter ticks per instruction, one wave)\n", names[i], tp[i],
               lat[i]);
    return 0;
}
