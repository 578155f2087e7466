// Microbenchmark: cycles per instruction for ONE wave on a CU (dependent / independent SALU and VALU chains,
// scalar 64-bit bit ops, v_readlane round trips).  s_memtime deltas; prints cycles per op.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int KIND>
__global__ void k_rate(uint64_t *out, uint32_t seed, int iters) {
    uint32_t a = seed, b = seed * 3u + 1u, c = seed ^ 0x55u, d = seed + 7u;
    uint64_t w = (uint64_t)seed << 17 | 1u;
    uint32_t v = threadIdx.x + seed;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        if constexpr (KIND == 0) {  // dependent SALU adds (uniform)
#pragma unroll
            for (int k = 0; k < 16; k++) { a = a + b; asm volatile("" : "+s"(a)); }
        } else if constexpr (KIND == 1) {  // 4 independent SALU chains
#pragma unroll
            for (int k = 0; k < 4; k++) {
                a += 1u; b += 3u; c ^= a; d += c;
                asm volatile("" : "+s"(a), "+s"(b), "+s"(c), "+s"(d));
            }
        } else if constexpr (KIND == 2) {  // dependent 64-bit scalar shift + clz chain (rice-like)
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int z = __builtin_clzll(w | 1);
                w = (w << ((z & 7) + 1)) ^ 0x9E3779B97F4A7C15ull;
                asm volatile("" : "+s"(w));
            }
        } else if constexpr (KIND == 3) {  // dependent VALU adds
#pragma unroll
            for (int k = 0; k < 16; k++) { v = v + 0x1234u; asm volatile("" : "+v"(v)); }
        } else if constexpr (KIND == 4) {  // 4 independent VALU chains
            uint32_t v1 = v + 1, v2 = v + 2, v3 = v + 3;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                v += 1u; v1 += 3u; v2 ^= v; v3 += v1;
                asm volatile("" : "+v"(v), "+v"(v1), "+v"(v2), "+v"(v3));
            }
            v ^= v1 ^ v2 ^ v3;
        } else if constexpr (KIND == 5) {  // v_readlane -> scalar use round trip
#pragma unroll
            for (int k = 0; k < 8; k++) {
                a = (uint32_t)__builtin_amdgcn_readlane((int)(v + a), (int)(a & 63));
                asm volatile("" : "+s"(a));
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = a + b + c + d + (uint32_t)w + v; }
}

int main() {
    uint64_t *d, h[2];
    hipMalloc(&d, 16);
    const char *names[] = {"salu dependent add", "salu 4 indep chains (per op)", "salu clz+shl64+xor dep (per op)",
                           "valu dependent add", "valu 4 indep chains (per op)", "readlane->salu round trip"};
    const double ops[] = {16, 16, 24, 16, 16, 8};
    const int iters = 4096;
    for (int kind = 0; kind < 6; kind++) {
        for (int rep = 0; rep < 2; rep++) {
            switch (kind) {
            case 0: k_rate<0><<<1, 64>>>(d, 5, iters); break;
            case 1: k_rate<1><<<1, 64>>>(d, 5, iters); break;
            case 2: k_rate<2><<<1, 64>>>(d, 5, iters); break;
            case 3: k_rate<3><<<1, 64>>>(d, 5, iters); break;
            case 4: k_rate<4><<<1, 64>>>(d, 5, iters); break;
            case 5: k_rate<5><<<1, 64>>>(d, 5, iters); break;
            }
            hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        }
        // s_memtime counts at the shader clock on gfx950 (compare with the 100 MHz s_memrealtime if unsure)
        printf("%-36s %8.2f memtime ticks per op\n", names[kind], (double)h[0] / (iters * ops[kind]));
    }
    return 0;
}
