// Micro: HBM read rate of the selection pass's access pattern on a 3.2 GB buffer (round 6).  k_sync_count reads
// the C4 arena at ~3.6 TB/s while tools/micro/reread.hip's persistent streaming form reaches ~6 TB/s; the forms here
// do the same loads with a trivial reduction instead of the sync-pattern test, to separate the pattern from the work:
//   F0  one 256-thread work-group per 64 KB, each wave 16 x 1 KB loads in flight (k_sync_count's pattern)
//   F1  one 256-thread work-group per 32 KB, 8 loads per wave
//   F2  one 1024-thread work-group per 256 KB, 16 loads per wave
//   F3  persistent: 4 work-groups per CU walking the 64 KB blocks (grid stride), 16 loads per wave per block
//   F4  F0 with the loads issued in two halves of 8 (the second half after the first is reduced)
// build: hipcc --offload-arch=gfx950 -O3 -o sel_pattern sel_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int STEPS>
__device__ inline uint32_t wave_read(const uint8_t *wb, int lane) {
    uint4 v[STEPS];
#pragma unroll
    for (int k = 0; k < STEPS; k++) v[k] = *reinterpret_cast<const uint4 *>(wb + 1024 * k + 16 * lane);
    uint32_t a = 0;
#pragma unroll
    for (int k = 0; k < STEPS; k++) a ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    return a;
}

template <int STEPS, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) k_block(const uint8_t *buf, uint32_t *out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint8_t *wb = buf + (int64_t)blockIdx.x * (1024 * STEPS * WAVES) + (int64_t)(1024 * STEPS) * wv;
    const uint32_t a = wave_read<STEPS>(wb, lane);
    if (a == 0x12345678u) out[blockIdx.x] = a;  // (never: keeps the loads)
}

__global__ void __launch_bounds__(256) k_persist(const uint8_t *buf, int64_t nblocks, uint32_t *out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t a = 0;
    for (int64_t b = blockIdx.x; b < nblocks; b += gridDim.x)
        a ^= wave_read<16>(buf + b * 65536 + 16384 * wv, lane);
    if (a == 0x12345678u) out[blockIdx.x] = a;
}

__global__ void __launch_bounds__(256) k_halves(const uint8_t *buf, uint32_t *out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint8_t *wb = buf + (int64_t)blockIdx.x * 65536 + 16384 * wv;
    uint32_t a = wave_read<8>(wb, lane);
    a ^= wave_read<8>(wb + 8192, lane);
    if (a == 0x12345678u) out[blockIdx.x] = a;
}

int main() {
    const int64_t bytes = 3200000000ll / 262144 * 262144;
    uint8_t *buf;
    uint32_t *out;
    if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
    (void)hipMemset(buf, 0x5A, bytes);
    (void)hipMalloc(&out, 1 << 24);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int form = 0; form < 5; form++) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; rep++) {
            (void)hipEventRecord(a);
            if (form == 0) k_block<16, 4><<<(unsigned)(bytes / 65536), 256>>>(buf, out);
            if (form == 1) k_block<8, 4><<<(unsigned)(bytes / 32768), 256>>>(buf, out);
            if (form == 2) k_block<16, 16><<<(unsigned)(bytes / 262144), 1024>>>(buf, out);
            if (form == 3) k_persist<<<cus * 4, 256>>>(buf, bytes / 65536, out);
            if (form == 4) k_halves<<<(unsigned)(bytes / 65536), 256>>>(buf, out);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        printf("F%d: %.3f ms, %.0f GB/s\n", form, best, bytes / best / 1e6);
    }
    return 0;
}
