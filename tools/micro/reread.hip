// Micro: can a tile's second read come from on-die caches (Infinity Cache / L2) when each CU works on ONE 512 KB
// tile at a time?  The analysis reads every C4 tile twice (min/max, then the autocorrelation pass); with one wave per
// tile and ~4096 tiles in flight the second read goes back to HBM.  Here a persistent work-group per CU (or two) takes
// 512 KB tiles from a counter and reads each twice back to back (form 1), or reads it once (form 0, the HBM baseline),
// or reads tile k's second pass after tile k+1's first (form 2, one tile of lag).  Prints ms and effective GB/s of the
// bytes loaded (2x for forms 1, 2).
// build: hipcc --offload-arch=gfx950 -O3 -o reread reread.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr int64_t kTile = 512 * 1024;  // bytes

__device__ inline uint32_t read_tile(const uint4 *p, int tid, int nthr) {
    uint32_t acc = 0;
    const int nvec = (int)(kTile / 16);
    for (int i = tid; i < nvec; i += nthr * 8) {
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int k = i + u * nthr;
            v[u] = k < nvec ? p[k] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    return acc;
}

template <int FORM>
__global__ void __launch_bounds__(256) k_reread(const uint4 *buf, int64_t ntiles, int *ctr, uint32_t *out) {
    __shared__ int s_t;
    uint32_t acc = 0;
    int prev = -1;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) s_t = atomicAdd(ctr, 1);
        __syncthreads();
        const int t = s_t;
        if (t >= ntiles) break;
        const uint4 *p = buf + (int64_t)t * (kTile / 16);
        acc += read_tile(p, threadIdx.x, blockDim.x);
        if constexpr (FORM == 1) acc += 3u * read_tile(p, threadIdx.x, blockDim.x);
        if constexpr (FORM == 2) {
            if (prev >= 0) acc += 3u * read_tile(buf + (int64_t)prev * (kTile / 16), threadIdx.x, blockDim.x);
            prev = t;
        }
    }
    if constexpr (FORM == 2)
        if (prev >= 0) acc += 3u * read_tile(buf + (int64_t)prev * (kTile / 16), threadIdx.x, blockDim.x);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    const int64_t bytes = 3200000000ll;
    const int64_t ntiles = bytes / kTile;
    uint4 *buf;
    int *ctr;
    uint32_t *out;
    if (hipMalloc(&buf, ntiles * kTile) != hipSuccess) return 1;
    (void)hipMemset(buf, 0x5A, ntiles * kTile);
    (void)hipMalloc(&ctr, 4);
    (void)hipMalloc(&out, 4 << 20);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int per_cu : {1, 2, 4}) {
        for (int form = 0; form < 3; form++) {
            float best = 1e9f;
            for (int rep = 0; rep < 3; rep++) {
                (void)hipMemset(ctr, 0, 4);
                (void)hipEventRecord(a);
                const int grid = cus * per_cu;
                if (form == 0) k_reread<0><<<grid, 256>>>(buf, ntiles, ctr, out);
                else if (form == 1) k_reread<1><<<grid, 256>>>(buf, ntiles, ctr, out);
                else k_reread<2><<<grid, 256>>>(buf, ntiles, ctr, out);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
            }
            const double loaded = (double)ntiles * kTile * (form ? 2 : 1);
            printf("WGs/CU %d form %d: %.3f ms, %.0f GB/s of loaded bytes\n", per_cu, form, best, loaded / best / 1e6);
        }
    }
    return 0;
}
