// Micro: the C5 pipe decoder's LPC restore (one wave, x[i] = (R[i] + sum_j q_j x[i-1-j]) >> shift, 16-bit samples,
// order 8, residuals pre-shifted in LDS) in two forms, ns per sample on one wave:
//   A  the round-5 pair step: 8 v_dot2 per pair, the newest pair (x[2m-1], x[2m-2]) through a dot2 (chain per pair:
//      perm -> dot2 -> ashr -> mul24 -> add -> ashr)
//   B  the newest two samples as 24-bit multiplies (the compiler sums them with v_add3: chain per pair mul -> add3 ->
//      ashr -> mul -> add3 -> ashr), the older pairs by dot2 one step ahead
//   C  B with v_mad_i32_i24 forced on the chain (mad -> ashr -> mad -> ashr)
//   D  A with the 64-sample group's residuals read from LDS up front (16 ds_read_b128 back to back): A reads four
//      residuals every second pair and waits for them at once (s_waitcnt lgkmcnt(0): an LDS round trip per 4 samples
//      on the lone wave's chain)
//   E, F  B and C with the group's residuals read up front as in D
// The outputs are checked against a host restore.
// build: hipcc --offload-arch=gfx950 -O3 -o restore_chain restore_chain.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef short v2s16 __attribute__((ext_vector_type(2)));
__device__ inline int32_t dot2(uint32_t a, uint32_t b, int32_t c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s16, a), __builtin_bit_cast(v2s16, b), c, false);
}
__device__ inline uint32_t pk(int32_t hi, int32_t lo) { return ((uint32_t)hi << 16) | ((uint32_t)lo & 0xFFFFu); }

constexpr int N = 4096;

template <int FORM>
__global__ void __launch_bounds__(64) k_restore(const int32_t *R, const int32_t *q, int shift, int reps, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) int32_t res[N + 64];
    __shared__ __attribute__((aligned(16))) uint32_t xout[N / 2];
    for (int i = threadIdx.x; i < N; i += 64) res[i] = R[i];
    // warm-up: x[0..7] = 0 (the restore starts at sample 8 on pair-aligned history)
    for (int i = threadIdx.x; i < 4; i += 64) xout[i] = 0;
    __syncthreads();
    int32_t q0 = q[0], q1 = q[1], q2 = q[2];
    // (the real decoder's operands live in VGPRs: keep the compiler from moving the wave-uniform math to the SALU)
    asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2));
    uint32_t Ce[4], Co[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        Ce[k] = pk(q[2 * k], q[2 * k + 1]);
        Co[k] = pk(q[2 * k + 1], k < 3 ? q[2 * k + 2] : 0);
        asm volatile("" : "+v"(Ce[k]), "+v"(Co[k]));
    }
    for (int rep = 0; rep < reps; rep++) {
        uint32_t Qr[4] = {0, 0, 0, 0};
        int32_t xe_p = 0, xo_p = 0;
        for (int i = 8; i < N; i += 64) {
            int4 rr = make_int4(0, 0, 0, 0);
            const int4 *rp = reinterpret_cast<const int4 *>(&res[i]);
            uint32_t *xp = xout + (i >> 1);
            int4 rall[FORM >= 3 ? 16 : 1];
            if constexpr (FORM >= 3) {
#pragma unroll
                for (int j = 0; j < 16; j++) rall[j] = rp[j];
            }
#pragma unroll
            for (int p2 = 0; p2 < 32; p2++) {
                if (i + 2 * p2 >= N) break;
                if (!(p2 & 1)) {
                    if constexpr (FORM >= 3) rr = rall[p2 >> 1];
                    else rr = rp[p2 >> 1];
                    asm volatile("" : "+v"(rr.x), "+v"(rr.y), "+v"(rr.z), "+v"(rr.w));
                }
                const int32_t Re = (p2 & 1) ? rr.z : rr.x, Ro = (p2 & 1) ? rr.w : rr.y;
                const uint32_t A = Qr[(p2 + 3) & 3], B = Qr[(p2 + 2) & 3], Cc = Qr[(p2 + 1) & 3], Dd = Qr[p2 & 3];
                uint32_t qn;
                if constexpr (FORM == 0 || FORM == 3) {
                    int32_t pe = dot2(Dd, Ce[3], Re);
                    pe = dot2(Cc, Ce[2], pe);
                    pe = dot2(B, Ce[1], pe);
                    int32_t po = dot2(Dd, Co[3], Ro);
                    po = dot2(Cc, Co[2], po);
                    po = dot2(B, Co[1], po);
                    po = dot2(A, Co[0], po);
                    pe = dot2(A, Ce[0], pe);
                    const int32_t xe = pe >> shift;
                    const int32_t xo = (__mul24(q0, xe) + po) >> shift;
                    qn = __builtin_amdgcn_perm((uint32_t)xo, (uint32_t)xe, 0x05040100u);
                } else if constexpr (FORM == 2 || FORM == 5) {
                    // B with explicit v_mad_i32_i24 on the chain: x[i-1] -> mad -> ashr -> mad -> ashr
                    int32_t pe = dot2(Dd, Ce[3], Re);
                    pe = dot2(Cc, Ce[2], pe);
                    pe = dot2(B, Ce[1], pe);
                    int32_t po = dot2(Dd, Co[3], Ro);
                    po = dot2(Cc, Co[2], po);
                    po = dot2(B, Co[1], po);
                    int32_t te, to, xe, xo;
                    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(te) : "v"(q1), "v"(xe_p), "v"(pe));
                    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(to) : "v"(q2), "v"(xe_p), "v"(po));
                    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(to) : "v"(q1), "v"(xo_p), "v"(to));
                    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(te) : "v"(q0), "v"(xo_p), "v"(te));
                    xe = te >> shift;
                    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(to) : "v"(q0), "v"(xe), "v"(to));
                    xo = to >> shift;
                    qn = __builtin_amdgcn_perm((uint32_t)xo, (uint32_t)xe, 0x05040100u);
                    xe_p = xe;
                    xo_p = xo;
                } else {
                    // older pairs (B, Cc, Dd) by dot2; the newest pair's samples (xe_p = x[2m-2], xo_p = x[2m-1]) and
                    // this step's even sample by multiply-adds: only q0 * x[i-1] waits on the previous sample
                    int32_t pe = dot2(Dd, Ce[3], Re);
                    pe = dot2(Cc, Ce[2], pe);
                    pe = dot2(B, Ce[1], pe);
                    int32_t po = dot2(Dd, Co[3], Ro);
                    po = dot2(Cc, Co[2], po);
                    po = dot2(B, Co[1], po);
                    pe = __mul24(q1, xe_p) + pe;
                    po = __mul24(q2, xe_p) + po;
                    po = __mul24(q1, xo_p) + po;
                    const int32_t xe = (__mul24(q0, xo_p) + pe) >> shift;
                    const int32_t xo = (__mul24(q0, xe) + po) >> shift;
                    qn = __builtin_amdgcn_perm((uint32_t)xo, (uint32_t)xe, 0x05040100u);
                    xe_p = xe;
                    xo_p = xo;
                }
                xp[p2] = qn;
                Qr[p2 & 3] = qn;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < N / 2; i += 64) out[i] = xout[i];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const int32_t qh[8] = {1800, -900, 420, -260, 130, -70, 30, -9};
    const int shift = 10;
    std::vector<int32_t> x(N, 0), R(N, 0);
    srand(7);
    for (int i = 8; i < N; i++) {
        int64_t s = 0;
        for (int j = 0; j < 8; j++) s += (int64_t)qh[j] * x[i - 1 - j];
        const int32_t r = (rand() % 2001) - 1000;
        int32_t v = (int32_t)((((int32_t)s) + (r << shift)) >> shift);
        if (v > 32767 || v < -32768) v = 0;
        x[i] = v;
        R[i] = (int32_t)(((int64_t)x[i] << shift) - (int32_t)s);  // so that (R + s) >> shift == x[i]
    }
    int32_t *dR, *dq;
    uint32_t *dout;
    hipMalloc(&dR, N * 4);
    hipMalloc(&dq, 32);
    hipMalloc(&dout, N * 2);
    hipMemcpy(dR, R.data(), N * 4, hipMemcpyHostToDevice);
    hipMemcpy(dq, qh, 32, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int form = 0; form < 6; form++) {
        for (int pass = 0; pass < 2; pass++) {
            hipEventRecord(a);
            if (form == 0) k_restore<0><<<1, 64>>>(dR, dq, shift, reps, dout);
            else if (form == 1) k_restore<1><<<1, 64>>>(dR, dq, shift, reps, dout);
            else if (form == 2) k_restore<2><<<1, 64>>>(dR, dq, shift, reps, dout);
            else if (form == 3) k_restore<3><<<1, 64>>>(dR, dq, shift, reps, dout);
            else if (form == 4) k_restore<4><<<1, 64>>>(dR, dq, shift, reps, dout);
            else k_restore<5><<<1, 64>>>(dR, dq, shift, reps, dout);
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        std::vector<uint32_t> o(N / 2);
        hipMemcpy(o.data(), dout, N * 2, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 8; i < N; i++) {
            const int16_t g = (int16_t)(o[i >> 1] >> (16 * (i & 1)));
            bad += g != (int16_t)x[i];
        }
        printf("form %c: %.2f ns/sample (%d reps), mismatches %d\n", "ABCDEF"[form], ms * 1e6 / ((double)reps * (N - 8)),
               reps, bad);
    }
    return 0;
}
