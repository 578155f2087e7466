"""Round-4 analysis variant: software-pipelined sample loads in k_analyze_v3's lean launch (32-sample chunks, the next
chunk's loads in flight while the current one is summed: two 16-VGPR chunks where one 64-sample chunk held 32)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from build_variant import build_variant

ANCHOR = "// min/max of a whole tile by one wave (16-bit samples, 16-B aligned rows)"
PF = r'''
template <int DT, int KIND, int kAnaChunk>
__device__ inline void ana_autoc_pf(const typename Elem<DT>::T *base, const EncodeParams &P, const TileGeom &g,
                                    int64_t s0, const TileNorm &tn, const int16_t *slut, const int16_t *glut,
                                    const float *__restrict__ swin, int vec, double *acc, uint32_t &or_acc, uint32_t *ft) {
    using Ch = ChunkN<DT, kAnaChunk>;
    const uint32_t r0 = udiv_inv((uint32_t)s0, (uint32_t)g.w, 1.0 / (double)g.w);
    int64_t crow = r0;
    int ccol = (int)((uint32_t)s0 - r0 * (uint32_t)g.w);
    double prev[8];
#pragma unroll
    for (int j = 0; j < 8; j++) prev[j] = 0.0;
    uint32_t x1 = 0x80000000u, e1p = 0x80000000u, e2p = 0x80000000u, e3p = 0x80000000u;
    uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, s0t = 0, s1t = 0, s2t = 0, s3t = 0, s4t = 0;
    auto fetch = [&](Ch &ch) {
        ch.template load<true>(base, P.row_stride, g.w, crow, ccol, vec, kAnaChunk);
        ccol += kAnaChunk;
        while (ccol >= g.w) {
            ccol -= g.w;
            crow++;
        }
    };
    auto sum = [&](const Ch &ch, int i0, bool first) {
#pragma unroll
        for (int b = 0; b < kAnaChunk / 8; b++) {
            double cur[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int32_t x = ana_norm<DT, KIND>(ch.get(8 * b + j), tn, slut, glut);
                or_acc |= (uint32_t)x;
                cur[j] = (double)((float)x * swin[i0 + 8 * b + j]);
                const uint32_t y0 = (uint32_t)x ^ 0x80000000u;
                const uint32_t y1 = (y0 - x1) ^ 0x80000000u, y2 = (y1 - e1p) ^ 0x80000000u, y3 = (y2 - e2p) ^ 0x80000000u;
                t0 = ana_sad(y0, 0x80000000u, t0);
                t1 = ana_sad(y0, x1, t1);
                t2 = ana_sad(y1, e1p, t2);
                t3 = ana_sad(y2, e2p, t3);
                t4 = ana_sad(y3, e3p, t4);
                x1 = y0;
                e1p = y1;
                e2p = y2;
                e3p = y3;
                if (b == 0 && j == 3 && first) {
                    s0t = t0;
                    s1t = t1;
                    s2t = t2;
                    s3t = t3;
                    s4t = t4;
                }
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
#pragma unroll
                for (int l = 0; l <= kMaxLpc; l++) acc[l] = fma(cur[j], (j - l >= 0) ? cur[j - l] : prev[8 + j - l], acc[l]);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) prev[j] = cur[j];
        }
    };
    constexpr int nch = kMaxBlock / kAnaChunk;
    static_assert(nch % 2 == 0, "pairs of chunks");
    Ch a, b;
    fetch(a);
    for (int c = 0; c < nch; c += 2) {
        fetch(b);  // chunk c + 1 in flight while chunk c is summed
        sum(a, c * kAnaChunk, c == 0);
        if (c + 2 < nch) fetch(a);
        sum(b, (c + 1) * kAnaChunk, false);
    }
    ft[0] = t0 - s0t;
    ft[1] = t1 - s1t;
    ft[2] = t2 - s2t;
    ft[3] = t3 - s3t;
    ft[4] = t4 - s4t;
}

'''
CALL_LDS = "            ana_autoc<DT, kAnaKindLds, kChunk>(base, P, g, s0, tn, wl, glut, window, vec, acc, or_acc, ft);\n        } else {\n            ana_autoc<DT, kAnaKindZero, kChunk>(base, P, g, s0, tn, wl, glut, window, vec, acc, or_acc, ft);"
CALL_PF = "            ana_autoc_pf<DT, kAnaKindLds, 32>(base, P, g, s0, tn, wl, glut, window, vec32, acc, or_acc, ft);\n        } else {\n            ana_autoc_pf<DT, kAnaKindZero, 32>(base, P, g, s0, tn, wl, glut, window, vec32, acc, or_acc, ft);"
VEC = "fp64 division)\n    const int vec = (g.w % kChunk) == 0 ? P.vec_ok : 0;\n"
VEC_PF = "fp64 division)\n    const int vec = (g.w % kChunk) == 0 ? P.vec_ok : 0;\n    const int vec32 = (g.w % 32) == 0 ? P.vec_ok : 0;\n"


LB_A = "template <int DT, bool SLOW, bool STATS = false>\n__global__ void __launch_bounds__(256) k_analyze_v3("
LB_B = "template <int DT, bool SLOW, bool STATS = false>\n__global__ void __launch_bounds__(256, SLOW ? 1 : 4) k_analyze_v3("


def patch(s):
    assert ANCHOR in s and CALL_LDS in s and s.count(VEC) == 1 and LB_A in s
    return s.replace(ANCHOR, PF + ANCHOR).replace(CALL_LDS, CALL_PF).replace(VEC, VEC_PF).replace(LB_A, LB_B)


if __name__ == "__main__":
    print(build_variant("base", lambda s: s))
    print(build_variant("anapf", patch))
