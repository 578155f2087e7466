#!/usr/bin/env python3
"""Timing-only ablations of k_encode_v3: each variant removes one pass of encode_frame_v3 (its output is wrong),
so the kernel time it saves is that pass's share.  Builds variants/lib<name>.so (tools/build_variant.py); run
them on the GPU box with tools/gpu/gpu_variants.sh and compare kernels_ms.encode."""
import sys

from build_variant import build_variant


def sub(old, new):
    def f(src):
        assert old in src, old[:60]
        return src.replace(old, new, 1)
    return f


def chain(*fs):
    def f(src):
        for g in fs:
            src = g(src)
        return src
    return f


NOCRC = sub("    if (ok) {\n        // slice-by-4", "    if (false) {\n        // slice-by-4")
NOPACK = sub("    } else if (type >= 2 && ok) {\n        // code = stop bit",
             "    } else if (false) {\n        // code = stop bit")
NOLENS = sub("        uint32_t lens = 0;\n#pragma unroll\n        for (int m = 0; m < 32; m++) {",
             "        uint32_t lens = 900;\n#pragma unroll\n        for (int m = 0; m < 0; m++) {")
NOLPCSUM = sub("    uint32_t sl = 0;\n    if (cand_lpc) {", "    uint32_t sl = 5000;\n    if (false) {")
NOFIXED = sub("    uint32_t sf = 0;  // the lane's sum of |e_of(i)| (lane 0 from i = of)\n    if (cand_fixed) {",
              "    uint32_t sf = 6000;\n    if (false) {")
NOSTORE = sub("    } else if (fbytes) {\n        // ---- store", "    } else if (false) {\n        // ---- store")

VARIANTS = {
    "base": lambda s: s,
    "nocrc": NOCRC,
    "nopack": NOPACK,
    "nolens_nopack": chain(NOLENS, NOPACK),
    "nolpcsum": NOLPCSUM,
    "nofixed": NOFIXED,
    "nostore": NOSTORE,
}

# ---- per-phase wave clocks (s_memtime deltas summed over waves), printed to stderr after each encode launch
PH_DECL = """__device__ unsigned long long g_ph[16];
#define PH(i) do { const uint64_t _t = __builtin_amdgcn_s_memtime(); ph[i] += _t - _pt; _pt = _t; } while (0)
template <int K>
__device__ inline uint32_t fixed_lane_sum("""


def phases(src):
    s = src
    rep = [
        ("template <int K>\n__device__ inline uint32_t fixed_lane_sum(", PH_DECL),
        ("    TileNorm tn = norms[t];\n    // the WG's LDS LUT", "    uint64_t _pt = __builtin_amdgcn_s_memtime();\n    TileNorm tn = norms[t];\n    // the WG's LDS LUT"),
        ("    reg_fence(E);  // keeps the load/normalise phase", "    PH(0);\n    reg_fence(E);  // keeps the load/normalise phase"),
        ("    uint32_t CL[4];\n", "    PH(1);\n    uint32_t CL[4];\n"),
        ("    reg_fence(E);\n    // ---- set_partitioned_rice_", "    PH(2);\n    reg_fence(E);\n    // ---- set_partitioned_rice_"),
        ("    // ---- choose (process_subframe_", "    PH(3);\n    // ---- choose (process_subframe_"),
        ("    if (!ok) {\n        if (l0) atomicOr(err, 2);\n        end_bits = 0;\n    }\n",
         "    if (!ok) {\n        if (l0) atomicOr(err, 2);\n        end_bits = 0;\n    }\n    PH(4);\n"),
        ("    if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);\n    reg_fence(E);\n",
         "    PH(5);\n    if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);\n    PH(6);\n    reg_fence(E);\n"),
        ("    if (type >= 2 && ok && (lane & (lanes_per - 1)) == 0) lds_put_bits2(fbuf, M, run - 4u, (uint32_t)k, 4);\n",
         "    PH(7);\n    if (type >= 2 && ok && (lane & (lanes_per - 1)) == 0) lds_put_bits2(fbuf, M, run - 4u, (uint32_t)k, 4);\n"),
        ("    uint32_t crc = 0;\n    if (ok) {\n        // slice-by-4", "    PH(8);\n    uint32_t crc = 0;\n    if (ok) {\n        // slice-by-4"),
        ("    prev.f = f;\n    prev.fbytes = fbytes;\n    prev.ok = ok;\n    prev.map = M;\n}\n\ntemplate <int DT>\n__global__",
         "    PH(9);\n    prev.f = f;\n    prev.fbytes = fbytes;\n    prev.ok = ok;\n    prev.map = M;\n}\n\ntemplate <int DT>\n__global__"),
        ("                                       const uint32_t *pslots, const int64_t *pbytes) {\n    using T",
         "                                       const uint32_t *pslots, const int64_t *pbytes, uint64_t *ph) {\n    using T"),
        ("lane, ftile, prev, hdr_tab, hdr_n, pslots, pbytes);\n    }\n    if (prev.f",
         "lane, ftile, prev, hdr_tab, hdr_n, pslots, pbytes, ph);\n    }\n    if (prev.f"),
        ("    if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);\n}\n",
         "    if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);\n"
         "    if (lane == 0) for (int i = 0; i < 11; i++) atomicAdd(&g_ph[i], ph[i]);\n}\n"),
        ("    while (true) {\n        __syncthreads();  // previous ticket's readers",
         "    uint64_t ph[11] = {0,0,0,0,0,0,0,0,0,0,0};\n    uint64_t _pt = __builtin_amdgcn_s_memtime();\n    while (true) {\n        __syncthreads();  // previous ticket's readers"),
        ("        const int64_t f = fbase + wave;\n        if (f < P.nframes)\n",
         "        PH(10);\n        const int64_t f = fbase + wave;\n        if (f < P.nframes)\n"),
        ("                                lane, ftile, prev, hdr_tab, hdr_n, pslots, pbytes, ph);\n    }\n",
         "                                lane, ftile, prev, hdr_tab, hdr_n, pslots, pbytes, ph);\n        _pt = __builtin_amdgcn_s_memtime();\n    }\n"),
        ("        prof_end(ctx, \"encode\", ev);\n",
         "        prof_end(ctx, \"encode\", ev);\n        if (getenv(\"FRS_PHASES\")) {\n            unsigned long long h[16];\n"
         "            hipStreamSynchronize(st);\n            hipMemcpyFromSymbol(h, HIP_SYMBOL(g_ph), sizeof(h));\n"
         "            fprintf(stderr, \"PHASES\");\n            for (int i = 0; i < 11; i++) fprintf(stderr, \" %llu\", h[i]);\n"
         "            fprintf(stderr, \"\\n\");\n            memset(h, 0, sizeof(h));\n            hipMemcpyToSymbol(HIP_SYMBOL(g_ph), h, sizeof(h));\n        }\n"),
    ]
    for a, b in rep:
        assert a in s, a[:70]
        s = s.replace(a, b, 1)
    return s


VARIANTS["phases"] = phases

LB3 = sub("__global__ void __launch_bounds__(256) k_encode_v3", "__global__ void __launch_bounds__(256, 3) k_encode_v3")
RESOLVE_FIRST = chain(
    sub("    if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);\n"
        "    // ---- phase B", "    // ---- phase B"),
    sub("    TileNorm tn = norms[t];", "    if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);\n"
        "    TileNorm tn = norms[t];"))
VARIANTS["lb3"] = LB3
VARIANTS["lb3_rf"] = chain(LB3, RESOLVE_FIRST)
VARIANTS["rf"] = RESOLVE_FIRST


def hist(src):
    """(subframe type, order) histogram of the fast encoder's frames, printed to stderr after each launch"""
    s = src
    rep = [
        ("template <int DT>\n__device__ inline void encode_frame_v3(",
         "__device__ unsigned int g_hist[64];\ntemplate <int DT>\n__device__ inline void encode_frame_v3("),
        ("    // ---- phase A: sizes only", "    if (l0) atomicAdd(&g_hist[type * 16 + (type == 2 ? of : type == 3 ? ol : 0)], 1u);\n"
         "    // ---- phase A: sizes only"),
        ("        prof_end(ctx, \"encode\", ev);\n",
         "        prof_end(ctx, \"encode\", ev);\n        if (getenv(\"FRS_HIST\")) {\n            unsigned h[64];\n"
         "            hipStreamSynchronize(st);\n            hipMemcpyFromSymbol(h, HIP_SYMBOL(g_hist), sizeof(h));\n"
         "            fprintf(stderr, \"HIST\");\n            for (int i = 0; i < 64; i++) if (h[i]) fprintf(stderr, \" %d:%u\", i, h[i]);\n"
         "            fprintf(stderr, \"\\n\");\n            memset(h, 0, sizeof(h));\n            hipMemcpyToSymbol(HIP_SYMBOL(g_hist), h, sizeof(h));\n        }\n"),
    ]
    for a, b in rep:
        assert a in s, a[:70]
        s = s.replace(a, b, 1)
    return s


VARIANTS["hist"] = hist


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    for n in names:
        print(n, build_variant(n, VARIANTS[n]), flush=True)
