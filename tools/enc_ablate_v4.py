#!/usr/bin/env python3
"""Timing-only ablations of k_encode_v4 (each variant removes one pass of encode_frame_v4; its output is wrong): the
kernel time a variant saves is that pass's share.  Variants are int16-only builds (-DFRS_PROBE_I16, the C4 bench's
dtype) of variants/lib<name>.so; run them with tools/gpu/gpu_variants.sh and compare kernels_ms.encode."""
import sys

from build_variant import build_variant


def sub(old, new):
    def f(src):
        i0 = src.index("__device__ __forceinline__ void encode_frame_v4")
        assert old in src[i0:], old[:70]
        return src[:i0] + src[i0:].replace(old, new, 1)
    return f


def gsub(old, new):
    def f(src):
        assert src.count(old) == 1, old[:70]
        return src.replace(old, new, 1)
    return f


def chain(*fs):
    def f(src):
        for g in fs:
            src = g(src)
        return src
    return f


NOASM = sub("                    if (!three) atomicOr(((uint32_t)i < split ? A : B) + 64 * i, v);",
            "                    if (!three) asm volatile(\"\" :: \"v\"(v), \"v\"(A), \"v\"(B));")
NOPV = chain(sub("        for (int i = 0; i <= kPrivRows; i++) Pv[i] = pcol[i << 6];\n        __builtin_amdgcn_s_waitcnt(0xC07F);  // every lane's column is in registers before the zeroing\n        __builtin_amdgcn_wave_barrier();\n        zero_wave_buf(fbuf, lane);",
                 "        for (int i = 0; i <= kPrivRows; i++) Pv[i] = seglen * (i + 1);"))
NOCRC = sub("        const uint32_t crc = crc16_cols(fbuf, M, body, S, lane);", "        const uint32_t crc = body * 3;")
NOPACK = sub("                atomicOr(a, __builtin_amdgcn_alignbit(0u, codeL, p));\n                atomicOr(a + 64, __builtin_amdgcn_alignbit(codeL, 0u, p));",
             "                asm volatile(\"\" :: \"v\"(a), \"v\"(codeL), \"v\"(p));")
NOLPCSUM = sub("    uint32_t sl = 0;\n    if (cand_lpc) {", "    uint32_t sl = 5000;\n    if (false) {")
NOHDR = sub("    if (type >= 2) {\n        // warm-up samples and quantised coefficients in parallel",
            "    if (false) {\n        // warm-up samples and quantised coefficients in parallel")

# timing only: publish the frame's Rice-estimate size before the look-back of the previous frame (as v3 publishes its
# exact size), and not after the packing
EARLYPUB = chain(sub("""    if constexpr (!SUB)
        if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);
    if (type >= 2) {""", """    if (!SUB && l0) {
        const uint64_t v = (f == 0 ? kFlagIncl : kFlagAgg) | (uint64_t)(((best + pos0 + 64) >> 3) + 2);
        __hip_atomic_store(&status[f], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (!SUB)
        if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);
    if (type >= 2) {"""),
    sub("""    if (!SUB && l0) {  // publish our aggregate
        const uint64_t v = (f == 0 ? kFlagIncl : kFlagAgg) | fbytes;""", """    if (false) {  // publish our aggregate
        const uint64_t v = (f == 0 ? kFlagIncl : kFlagAgg) | fbytes;"""))

# tickets of 8 frames: wave w codes frames fbase + w and fbase + 4 + w (one barrier pair per two frames)
T8 = chain(
    sub("            const int64_t u0 = (int64_t)tk * 4;\n            S.want = (u0 < nunits) ? ftile[SUB ? u0 / P.nch : u0] : -1;\n        }\n        __syncthreads();\n        const int64_t fbase = (int64_t)S.ticket * 4;",
        "            const int64_t u0 = (int64_t)tk * 8;\n            S.want = (u0 < nunits) ? ftile[SUB ? u0 / P.nch : u0] : -1;\n        }\n        __syncthreads();\n        const int64_t fbase = (int64_t)S.ticket * 8;"),
    sub("""            const int64_t f = fbase + wave;
            if (f < nunits)
                encode_frame_v4<DT>(raster, P, tiles, norms, ana, arena, arena_cap, frame_off, status, err, S, want, f,
                                    lane, ftile, prev, hdr_tab, hdr_n, pslots, pbytes, 0, nullptr, nullptr, dbg);""",
        """            for (int h = 0; h < 2; h++) {
            const int64_t f = fbase + wave + 4 * h;
            if (f < nunits)
                encode_frame_v4<DT>(raster, P, tiles, norms, ana, arena, arena_cap, frame_off, status, err, S, want, f,
                                    lane, ftile, prev, hdr_tab, hdr_n, pslots, pbytes, 0, nullptr, nullptr, dbg);
            }"""))
# the frame CRC in two interleaved chains per lane (halves of its column), joined with one x^(8m) factor
CRC2 = gsub("""    uint32_t c = 0;
    const uint32_t *colp = fbuf + lane;
    const uint16_t(*T)[256] = S.crc8x;
    uint32_t i = wb;
    for (; i + 3 < we; i += 4, colp += 256) {""", """    uint32_t c = 0;
    const uint32_t *colp = fbuf + lane;
    const uint16_t(*T)[256] = S.crc8x;
    uint32_t i = wb;
    const uint32_t nst = (we - wb) >> 3;  // 4-word steps of each chain
    if (nst) {
        uint32_t ca = 0, cb = 0;
        const uint32_t *pa = colp, *pb = colp + 256 * nst;
        for (uint32_t st = 0; st < nst; st++, pa += 256, pb += 256) {
            const uint32_t w0 = pa[0], w1 = pa[64], w2 = pa[128], w3 = pa[192];
            const uint32_t x0 = pb[0], x1 = pb[64], x2 = pb[128], x3 = pb[192];
            ca = (uint32_t)T[15][((ca >> 8) ^ (w0 >> 24)) & 0xFF] ^ T[14][((ca & 0xFF) ^ (w0 >> 16)) & 0xFF] ^
                T[13][(w0 >> 8) & 0xFF] ^ T[12][w0 & 0xFF] ^ T[11][w1 >> 24] ^ T[10][(w1 >> 16) & 0xFF] ^
                T[9][(w1 >> 8) & 0xFF] ^ T[8][w1 & 0xFF] ^ T[7][w2 >> 24] ^ T[6][(w2 >> 16) & 0xFF] ^
                T[5][(w2 >> 8) & 0xFF] ^ T[4][w2 & 0xFF] ^ T[3][w3 >> 24] ^ T[2][(w3 >> 16) & 0xFF] ^
                T[1][(w3 >> 8) & 0xFF] ^ T[0][w3 & 0xFF];
            cb = (uint32_t)T[15][((cb >> 8) ^ (x0 >> 24)) & 0xFF] ^ T[14][((cb & 0xFF) ^ (x0 >> 16)) & 0xFF] ^
                T[13][(x0 >> 8) & 0xFF] ^ T[12][x0 & 0xFF] ^ T[11][x1 >> 24] ^ T[10][(x1 >> 16) & 0xFF] ^
                T[9][(x1 >> 8) & 0xFF] ^ T[8][x1 & 0xFF] ^ T[7][x2 >> 24] ^ T[6][(x2 >> 16) & 0xFF] ^
                T[5][(x2 >> 8) & 0xFF] ^ T[4][x2 & 0xFF] ^ T[3][x3 >> 24] ^ T[2][(x3 >> 16) & 0xFF] ^
                T[1][(x3 >> 8) & 0xFF] ^ T[0][x3 & 0xFF];
        }
        const uint32_t mb = 16 * nst;  // chain b's bytes: ca advanced past them
        c = gf_mulmod(gf_mulmod(ca, S.xlo[mb & 63]), S.xhi[mb >> 6]) ^ cb;
        i = wb + 8 * nst;
        colp += 512 * nst;
    }
    for (; i + 3 < we; i += 4, colp += 256) {""")

VARIANTS = {
    "v4t8": T8,
    "v4crc2": CRC2,
    "v4earlypub": EARLYPUB,
    "v4base": lambda s: s,
    "v4noasm": NOASM,
    "v4nopv": NOPV,
    "v4nocrc": NOCRC,
    "v4nopack": NOPACK,
    "v4nolpcsum": NOLPCSUM,
    "v4nowarm": NOHDR,
}

def phases(src):
    """per-phase wave clocks of encode_frame_v4 (s_memtime deltas summed per wave, then over waves), printed to
    stderr after each encode launch when $FRS_PHASES is set"""
    i0 = src.index("template <int DT, bool SUB = false>\n__device__ __forceinline__ void encode_frame_v4")
    head, s = src[:i0], src[i0:]
    rep = [
        ("unsigned long long *dbg = nullptr) {\n    using T = typename Elem<DT>::T;",
         "unsigned long long *dbg = nullptr, uint64_t *ph = nullptr) {\n    using T = typename Elem<DT>::T;"),
        ("    uint32_t E[36];\n    load_E(E);\n", "    uint32_t E[36];\n    load_E(E);\n    PH(0);\n"),
        ("    rice_candidates(sf, sl, of, ol,", "    PH(1);\n    rice_candidates(sf, sl, of, ol,"),
        ("    // ---- the previous frame of this wave: its successors", "    PH(2);\n    // ---- the previous frame of this wave: its successors"),
        ("    if (type >= 2) {\n        // ---- private packing", "    PH(3);\n    if (type >= 2) {\n        // ---- private packing"),
        ("    __builtin_amdgcn_s_setprio(0);\n    // ---- assembly into the v3 frame layout", "    PH(4);\n    __builtin_amdgcn_s_setprio(0);\n    // ---- assembly into the v3 frame layout"),
        ("    // ---- header, subframe header, warm-up, coefficients, partition order (fixed positions below pos)",
         "    PH(5);\n    // ---- header, subframe header, warm-up, coefficients, partition order (fixed positions below pos)"),
        ("    if (ok) {\n        const uint32_t crc = crc16_cols(", "    PH(6);\n    if (ok) {\n        const uint32_t crc = crc16_cols("),
        ("    prev.f = f, prev.fbytes = fbytes, prev.ok = ok, prev.map = M;\n}\n",
         "    PH(7);\n    prev.f = f, prev.fbytes = fbytes, prev.ok = ok, prev.map = M;\n}\n"),
        ("    PendingFrame prev;\n    uint32_t *fbuf = S.bits[wave];\n    while (true) {",
         "    PendingFrame prev;\n    uint32_t *fbuf = S.bits[wave];\n    uint64_t ph[16] = {0};\n    ph[15] = __builtin_amdgcn_s_memtime();\n    while (true) {"),
        ("            const int64_t f = fbase + wave;\n            if (f < nunits)\n                encode_frame_v4<DT>(",
         "            const int64_t f = fbase + wave;\n            PH(8);\n            if (f < nunits)\n                encode_frame_v4<DT>("),
        ("pslots, pbytes, 0, nullptr, nullptr, dbg);\n        }\n    }\n    if constexpr (!SUB)\n        if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);\n}",
         "pslots, pbytes, 0, nullptr, nullptr, dbg, ph);\n        }\n    }\n    if constexpr (!SUB)\n        if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);\n"
         "    if (lane == 0) for (int i = 0; i < 9; i++) atomicAdd(&g_ph4[i], (unsigned long long)ph[i]);\n}"),
    ]
    for a, b in rep:
        assert a in s, a[:70]
        s = s.replace(a, b, 1)
    decl = ("__device__ unsigned long long g_ph4[16];\n"
            "#define PH(i) do { if (ph) { const uint64_t _t = __builtin_amdgcn_s_memtime(); ph[i] += _t - ph[15]; ph[15] = _t; } } while (0)\n")
    s = head + decl + s
    a = "            prof_end(ctx, \"encode\", ev);\n            if (dbg) {"
    b = ("            prof_end(ctx, \"encode\", ev);\n            if (getenv(\"FRS_PHASES\")) {\n                unsigned long long h[16];\n"
         "                hipStreamSynchronize(st);\n                hipMemcpyFromSymbol(h, HIP_SYMBOL(g_ph4), sizeof(h));\n"
         "                fprintf(stderr, \"PHASES\");\n                for (int i = 0; i < 9; i++) fprintf(stderr, \" %llu\", h[i]);\n"
         "                fprintf(stderr, \"\\n\");\n                memset(h, 0, sizeof(h));\n                hipMemcpyToSymbol(HIP_SYMBOL(g_ph4), h, sizeof(h));\n            }\n            if (dbg) {")
    assert a in s
    s = s.replace(a, b, 1)
    return s


VARIANTS["v4phases"] = phases


# analysis at 5 waves per SIMD (32-sample loads per lane: 94 VGPRs; 5 x 32 KB of LUTs fill the LDS)
VARIANTS["ana5"] = chain(
    gsub("__global__ void __launch_bounds__(256) k_analyze_v3(", "__global__ void __launch_bounds__(256, SLOW ? 1 : 5) k_analyze_v3("),
    gsub("    constexpr int kChunk = SLOW ? 16 : 64;", "    constexpr int kChunk = SLOW ? 16 : 32;"))
VARIANTS["ana5c64"] = gsub("__global__ void __launch_bounds__(256) k_analyze_v3(",
                           "__global__ void __launch_bounds__(256, SLOW ? 1 : 5) k_analyze_v3(")


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    for n in names:
        print(build_variant(n, VARIANTS[n], extra_flags=("-DFRS_PROBE_I16",)))
