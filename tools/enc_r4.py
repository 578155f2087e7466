#!/usr/bin/env python3
"""Round-4 encoder variants of frs_encode.hip (tools/build_variant.py -> variants/lib<name>.so), A/B'd on the GPU box
with tools/gpu/gpu_var_ab.sh.

pwt: per-wave frame tickets.  Every wave claims its own frame (one atomic per frame, in frame order) instead of a
     work-group claiming four and meeting at two barriers per ticket; each wave keeps its own LDS LUT slot of
     kLutWave entries (the four slots take the LDS of the old shared 4096-entry LUT), refreshed from the tile's global
     LUT after the frame's sample loads are issued.  Tiles whose LUT does not fit a slot take the exact division.
"""
import sys

from build_variant import build_variant


def sub(old, new, count=1):
    def f(src):
        assert old in src, old[:80]
        return src.replace(old, new, count)
    return f


def chain(*fs):
    def f(src):
        for g in fs:
            src = g(src)
        return src
    return f


PWT = chain(
    sub("""struct EncV3Shared {
    uint32_t bits[4][kBufWordsV3];
    int16_t lut[kLutCap];""", """constexpr int kLutWave = kLutCap / 4;  // LUT entries of a wave's own slot
struct EncV3Shared {
    uint32_t bits[4][kBufWordsV3];
    int16_t lut[4][kLutWave];"""),
    sub("""    int ticket;
    int want;
    int lut_tile;
};""", """};"""),
    sub("""static_assert(offsetof(EncV3Shared, lut) + sizeof(int16_t) * kLutCap <= 65536, "LUT beyond 64 KiB of LDS");""",
        """static_assert(offsetof(EncV3Shared, lut) + sizeof(int16_t) * 4 * kLutWave <= 65536, "LUT beyond 64 KiB of LDS");"""),
    # encode_frame_v3: `want` becomes the wave's slot tile (in/out); the slot is refreshed after the sample loads
    sub("""uint64_t *status, int *err, EncV3Shared &S, int want, int64_t f, int lane,""",
        """uint64_t *status, int *err, EncV3Shared &S, int &want, int64_t f, int lane,"""),
    sub("""    TileNorm tn = norms[t];
    // the WG's LDS LUT belongs to tile `want`; a frame of another tile takes the exact division instead
    if (t != want && tn.mode == kNormLut) tn.mode = kNormSlow;
    const int16_t *lut = S.lut;""", """    TileNorm tn = norms[t];
    // the wave's LDS LUT slot holds tile `want`'s table; refreshed below (after the sample loads are in flight) when
    // the frame is of another tile; a tile whose table does not fit the slot takes the exact division
    const bool lut_fits = tn.mode == kNormLut && tn.imax - tn.imin < kLutWave;
    if (tn.mode == kNormLut && !lut_fits) tn.mode = kNormSlow;
    int16_t *lut = S.lut[threadIdx.x >> 6];"""),
    sub("""        ch.load(base, P.row_stride, g.w, row, (int)(sl0 - row * (uint32_t)g.w), (g.w % 64) == 0 ? P.vec_ok : 0, 64);
        if (sizeof(T) == 2 && tn.mode == kNormLut && w == 0) {""",
        """        ch.load(base, P.row_stride, g.w, row, (int)(sl0 - row * (uint32_t)g.w), (g.w % 64) == 0 ? P.vec_ok : 0, 64);
        if (lut_fits && t != want) {  // (wave-uniform) 16-B copies of the tile's table (entries up to a multiple of 8)
            const int R = (int)(tn.imax - tn.imin);
            const uint4 *src = reinterpret_cast<const uint4 *>(luts + (int64_t)t * kLutCap);
            uint4 *dst = reinterpret_cast<uint4 *>(lut);
            for (int q = lane; q * 8 <= R; q += 64) dst[q] = src[q];
            want = t;
        }
        if (sizeof(T) == 2 && tn.mode == kNormLut && w == 0) {"""),
    # kernel: per-wave tickets, no barriers in the loop
    sub("""    for (int i = threadIdx.x; i < 4 * kBufWordsV3; i += blockDim.x) (&S.bits[0][0])[i] = 0;
    if (threadIdx.x == 0) S.lut_tile = -1;
    PendingFrame prev;
    uint32_t *fbuf = S.bits[wave];
    while (true) {
        __syncthreads();  // previous ticket's readers of S.ticket / S.lut are done
        const int64_t nunits = uend < 0 ? (SUB ? P.nframes * P.nch : P.nframes) : uend;
        if (threadIdx.x == 0) {
            const int tk = atomicAdd(ticket_ctr, 1);
            S.ticket = tk;
            const int64_t u0 = ubeg + (int64_t)tk * 4;
            S.want = (u0 < nunits) ? ftile[SUB ? u0 / P.nch : u0] : -1;
        }
        __syncthreads();
        const int64_t fbase = ubeg + (int64_t)S.ticket * 4;
        if (fbase >= nunits) break;
        const int want = S.want;
        if (want != S.lut_tile) {  // WG-uniform
            const TileNorm tw = norms[want];
            if (tw.mode == kNormLut) {
                const int64_t R = tw.imax - tw.imin;
                const int16_t *src = luts + (int64_t)want * kLutCap;
                for (int64_t d = threadIdx.x; d <= R; d += blockDim.x) S.lut[d] = src[d];
            }
            __syncthreads();
            if (threadIdx.x == 0) S.lut_tile = want;
        }
        if constexpr (SUB) {
            const int64_t v = fbase + wave;
            if (v < nunits) {""", """    for (int i = threadIdx.x; i < 4 * kBufWordsV3; i += blockDim.x) (&S.bits[0][0])[i] = 0;
    __syncthreads();
    PendingFrame prev;
    uint32_t *fbuf = S.bits[wave];
    int want = -1;  // tile whose LUT sits in this wave's slot
    const int64_t nunits = uend < 0 ? (SUB ? P.nframes * P.nch : P.nframes) : uend;
    while (true) {
        // this wave's next unit, claimed in unit order (the look-back waits only on units resident waves own)
        int tk = 0;
        if (lane == 0) tk = atomicAdd(ticket_ctr, 1);
        tk = __builtin_amdgcn_readfirstlane(tk);
        const int64_t fbase = ubeg + (int64_t)tk;
        if (fbase >= nunits) break;
        if constexpr (SUB) {
            const int64_t v = fbase;
            if (v < nunits) {"""),
    sub("""        } else {
            const int64_t f = fbase + wave;
            if (f < nunits)""", """        } else {
            const int64_t f = fbase;
            if (f < nunits)"""),
    # host: grid cap by units (one per wave)
    sub("""                grid = std::min<int64_t>(grid, (f1 - f0 + 3) / 4);""",
        """                grid = std::min<int64_t>(grid, (f1 - f0 + 3) / 4);  // (one unit per wave and ticket)"""),
)

# crc2: each lane's CRC column as two independent chains (the dependent table lookups per chain halve), joined by
#       one multiply by x^(8 bytes of the second chain) from an LDS table; the lane's final shift by x^(8 m) is one
#       multiply by the global x^(8m) table entry (L1/L2-resident) instead of two by the LDS split tables
CRC2 = chain(
    sub("""    uint16_t xlo[64];       // x^(8m) mod P, m = 0..63""",
        """    uint16_t xlo[80];       // x^(8m) mod P, m = 0..79"""),
    sub("""    for (int i = threadIdx.x; i < 64; i += blockDim.x) S.xlo[i] = g_xpow_bytes[i];""",
        """    for (int i = threadIdx.x; i < 80; i += blockDim.x) S.xlo[i] = g_xpow_bytes[i];"""),
    sub("""        uint32_t c = 0;
        const uint32_t *colp = fbuf + lane;
        // slice-by-8 (two words per step: the table lookups that depend on the running CRC, and so the
        // latency chain, are halved), then one slice-by-4 step for an odd word
        const uint16_t(*T)[256] = S.crc8x;
        uint32_t i = wb;
        for (; i + 1 < we; i += 2, colp += 128) {
            const uint32_t w0 = colp[0], w1 = colp[64];
            c = (uint32_t)T[7][((c >> 8) ^ (w0 >> 24)) & 0xFF] ^ T[6][((c & 0xFF) ^ (w0 >> 16)) & 0xFF] ^
                T[5][(w0 >> 8) & 0xFF] ^ T[4][w0 & 0xFF] ^ T[3][w1 >> 24] ^ T[2][(w1 >> 16) & 0xFF] ^
                T[1][(w1 >> 8) & 0xFF] ^ T[0][w1 & 0xFF];
        }
        if (i < we) {
            const uint32_t word = *colp;
            c = (uint32_t)T[3][((c >> 8) ^ (word >> 24)) & 0xFF] ^ T[2][((c & 0xFF) ^ (word >> 16)) & 0xFF] ^
                T[1][(word >> 8) & 0xFF] ^ T[0][word & 0xFF];
        }
        uint32_t end = we * 4;""",
        """        // slice-by-8 (two words per step), the column as two independent chains A = [wb, wb + na) and
        // B = [wb + na, we) in lockstep (na even, nb = n - na in [na, na + 3]); c = cA x^(8 * 4 nb) + cB
        const uint16_t(*T)[256] = S.crc8x;
        auto step8 = [&](uint32_t c, uint32_t w0, uint32_t w1) -> uint32_t {
            return (uint32_t)T[7][((c >> 8) ^ (w0 >> 24)) & 0xFF] ^ T[6][((c & 0xFF) ^ (w0 >> 16)) & 0xFF] ^
                   T[5][(w0 >> 8) & 0xFF] ^ T[4][w0 & 0xFF] ^ T[3][w1 >> 24] ^ T[2][(w1 >> 16) & 0xFF] ^
                   T[1][(w1 >> 8) & 0xFF] ^ T[0][w1 & 0xFF];
        };
        const uint32_t n = we - wb, na = (n >> 1) & ~1u, nb = n - na;
        const uint32_t *pa = fbuf + lane, *pb = fbuf + lane + (na << 6);
        uint32_t ca = 0, cb = 0, i = 0;
        for (; i < na; i += 2, pa += 128, pb += 128) {
            ca = step8(ca, pa[0], pa[64]);
            cb = step8(cb, pb[0], pb[64]);
        }
        if (i + 1 < nb) {
            cb = step8(cb, pb[0], pb[64]);
            i += 2;
            pb += 128;
        }
        if (i < nb) {
            const uint32_t word = *pb;
            cb = (uint32_t)T[3][((cb >> 8) ^ (word >> 24)) & 0xFF] ^ T[2][((cb & 0xFF) ^ (word >> 16)) & 0xFF] ^
                 T[1][(word >> 8) & 0xFF] ^ T[0][word & 0xFF];
        }
        uint32_t c = (na ? gf_mulmod(ca, S.xlo[4 * nb]) : 0u) ^ cb;
        uint32_t end = we * 4;"""),
    sub("""        crc = dpp_wave_xor_u32(gf_mulmod(gf_mulmod(c, S.xlo[m & 63]), S.xhi[m >> 6]));""",
        """        crc = dpp_wave_xor_u32(gf_mulmod(c, g_xpow_bytes[m]));"""),
)

# pwt2: per-wave LUT slots (as pwt) and no barriers, but units still claimed from the global counter in blocks of
#       four (one global atomic per four units, as the work-group tickets): the waves of a work-group take units from
#       an LDS counter; the wave that takes a block's first unit claims the block's global ticket and posts it in an
#       LDS ring (tag, ticket); the others wait only for that post, not for each other's frames.
PWT2_LOOP = sub("""    int want = -1;  // tile whose LUT sits in this wave's slot
    const int64_t nunits = uend < 0 ? (SUB ? P.nframes * P.nch : P.nframes) : uend;
    while (true) {
        // this wave's next unit, claimed in unit order (the look-back waits only on units resident waves own)
        int tk = 0;
        if (lane == 0) tk = atomicAdd(ticket_ctr, 1);
        tk = __builtin_amdgcn_readfirstlane(tk);
        const int64_t fbase = ubeg + (int64_t)tk;
        if (fbase >= nunits) break;""", """    int want = -1;  // tile whose LUT sits in this wave's slot
    const int64_t nunits = uend < 0 ? (SUB ? P.nframes * P.nch : P.nframes) : uend;
    while (true) {
        // this wave's next unit: local index i from the LDS counter; block i / 4 of the WG is global ticket tk
        int i = 0;
        if (lane == 0) i = atomicAdd(&S.taken, 1);
        i = __builtin_amdgcn_readfirstlane(i);
        const int blk = i >> 2;
        int2 *ring = &S.ring[blk & 7];
        if ((i & 3) == 0 && lane == 0) {  // the block's first taker claims it
            const int tk = atomicAdd(ticket_ctr, 1);
            __hip_atomic_store(&ring->y, tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(&ring->x, blk, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        int tk = 0;
        for (int spin = 0;; spin++) {  // (the claimer's own post is already visible)
            int tag = 0, v = 0;
            if (lane == 0) {
                tag = __hip_atomic_load(&ring->x, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                v = __hip_atomic_load(&ring->y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            tag = __builtin_amdgcn_readfirstlane(tag);
            if (tag == blk) {
                tk = __builtin_amdgcn_readfirstlane(v);
                break;
            }
            if (spin > (1 << 24)) {  // a lost post (cannot happen: 8 slots, a block is read right after its claim)
                if (lane == 0) atomicOr(err, 32);
                tk = 1 << 30;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const int64_t fbase = ubeg + (int64_t)tk * 4 + (i & 3);
        if (fbase >= nunits) break;""")
PWT2 = chain(PWT,
             sub("""    int16_t lut[4][kLutWave];""", """    int16_t lut[4][kLutWave];
    int2 ring[8];  // (block tag, global ticket) of the WG's last eight blocks
    int taken;     // units taken by the WG's waves"""),
             sub("""    for (int i = threadIdx.x; i < 4 * kBufWordsV3; i += blockDim.x) (&S.bits[0][0])[i] = 0;
    __syncthreads();""", """    for (int i = threadIdx.x; i < 4 * kBufWordsV3; i += blockDim.x) (&S.bits[0][0])[i] = 0;
    if (threadIdx.x < 8) S.ring[threadIdx.x] = make_int2(-1, 0);
    if (threadIdx.x == 0) S.taken = 0;
    __syncthreads();"""),
             PWT2_LOOP)

# early: the previous frame's look-back + store + buffer re-zero right after this frame's sample loads are issued (its
#        latency hides behind them) instead of between this frame's phases A and B
EARLY = chain(
    sub("""        ch.load(base, P.row_stride, g.w, row, (int)(sl0 - row * (uint32_t)g.w), (g.w % 64) == 0 ? P.vec_ok : 0, 64);
        if (sizeof(T) == 2 && tn.mode == kNormLut && w == 0) {  // (wave-uniform) the common case""",
        """        ch.load(base, P.row_stride, g.w, row, (int)(sl0 - row * (uint32_t)g.w), (g.w % 64) == 0 ? P.vec_ok : 0, 64);
        if constexpr (!SUB)
            if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);
        if (sizeof(T) == 2 && tn.mode == kNormLut && w == 0) {  // (wave-uniform) the common case"""),
    sub("""    if constexpr (!SUB)
        if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);
    __builtin_amdgcn_s_setprio(0);""", """    __builtin_amdgcn_s_setprio(0);"""),
)

VARIANTS = {"base": lambda s: s, "pwt": PWT, "crc2": CRC2, "pwt_crc2": chain(PWT, CRC2), "pwt2": PWT2, "pwt2_crc2": chain(PWT2, CRC2), "early": EARLY, "early_crc2": chain(EARLY, CRC2)}

if __name__ == "__main__":
    for name in sys.argv[1:] or list(VARIANTS):
        print(build_variant(name, VARIANTS[name]))
