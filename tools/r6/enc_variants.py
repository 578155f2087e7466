#!/usr/bin/env python3
"""Round 6 encoder variants of frs_encode.hip (libraries in variants/, selected with FRS_LIB_PATH):
eA = k_encode_v4's ticket loop with ONE barrier per ticket: the ticket and the tile it wants are double-buffered in
LDS (slot = iteration & 1), so thread 0 can write the next ticket while slower waves still read the current one and
the barrier in front of the atomic goes (all waves still meet once per ticket, after the atomic)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from build_variant import build_variant  # noqa: E402


def one_barrier(src):
    subs = [
        ("""    int ticket;
    int want;
    int lut_tile;""", """    int ticket[2];
    int want[2];
    int lut_tile;"""),
        ("""    while (true) {
        __syncthreads();  // previous ticket's readers of S.ticket / S.lut are done
        constexpr int kUpfSt = WIDE ? 1 : 3;  // units per frame of a two-channel launch""",
         """    int it = 0;
    while (true) {
        const int sl = it & 1;  // (slot sl is read after this iteration's barrier; the previous one's slot is sl ^ 1)
        it++;
        constexpr int kUpfSt = WIDE ? 1 : 3;  // units per frame of a two-channel launch"""),
        ("""            S.ticket = tk;""", """            S.ticket[sl] = tk;"""),
        ("""            S.want = (u0 < nunits) ? ftile[SUB ? u0 / upf : u0] : -1;""",
         """            S.want[sl] = (u0 < nunits) ? ftile[SUB ? u0 / upf : u0] : -1;"""),
        ("""        const int64_t fbase = (int64_t)S.ticket * 4;""", """        const int64_t fbase = (int64_t)S.ticket[sl] * 4;"""),
        ("""        const int want = S.want;""", """        const int want = S.want[sl];"""),
    ]
    for a, b in subs:
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    return src


def no_barrier(src):
    """eB (on the tree's eA form): no barrier per ticket.  Thread 0 fills a ring of four ticket slots, each once the
    four waves have read its previous use (an LDS read counter); every wave waits (LDS poll) for its iteration's slot
    and reads it; the work-group meets only when the LUT's tile changes (all waves are then past their frames of the
    old tile).  Spins are bounded (err |= 32, the wave returns: an ended wave no longer counts at a barrier)."""
    subs = [
        ("""    int ticket[2];
    int want[2];
    int lut_tile;""", """    int ticket[4];
    int want[4];
    int seq[4];
    int nread[4];
    int lut_tile;"""),
        ("""    if (threadIdx.x == 0) S.lut_tile = -1;
    PendingFrame prev;""", """    if (threadIdx.x == 0) S.lut_tile = -1;
    if (threadIdx.x < 4) {
        S.seq[threadIdx.x] = 0;
        S.nread[threadIdx.x] = 4;
    }
    __syncthreads();
    PendingFrame prev;"""),
        ("""    int it = 0;
    while (true) {
        const int sl = it & 1;  // (slot sl is read after this iteration's barrier; the previous one's slot is sl ^ 1)
        it++;
        constexpr int kUpfSt = WIDE ? 1 : 3;  // units per frame of a two-channel launch
        const int upf = ST ? kUpfSt : P.nch;
        const int64_t nunits = SUB ? P.nframes * upf : P.nframes;
        if (threadIdx.x == 0) {
            const int tk = atomicAdd(ticket_ctr, 1);
            S.ticket[sl] = tk;
            const int64_t u0 = (int64_t)tk * 4;
            S.want[sl] = (u0 < nunits) ? ftile[SUB ? u0 / upf : u0] : -1;
        }
        __syncthreads();
        const int64_t fbase = (int64_t)S.ticket[sl] * 4;
        if (fbase >= nunits) break;
        const int want = S.want[sl];
        if (want != S.lut_tile) {  // WG-uniform
            const TileNorm tw = norms[want];""", """    int it = 0;
    volatile int *vseq = S.seq, *vnread = S.nread;
    while (true) {
        const int sl = it & 3;
        it++;
        constexpr int kUpfSt = WIDE ? 1 : 3;  // units per frame of a two-channel launch
        const int upf = ST ? kUpfSt : P.nch;
        const int64_t nunits = SUB ? P.nframes * upf : P.nframes;
        if (threadIdx.x == 0) {
            long spins = 0;
            while (vnread[sl] < 4) {  // the slot's previous use read by every wave
                if (++spins > (1l << 24)) {
                    atomicOr(err, 32);
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            vnread[sl] = 0;
            const int tk = atomicAdd(ticket_ctr, 1);
            S.ticket[sl] = tk;
            const int64_t u0 = (int64_t)tk * 4;
            S.want[sl] = (u0 < nunits) ? ftile[SUB ? u0 / upf : u0] : -1;
            __builtin_amdgcn_s_waitcnt(0xC07F);  // the slot's words have landed before its sequence number
            vseq[sl] = it;
        }
        {
            long spins = 0;
            while (vseq[sl] != it) {
                if (++spins > (1l << 24)) {
                    if (lane == 0) atomicOr(err, 32);
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __asm__ volatile("" ::: "memory");
        const int64_t fbase = (int64_t)S.ticket[sl] * 4;
        const int want = S.want[sl];
        __builtin_amdgcn_s_waitcnt(0xC07F);  // (the reads above have returned before the read count moves)
        if (lane == 0) atomicAdd(&S.nread[sl], 1);
        if (fbase >= nunits) break;
        if (want != S.lut_tile) {  // WG-uniform
            __syncthreads();  // every wave is past its frames of the previous tile
            const TileNorm tw = norms[want];"""),
    ]
    for a, b in subs:
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    return src


def early_ticket(src):
    """eC (on the tree's eA form, mono launches): thread 0 takes the work-group's next ticket right after its own frame
    has published its size (the atomic's latency then hides behind the frame's assembly and CRC) instead of at the
    loop top; a ticket taken a whole frame early measured +0.4 ms in round 2 (its frames publish late)."""
    subs = [
        ("""                                                uint32_t *sub_slots = nullptr, int32_t *sub_bits = nullptr,
                                                int32_t *sub_est = nullptr) {
    using T = typename Elem<DT>::T;
    using Lane = std::conditional_t<WIDE, LaneWide, LanePairs>;""",
         """                                                uint32_t *sub_slots = nullptr, int32_t *sub_bits = nullptr,
                                                int32_t *sub_est = nullptr, int *tk_ctr = nullptr,
                                                int *tk_next = nullptr) {
    using T = typename Elem<DT>::T;
    using Lane = std::conditional_t<WIDE, LaneWide, LanePairs>;"""),
        ("""    if (!SUB && l0) {  // publish our aggregate
        const uint64_t v = (f == 0 ? kFlagIncl : kFlagAgg) | fbytes;
        __hip_atomic_store(&status[f], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }""", """    if (!SUB && l0) {  // publish our aggregate
        const uint64_t v = (f == 0 ? kFlagIncl : kFlagAgg) | fbytes;
        __hip_atomic_store(&status[f], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!SUB && tk_next && threadIdx.x == 0) *tk_next = atomicAdd(tk_ctr, 1);  // the work-group's next ticket"""),
        ("""    int it = 0;
    while (true) {""", """    int it = 0;
    int tk_next = -1;  // (thread 0) a ticket taken during the last frame
    while (true) {"""),
        ("""        if (threadIdx.x == 0) {
            const int tk = atomicAdd(ticket_ctr, 1);
            S.ticket[sl] = tk;""", """        if (threadIdx.x == 0) {
            const int tk = tk_next >= 0 ? tk_next : atomicAdd(ticket_ctr, 1);
            tk_next = -1;
            S.ticket[sl] = tk;"""),
        ("""                encode_frame_v4<DT>(raster, P, tiles, norms, ana, arena, arena_cap, frame_off, status, err, S, want, f,
                                    lane, ftile, prev, hdr_tab, hdr_n, pslots, pbytes);""",
         """                encode_frame_v4<DT>(raster, P, tiles, norms, ana, arena, arena_cap, frame_off, status, err, S, want, f,
                                    lane, ftile, prev, hdr_tab, hdr_n, pslots, pbytes, 0, nullptr, nullptr, nullptr,
                                    ticket_ctr, wave == 0 ? &tk_next : nullptr);"""),
    ]
    for a, b in subs:
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    return src


if __name__ == "__main__":
    for name in sys.argv[1:] or ["eA"]:
        print(build_variant(name, {"eA": one_barrier, "eB": no_barrier, "eC": early_ticket}[name]))
