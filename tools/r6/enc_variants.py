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


if __name__ == "__main__":
    for name in sys.argv[1:] or ["eA"]:
        print(build_variant(name, {"eA": one_barrier}[name]))
