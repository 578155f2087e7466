#!/usr/bin/env python3
"""Round-4 lane-decoder variants of frs_decode.hip (tools/build_variant.py -> variants/lib<name>.so).

dlean: an 8-sample step takes a lean body unless some lane of the wave needs the general one (warm-up samples in
       step 0, the block's end, or a partition boundary of a Rice-coded subframe inside the step): one code per
       sample read branch-free for VERBATIM and Rice lanes alike (a VERBATIM code is sbps raw bits, a Rice code its
       unary run, stop bit and k low bits; CONSTANT lanes read nothing), no per-sample partition or warm-up tests.
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


DLEAN = sub("""                    for (int i0 = 0; i0 < bs && take; i0 += 8) {
                        br.top_up();
                        uint32_t ob[8];
#pragma unroll
                        for (int u = 0; u < 8; u++) {""", """                    for (int i0 = 0; i0 < bs && take; i0 += 8) {
                        br.top_up();
                        uint32_t ob[8];
                        // the general per-sample body only where some lane needs it: warm-up samples (step 0), the
                        // block's end, a partition boundary of a Rice-coded subframe inside this step
                        const bool gen = i0 == 0 || i0 + 8 > bs || (!raw && !cst && part_end < i0 + 8);
                        if (!__ballot(gen)) {
#pragma unroll
                            for (int u = 0; u < 8; u++) {
                                // one code per sample: VERBATIM = sbps raw bits, Rice = unary run + stop bit + k low
                                // bits, CONSTANT = nothing read
                                const int z = br.c ? __builtin_clzll(br.c) : 64;
                                const int pre = (raw || cst) ? 0 : z + 1;
                                const int kk = raw ? sbps : (cst ? 0 : k);
                                const int used = pre + kk;
                                uint32_t v;
                                if (used > br.n) {  // (rare: a Rice code longer than the >= 33 cached bits)
                                    const uint32_t q = br.unary();
                                    v = (q << k) | br.bits(k);
                                } else {
                                    const uint64_t tb = pre >= 64 ? 0ull : (br.c << pre);
                                    const uint32_t low = kk ? (uint32_t)(tb >> (64 - kk)) : 0u;
                                    br.c = used >= 64 ? 0ull : (br.c << used);
                                    br.n -= used;
                                    br.ensure();
                                    v = raw ? low : (((uint32_t)z << k) | low);
                                }
                                const int32_t r = raw ? ((int32_t)(v << (32 - sbps)) >> (32 - sbps))
                                                      : (int32_t)((v >> 1) ^ (uint32_t)(-(int32_t)(v & 1)));
                                int32_t pred = 0;
#pragma unroll
                                for (int m = 0; m < 8; m++) pred += __mul24(cq[m], R[(u + 7 - m) & 7]);
                                const int32_t x = cst ? cval : r + (pred >> shift);
                                R[u] = x;
                                const int32_t xo = (int32_t)((uint32_t)x << w);
                                if constexpr (OUT == kOutAny) {
                                    dn_store(dout, obase + i0 + u, xo, dnp);
                                    ob[u] = 0;
                                } else {
                                    ob[u] = dn_bits_t<OUT>(dout, xo, dnp);
                                }
                            }
                        } else
#pragma unroll
                        for (int u = 0; u < 8; u++) {""")

VARIANTS = {"dbase": lambda s: s, "dlean": DLEAN}

if __name__ == "__main__":
    for name in sys.argv[1:] or list(VARIANTS):
        print(build_variant(name, VARIANTS[name], src_name="frs_decode.hip"))
