#!/usr/bin/env python3
"""Round 6: C5 restore-chain variants of frs_decode.hip (tools/micro/restore_chain.hip measures the same forms):
dA = the round-5 pair step (newest pair through a dot2), dC = the newest samples by forced v_mad_i32_i24.
The tree's own source carries form B (24-bit multiplies summed by the compiler).  Libraries land in variants/."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from build_variant import build_variant  # noqa: E402

B_STEP = """                pe = __mul24(q1, xe_p) + pe;
                po = __mul24(q2, xe_p) + po;
                po = __mul24(q1, xo_p) + po;
                const int32_t xe = (__mul24(q0, xo_p) + pe) >> shift;
                const int32_t xo = (__mul24(q0, xe) + po) >> shift;"""
C_STEP = """                int32_t te, to;
                asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(te) : "v"(q1), "v"(xe_p), "v"(pe));
                asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(to) : "v"(q2), "v"(xe_p), "v"(po));
                asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(to) : "v"(q1), "v"(xo_p), "v"(to));
                asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(te) : "v"(q0), "v"(xo_p), "v"(te));
                const int32_t xe = te >> shift;
                asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(to) : "v"(q0), "v"(xe), "v"(to));
                const int32_t xo = to >> shift;"""
A_STEP = """                po = dec_dot2(Qr[(p2 + 3) & 3], Co[0], po);
                pe = dec_dot2(Qr[(p2 + 3) & 3], Ce[0], pe);
                const int32_t xe = pe >> shift;
                const int32_t xo = (__mul24(q0, xe) + po) >> shift;"""


def sub(old, new):
    def f(src):
        assert old in src, "pattern"
        return src.replace(old, new)
    return f


if __name__ == "__main__":
    which = sys.argv[1:] or ["dA", "dC"]
    for name in which:
        step = {"dA": A_STEP, "dC": C_STEP}[name]
        print(build_variant(name, sub(B_STEP, step), src_name="frs_decode.hip"))
