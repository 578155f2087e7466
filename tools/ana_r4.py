"""Round-4 analysis variants: k_analyze_v3's lean launch at 5 waves per SIMD (16- or 32-sample chunks per lane load
instead of 64, __launch_bounds__(256, 5)): 5120 wave slots for C4's 6241 tiles (1.22 rounds instead of 1.52)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from build_variant import build_variant

LB_A = "template <int DT, bool SLOW, bool STATS = false>\n__global__ void __launch_bounds__(256) k_analyze_v3("
LB_B = "template <int DT, bool SLOW, bool STATS = false>\n__global__ void __launch_bounds__(256, SLOW ? 1 : 5) k_analyze_v3("
CH_A = "    constexpr int kChunk = SLOW ? 16 : 64;"


def ana(chunk):
    def patch(s):
        assert LB_A in s and CH_A in s
        return s.replace(LB_A, LB_B).replace(CH_A, f"    constexpr int kChunk = SLOW ? 16 : {chunk};")
    return patch


if __name__ == "__main__":
    print(build_variant("base", lambda s: s))
    print(build_variant("ana16", ana(16)))
    print(build_variant("ana32", ana(32)))
