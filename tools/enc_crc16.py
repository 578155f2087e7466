"""Round-4 encoder variant: the frame CRC-16 by slice-by-16 (four buffer words per step, 16 tables = 8 KB of LDS per
work-group instead of 4 KB; 3 work-groups per CU still fit) instead of slice-by-8: half the dependent steps."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from build_variant import build_variant

REPL = [
    ("__constant__ uint16_t c_crc16x8[8][256];", "__constant__ uint16_t c_crc16x8[16][256];"),
    ("    uint16_t crc8x[8][256];  // slice-by-8 tables", "    uint16_t crc8x[16][256];  // slice-by-16 tables"),
    ("    static uint16_t t4[8][256];", "    static uint16_t t4[16][256];"),
    ("    for (int k = 1; k < 8; k++)\n        for (int i = 0; i < 256; i++) {\n            const uint16_t c = t4[k - 1][i];",
     "    for (int k = 1; k < 16; k++)\n        for (int i = 0; i < 256; i++) {\n            const uint16_t c = t4[k - 1][i];"),
    ("        for (; i + 1 < we; i += 2, colp += 128) {\n            const uint32_t w0 = colp[0], w1 = colp[64];",
     """        for (; i + 3 < we; i += 4, colp += 256) {
            const uint32_t w0 = colp[0], w1 = colp[64], w2 = colp[128], w3 = colp[192];
            c = (uint32_t)T[15][((c >> 8) ^ (w0 >> 24)) & 0xFF] ^ T[14][((c & 0xFF) ^ (w0 >> 16)) & 0xFF] ^
                T[13][(w0 >> 8) & 0xFF] ^ T[12][w0 & 0xFF] ^ T[11][w1 >> 24] ^ T[10][(w1 >> 16) & 0xFF] ^
                T[9][(w1 >> 8) & 0xFF] ^ T[8][w1 & 0xFF] ^ T[7][w2 >> 24] ^ T[6][(w2 >> 16) & 0xFF] ^
                T[5][(w2 >> 8) & 0xFF] ^ T[4][w2 & 0xFF] ^ T[3][w3 >> 24] ^ T[2][(w3 >> 16) & 0xFF] ^
                T[1][(w3 >> 8) & 0xFF] ^ T[0][w3 & 0xFF];
        }
        for (; i + 1 < we; i += 2, colp += 128) {
            const uint32_t w0 = colp[0], w1 = colp[64];"""),
]


def patch(s):
    for a, b in REPL:
        assert a in s, a[:60]
        s = s.replace(a, b)
    n = s.count("for (int i = threadIdx.x; i < 2048; i += blockDim.x) (&S.crc8x[0][0])[i] = (&c_crc16x8[0][0])[i];")
    assert n == 2, n
    return s.replace("for (int i = threadIdx.x; i < 2048; i += blockDim.x) (&S.crc8x[0][0])[i] = (&c_crc16x8[0][0])[i];",
                     "for (int i = threadIdx.x; i < 4096; i += blockDim.x) (&S.crc8x[0][0])[i] = (&c_crc16x8[0][0])[i];")


if __name__ == "__main__":
    print(build_variant("ebase", lambda s: s + "\n"))
    print(build_variant("ecrc16", patch))
