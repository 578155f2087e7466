// frs_decode.hip -- gfx950 decode path: FLAC frames -> int32 PCM -> de-normalised raster samples.
//
// Reference path replaced: converter.py:241-242 (pyflac.FileDecoder -> libFLAC
// FLAC__stream_decoder_process_until_end_of_stream, docs/sonos-pyflac.txt:1584-1640, 1809-1854) and
// converter.py:88-110 (_denormalize_from_audio), as used by cli.py:1022-1023 (extract-streaming).
//
// Frames carry no size field and STREAMINFO min/max framesize are 0 in these files, so frames are
// located in parallel: k_sync_select finds every byte that starts a sync code with a parseable,
// CRC-8-correct header and compacts them, in one pass (block counts + decoupled look-back), into the
// sorted candidate list (bounded: overflow is counted, never written); k_span_crc_wave finds for each
// candidate the first later candidate (or stream end) whose preceding two bytes are the CRC-16 of the
// span; k_chain_lds follows those spans from each stream's first byte (so false syncs inside frame data
// are never used); the frame decoders decode the true frames and check that the subframes end exactly at
// the CRC footer.  Positions are 64-bit throughout (a C4 arena is 3.1 GB); candidate indices are int32
// and the candidate buffer is capped below 2^31.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <type_traits>
#include <vector>

#include "frs_internal.h"

namespace frs {

__constant__ uint8_t d_crc8[256];
__constant__ uint16_t d_crc16[256];
__device__ __attribute__((aligned(16))) uint16_t d_crc16x4[4][256];  // slice-by-4 tables (T_0 = d_crc16), host-computed once per device
__device__ __attribute__((aligned(16))) uint16_t d_xpow_lo[256];   // x^(8m) mod P, m < 256
__device__ uint16_t d_xpow_hi[4096];  // x^(8*256*m) mod P

// a * b mod P (CRC-16 polynomial P = x^16 + x^15 + x^2 + 1), bitwise
__device__ inline uint32_t dec_gfmul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 15; i >= 0; i--) {
        r <<= 1;
        if (r & 0x10000u) r ^= 0x18005u;
        if ((b >> i) & 1u) r ^= a;
    }
    return r;
}
// c * x^(8m) mod P: the CRC state c advanced over m zero bytes (m < 2^20)
__device__ inline uint32_t crc_xpow(uint32_t c, uint32_t m) {
    if (c == 0 || m == 0) return c;
    return dec_gfmul(dec_gfmul(c, d_xpow_lo[m & 255]), d_xpow_hi[m >> 8]);
}
__device__ inline uint32_t gf_pow16(uint32_t b, uint64_t e) {  // b^e mod P
    uint32_t r = 1;
    while (e) {
        if (e & 1) r = dec_gfmul(r, b);
        b = dec_gfmul(b, b);
        e >>= 1;
    }
    return r;
}

struct FrameHdr {
    int32_t ok;
    int32_t frame_no;  // frame number from the header
    int32_t bs;        // block size
    int32_t hdr_len;   // header bytes incl. CRC-8
    int32_t chass;     // channel assignment
    int32_t bps;       // sample size
};

__device__ inline int stream_of(const int64_t *soff, int ns, int64_t p) {
    int lo = 0, hi = ns - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (soff[mid] <= p) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Parse + CRC-8-check a frame header at p (RFC 9639 9.1); end = end of the containing stream.
__device__ FrameHdr parse_header(const uint8_t *blob, int64_t p, int64_t end, int channels, int stream_bps) {
    FrameHdr h;
    h.ok = 0;
    if (p + 6 > end) return h;
    if (blob[p] != 0xFF || (blob[p + 1] & 0xFE) != 0xF8) return h;
    const uint8_t b2 = blob[p + 2], b3 = blob[p + 3];
    const int bsc = b2 >> 4, src = b2 & 15, chass = b3 >> 4, ssc = (b3 >> 1) & 7;
    if (bsc == 0 || src == 15 || chass > 10 || ssc == 3 || (b3 & 1)) return h;
    int64_t q = p + 4;
    uint32_t v = blob[q++];
    int extra = 0;
    if (v & 0x80) {
        if ((v & 0xE0) == 0xC0) { extra = 1; v &= 0x1F; }
        else if ((v & 0xF0) == 0xE0) { extra = 2; v &= 0x0F; }
        else if ((v & 0xF8) == 0xF0) { extra = 3; v &= 0x07; }
        else if ((v & 0xFC) == 0xF8) { extra = 4; v &= 0x03; }
        else if ((v & 0xFE) == 0xFC) { extra = 5; v &= 0x01; }
        else return h;
    }
    for (int i = 0; i < extra; i++) {
        if (q >= end) return h;
        const uint8_t c = blob[q++];
        if ((c & 0xC0) != 0x80) return h;
        v = (v << 6) | (c & 0x3F);
    }
    int bs;
    if (bsc == 1) bs = 192;
    else if (bsc >= 2 && bsc <= 5) bs = 576 << (bsc - 2);
    else if (bsc == 6) { if (q >= end) return h; bs = blob[q++] + 1; }
    else if (bsc == 7) { if (q + 1 >= end) return h; bs = ((blob[q] << 8) | blob[q + 1]) + 1; q += 2; }
    else bs = 256 << (bsc - 8);
    if (src == 12) q += 1;
    else if (src == 13 || src == 14) q += 2;
    if (q >= end) return h;
    uint8_t c = 0;
    for (int64_t i = p; i < q; i++) c = d_crc8[c ^ blob[i]];
    if (c != blob[q]) return h;
    const int nch = chass < 8 ? chass + 1 : 2;
    if (nch != channels) return h;
    h.ok = 1;
    h.frame_no = (int32_t)v;
    h.bs = bs;
    h.hdr_len = (int32_t)(q + 1 - p);
    h.chass = chass;
    h.bps = ssc == 1 ? 8 : ssc == 2 ? 12 : ssc == 4 ? 16 : ssc == 5 ? 20 : ssc == 6 ? 24 : ssc == 7 ? 32 : stream_bps;
    return h;
}

// ---------------------------------------------------------------------------------- candidate selection
// One pass over the blob: a block takes 64 KB (16 KB per wave, coalesced 16-byte loads: sel_masks_co), flags the bytes that
// start a sync code with a parseable CRC-8-correct header, and writes their positions, in order, at its
// exclusive prefix -- found by decoupled look-back over the blocks' published counts, 64 predecessors per step
// (one wave).  Blocks take their ordinal from a ticket (the block that draws the last ticket re-arms the counter
// for the next call), so a predecessor is always resident or done.  Status word: [63:40] call epoch, [39:38]
// flag, [37:0] count; words of another epoch read as "not published", so the buffer is never cleared.
constexpr int kSelThreads = 256, kSelBytes = 64 * 1024;  // 4 waves x 16 KB per block
constexpr uint64_t kSelAgg = 1ull << 38, kSelIncl = 2ull << 38, kSelVal = (1ull << 38) - 1;

__device__ inline int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Coalesced candidate flags: wave w of a 64 KB block takes the contiguous 16 KB at qw = block base + 16 KB w; step k
// of it is the 1 KB at qw + 1024 k, lane L its 16 bytes at + 16 L (one fully coalesced 16-byte load per lane and
// step), and the byte after them comes from lane L + 1 (lane 63: the next step's lane 0, or one guarded byte after
// the last step).  Bit j of m[k] marks a sync code with a parseable, CRC-8-correct header at qw + 1024 k + 16 L + j,
// so candidates are ordered by (k, lane, j).  Returns the lane's candidate count.
constexpr int kSelSteps = kSelBytes / (kSelThreads / 64) / 1024;  // 16 steps of 1 KB per wave
static_assert(kSelSteps == 16, "64 KB blocks of 4 waves");
// small ranges (a C5 query's tile, <= 4 MB): 16 KB blocks of 4 waves x 4 steps, so a 0.5 MB tile spreads over 32
// work-groups instead of 8 (the one-pass selection is latency-bound there)
constexpr int kSelStepsSmall = 4;

// CRC-8 (poly 0x07) of one byte folded into c, bitwise (no table: the header check runs from registers)
__device__ inline uint32_t crc8_byte(uint32_t c, uint32_t b) {
    c ^= b;
#pragma unroll
    for (int k = 0; k < 8; k++) c = (c & 0x80u) ? ((c << 1) ^ 0x07u) & 0xFFu : (c << 1) & 0xFFu;
    return c;
}

// parse_header on the 16 bytes h (little-endian dwords) that start at a sync code, `avail` bytes of the blob from
// there: the same acceptance test (RFC 9639 9.1: reserved codes, UTF-8 frame number, CRC-8, channel count).
__device__ inline bool header_ok_regs(const uint32_t *h, int64_t avail, int channels) {
    auto B = [&](int t) -> uint32_t { return (h[t >> 2] >> (8 * (t & 3))) & 0xFFu; };
    if (avail < 6) return false;
    const uint32_t b2 = B(2), b3 = B(3);
    const uint32_t bsc = b2 >> 4, src = b2 & 15, chass = b3 >> 4, ssc = (b3 >> 1) & 7;
    if (bsc == 0 || src == 15 || chass > 10 || ssc == 3 || (b3 & 1)) return false;
    const uint32_t v = B(4);
    int extra = 0;
    if (v & 0x80) {
        if ((v & 0xE0) == 0xC0) extra = 1;
        else if ((v & 0xF0) == 0xE0) extra = 2;
        else if ((v & 0xF8) == 0xF0) extra = 3;
        else if ((v & 0xFC) == 0xF8) extra = 4;
        else if ((v & 0xFE) == 0xFC) extra = 5;
        else return false;
    }
    int q = 5;
#pragma unroll
    for (int i = 0; i < 5; i++) {
        if (i < extra) {
            if (q >= avail || (B(5 + i) & 0xC0) != 0x80) return false;
            q++;
        }
    }
    if (bsc == 6) {
        if (q >= avail) return false;
        q += 1;
    } else if (bsc == 7) {
        if (q + 1 >= avail) return false;
        q += 2;
    }
    if (src == 12) q += 1;
    else if (src == 13 || src == 14) q += 2;
    if (q >= avail) return false;  // q <= 14: the CRC-8 byte is h's byte q
    uint32_t c = 0;
#pragma unroll
    for (int t = 0; t < 15; t++)
        if (t < q) c = crc8_byte(c, B(t));
    if (c != B(q)) return false;
    const int nch = chass < 8 ? (int)chass + 1 : 2;
    return nch == channels;
}

// dword idx (0..7) of the 32-byte window w0 | w1, idx dynamic (a select chain, no register indexing)
__device__ inline uint32_t win_dword(const uint4 &w0, const uint4 &w1, int idx) {
    uint32_t r = w0.x;
    r = idx == 1 ? w0.y : r;
    r = idx == 2 ? w0.z : r;
    r = idx == 3 ? w0.w : r;
    r = idx == 4 ? w1.x : r;
    r = idx == 5 ? w1.y : r;
    r = idx == 6 ? w1.z : r;
    r = idx == 7 ? w1.w : r;
    return r;
}

// ---- prefix CRC-16 of the selection range (two-pass form): the span check without a second read of the bytes.
// A frame's CRC-16 footer verifies iff CRC([p, e)) == 0, and with pc(p) = CRC-16 of the range's bytes [0, p)
// (init 0, no final xor: CRC(A B) = CRC(A) x^(8|B|) + CRC(B)), CRC([p, e)) = pc(e) + pc(p) x^(8(e - p)).  So the
// selection pass, which reads every byte anyway, also folds them: each lane the CRC of its 16 bytes (slice-by-16),
// a Horner state per lane over the wave's 16 steps, and -- only on steps holding a candidate or a stream boundary --
// the step's prefix (the 64 lanes' states reduced) and the lanes' exclusive in-step scan, from which a point's
// prefix within its 64 KB block follows.  A one-work-group scan chains the blocks; the span check is then one
// comparison per candidate pair (k_span_pcrc) instead of re-reading every frame (k_span_crc_lane).
constexpr int kSelCrcTab = 16 * 256 + 2 * 256 + 12 * 256;  // u16 entries: T16 | MK | ML[6]
__device__ __attribute__((aligned(16))) uint16_t d_selcrc_tab[kSelCrcTab];  // host-computed once per device
struct SelCrcLds {
    uint16_t T[16][256];     // T[k][v]: CRC-16 of byte v followed by k zero bytes
    uint16_t MK[2][256];     // multiply by x^(8 * 1024) (one step): [0] high byte, [1] low byte of the operand
    uint16_t ML[6][2][256];  // multiply by x^(8 * 16 * 2^i) (lane tree level i)
    uint16_t E[4][16][64];   // wave, step, lane: CRC of the step's bytes before the lane's 16 (point steps only)
    uint32_t SW[4][16];      // wave, step: CRC of the wave's bytes before the step (point steps only)
    uint32_t W[4];           // wave: CRC of its 16 KB
    uint32_t WP[4];          // wave: CRC of the block's bytes before it
};
static_assert(offsetof(SelCrcLds, E) == 2 * kSelCrcTab, "tables first, contiguous");
__device__ inline void sel_crc_load_tables(SelCrcLds *cx, int tid, int nthreads) {
    for (int i = tid; i < kSelCrcTab / 8; i += nthreads)
        reinterpret_cast<uint4 *>(&cx->T[0][0])[i] = reinterpret_cast<const uint4 *>(d_selcrc_tab)[i];
}
__device__ inline uint32_t crc_mul_tab(uint32_t c, const uint16_t (*M)[256]) { return (uint32_t)M[0][c >> 8] ^ M[1][c & 0xFFu]; }
__device__ inline uint32_t chunk_crc16(const uint4 &v, const uint16_t (*T)[256]) {  // 16 bytes (LE dwords) from 0
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
        for (int b = 0; b < 4; b++) c ^= T[15 - (4 * q + b)][(w[q] >> (8 * b)) & 0xFFu];
    return c;
}
// every lane: XOR over lanes L of a_L x^(128 (63 - L)) -- the CRC of the 64 consecutive 16-byte pieces
__device__ inline uint32_t lane_reduce_crc(uint32_t a, int lane, const uint16_t (*ML)[2][256]) {
#pragma unroll
    for (int i = 0; i < 6; i++) {
        const uint32_t o = (uint32_t)__shfl_xor((int)a, 1 << i);
        const bool hi = (lane >> i) & 1;
        a = crc_mul_tab(hi ? o : a, ML[i]) ^ (hi ? a : o);
    }
    return a;
}
// lane L: the CRC of pieces 0 .. L - 1 (Kogge-Stone over the lanes)
__device__ inline uint32_t lane_excl_scan_crc(uint32_t c, int lane, const uint16_t (*ML)[2][256]) {
    uint32_t x = c;
#pragma unroll
    for (int i = 0; i < 6; i++) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, 1 << i);
        if (lane >= (1 << i)) x = crc_mul_tab(y, ML[i]) ^ x;
    }
    const uint32_t e = (uint32_t)__shfl_up((int)x, 1);
    return lane ? e : 0u;
}
// CRC of the wave's bytes [wave start, point) for a point at step k, lane `lane`, byte j of its 16 (point steps'
// SW / E recorded); the lane's first j bytes are read again (rare: candidates and stream boundaries)
__device__ inline uint32_t sel_point_crc(const SelCrcLds *cx, int wv, int k, int lane, int j, const uint8_t *abase,
                                         int64_t qc, int lead) {
    uint32_t r = crc_xpow(cx->SW[wv][k], 16u * (uint32_t)lane + (uint32_t)j) ^ crc_xpow(cx->E[wv][k][lane], (uint32_t)j);
    uint32_t c = 0;
    for (int b = 0; b < j; b++) {
        const uint32_t byte = qc + b >= lead ? abase[qc + b] : 0u;
        c = ((c << 8) & 0xFFFFu) ^ cx->T[0][((c >> 8) ^ byte) & 0xFFu];
    }
    return r ^ c;
}

// The sync patterns `raw` (bit j: a 0xFF 0xF8/F9 pair at byte j) of one lane's 16 bytes `cur` (blob position p0),
// `nxt` = the following 16 bytes: the bits whose header parses (header_ok_regs on the 32-byte window; the global
// parse when the window does not hold the next 16 bytes).  Out of line: the rare path must not keep the caller's
// step loop from unrolling (a rolled loop indexed the 16 loaded chunks dynamically, i.e. through scratch memory).
__device__ inline uint32_t sel_check_body(uint4 cur, uint4 nxt, uint32_t raw, int64_t p0, int64_t nbytes,
                                          const uint8_t *blob, const int64_t *soff, int ns, int channels,
                                          int stream_bps, bool regs_ok) {
    uint32_t mask = 0;
    while (raw) {
        const int j = __builtin_ctz(raw);
        raw &= raw - 1;
        const int64_t p = p0 + j;
        if (p < 0 || p + 1 >= nbytes) continue;
        bool ok;
        if (regs_ok) {
            uint32_t h[4];
            const int wi = j >> 2, sh = j & 3;
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const uint32_t lo = win_dword(cur, nxt, wi + d), hi = win_dword(cur, nxt, min(wi + d + 1, 7));
                h[d] = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)sh);
            }
            ok = header_ok_regs(h, min<int64_t>(nbytes - p, 16), channels);
        } else {
            // (one stream: its end is the range end -- the single-stream latency path passes its tables as kernel
            // arguments, so soff may not be in device memory yet)
            const int st = stream_of(soff, ns, p);
            ok = parse_header(blob, p, ns == 1 ? nbytes : soff[st + 1], channels, stream_bps).ok;
        }
        if (ok) mask |= 1u << j;
    }
    return mask;
}

__device__ __attribute__((noinline)) uint32_t sel_check_candidates(uint4 cur, uint4 nxt, uint32_t raw, int64_t p0,
                                                                   int64_t nbytes, const uint8_t *blob,
                                                                   const int64_t *soff, int ns, int channels,
                                                                   int stream_bps, bool regs_ok) {
    return sel_check_body(cur, nxt, raw, p0, nbytes, blob, soff, ns, channels, stream_bps, regs_ok);
}

// Coalesced candidate flags: wave w of a 64 KB block takes the contiguous 16 KB at qw = block base + 16 KB w; step k
// of it is the 1 KB at qw + 1024 k, lane L its 16 bytes at + 16 L (one fully coalesced 16-byte load per lane and
// step).  Bit j of m[k] marks a sync code with a parseable, CRC-8-correct header at qw + 1024 k + 16 L + j, so
// candidates are ordered by (k, lane, j).  The header check runs on registers: a step with a sync pattern fetches
// each lane's successor 16 bytes (lane L + 1; lane 63: the next step's lane 0) by shuffles, so a header (<= 16 bytes)
// lies in the lane's 32-byte window -- no dependent global loads, which had made the pass latency-bound (~1 TB/s).
// Only a header starting in the wave's last 16 bytes takes the global parse.  Headers are bounded by the blob end
// (not the stream end: a header straddling a stream boundary becomes a candidate whose CRC span never verifies).
// Returns the lane's candidate count.
// FULL: the caller knows the wave's 16 KB lie inside the range: no per-lane guards.  (A separate kernel instance:
// with both load forms in one kernel the compiler keeps a second register set live -- 116 instead of 87 VGPRs.)
template <int STEPS = kSelSteps, bool CRC = false, bool FULL = false>
__device__ inline int sel_masks_co(const uint8_t *blob, int64_t nbytes, const int64_t *soff, int ns, int channels,
                                   int stream_bps, int64_t qw, int lane, uint32_t *m, SelCrcLds *cx = nullptr,
                                   int wv = 0, uint32_t bsteps = 0) {
    constexpr int kSelSteps = STEPS;
    const int lead = (int)(reinterpret_cast<uintptr_t>(blob) & 15);
    const uint8_t *base = blob - lead;
    const int64_t qend = nbytes + lead;
    // all 16 loads in flight at once: unconditional (a chunk past the end re-reads chunk 0 and is zeroed after) --
    // a guarded load per step compiled to 16 load/wait round trips
    uint4 v[kSelSteps];
    if constexpr (FULL) {
        const uint8_t *wb = base + qw;
#pragma unroll
        for (int k = 0; k < kSelSteps; k++)
            v[k] = *reinterpret_cast<const uint4 *>(wb + (uint32_t)(1024 * k + 16 * lane));
    } else {
#pragma unroll
        for (int k = 0; k < kSelSteps; k++) {
            const int64_t q = qw + 1024 * k + 16 * lane;
            v[k] = *reinterpret_cast<const uint4 *>(base + (q < qend ? q : 0));
        }
#pragma unroll
        for (int k = 0; k < kSelSteps; k++)
            if (qw + 1024 * k + 16 * lane >= qend) v[k] = make_uint4(0, 0, 0, 0);
    }
    const int64_t qlast = qw + 1024 * kSelSteps;  // the byte after the wave's 16 KB
    const uint32_t after = (lane == 63 && qlast < qend) ? base[qlast] : 0u;
    int cnt = 0;
    uint32_t acc = 0;  // CRC: Horner state of this lane's pieces over the steps so far
    // no CRC fold (round 6; the one-pass selection and the placement pass's re-scan -- k_sync_count has its own
    // queue form, sel_count_queue): the header checks wait until every step is flagged -- the steps keep only their
    // patterns (16 bits each, two steps per register) and the steps holding one (rsteps), so the call to the
    // rare-path check no longer sits between the 16 loaded chunks and the steps that read them
    uint32_t rp[(kSelSteps + 1) / 2];
#pragma unroll
    for (int i = 0; i < (kSelSteps + 1) / 2; i++) rp[i] = 0;
    uint32_t rsteps = 0;
#pragma unroll
    for (int k = 0; k < kSelSteps; k++) {
        // first byte of the next 16 bytes: lane L + 1's word 0 (lane 63: next step's lane 0)
        uint32_t nx = (uint32_t)__shfl_down((int)v[k].x, 1);
        const uint32_t n0 = k + 1 < kSelSteps ? (uint32_t)__builtin_amdgcn_readlane((int)v[k + 1 < kSelSteps ? k + 1 : k].x, 0)
                                              : after;
        if (lane == 63) nx = n0;
        const uint32_t w[5] = {v[k].x, v[k].y, v[k].z, v[k].w, nx & 0xFFu};
        // sync patterns (0xFF then 0xF8 / 0xF9) of this lane's 16 bytes.  Branch-free test first (round 6): per dword
        // t = ~x | ((x >> 8 | next byte << 24) & 0xFE..FE ^ 0xF8..F8) has a zero byte exactly where a pattern starts,
        // and haszero(t) is exact as a boolean; a 0xFF alone (1.6 % of dwords, so nearly every step of some lane) no
        // longer sends the whole wave through the per-byte test, which runs only on steps with a pattern (~3 %)
        uint32_t hit = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t sh = __builtin_amdgcn_alignbyte(w[i + 1], w[i], 1u);
            const uint32_t t = ~w[i] | ((sh & 0xFEFEFEFEu) ^ 0xF8F8F8F8u);
            hit |= (t - 0x01010101u) & ~t & 0x80808080u;
        }
        uint32_t raw = 0;
        if (__ballot(hit != 0)) {  // (wave-uniform, rare) the exact per-byte flags
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t x = w[i];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t b0 = (x >> (8 * j)) & 0xFF;
                    const uint32_t b1 = j < 3 ? (x >> (8 * j + 8)) & 0xFF : w[i + 1] & 0xFF;
                    if (b0 == 0xFF && (b1 & 0xFE) == 0xF8) raw |= 1u << (4 * i + j);
                }
            }
        }
        if constexpr (!CRC) {
            rp[k >> 1] |= raw << (16 * (k & 1));
            if (__ballot(raw != 0)) rsteps |= 1u << k;
            continue;
        }
        uint32_t mask = 0;
        if (__ballot(raw != 0)) {  // (wave-uniform, ~3 % of steps) the successor 16 bytes of every lane
            // lane L reads lane L + 1's chunk; lane 63 lane 0's chunk of the next step (all lanes shuffle: no
            // cross-lane read inside a divergent branch)
            const uint4 &vn = v[k + 1 < kSelSteps ? k + 1 : k];
            const uint4 src = lane == 0 ? vn : v[k];
            const int from = (lane + 1) & 63;
            uint4 nv;
            nv.x = (uint32_t)__shfl((int)src.x, from);
            nv.y = (uint32_t)__shfl((int)src.y, from);
            nv.z = (uint32_t)__shfl((int)src.z, from);
            nv.w = (uint32_t)__shfl((int)src.w, from);
            const int64_t q0 = qw + 1024 * k + 16 * lane;
            const bool regs_ok = k + 1 < kSelSteps || lane < 63;  // the window holds the next 16 bytes
            if (raw) mask = sel_check_candidates(v[k], nv, raw, q0 - lead, nbytes, blob, soff, ns, channels,
                                                 stream_bps, regs_ok);
        }
        m[k] = mask;
        cnt += __builtin_popcount(mask);
        if constexpr (CRC) {
            uint4 cv = v[k];
            if (qw + 1024 * k + 16 * lane == 0 && lead) {  // bytes before the blob start count as zeros
                auto keep = [&](uint32_t w, int d) -> uint32_t {
                    const int nb = lead - 4 * d;  // leading bytes of this dword to clear
                    return nb >= 4 ? 0u : nb <= 0 ? w : (w & ~((1u << (8 * nb)) - 1u));
                };
                cv = make_uint4(keep(cv.x, 0), keep(cv.y, 1), keep(cv.z, 2), keep(cv.w, 3));
            }
            const uint32_t c = chunk_crc16(cv, cx->T);
            if (__ballot(mask != 0) || ((bsteps >> k) & 1u)) {  // (wave-uniform) a point step
                const uint32_t sw = lane_reduce_crc(acc, lane, cx->ML);
                const uint32_t e = lane_excl_scan_crc(c, lane, cx->ML);
                cx->E[wv][k][lane] = (uint16_t)e;
                if (lane == 0) cx->SW[wv][k] = sw;
            }
            acc = crc_mul_tab(acc, cx->MK) ^ c;
        }
    }
    if constexpr (CRC) {
        const uint32_t w = lane_reduce_crc(acc, lane, cx->ML);
        if (lane == 0) cx->W[wv] = w;
    } else {
        // the header checks of the flagged steps: the lane's 16 bytes and the next 16 read again (L2-hot; the next
        // 16 zero past the range end, as the in-register window had them)
#pragma unroll
        for (int k = 0; k < kSelSteps; k++) {
            uint32_t mask = 0;
            if ((rsteps >> k) & 1u) {  // (wave-uniform)
                const uint32_t raw = (rp[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                if (raw) {
                    const int64_t q0 = qw + 1024 * k + 16 * lane;
                    const uint4 cur = *reinterpret_cast<const uint4 *>(base + q0);
                    const uint4 nxt = q0 + 16 < qend ? *reinterpret_cast<const uint4 *>(base + q0 + 16)
                                                     : make_uint4(0, 0, 0, 0);
                    const bool regs_ok = k + 1 < kSelSteps || lane < 63;  // the window holds the next 16 bytes
                    mask = sel_check_candidates(cur, nxt, raw, q0 - lead, nbytes, blob, soff, ns, channels,
                                                stream_bps, regs_ok);
                }
            }
            m[k] = mask;
            cnt += __builtin_popcount(mask);
        }
    }
    return cnt;
}

__device__ inline int wave_excl_scan_i32(int v, int lane, int &total) {
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    total = __builtin_amdgcn_readlane(x, 63);
    return x - v;
}

// candidate positions of one wave in (k, lane, j) order from output index `base`; past the cap only counted
// CRC: ccrc[idx] = CRC of [origin, candidate), `pre` = CRC of [origin, wave start)
template <int STEPS = kSelSteps, bool CRC = false>
__device__ inline void sel_emit_co(const uint32_t *m, int64_t qw, int lane, int lead, int64_t base, int64_t *cpos,
                                   int64_t cap, uint16_t *ccrc = nullptr, const SelCrcLds *cx = nullptr, int wv = 0,
                                   const uint8_t *abase = nullptr, uint32_t pre = 0) {
    constexpr int kSelSteps = STEPS;
#pragma unroll
    for (int k = 0; k < kSelSteps; k++) {
        if (__ballot(m[k] != 0) == 0) continue;  // (wave-uniform) most steps hold no candidate: no scan
        int tot;
        const int ex = wave_excl_scan_i32(__builtin_popcount(m[k]), lane, tot);
        if (tot) {
            int64_t idx = base + ex;
            uint32_t mask = m[k];
            while (mask) {
                const int j = __builtin_ctz(mask);
                mask &= mask - 1;
                if (idx < cap) {
                    cpos[idx] = qw + 1024 * k + 16 * lane + j - lead;
                    if constexpr (CRC) {
                        const int64_t qc = qw + 1024 * k + 16 * lane;
                        ccrc[idx] = (uint16_t)(crc_xpow(pre, (uint32_t)(qc + j - qw)) ^
                                               sel_point_crc(cx, wv, k, lane, j, abase, qc, lead));
                    }
                }
                idx++;
            }
        }
        base += tot;
    }
}

// Two-pass selection count without the CRC fold (round 6, the batched mono decode): the steps only flag sync patterns
// (a branch-free test per dword, sel_masks_co) and append each lane holding one to the wave's queue in LDS -- entry =
// step << 22 | lane << 16 | pattern bits, appended in (step, lane) order; then the queue's header checks run 64 at a
// time, one entry per lane (the entry's 32-byte window read again, L2-hot), each entry's low 16 bits replaced by its
// candidate bits.  Round 5 checked each flagged step for the whole wave in turn with the 16 chunks still in registers
// (a call holding them live: 124 VGPRs) -- per wave ~2 K VALU, most of it the per-byte test that any 0xFF byte in
// any lane triggered.  Candidates keep the (k, lane, j) order of sel_masks_co / sel_emit_co (the queue's order), so the
// placement pass's re-scan of an overflowing block agrees.  Returns the lane's candidate count; qn = queue length.
constexpr int kSelQueue = kSelSteps * 64;  // entries per wave (every lane of every step)
// CRC (the prefix-CRC span check): also the lanes' CRC fold of sel_masks_co<CRC> -- a step is a point step (E / SW
// recorded) when some lane holds a sync pattern (a superset of the candidate steps) or a stream boundary.
template <bool FULL, bool CRC = false>
__device__ inline int sel_count_queue(const uint8_t *blob, int64_t nbytes, const int64_t *soff, int ns, int channels,
                                      int stream_bps, int64_t qw, int lane, uint32_t *q, int &qn_out,
                                      SelCrcLds *cx = nullptr, int wv = 0, uint32_t bsteps = 0) {
    const int lead = (int)(reinterpret_cast<uintptr_t>(blob) & 15);
    const uint8_t *base = blob - lead;
    const int64_t qend = nbytes + lead;
    uint4 v[kSelSteps];
    if constexpr (FULL) {
        const uint8_t *wb = base + qw;
#pragma unroll
        for (int k = 0; k < kSelSteps; k++)
            v[k] = *reinterpret_cast<const uint4 *>(wb + (uint32_t)(1024 * k + 16 * lane));
    } else {
#pragma unroll
        for (int k = 0; k < kSelSteps; k++) {
            const int64_t qq = qw + 1024 * k + 16 * lane;
            v[k] = *reinterpret_cast<const uint4 *>(base + (qq < qend ? qq : 0));
        }
#pragma unroll
        for (int k = 0; k < kSelSteps; k++)
            if (qw + 1024 * k + 16 * lane >= qend) v[k] = make_uint4(0, 0, 0, 0);
    }
    const int64_t qlast = qw + 1024 * kSelSteps;  // the byte after the wave's 16 KB
    const uint32_t after = (lane == 63 && qlast < qend) ? base[qlast] : 0u;
    int qn = 0;  // (wave-uniform)
    uint32_t acc = 0;  // CRC: Horner state of this lane's pieces over the steps so far
#pragma unroll
    for (int k = 0; k < kSelSteps; k++) {
        uint32_t nx = (uint32_t)__shfl_down((int)v[k].x, 1);
        const uint32_t n0 = k + 1 < kSelSteps ? (uint32_t)__builtin_amdgcn_readlane((int)v[k + 1 < kSelSteps ? k + 1 : k].x, 0)
                                              : after;
        if (lane == 63) nx = n0;
        const uint32_t w[5] = {v[k].x, v[k].y, v[k].z, v[k].w, nx & 0xFFu};
        uint32_t hit = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t sh = __builtin_amdgcn_alignbyte(w[i + 1], w[i], 1u);
            const uint32_t t = ~w[i] | ((sh & 0xFEFEFEFEu) ^ 0xF8F8F8F8u);
            hit |= (t - 0x01010101u) & ~t & 0x80808080u;
        }
        const uint64_t bm = __ballot(hit != 0);
        if (bm) {  // (wave-uniform, ~3 % of steps) the exact per-byte flags of the lanes with one, queued
            if (hit) {
                uint32_t raw = 0;
#pragma unroll
                for (int i = 0; i < 4; i++) {
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t b0 = (w[i] >> (8 * j)) & 0xFF;
                        const uint32_t b1 = j < 3 ? (w[i] >> (8 * j + 8)) & 0xFF : w[i + 1] & 0xFF;
                        if (b0 == 0xFF && (b1 & 0xFE) == 0xF8) raw |= 1u << (4 * i + j);
                    }
                }
                const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
                q[qn + below] = ((uint32_t)k << 22) | ((uint32_t)lane << 16) | raw;  // (hit exact: raw != 0)
            }
            qn += __builtin_popcountll(bm);
        }
        if constexpr (CRC) {
            uint4 cv = v[k];
            if (qw + 1024 * k + 16 * lane == 0 && lead) {  // bytes before the blob start count as zeros
                auto keep = [&](uint32_t x, int d) -> uint32_t {
                    const int nb = lead - 4 * d;  // leading bytes of this dword to clear
                    return nb >= 4 ? 0u : nb <= 0 ? x : (x & ~((1u << (8 * nb)) - 1u));
                };
                cv = make_uint4(keep(cv.x, 0), keep(cv.y, 1), keep(cv.z, 2), keep(cv.w, 3));
            }
            const uint32_t c = chunk_crc16(cv, cx->T);
            if (bm || ((bsteps >> k) & 1u)) {  // (wave-uniform) a point step
                const uint32_t sw = lane_reduce_crc(acc, lane, cx->ML);
                const uint32_t e = lane_excl_scan_crc(c, lane, cx->ML);
                cx->E[wv][k][lane] = (uint16_t)e;
                if (lane == 0) cx->SW[wv][k] = sw;
            }
            acc = crc_mul_tab(acc, cx->MK) ^ c;
        }
    }
    if constexpr (CRC) {
        const uint32_t wc = lane_reduce_crc(acc, lane, cx->ML);
        if (lane == 0) cx->W[wv] = wc;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // the queue's LDS writes have landed (one wave: in order)
    __builtin_amdgcn_wave_barrier();
    int cnt = 0;
    for (int r0 = 0; r0 < qn; r0 += 64) {  // (wave-uniform) the header checks, one queue entry per lane
        const int i = r0 + lane;
        if (i < qn) {
            const uint32_t e = q[i];
            const int k = (int)(e >> 22), ln = (int)((e >> 16) & 63);
            const int64_t q0 = qw + 1024 * k + 16 * ln;
            const uint4 cur = *reinterpret_cast<const uint4 *>(base + q0);
            const uint4 nxt = q0 + 16 < qend ? *reinterpret_cast<const uint4 *>(base + q0 + 16) : make_uint4(0, 0, 0, 0);
            const bool regs_ok = k + 1 < kSelSteps || ln < 63;  // as sel_masks_co: the window holds the next 16 bytes
            const uint32_t mask = sel_check_body(cur, nxt, e & 0xFFFFu, q0 - lead, nbytes, blob, soff, ns, channels,
                                                 stream_bps, regs_ok);
            q[i] = (e & 0xFFFF0000u) | mask;
            cnt += __builtin_popcount(mask);
        }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    qn_out = qn;
    return cnt;
}

// the candidate positions of sel_count_queue's checked queue, from output index `base` (past `cap` only counted);
// CRC: ccrc[idx] = CRC of [origin, candidate) as sel_emit_co<CRC> forms it (`pre` = CRC of [origin, wave start))
template <bool CRC = false>
__device__ inline void sel_emit_queue(const uint32_t *q, int qn, int64_t qw, int lane, int lead, int64_t base,
                                      int64_t *cpos, int64_t cap, uint16_t *ccrc = nullptr,
                                      const SelCrcLds *cx = nullptr, int wv = 0, const uint8_t *abase = nullptr,
                                      uint32_t pre = 0) {
    for (int r0 = 0; r0 < qn; r0 += 64) {  // (wave-uniform)
        const int i = r0 + lane;
        const uint32_t e = i < qn ? q[i] : 0u;
        uint32_t mask = e & 0xFFFFu;
        int tot;
        const int ex = wave_excl_scan_i32(__builtin_popcount(mask), lane, tot);
        int64_t idx = base + ex;
        const int ek = (int)(e >> 22), eln = (int)((e >> 16) & 63);
        const int64_t qc = qw + 1024 * ek + 16 * eln;
        while (mask) {
            const int j = __builtin_ctz(mask);
            mask &= mask - 1;
            if (idx < cap) {
                cpos[idx] = qc - lead + j;
                if constexpr (CRC)
                    ccrc[idx] = (uint16_t)(crc_xpow(pre, (uint32_t)(qc + j - qw)) ^
                                           sel_point_crc(cx, wv, ek, eln, j, abase, qc, lead));
            }
            idx++;
        }
        base += tot;
    }
}

// One stream (a bbox query's tile): its call tables [soff | fbase | poff | (max - min, min)] ride in the kernel
// arguments and block 0 writes them to `tabdst` for the later kernels (no host-to-device copy per query)
struct SmallTabs {
    int64_t v[7];
};
template <int STEPS>
__global__ void __launch_bounds__(kSelThreads) k_sync_select(const uint8_t *blob, int64_t nbytes, const int64_t *soff,
                                                           int ns, int channels, int stream_bps, uint64_t *status,
                                                           unsigned long long *ticket, uint32_t epoch, int64_t nblocks,
                                                           int64_t *cpos, int64_t cap, int *counts,
                                                           int64_t *tabdst = nullptr, SmallTabs tabs = {}) {
    constexpr int kSelSteps = STEPS, kSelBytes = STEPS * 1024 * (kSelThreads / 64);
    __shared__ int64_t s_ord, s_base;
    __shared__ int s_wsum[kSelThreads / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (tabdst && blockIdx.x == 0 && t < 7) tabdst[t] = tabs.v[t];
    if (t == 0) {
        const int64_t o = (int64_t)atomicAdd(ticket, 1ull);
        if (o == nblocks - 1) atomicExch(ticket, 0ull);  // every ticket of this launch is drawn: re-arm
        s_ord = o;
    }
    __syncthreads();
    const int64_t ord = s_ord;
    const int lead = (int)(reinterpret_cast<uintptr_t>(blob) & 15);
    const int64_t qw = ord * kSelBytes + (int64_t)(kSelBytes / 4) * wv;
    uint32_t m[kSelSteps];
    int cnt = sel_masks_co<STEPS>(blob, nbytes, soff, ns, channels, stream_bps, qw, lane, m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (lane == 0) s_wsum[wv] = cnt;
    __syncthreads();
    int wbase = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kSelThreads / 64; k++) {
        const int sv = s_wsum[k];
        wbase += k < wv ? sv : 0;
        tot += sv;
    }
    if (wv == 0) {  // publish, then look back 64 predecessors at a time
        const uint64_t tag = (uint64_t)epoch << 40;
        int64_t excl = 0;
        if (ord == 0) {
            if (lane == 0) {
                __hip_atomic_store(&status[0], tag | kSelIncl | (uint64_t)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                counts[1] = 0;  // nvalid, bad, lane-decoder queue, optimistic-decode fallback flag and count:
                counts[2] = 0;  // zeroed here (later kernels run after this one)
                counts[3] = 0;
                counts[6] = 0;  // (ints 4-5 hold the selection ticket)
                counts[7] = 0;
            }
        } else {
            if (lane == 0)
                __hip_atomic_store(&status[ord], tag | kSelAgg | (uint64_t)tot, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            for (int64_t hi = ord - 1;;) {
                const int64_t j = hi - lane;
                uint64_t sv = tag | kSelIncl;  // before block 0: inclusive 0
                if (j >= 0) sv = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool valid = (sv >> 40) == epoch && (sv & (kSelAgg | kSelIncl));
                const uint64_t has = __ballot(valid && (sv & kSelIncl));
                const int fl = has ? __builtin_ctzll(has) : 64;  // nearest inclusive predecessor
                const bool need = lane <= fl;
                if (__ballot(need && !valid)) {
                    __builtin_amdgcn_s_sleep(2);
                    continue;
                }
                excl += wave_sum_i64(need ? (int64_t)(sv & kSelVal) : 0);
                if (fl < 64) break;
                hi -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&status[ord], tag | kSelIncl | (uint64_t)(excl + tot), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            if (ord == nblocks - 1) counts[0] = (int)min<int64_t>(excl + tot, (int64_t)0x7FFFFFFF);
            s_base = excl;
        }
    }
    __syncthreads();
    sel_emit_co<STEPS>(m, qw, lane, lead, s_base + wbase, cpos, cap);
}

// Large ranges (a whole arena): the single pass above serialises on its look-back (the inclusive prefix advances one
// 64-block window per status round trip: ~7 ms over a 3.1 GB arena), so large ranges take two passes instead --
// per-block counts (each block also keeps up to kSelBlkCap of its candidate positions, in order, in a per-block
// scratch), one work-group's scan of the counts, and a placement pass that copies the kept positions to their place;
// only a block with more candidates than its scratch holds reads its 64 KB again (the range used to be read twice in
// full: 3.1 GB more per whole-arena decode).
constexpr int kSelBlkCap = 32;  // candidates kept per 64 KB block (a C4 block holds ~8 frame starts)

// CRC combine of the block's four 16 KB waves (thread 0): WP[w] = CRC of the block's bytes before wave w; returns the
// block's CRC
__device__ inline uint32_t sel_crc_block(SelCrcLds *cx) {
    const uint32_t X = d_xpow_hi[64];  // x^(8 * 16384)
    uint32_t pre = 0;
#pragma unroll
    for (int w = 0; w < kSelThreads / 64; w++) {
        cx->WP[w] = pre;
        pre = dec_gfmul(pre, X) ^ cx->W[w];
    }
    return pre;
}

// CRC (prefix-CRC span check): the block's CRC to bcrc[b], each kept candidate's CRC from the block start to bipc
// (beside bpos), and each stream boundary inside the block (bfirst[b]: the first such stream index, soff[s] + lead
// past the block start) to sbib[s]
// FULL: blocks [blk0, blk0 + grid) lie inside the range (the host launches the range's last block apart)
template <bool CRC = false, bool FULL = false>
__global__ void __launch_bounds__(kSelThreads) k_sync_count(const uint8_t *blob, int64_t nbytes, const int64_t *soff,
                                                          int ns, int channels, int stream_bps, int32_t *bcount,
                                                          int64_t *bpos, uint16_t *bcrc = nullptr,
                                                          uint16_t *bipc = nullptr, const uint32_t *bfirst = nullptr,
                                                          uint16_t *sbib = nullptr, int64_t blk0 = 0) {
    const int64_t blk = blk0 + blockIdx.x;
    __shared__ int s_wsum[kSelThreads / 64];
    __shared__ typename std::conditional<CRC, SelCrcLds, char>::type cxs;
    __shared__ uint32_t s_queue[kSelThreads / 64][kSelQueue];  // sel_count_queue's queues
    SelCrcLds *cx = CRC ? reinterpret_cast<SelCrcLds *>(&cxs) : nullptr;
    const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);  // (wave-uniform: scalar)
    const int lead = (int)(reinterpret_cast<uintptr_t>(blob) & 15);
    const int64_t qw = blk * kSelBytes + (int64_t)(kSelBytes / 4) * wv;
    uint32_t bsteps = 0;  // this wave's steps holding a stream boundary
    const int sb0 = CRC ? (int)bfirst[blk] : -1;
    if constexpr (CRC) {
        sel_crc_load_tables(cx, t, kSelThreads);
        for (int sidx = sb0; sidx >= 0 && sidx <= ns; sidx++) {
            const int64_t q = soff[sidx] + lead;
            if (q >= qw + kSelBytes / 4) break;
            if (q >= qw) bsteps |= 1u << ((q - qw) >> 10);
        }
        __syncthreads();
    }
    int qn = 0;
    int c = sel_count_queue<FULL, CRC>(blob, nbytes, soff, ns, channels, stream_bps, qw, lane, &s_queue[wv][0], qn, cx,
                                       wv, bsteps);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) s_wsum[wv] = c;
    __syncthreads();
    int wbase = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kSelThreads / 64; k++) {
        wbase += k < wv ? s_wsum[k] : 0;
        tot += s_wsum[k];
    }
    if (t == 0) bcount[blk] = tot;
    const int64_t slot = blk * kSelBlkCap;
    if constexpr (CRC) {
        if (t == 0) bcrc[blk] = (uint16_t)sel_crc_block(cx);
        __syncthreads();
        const uint8_t *abase = blob - lead;
        if (tot <= kSelBlkCap)
            sel_emit_queue<true>(&s_queue[wv][0], qn, qw, lane, lead, slot + wbase, bpos, slot + kSelBlkCap, bipc, cx, wv,
                                 abase, cx->WP[wv]);
        for (int sidx = sb0; sidx >= 0 && sidx <= ns; sidx++) {  // (wave-uniform loop) stream boundaries
            const int64_t q = soff[sidx] + lead;
            if (q >= qw + kSelBytes / 4) break;
            if (q < qw) continue;
            const int64_t d = q - qw;
            if (lane == (int)((d >> 4) & 63))
                sbib[sidx] = (uint16_t)(crc_xpow(cx->WP[wv], (uint32_t)d) ^
                                        sel_point_crc(cx, wv, (int)(d >> 10), lane, (int)(d & 15), abase, q - (d & 15),
                                                      lead));
        }
    } else if (tot <= kSelBlkCap) {  // (block-uniform) keep the positions: the placement pass copies them
        sel_emit_queue(&s_queue[wv][0], qn, qw, lane, lead, slot + wbase, bpos, slot + kSelBlkCap);
    }
}

// stream boundaries for the prefix-CRC span check: bfirst[b] = the smallest stream index s >= 1 whose start
// soff[s] + lead lies inside 64 KB block b (not at its first byte); bfirst is 0xFF-filled before
__global__ void k_bound_mark(const int64_t *soff, int ns, int lead, uint32_t *bfirst) {
    const int sidx = (int)(blockIdx.x * blockDim.x + threadIdx.x) + 1;
    if (sidx > ns) return;
    const int64_t q = soff[sidx] + lead;
    if (q & (kSelBytes - 1)) atomicMin(&bfirst[q / kSelBytes], (uint32_t)sidx);
}

// exclusive scan of the block counts in one work-group (bbase[n] = total -> counts[0]); zeroes the later counters
// CRC (bcrc != nullptr): also BP[i] = CRC of the range's bytes before block i, i = 0 .. n (BP[n]: all n blocks)
__global__ void __launch_bounds__(1024) k_sync_scan(const int32_t *bcount, int64_t *bbase, int64_t n, int *counts,
                                                  const uint16_t *bcrc = nullptr, uint32_t *BP = nullptr) {
    __shared__ int64_t wsum[16];
    __shared__ uint32_t wcrc[16];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t c = (n + 1023) / 1024;
    const int64_t a = min(n, (int64_t)t * c), b = min(n, a + c);
    int64_t run = 0;
#pragma unroll 8
    for (int64_t i = a; i < b; i++) run += bcount[i];  // (unrolled: the loads of a thread's range issue together)
    int64_t x = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int64_t base = 0, total = 0;
    for (int k = 0; k < 16; k++) {
        base += k < wv ? wsum[k] : 0;
        total += wsum[k];
    }
    int64_t acc = base + x - run;
#pragma unroll 8
    for (int64_t i = a; i < b; i++) {
        bbase[i] = acc;
        acc += bcount[i];
    }
    if (t == 0) {
        counts[0] = (int)min<int64_t>(total, (int64_t)0x7FFFFFFF);
        counts[1] = 0;
        counts[2] = 0;
        counts[3] = 0;
        counts[6] = 0;  // (ints 4-5 hold the selection ticket)
        counts[7] = 0;
    }
    if (!bcrc) return;
    // thread t folds blocks [t c, t c + c) (blocks >= n: zeros), Kogge-Stone over the threads with the uniform
    // multipliers KB^(c 2^i), KB = x^(8 * 64 KB); then each thread re-walks its blocks from its exclusive prefix
    const uint32_t KB = d_xpow_hi[256];
    const int64_t a2 = (int64_t)t * c;
    uint32_t h = 0;
    for (int64_t i = a2; i < a2 + c; i++) h = dec_gfmul(h, KB) ^ (i < n ? (uint32_t)bcrc[i] : 0u);
    const uint32_t Mc = gf_pow16(KB, (uint64_t)c);  // one thread's span
    uint32_t x2 = h, mo = Mc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x2, o);
        if (lane >= o) x2 = dec_gfmul(y, mo) ^ x2;
        mo = dec_gfmul(mo, mo);  // Mc^(2o)
    }
    if (lane == 63) wcrc[wv] = x2;  // the wave's 64 c blocks
    __syncthreads();
    const uint32_t M64 = mo;  // Mc^64
    uint32_t pre = 0;
    for (int k = 0; k < wv; k++) pre = dec_gfmul(pre, M64) ^ wcrc[k];
    const uint32_t incl = dec_gfmul(pre, gf_pow16(Mc, (uint64_t)(lane + 1))) ^ x2;  // blocks [0, (t + 1) c)
    const uint32_t up = (uint32_t)__shfl_up((int)incl, 1);
    uint32_t rc = lane ? up : pre;  // blocks [0, t c)
    for (int64_t i = a2; i < a2 + c && i <= n; i++) {
        BP[i] = rc;
        if (i < n) rc = dec_gfmul(rc, KB) ^ bcrc[i];
    }
    if (a2 + c == n) BP[n] = rc;  // (n a multiple of c: no thread's range holds index n)
}

// placement: a block's kept positions to cpos[bbase ...]; a block whose candidates overflowed its scratch recomputes
// its flags (re-reads its 64 KB) and emits them directly.  CRC: pcrc[i] = CRC of the range's bytes before candidate i
template <bool CRC = false>
__global__ void __launch_bounds__(kSelThreads) k_sync_scatter(const uint8_t *blob, int64_t nbytes, const int64_t *soff,
                                                            int ns, int channels, int stream_bps, const int64_t *bbase,
                                                            int64_t *cpos, int64_t cap, const int32_t *bcount,
                                                            const int64_t *bpos, uint16_t *pcrc = nullptr,
                                                            const uint32_t *BP = nullptr,
                                                            const uint16_t *bipc = nullptr) {
    __shared__ int s_wsum[kSelThreads / 64];
    __shared__ typename std::conditional<CRC, SelCrcLds, char>::type cxs;
    SelCrcLds *cx = CRC ? reinterpret_cast<SelCrcLds *>(&cxs) : nullptr;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int tot = bcount[blockIdx.x];
    const int lead = (int)(reinterpret_cast<uintptr_t>(blob) & 15);
    const int64_t bq0 = (int64_t)blockIdx.x * kSelBytes;
    if (tot <= kSelBlkCap) {  // (block-uniform)
        const int64_t dst = bbase[blockIdx.x] + t;
        if (t < tot && dst < cap) {
            const int64_t src = (int64_t)blockIdx.x * kSelBlkCap + t;
            const int64_t p = bpos[src];
            cpos[dst] = p;
            if constexpr (CRC) pcrc[dst] = (uint16_t)(crc_xpow(BP[blockIdx.x], (uint32_t)(p + lead - bq0)) ^ bipc[src]);
        }
        return;
    }
    if constexpr (CRC) {
        sel_crc_load_tables(cx, t, kSelThreads);
        __syncthreads();
    }
    const int64_t qw = bq0 + (int64_t)(kSelBytes / 4) * wv;
    uint32_t m[kSelSteps];
    int c = sel_masks_co<kSelSteps, CRC>(blob, nbytes, soff, ns, channels, stream_bps, qw, lane, m, cx, wv, 0u);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) s_wsum[wv] = c;
    __syncthreads();
    int wbase = 0;
#pragma unroll
    for (int k = 0; k < kSelThreads / 64; k++) wbase += k < wv ? s_wsum[k] : 0;
    if constexpr (CRC) {
        if (t == 0) (void)sel_crc_block(cx);
        __syncthreads();
        const uint32_t pre = crc_xpow(BP[blockIdx.x], (uint32_t)(qw - bq0)) ^ cx->WP[wv];  // bytes before the wave
        sel_emit_co<kSelSteps, true>(m, qw, lane, lead, bbase[blockIdx.x] + wbase, cpos, cap, pcrc, cx, wv, blob - lead,
                                     pre);
    } else {
        sel_emit_co(m, qw, lane, lead, bbase[blockIdx.x] + wbase, cpos, cap);
    }
}

// Fused de-normalisation of decoded samples (converter.py:88-110 after pyflac + soundfile's PCM_16 WAV round
// trip, sonos-pyflac.txt:1629): v = float32(pcm16 / 32768); out = rint(((v + 1) / 2) * f32(max - min) + f32(min))
// in fp32 without contraction, cast to the raster dtype; float dtypes get v itself.
struct DecOut {
    void *out;         // nullptr: the decoders write int32 PCM
    const float2 *dn;  // per stream: (float32(data_max - data_min), float32(data_min))
    int dtype;         // enum frs_dtype of out
    int shift;         // 16 for 32-bit streams (libsndfile int -> short keeps the high half), else 0
};

__device__ inline void dn_store(const DecOut &o, int64_t i, int32_t pcm, float2 p) {
    const float v = (float)(pcm >> o.shift) * (1.0f / 32768.0f);
    if (o.dtype == FRS_DT_F32) { static_cast<float *>(o.out)[i] = v; return; }
    if (o.dtype == FRS_DT_F64) { static_cast<double *>(o.out)[i] = (double)v; return; }
    float a = __fadd_rn(v, 1.0f);
    a = __fdiv_rn(a, 2.0f);
    a = __fmul_rn(a, p.x);
    a = __fadd_rn(a, p.y);
    const int64_t r = (int64_t)rintf(a);
    switch (o.dtype) {
    case FRS_DT_U8: static_cast<uint8_t *>(o.out)[i] = (uint8_t)r; break;
    case FRS_DT_U16: static_cast<uint16_t *>(o.out)[i] = (uint16_t)r; break;
    case FRS_DT_I16: static_cast<int16_t *>(o.out)[i] = (int16_t)r; break;
    case FRS_DT_I32: static_cast<int32_t *>(o.out)[i] = (int32_t)r; break;
    default: static_cast<uint32_t *>(o.out)[i] = (uint32_t)r; break;
    }
}

// Span check for frames too large for the wave kernel's tables (max frame >= 1 MiB: many channels of
// 32-bit samples), one thread per candidate: the CRC-16 runs incrementally over the bytes from the
// candidate, compared at every later candidate start (and the stream end).  Same outputs as
// k_span_crc_wave: ends[i] = e or -1, nexti[i] = candidate index at e, -2 at the stream end.
__global__ void k_span_crc(const uint8_t *blob, const int64_t *soff, int ns, const int64_t *cpos, const int *ncand,
                           int cand_cap, int64_t max_frame, int64_t *ends, int32_t *nexti) {
    const int nc = *ncand;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (nc > cand_cap || i >= nc) return;
    const int64_t p = cpos[i];
    const int s = stream_of(soff, ns, p);
    const int64_t send = soff[s + 1];
    const int64_t lim = min(send, p + max_frame);
    uint32_t crc = 0;  // covers [p, b)
    int64_t b = p, result = -1;
    int32_t rnext = -1;
    for (int j = i + 1;; j++) {
        int64_t e = j < nc ? cpos[j] : send;
        if (e > send) e = send;
        if (e > lim) break;
        if (e >= p + 7) {
            for (; b < e - 2; b++) crc = ((crc << 8) & 0xFFFFu) ^ d_crc16[((crc >> 8) ^ blob[b]) & 0xFF];
            if (crc == (((uint32_t)blob[e - 2] << 8) | blob[e - 1])) {
                result = e;
                rnext = (j < nc && cpos[j] < send) ? j : -2;
                break;
            }
        }
        if (e >= send) break;
    }
    ends[i] = result;
    nexti[i] = rnext;
}


// Span check, one wave per candidate: the span [p, e) to the next candidate e (or the stream end) is
// staged in LDS and its CRC-16 computed by all 64 lanes (slice-by-4 per lane, lanes combined with
// x^(8m) factors); on a mismatch the next candidate is tried.  Spans longer than the LDS stage use the
// single-lane byte loop.  ends[i] = e or -1.
// dword k of the blob (bytes 4k..4k+3, little-endian), never touching bytes at or past `end`
__device__ inline uint32_t load_word_guarded(const uint8_t *blob, int64_t k, int64_t end) {
    const int64_t b = 4 * k;
    if (b + 4 <= end) return *reinterpret_cast<const uint32_t *>(blob + b);
    uint32_t v = 0;
    for (int j = 0; j < 4; j++)
        if (b + j < end) v |= (uint32_t)blob[b + j] << (8 * j);
    return v;
}

// words [wb, wb + nwords) of the blob (little-endian dwords, zero past `end`; byte-swapped when BSWAP) into an LDS
// stage by NT threads (tid < NT): eight unconditional dword loads per thread in flight per round (a guarded load per
// word compiled to a branch and a vmcnt(0) per word: one load in flight, ~10 us to stage an 8 KB frame on one wave).
// The caller guarantees 4 wb + 4 <= end (the fallback address of a word past the end).
template <int NT, bool BSWAP = false>
__device__ inline void stage_words(uint32_t *stage, const uint8_t *blob, int64_t wb, int64_t nwords, int64_t end,
                                   int tid) {
    for (int64_t k0 = 0; k0 < nwords; k0 += 8 * NT) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int64_t b = 4 * (wb + k0 + NT * u + tid);
            v[u] = *reinterpret_cast<const uint32_t *>(blob + (b + 4 <= end ? b : 4 * wb));
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int64_t k = k0 + NT * u + tid;
            if (k < nwords) {
                const uint32_t w = 4 * (wb + k) + 4 <= end ? v[u] : load_word_guarded(blob, wb + k, end);
                stage[k] = BSWAP ? __builtin_bswap32(w) : w;
            }
        }
    }
}
constexpr int kSpanWords = 6144;  // 24 KB stage

__global__ void __launch_bounds__(64) k_span_crc_wave(const uint8_t *blob, const int64_t *soff, int ns,
                                                     const int64_t *cpos, const int *ncand, int cand_cap,
                                                     int64_t max_frame, int64_t *ends, int32_t *nexti) {
    // launched before the host knows the candidate count (no mid-query sync): idle work-groups leave at once and
    // the rest stride over the candidates; an overflowing selection is reported by the host, not walked here
    const int nc = *ncand;
    if ((int)blockIdx.x >= nc || nc > cand_cap) return;
    __shared__ uint32_t stage[kSpanWords + 1];
    __shared__ __attribute__((aligned(16))) uint16_t t4[4][256];
    __shared__ __attribute__((aligned(16))) uint16_t xlo[256];
    const int lane = threadIdx.x;
    // tables from their global copies: independent 16-byte loads (deriving T_1..T_3 from T_0 here was three
    // dependent constant-memory lookups per entry at the start of every work-group)
    for (int k = lane; k < 128; k += 64) reinterpret_cast<uint4 *>(&t4[0][0])[k] = reinterpret_cast<const uint4 *>(&d_crc16x4[0][0])[k];
    for (int k = lane; k < 32; k += 64) reinterpret_cast<uint4 *>(xlo)[k] = reinterpret_cast<const uint4 *>(d_xpow_lo)[k];
    __syncthreads();
    for (int i = blockIdx.x; i < nc; i += gridDim.x) {
        const int64_t p = cpos[i];
        const int s = stream_of(soff, ns, p);
        const int64_t send = soff[s + 1];
        const int64_t lim = min(send, p + max_frame);
        int64_t result = -1;
        int32_t rnext = -1;  // candidate index at the span's end, -2 = the stream's end
        for (int j = i + 1;; j++) {
            int64_t e = (j < nc) ? cpos[j] : send;
            if (e > send) e = send;
            if (e > lim) break;
            if (e >= p + 7) {
                const int64_t wb = p >> 2, we = (e + 3) >> 2;  // aligned words covering [p, e)
                const int64_t nwords = we - wb;
                uint32_t crc = 0;
                if (nwords <= kSpanWords) {
                    stage_words<64>(stage, blob, wb, nwords, send, lane);  // (e >= p + 7: 4 wb + 4 <= send)
                    __builtin_amdgcn_s_waitcnt(0xC07F);
                    __builtin_amdgcn_wave_barrier();
                    const uint32_t nb = (uint32_t)(e - 2 - p);  // bytes covered by the CRC
                    const uint32_t off0 = (uint32_t)(p & 3);    // byte offset of p in stage
                    auto byte_at = [&](uint32_t b) -> uint32_t {  // b relative to p
                        const uint32_t a = b + off0;
                        return (stage[a >> 2] >> (8 * (a & 3))) & 0xFFu;
                    };
                    // bytes per lane: a multiple of 4 whose word count is odd (lane bases in distinct LDS banks)
                    uint32_t ch = ((nb + 63) / 64 + 3) & ~3u;
                    if (!((ch >> 2) & 1u)) ch += 4;
                    const uint32_t b0 = min(nb, (uint32_t)lane * ch), b1 = min(nb, b0 + ch);
                    uint32_t c = 0, b = b0;
                    for (; b + 4 <= b1; b += 4) {
                        const uint32_t a = b + off0;
                        const uint32_t lo = stage[a >> 2], hi = stage[(a >> 2) + 1];
                        const uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, a & 3);  // bytes b..b+3, LE
                        c = (uint32_t)t4[3][((c >> 8) ^ (w & 0xFF)) & 0xFF] ^ t4[2][((c & 0xFF) ^ ((w >> 8) & 0xFF)) & 0xFF] ^
                            t4[1][(w >> 16) & 0xFF] ^ t4[0][w >> 24];
                    }
                    for (; b < b1; b++) c = ((c << 8) & 0xFFFFu) ^ t4[0][((c >> 8) ^ byte_at(b)) & 0xFF];
                    const uint32_t m = nb - b1;  // bytes after this lane's chunk
                    c = dec_gfmul(dec_gfmul(c, xlo[m & 255]), d_xpow_hi[m >> 8]);
    #pragma unroll
                    for (int o = 32; o > 0; o >>= 1) c ^= __shfl_xor(c, o);
                    crc = c;
                    const uint32_t got = (byte_at(nb) << 8) | byte_at(nb + 1);
                    __builtin_amdgcn_wave_barrier();
                    if (crc == got) {
                        result = e;
                        rnext = (j < nc && cpos[j] < send) ? j : -2;
                        break;
                    }
                } else {  // rare: a span longer than the stage
                    uint32_t c = 0;
                    for (int64_t b = p; b < e - 2; b++) c = ((c << 8) & 0xFFFFu) ^ d_crc16[((c >> 8) ^ blob[b]) & 0xFF];
                    const uint32_t got = ((uint32_t)blob[e - 2] << 8) | blob[e - 1];
                    if (c == got) {
                        result = e;
                        rnext = (j < nc && cpos[j] < send) ? j : -2;
                        break;
                    }
                }
            }
            if (e >= send) break;
        }
        if (lane == 0) {
            ends[i] = result;
            nexti[i] = rnext;
        }
    }
}

// Span check for batched decodes, one lane per candidate (the wave form above spends a work-group's LDS stage per
// candidate and runs at ~1.5 waves per SIMD): the lane folds the bytes from its candidate into a CRC-16 with
// aligned loads and compares it at every later candidate start (and the stream end).  Same outputs as
// k_span_crc_wave.  The fold is a dependency chain through LDS table lookups; slice-by-16 (16 tables, 8 KB of LDS,
// derived in the work-group from the slice-by-4 ones) puts only two of a 16-byte step's lookups on that chain
// instead of two of every 4 bytes' (slice-by-4: the span check was 1.27 ms of the 7.4 ms batched C4 decode).
__global__ void __launch_bounds__(256) k_span_crc_lane(const uint8_t *blob, const int64_t *soff, int ns,
                                                      const int64_t *cpos, const int *ncand, int cand_cap,
                                                      int64_t max_frame, int64_t *ends, int32_t *nexti) {
    __shared__ __attribute__((aligned(16))) uint16_t t4[16][256];  // t4[k][x]: byte x followed by k zero bytes
    for (int k = threadIdx.x; k < 128; k += blockDim.x)
        reinterpret_cast<uint4 *>(&t4[0][0])[k] = reinterpret_cast<const uint4 *>(&d_crc16x4[0][0])[k];
    __syncthreads();
    for (int k = 4; k < 16; k++) {  // t[k][x] = t[k-1][x] advanced by one zero byte
        for (int x = threadIdx.x; x < 256; x += blockDim.x) {
            const uint32_t v = t4[k - 1][x];
            t4[k][x] = (uint16_t)(((v << 8) & 0xFFFFu) ^ t4[0][v >> 8]);
        }
        __syncthreads();
    }
    const int nc = *ncand;
    if (nc > cand_cap) return;
    const int64_t lead = (int64_t)(reinterpret_cast<uintptr_t>(blob) & 15);
    const uint8_t *abase = blob - lead;  // 16-byte aligned view: blob[b] = abase[b + lead]
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nc; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = cpos[i];
    const int s = stream_of(soff, ns, p);
    const int64_t send = soff[s + 1];
    const int64_t lim = min(send, p + max_frame);
    uint32_t crc = 0;  // CRC-16 of [p, b)
    int64_t b = p, result = -1;
    int32_t rnext = -1;
    for (int64_t j = i + 1;; j++) {
        int64_t e = j < nc ? cpos[j] : send;
        if (e > send) e = send;
        if (e > lim) break;
        if (e >= p + 7) {
            const int64_t stop = e - 2;
            auto fold4 = [&](uint32_t w) {  // bytes of w (little-endian) in order
                crc = (uint32_t)t4[3][((crc >> 8) ^ (w & 0xFF)) & 0xFF] ^ t4[2][((crc & 0xFF) ^ ((w >> 8) & 0xFF)) & 0xFF] ^
                      t4[1][(w >> 16) & 0xFF] ^ t4[0][w >> 24];
            };
            for (; b < stop && ((b + lead) & 3); b++) crc = ((crc << 8) & 0xFFFFu) ^ t4[0][((crc >> 8) ^ blob[b]) & 0xFF];
            for (; b + 4 <= stop && ((b + lead) & 15); b += 4) fold4(*reinterpret_cast<const uint32_t *>(abase + b + lead));
            // whole 128-byte lines, all eight 16-byte loads issued together: a lane streams its own span, and with
            // one 16-byte load per step the ~1500 concurrent streams of a CU evicted each line from L2 between its
            // eight visits (PMC: 7x the span bytes fetched)
            auto fold16 = [&](const uint4 &v) {  // 16 bytes (little-endian dwords) in order: slice-by-16
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                uint32_t r = (uint32_t)t4[15][((crc >> 8) ^ (w[0] & 0xFF)) & 0xFF] ^
                             t4[14][((crc & 0xFF) ^ ((w[0] >> 8) & 0xFF)) & 0xFF];
                r ^= (uint32_t)t4[13][(w[0] >> 16) & 0xFF] ^ t4[12][w[0] >> 24];
#pragma unroll
                for (int q = 1; q < 4; q++)
                    r ^= (uint32_t)t4[15 - 4 * q][w[q] & 0xFF] ^ t4[14 - 4 * q][(w[q] >> 8) & 0xFF] ^
                         t4[13 - 4 * q][(w[q] >> 16) & 0xFF] ^ t4[12 - 4 * q][w[q] >> 24];
                crc = r;
            };
            for (; b + 128 <= stop && ((b + lead) & 127); b += 16) fold16(*reinterpret_cast<const uint4 *>(abase + b + lead));
            for (; b + 128 <= stop; b += 128) {
                uint4 v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = *reinterpret_cast<const uint4 *>(abase + b + lead + 16 * u);
#pragma unroll
                for (int u = 0; u < 8; u++) fold16(v[u]);
            }
            for (; b + 16 <= stop; b += 16) fold16(*reinterpret_cast<const uint4 *>(abase + b + lead));
            for (; b + 4 <= stop; b += 4) fold4(*reinterpret_cast<const uint32_t *>(abase + b + lead));
            for (; b < stop; b++) crc = ((crc << 8) & 0xFFFFu) ^ t4[0][((crc >> 8) ^ blob[b]) & 0xFF];
            if (crc == (((uint32_t)blob[e - 2] << 8) | blob[e - 1])) {
                result = e;
                rnext = (j < nc && cpos[j] < send) ? (int32_t)j : -2;
                break;
            }
        }
        if (e >= send) break;
    }
    ends[i] = result;
    nexti[i] = rnext;
    }
}

// Span check from the selection's prefix CRCs (two-pass form), one lane per candidate: the first later candidate e
// (or the stream end) with pc(e) == pc(p) x^(8(e - p)), i.e. the span's CRC-16 footer verifies -- the same candidates
// tried in the same order as k_span_crc_lane, without reading a byte.  The stream end's prefix comes from its block's
// prefix and the in-block value the count pass left (sbib).
__global__ void __launch_bounds__(256) k_span_pcrc(const int64_t *soff, int ns, const int64_t *cpos, const int *ncand,
                                                  int cand_cap, int64_t max_frame, const uint16_t *pcrc,
                                                  const uint32_t *BP, const uint16_t *sbib, int lead, int64_t *ends,
                                                  int32_t *nexti) {
    const int nc = *ncand;
    if (nc > cand_cap) return;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nc; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = cpos[i];
        const int s = stream_of(soff, ns, p);
        const int64_t send = soff[s + 1];
        const int64_t lim = min(send, p + max_frame);
        const uint32_t pp = pcrc[i];
        int64_t result = -1;
        int32_t rnext = -1;
        for (int64_t j = i + 1;; j++) {
            const int64_t cj = j < nc ? cpos[j] : send;
            const int64_t e = cj > send ? send : cj;
            if (e > lim) break;
            if (e >= p + 7) {
                uint32_t pe;
                if (j < nc && cj == e) {
                    pe = pcrc[j];
                } else {  // the stream end
                    const int64_t q = send + lead;
                    const int64_t off = q & (kSelBytes - 1);
                    pe = crc_xpow(BP[q / kSelBytes], (uint32_t)off) ^ (off ? (uint32_t)sbib[s + 1] : 0u);
                }
                if (pe == crc_xpow(pp, (uint32_t)(e - p))) {
                    result = e;
                    rnext = (j < nc && cpos[j] < send) ? (int32_t)j : -2;
                    break;
                }
            }
            if (e >= send) break;
        }
        ends[i] = result;
        nexti[i] = rnext;
    }
}

// Frame chain of each stream from its first byte: one work-group per stream loads the stream's candidate ->
// next-candidate links (the span kernels' nexti) into LDS and lane 0 walks them, one LDS read per frame (streams
// with more candidates than the LDS table walk global memory).  frame_cand[fbase[s] + k] = candidate of frame k,
// written only once that candidate's CRC span is verified (its link is not -1); frames the walk does not reach
// get -1 and are skipped by the decoders; any break is counted in *bad.
constexpr int kChainLds = 4096;
__device__ inline int lower_bound_pos(const int64_t *cpos, int n, int64_t p) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cpos[mid] < p) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__global__ void __launch_bounds__(1024) k_chain_lds(const int64_t *soff, int ns, const int64_t *cpos, const int *ncand,
                                                   int cand_cap,
                                                   const int32_t *nexti, const int64_t *fbase, int64_t *frame_cand,
                                                   int *bad) {
    __shared__ int32_t nx[kChainLds];
    __shared__ int32_t rng[2];
    __shared__ int32_t wcnt[16];
    __shared__ int32_t sbad;
    const int s = blockIdx.x;
    if (s >= ns) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nt = blockDim.x, nw = nt >> 6;
    const int nc = *ncand;
    const int64_t fb = fbase[s], nf = fbase[s + 1] - fb;
    if (nc > cand_cap) {  // uniform: the selection overflowed its buffer (the host reports it)
        for (int64_t k = tid; k < nf; k += nt) frame_cand[fb + k] = -1;
        if (tid == 0) atomicAdd(bad, 1);
        return;
    }
    if (tid < 64) {  // the stream's candidate range: wave 0 narrows both bounds 64 ways per step (3 dependent loads for
                     // 390 K candidates instead of 2 x 19 of a one-lane binary search)
        for (int e = 0; e < 2; e++) {
            const int64_t key = soff[s + e];
            int lo = 0, hi = nc;  // first index with cpos >= key lies in [lo, hi]
            if (ns == 1) {
                lo = hi = e ? nc : 0;
            }
            while (hi - lo > 64) {
                const int64_t span = hi - lo;
                const int piv = lo + (int)(span * (tid + 1) / 65);  // 64 pivots inside (lo, hi)
                const uint64_t below = __ballot(cpos[piv] < key);  // pivots with cpos < key: a prefix of the lanes
                const int nb = __popcll(below);
                const int nlo = nb ? lo + (int)(span * nb / 65) + 1 : lo;
                const int nhi = nb < 64 ? lo + (int)(span * (nb + 1) / 65) : hi;
                lo = nlo;
                hi = nhi;
            }
            const int i = lo + tid;
            const uint64_t below = __ballot(i < hi && cpos[i] < key);
            if (tid == 0) rng[e] = lo + __popcll(below);
        }
        if (tid == 0) sbad = 0;
    }
    __syncthreads();
    const int c0 = rng[0], c1 = rng[1];
    const bool in_lds = c1 - c0 <= kChainLds;
    if (c0 < c1 && cpos[c0] == soff[s] && nf > 0) {
        // a walk is one dependent load per frame (a long stream: tens of thousands of global loads; a C5 tile: 64
        // dependent LDS reads by one lane, ~10 us).  Optimistic parallel ranking instead: the verified candidates
        // (link != -1) in position order ARE the chain when there are nf of them, each links to the next and the last
        // to the stream end -- checked below; anything else (a false sync with a verified span) falls back to the
        // exact walk.  All of the work-group's waves rank (one wave per stream of a batched decode, 16 for the one
        // long stream of a plain multi-band convert).
        int64_t cnt = 0;
        for (int i0 = c0; i0 < c1; i0 += nt) {
            const int i = i0 + tid;
            const int32_t v = i < c1 ? nexti[i] : -1;
            const uint64_t m = __ballot(v != -1);
            if (lane == 0) wcnt[wv] = __popcll(m);
            __syncthreads();
            int64_t before = cnt, tot = 0;
            for (int k = 0; k < nw; k++) {
                before += k < wv ? wcnt[k] : 0;
                tot += wcnt[k];
            }
            const int64_t r = before + __popcll(m & ((1ull << lane) - 1ull));
            if (v != -1 && r < nf) frame_cand[fb + r] = i;
            cnt += tot;
            __syncthreads();  // wcnt reused
        }
        bool good = cnt == nf;
        if (good) {
            __threadfence();
            __syncthreads();
            bool bad_link = false;
            for (int64_t k = tid; k < nf; k += nt) {
                const int64_t ci = frame_cand[fb + k];
                const int32_t want = k + 1 < nf ? (int32_t)frame_cand[fb + k + 1] : -2;
                bad_link |= nexti[ci] != want || (k == 0 && ci != c0);  // frame 0 is the stream's first byte
            }
            if (bad_link) sbad = 1;
            __syncthreads();
            good = sbad == 0;
        }
        if (good) return;
        __threadfence();
    }
    if (in_lds)
        for (int k = tid; k < c1 - c0; k += nt) nx[k] = nexti[c0 + k];
    __syncthreads();
    if (tid != 0) return;
    bool ok = c0 < c1 && cpos[c0] == soff[s];
    int64_t k = 0;
    int idx = c0;
    if (ok) {
        for (; k < nf; k++) {
            const int n = in_lds ? nx[idx - c0] : nexti[idx];
            if (n == -1) {  // frame k failed its CRC span: not handed to the decoders
                ok = false;
                break;
            }
            frame_cand[fb + k] = idx;
            if (k + 1 < nf) {
                if (n < 0) {  // the stream ends before its last frame
                    ok = false;
                    k++;
                    break;
                }
                idx = n;
            } else if (n != -2) {
                ok = false;  // bytes after the last frame
            }
        }
    }
    for (; k < nf; k++) frame_cand[fb + k] = -1;
    if (!ok) atomicAdd(bad, 1);
}

constexpr int kDecResMax = 4096;  // residual buffer (LDS) of the fast subframe path

// MSB-first bit reader over global bytes (bounded)
struct BitReader {
    const uint8_t *base;
    int64_t pos_bits;
    int64_t end_bits;
    uint64_t cache;   // left-aligned
    int avail;
    bool err;
    __device__ void init(const uint8_t *b, int64_t start_byte, int64_t end_byte) {
        base = b;
        pos_bits = start_byte * 8;
        end_bits = end_byte * 8;
        cache = 0;
        avail = 0;
        err = false;
    }
    // reposition at an arbitrary bit (the cache invariant wants byte-aligned loads)
    __device__ inline void seek_bits(int64_t p) {
        pos_bits = (p >> 3) << 3;
        cache = 0;
        avail = 0;
        if (p & 7) bits((int)(p & 7));
    }
    __device__ inline void refill() {
        while (avail <= 32) {
            const int64_t byte = (pos_bits + avail) >> 3;  // next byte not yet in the cache (avail % 8 == 0)
            const int64_t endb = end_bits >> 3;
            if (byte + 8 <= endb) {
                // 4 bytes via the two aligned dwords around them (no per-byte loads)
                const uint32_t *w = reinterpret_cast<const uint32_t *>(base + (byte & ~(int64_t)3));
                const uint32_t v = __builtin_bswap32(__builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(byte & 3)));
                cache |= (uint64_t)v << (32 - avail);
                avail += 32;
            } else {
                uint64_t b = 0;
                if (byte < endb) b = base[byte];
                else if (byte >= endb + 8) {
                    err = true;
                    return;
                }
                cache |= b << (56 - avail);
                avail += 8;
            }
        }
    }
    __device__ inline uint32_t bits(int n) {  // n <= 32
        if (n == 0) return 0;
        if (avail < n) refill();
        const uint32_t v = (uint32_t)(cache >> (64 - n));
        cache <<= n;
        avail -= n;
        pos_bits += n;
        return v;
    }
    __device__ inline int32_t sbits(int n) {
        if (n == 0) return 0;
        uint32_t v = bits(n);
        if (n < 32 && (v >> (n - 1))) v |= ~0u << n;
        return (int32_t)v;
    }
    __device__ inline uint32_t unary() {  // count zeros before the next 1
        uint32_t q = 0;
        for (;;) {
            if (avail < 32) refill();
            if (err) return q;
            if (cache) {
                const int z = __builtin_clzll(cache);
                if (z < avail) {
                    q += z;
                    cache = (z + 1 >= 64) ? 0 : (cache << (z + 1));  // a 64-bit shift by 64 is a no-op on gfx950
                    avail -= z + 1;
                    pos_bits += z + 1;
                    return q;
                }
            }
            q += avail;
            pos_bits += avail;
            cache = 0;
            avail = 0;
            if (pos_bits > end_bits + 64) {
                err = true;
                return q;
            }
        }
    }
};

// Rice codes of one partition straight from the LDS stage (words w, MSB-first after a byte swap): a 64-bit
// cache refilled 32 bits at a time from a word fetched one refill ahead.  pos_bits (relative to w) is
// advanced; false if the codes run past max_bits.
__device__ __attribute__((always_inline)) inline bool rice_run_lds(const uint32_t *w, int64_t &pos_bits,
                                                                   int64_t max_bits, int ns, int k, int32_t *out) {
    uint32_t wi = (uint32_t)(pos_bits >> 5);
    const int off = (int)(pos_bits & 31);
    uint64_t c = ((((uint64_t)__builtin_bswap32(w[wi])) << 32) | __builtin_bswap32(w[wi + 1])) << off;
    int n = 64 - off;
    wi += 2;
    uint32_t nw = __builtin_bswap32(w[wi]);
    const uint32_t wmax = (uint32_t)((max_bits + 31) >> 5) + 2;
    for (int j = 0; j < ns; j++) {
        if (n < 32) {
            c |= (uint64_t)nw << (32 - n);
            n += 32;
            nw = __builtin_bswap32(w[++wi]);
        }
        uint32_t q;
        const int z = c ? __builtin_clzll(c) : 64;
        if (z < 32) {
            q = (uint32_t)z;
            c <<= z + 1;
            n -= z + 1;
        } else {  // long unary run
            q = 0;
            while (true) {
                const int zz = c ? __builtin_clzll(c) : 64;
                if (zz < n) {
                    q += (uint32_t)zz;
                    c = (zz + 1 >= 64) ? 0 : (c << (zz + 1));
                    n -= zz + 1;
                    break;
                }
                q += (uint32_t)n;
                c = (uint64_t)nw << 32;
                n = 32;
                nw = __builtin_bswap32(w[++wi]);
                if (wi > wmax) return false;
            }
        }
        if (n < 32) {
            c |= (uint64_t)nw << (32 - n);
            n += 32;
            nw = __builtin_bswap32(w[++wi]);
        }
        const uint32_t low = k ? (uint32_t)(c >> (64 - k)) : 0u;
        c <<= k;
        n -= k;
        const uint32_t u = (q << k) | low;
        out[j] = (int32_t)((u >> 1) ^ (uint32_t)(-(int32_t)(u & 1)));
        if (wi > wmax) return false;
    }
    pos_bits = (int64_t)wi * 32 - n;
    return pos_bits <= max_bits;
}

__device__ __attribute__((always_inline)) inline void decode_one_frame(const uint8_t *blob, const uint8_t *bits_base, int64_t bits_shift,
                                        const int64_t *soff, int ns, const int64_t *poff, const int64_t *cpos,
                                        const int64_t *ends, const int64_t *fbase, const int64_t *frame_cand,
                                        int64_t fi, int channels, int stream_bps, int32_t *pcm, int blocksize,
                                        int *nvalid, int32_t *resbuf, const uint32_t *lds_words,
                                        int32_t *outb_override = nullptr) {
    const int64_t ci = frame_cand[fi];
    if (ci < 0) return;  // not on a valid chain (the host reports it)
    const int64_t fpos = cpos[ci];
    const int64_t fend_known = ends[ci];
    if (fend_known < 0) return;  // no verified CRC span
    const int s = stream_of(soff, ns, fpos);
    const int64_t send = soff[s + 1];
    const FrameHdr cd = parse_header(blob, fpos, send, channels, stream_bps);
    const int64_t nsamp = poff[s + 1] - poff[s];
    const int64_t kk = fi - fbase[s];
    const int64_t first = kk * blocksize;
    if (!cd.ok || cd.frame_no != kk || cd.bs > blocksize || first + cd.bs > nsamp) return;
    // frame-local output (an LDS buffer of the fused decode) or the frame's place in the PCM array
    int32_t *outb = outb_override ? outb_override : pcm + (poff[s] + first) * channels;
    BitReader br;  // bits_base[k] = blob[k + bits_shift] (LDS stage or the blob itself)
    br.init(bits_base, fpos + cd.hdr_len - bits_shift, fend_known - bits_shift);
    const int nch = channels;
    bool combined = false;  // mid/side already undone while the 33-bit side was decoded
    // decode subframes straight into the output (interleaved), then verify the CRC
    for (int c = 0; c < nch; c++) {
        int sbps = cd.bps;
        const bool side = (cd.chass == 8 && c == 1) || (cd.chass == 9 && c == 0) || (cd.chass == 10 && c == 1);
        if (side) sbps++;
        br.bits(1);
        const int t = (int)br.bits(6);
        int w = 0;
        if (br.bits(1)) w = (int)br.unary() + 1;
        sbps -= w;
        if (br.err || sbps <= 0 || sbps > 33) return;
        int32_t *x = outb + c;
        const int bs = cd.bs;
        if (side && cd.bps == 32) {
            // The 33-bit side signal of a 32-bit stereo stream: an exact int64 walk (history ring of the last 32
            // samples).  Left-/right-side keep its low 32 bits (the other channel is L - S / R + S mod 2^32);
            // mid-side needs all 33, so L and R are formed here and the post-pass skips the frame.
            int64_t hist[32];
            auto rd = [&](int nb) -> int64_t {  // signed field of nb <= 33 bits
                if (nb <= 32) return (int64_t)br.sbits(nb);
                const uint64_t hi = br.bits(nb - 32), lo = br.bits(32);
                const uint64_t v = (hi << 32) | lo;
                return (int64_t)(v << (64 - nb)) >> (64 - nb);
            };
            auto put = [&](int i, int64_t v) {
                hist[i & 31] = v;
                const int64_t sd = (int64_t)((uint64_t)v << w);
                int32_t *pr = outb + (int64_t)i * nch;
                if (cd.chass == 10) {
                    const int64_t mid = (int64_t)((uint64_t)(int64_t)pr[0] << 1) | (sd & 1);
                    pr[0] = (int32_t)((mid + sd) >> 1);
                    pr[1] = (int32_t)((mid - sd) >> 1);
                } else {
                    x[(int64_t)i * nch] = (int32_t)sd;
                }
            };
            if (t == 0) {
                const int64_t v = rd(sbps);
                for (int i = 0; i < bs; i++) put(i, v);
            } else if (t == 1) {
                for (int i = 0; i < bs; i++) put(i, rd(sbps));
            } else if ((t >= 8 && t <= 12) || t >= 32) {
                const bool lpc = t >= 32;
                const int o = lpc ? t - 31 : t - 8;
                if (o > bs) return;
                int32_t q[32];
                int shift = 0;
                for (int i = 0; i < o; i++) put(i, rd(sbps));
                if (lpc) {
                    const int prec = (int)br.bits(4) + 1;
                    if (prec == 16) return;
                    shift = br.sbits(5);
                    if (shift < 0) return;
                    for (int i = 0; i < o; i++) q[i] = br.sbits(prec);
                }
                const int method = (int)br.bits(2);
                if (method > 1) return;
                const int po = (int)br.bits(4);
                const int pb = method == 0 ? 4 : 5, esc = (1 << pb) - 1;
                if ((bs >> po) < o || (bs & ((1 << po) - 1))) return;
                int i = o;
                for (int p = 0; p < (1 << po); p++) {
                    const int ns = (bs >> po) - (p == 0 ? o : 0);
                    const int kp = (int)br.bits(pb);
                    const int nb = kp == esc ? (int)br.bits(5) : 0;
                    for (int j = 0; j < ns; j++, i++) {
                        int64_t r;
                        if (kp == esc) r = nb ? (int64_t)br.sbits(nb) : 0;
                        else {
                            const uint32_t qq = br.unary();
                            const uint32_t u = (qq << kp) | br.bits(kp);
                            r = (int32_t)((u >> 1) ^ (uint32_t)(-(int32_t)(u & 1)));
                        }
                        int64_t pred = 0;
                        if (lpc) {
                            for (int m = 0; m < o; m++) pred += (int64_t)q[m] * hist[(i - 1 - m) & 31];
                            pred >>= shift;
                        } else {
                            const int64_t a = o > 0 ? hist[(i - 1) & 31] : 0, b = o > 1 ? hist[(i - 2) & 31] : 0,
                                          d = o > 2 ? hist[(i - 3) & 31] : 0, e = o > 3 ? hist[(i - 4) & 31] : 0;
                            pred = o == 1 ? a : o == 2 ? 2 * a - b : o == 3 ? 3 * a - 3 * b + d
                                 : o == 4 ? 4 * a - 6 * b + 4 * d - e : 0;
                        }
                        put(i, r + pred);
                        if (br.err) return;
                    }
                }
            } else {
                return;
            }
            if (cd.chass == 10) combined = true;
            continue;
        }
        if (t == 0) {
            const int32_t v = br.sbits(sbps);
            for (int i = 0; i < bs; i++) x[(int64_t)i * nch] = v;
        } else if (t == 1) {
            for (int i = 0; i < bs; i++) x[(int64_t)i * nch] = br.sbits(sbps);
        } else if ((t >= 8 && t <= 12) || t >= 32) {
            const bool lpc = t >= 32;
            const int o = lpc ? t - 31 : t - 8;
            if (o > bs) return;
            int32_t q[32];
            int shift = 0;
            int prec_lpc = 0;
            for (int i = 0; i < o; i++) x[(int64_t)i * nch] = br.sbits(sbps);
            if (lpc) {
                const int prec = (int)br.bits(4) + 1;
                prec_lpc = prec;
                if (prec == 16) return;
                shift = br.sbits(5);
                if (shift < 0) return;
                for (int i = 0; i < o; i++) q[i] = br.sbits(prec);
            }
            const int method = (int)br.bits(2);
            if (method > 1) return;
            const int po = (int)br.bits(4);
            const int pb = method == 0 ? 4 : 5, esc = (1 << pb) - 1;
            if ((bs >> po) < o || (bs & ((1 << po) - 1))) return;
            int i = o;
            int lg = 0;
            while ((1 << lg) < o) lg++;
            const bool safe32 = (lpc ? prec_lpc : 3) + sbps + lg <= 31;  // the 32-bit prediction cannot wrap
            // libFLAC's level-5 precision makes prec + 16 + log2(order) = 32 for every 16-bit LPC order >= 2, so the
            // 32-bit sum may wrap in principle; a wrapped sum moves the sample by a multiple of 2^(32 - shift),
            // which for sbps + shift <= 31 leaves the sbps range -- the restore checks every sample and redoes the
            // subframe on the exact 64-bit path if one is out (never on a stream libFLAC decodes in 32 bits)
            const bool wrap_checked = !safe32 && sbps <= 17 && sbps + shift <= 31;
            const bool narrow = sbps <= 23 && (safe32 || wrap_checked);
            bool done = false;
            if (resbuf && narrow && bs <= kDecResMax) {
                const auto br0 = br;
                // ---- phase 1: every residual of the subframe into LDS (tight Rice loop: refill only when
                //      fewer than 32 bits are cached, long unary runs via the generic reader)
                for (int p = 0; p < (1 << po); p++) {
                    const int ns = (bs >> po) - (p == 0 ? o : 0);
                    const int kp = (int)br.bits(pb);
                    if (kp == esc) {
                        const int nb = (int)br.bits(5);
                        for (int j = 0; j < ns; j++) resbuf[i++] = nb ? br.sbits(nb) : 0;
                    } else if (lds_words) {
                        int64_t pbits = br.pos_bits;
                        if (!rice_run_lds(lds_words, pbits, br.end_bits, ns, kp, resbuf + i)) return;
                        i += ns;
                        br.seek_bits(pbits);
                    } else {
                        for (int j = 0; j < ns; j++) {
                            if (br.avail < 32) br.refill();
                            const uint64_t c = br.cache;
                            const int z = c ? __builtin_clzll(c) : 64;
                            uint32_t qq;
                            if (z < br.avail) {
                                qq = (uint32_t)z;
                                br.cache = c << (z + 1);
                                br.avail -= z + 1;
                                br.pos_bits += z + 1;
                            } else {
                                qq = br.unary();
                            }
                            uint32_t low = 0;
                            if (kp) {
                                if (br.avail < kp) br.refill();
                                low = (uint32_t)(br.cache >> (64 - kp));
                                br.cache <<= kp;
                                br.avail -= kp;
                                br.pos_bits += kp;
                            }
                            const uint32_t u = (qq << kp) | low;
                            resbuf[i++] = (int32_t)((u >> 1) ^ (uint32_t)(-(int32_t)(u & 1)));
                        }
                    }
                    if (br.err) return;
                }
                // ---- phase 2: reconstruction with an 8-register ring R[k] = x[i0 - 8 + k]; the taps on older
                //      samples are summed first so only the newest tap is on the critical path
                int32_t cq[8], R[8];
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    int32_t cm = 0;
                    if (lpc) cm = m < o ? q[m] : 0;
                    else if (o == 1) cm = m == 0 ? 1 : 0;
                    else if (o == 2) cm = m == 0 ? 2 : m == 1 ? -1 : 0;
                    else if (o == 3) cm = m == 0 ? 3 : m == 1 ? -3 : m == 2 ? 1 : 0;
                    else if (o == 4) cm = m == 0 ? 4 : m == 1 ? -6 : m == 2 ? 4 : m == 3 ? -1 : 0;
                    cq[m] = cm;
                    const int src = o - 8 + m;
                    R[m] = src >= 0 ? x[(int64_t)src * nch] : 0;
                }
                // keep the ring, taps and output cursor in VGPRs (vector ALU; the scalar unit would spill)
                int32_t vshift = shift;
                int32_t *xo = x;
                const int32_t xlo = -(1 << (sbps - 1)), xhi = (1 << (sbps - 1)) - 1;
                uint32_t oor = 0;
#pragma unroll
                for (int m = 0; m < 8; m++) asm volatile("" : "+v"(cq[m]), "+v"(R[m]));
                asm volatile("" : "+v"(vshift));
                for (int i0 = o; i0 < bs; i0 += 8) {
                    int32_t rr[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) rr[u] = (i0 + u < bs) ? resbuf[i0 + u] : 0;
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        if (i0 + u < bs) {
                            int32_t older = 0;
#pragma unroll
                            for (int m = 1; m < 8; m++) older += __mul24(cq[m], R[(u - 1 - m + 16) & 7]);
                            const int32_t pred = older + __mul24(cq[0], R[(u - 1 + 8) & 7]);
                            const int32_t v = rr[u] + (pred >> vshift);
                            oor |= (uint32_t)(v < xlo) | (uint32_t)(v > xhi);
                            xo[(int64_t)(i0 + u) * nch] = v;
                            R[u] = v;
                        }
                    }
                }
                i = bs;
                done = !(wrap_checked && oor);
                if (!done) {  // a wrapped prediction: the subframe's residual bits again, exactly
                    br = br0;
                    i = o;
                }
            }
            if (done) {
            } else if (o <= 8) {
                // history in registers: h[m] = x[i-1-m]; coefficient m = 0 for m >= o (branch-free taps)
                int32_t cq[8];
                int32_t h[8];
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    int32_t cm = 0;
                    if (lpc) cm = m < o ? q[m] : 0;
                    else if (o == 1) cm = m == 0 ? 1 : 0;
                    else if (o == 2) cm = m == 0 ? 2 : m == 1 ? -1 : 0;
                    else if (o == 3) cm = m == 0 ? 3 : m == 1 ? -3 : m == 2 ? 1 : 0;
                    else if (o == 4) cm = m == 0 ? 4 : m == 1 ? -6 : m == 2 ? 4 : m == 3 ? -1 : 0;
                    cq[m] = cm;
                    h[m] = m < o ? x[(int64_t)(o - 1 - m) * nch] : 0;
                }
                for (int p = 0; p < (1 << po); p++) {
                    const int ns = (bs >> po) - (p == 0 ? o : 0);
                    const int kp = (int)br.bits(pb);
                    int nb = 0;
                    if (kp == esc) nb = (int)br.bits(5);
                    for (int j = 0; j < ns; j++, i++) {
                        int32_t r;
                        if (kp == esc) r = nb ? br.sbits(nb) : 0;
                        else {
                            const uint32_t qq = br.unary();
                            const uint32_t u = (qq << kp) | br.bits(kp);
                            r = (int32_t)((u >> 1) ^ (uint32_t)(-(int32_t)(u & 1)));
                        }
                        int64_t pred = 0;
#pragma unroll
                        for (int m = 0; m < 8; m++) pred += (int64_t)cq[m] * h[m];
                        pred >>= shift;
                        const int32_t v = (int32_t)(r + pred);
                        x[(int64_t)i * nch] = v;
#pragma unroll
                        for (int m = 7; m > 0; m--) h[m] = h[m - 1];
                        h[0] = v;
                    }
                    if (br.err) return;
                }
            } else
            for (int p = 0; p < (1 << po); p++) {
                const int ns = (bs >> po) - (p == 0 ? o : 0);
                const int kp = (int)br.bits(pb);
                int nb = 0;
                if (kp == esc) nb = (int)br.bits(5);
                for (int j = 0; j < ns; j++, i++) {
                    int32_t r;
                    if (kp == esc) r = nb ? br.sbits(nb) : 0;
                    else {
                        const uint32_t qq = br.unary();
                        const uint32_t u = (qq << kp) | br.bits(kp);
                        r = (int32_t)((u >> 1) ^ (uint32_t)(-(int32_t)(u & 1)));
                    }
                    int64_t pred = 0;
                    if (lpc) {
                        for (int m = 0; m < o; m++) pred += (int64_t)q[m] * x[(int64_t)(i - 1 - m) * nch];
                        pred >>= shift;
                    } else {
                        switch (o) {
                        case 0: pred = 0; break;
                        case 1: pred = x[(int64_t)(i - 1) * nch]; break;
                        case 2: pred = 2 * (int64_t)x[(int64_t)(i - 1) * nch] - x[(int64_t)(i - 2) * nch]; break;
                        case 3: pred = 3 * (int64_t)x[(int64_t)(i - 1) * nch] - 3 * (int64_t)x[(int64_t)(i - 2) * nch] + x[(int64_t)(i - 3) * nch]; break;
                        default: pred = 4 * (int64_t)x[(int64_t)(i - 1) * nch] - 6 * (int64_t)x[(int64_t)(i - 2) * nch] + 4 * (int64_t)x[(int64_t)(i - 3) * nch] - x[(int64_t)(i - 4) * nch]; break;
                        }
                    }
                    x[(int64_t)i * nch] = (int32_t)(r + pred);
                    if (br.err) return;
                }
            }
        } else {
            return;
        }
        if (w)
            for (int i = 0; i < bs; i++) x[(int64_t)i * nch] = (int32_t)((uint32_t)x[(int64_t)i * nch] << w);
    }
    if (cd.chass >= 8 && !combined) {
        for (int i = 0; i < cd.bs; i++) {
            int32_t *pr = outb + (int64_t)i * nch;
            const int64_t a = pr[0], sd = pr[1];
            if (cd.chass == 8) pr[1] = (int32_t)(a - sd);
            else if (cd.chass == 9) pr[0] = (int32_t)(a + sd);
            else {
                const int64_t mid = (a * 2) | (sd & 1);
                pr[0] = (int32_t)((mid + sd) >> 1);
                pr[1] = (int32_t)((mid - sd) >> 1);
            }
        }
    }
    // the decoded subframes must end exactly at the CRC-16 footer found by k_span_crc
    const int64_t fend = ((br.pos_bits + 7) >> 3) + bits_shift;
    if (br.err || fend + 2 != fend_known) return;
    atomicAdd(nvalid, 1);
}


// ------------------------------------------------------------------ wave-uniform (scalar-unit) frame decoder
// A subframe's Rice codes are a sequential bit walk and its LPC restore a nonlinear recurrence, so one frame is
// serial work.  It runs here on the scalar unit: every value is wave-uniform (SGPRs: s_flbit_i32_b64,
// s_lshl_b64, s_mul_i32 at scalar latency) instead of lane 0's dependent VALU chain.  Bitstream words reach the
// scalar unit through a VGPR window (lane i = stage word wbase + i, one ds_read per 64 words) and v_readlane;
// decoded samples leave through v_writelane into a VGPR stored by one coalesced write per 64 samples.
constexpr int kDecStageWords = 6144;  // 24 KB
// Rice window of the pipelined producer: kRiceWinQ candidates per lane (64 * kRiceWinQ bit positions); jump tables
// hold the window plus the fixed points a code can end on past it (< 64 bits further)
constexpr int kRiceWinQ = 16, kRiceWinBits = 64 * kRiceWinQ, kJumpN = kRiceWinBits + 128;

struct WaveBits {
    const uint32_t *stage;  // LDS: big-endian (byte-swapped) dwords of the blob from byte 4 * wb
    uint32_t win;           // stage[wbase + lane]
    uint32_t wbase, wi;     // window base and next word to take (stage word indices)
    uint32_t wlim;          // words staged
    uint64_t c;             // left-aligned bit cache
    int n;                  // valid bits in c
    int lane;
    __device__ inline uint32_t word(uint32_t i) {
        if (i - wbase >= 64u) {
            wbase = i & ~63u;
            win = stage[min(wbase + (uint32_t)lane, wlim)];
        }
        return (uint32_t)__builtin_amdgcn_readlane((int)win, (int)(i - wbase));
    }
    __device__ inline void refill() {
        while (n <= 32) refill1();
    }
    __device__ inline void refill1() {  // one word (callers guarantee 0 < n <= 32)
        c |= (uint64_t)word(wi++) << (32 - n);
        n += 32;
    }
    __device__ inline void init(const uint32_t *st, uint32_t nwords, uint32_t bitpos, int ln) {
        stage = st;
        wlim = nwords;
        lane = ln;
        wbase = 0u - 64u;
        wi = bitpos >> 5;
        c = (uint64_t)word(wi++) << 32;
        n = 32;
        const int off = (int)(bitpos & 31);
        c <<= off;
        n -= off;
        refill();
    }
    __device__ inline uint32_t bits(int k) {  // k <= 32; n > 32 on entry
        if (k == 0) return 0;
        const uint32_t v = (uint32_t)(c >> (64 - k));
        c <<= k;
        n -= k;
        refill();
        return v;
    }
    __device__ inline int32_t sbits(int k) {
        const uint32_t v = bits(k);
        return (k == 0 || k == 32) ? (int32_t)v : ((int32_t)(v << (32 - k)) >> (32 - k));
    }
    __device__ inline uint32_t pos() const { return wi * 32 - (uint32_t)n; }
    __device__ inline void seek(uint32_t bitpos) {
        wi = bitpos >> 5;
        c = (uint64_t)word(wi++) << 32;
        n = 32;
        const int off = (int)(bitpos & 31);
        c <<= off;
        n -= off;
        refill();
    }
    // zeros before the next 1 (the 1 is consumed); false past `lim` bits (corrupt data)
    __device__ inline bool unary(uint32_t &q, uint32_t lim) {
        q = 0;
        while (c == 0) {  // the cache holds n (> 32) zero bits
            q += (uint32_t)n;
            n = 0;
            refill();
            if (pos() > lim) return false;
        }
        const int z = __builtin_clzll(c);  // < n: the cache's bits below n are zero
        q += (uint32_t)z;
        c = (z + 1 >= 64) ? 0 : (c << (z + 1));
        n -= z + 1;
        refill();
        return true;
    }
};

// ------------------------------------------------------------------ two-wave pipelined frame decoder
// A lone wave issues one instruction every ~6 (SALU) to ~8 (VALU) cycles (tools/micro/issue_rates.hip), so a
// frame's decode time is its serial instruction count.  k_decode_frames_pipe splits that count over two waves of
// one work-group (same CU): wave 0 parses the frame on the scalar unit and Rice-decodes the residuals into LDS,
// 64 at a time, publishing progress; wave 1 restores the samples behind it -- the LPC recurrence as a v_dot2
// chain over the eight newest samples held as packed int16 pairs -- and writes them to LDS, copied to the PCM
// output at the end.  Mono 16-bit FIXED / LPC (order <= 8, 32-bit-safe prediction) / CONSTANT / VERBATIM
// subframes; anything else falls back to decode_one_frame on wave 0, lane 0.
// The jump tables of one Rice window (kRiceWinBits candidate bit positions from stage bit P, parameter k1 - 1) by
// one wave: jt[0][c] = 2 x the start of the code after a code starting at candidate c (absorbing -- c itself -- when
// that code's stop bit lies more than 64 bits past its lane's first candidate), jt[k+1][c] = jt[k][jt[k][c]].  Entries
// are BYTE offsets into a row (2 c), so a lookup's address is the entry itself plus the row's immediate offset.  Lane
// j owns the kRiceWinQ consecutive candidates c = kRiceWinQ j + t: their 64-bit windows lie in four stage words, and
// the lane's entries are one contiguous run (16-byte LDS stores).  The entries past the window (fixed points) are
// the caller's.
__device__ inline void rice_window_tables(const uint32_t *stage, uint32_t P, int k1, uint16_t (*jt)[kRiceWinBits + 128],
                                          int lane) {
    const uint32_t b = P + (uint32_t)(kRiceWinQ * lane), wi = b >> 5, sh = b & 31u;
    const uint64_t wA = ((uint64_t)stage[wi] << 32) | stage[wi + 1];
    const uint64_t wB = ((uint64_t)stage[wi + 2] << 32) | stage[wi + 3];
    int jq[kRiceWinQ];
    {
        // the lane's 64 bits from its first candidate; candidate t's code ends k1 bits after the first set bit at or
        // after t: those first-set positions by a backward select chain over the top 16 bits (one 64-bit clz for the
        // rest) instead of a shift + clz per candidate.  A code whose stop bit lies past these 64 bits is left
        // absorbing (the chain's long-code path decodes it).
        const uint64_t X = sh ? (wA << sh) | (wB >> (64u - sh)) : wA;
        const uint64_t X16 = X << 16;
        int f = (X16 ? __builtin_clzll(X16) : 64) + 16;  // 80: no set bit in [16, 64)
        const uint32_t top = (uint32_t)(X >> 48);
        const int c0 = kRiceWinQ * lane;
#pragma unroll
        for (int t = kRiceWinQ - 1; t >= 0; t--) {
            f = ((top >> (15 - t)) & 1u) ? t : f;
            jq[t] = 2 * (f + k1 - t <= 64 ? c0 + f + k1 : c0 + t);
        }
    }
    auto store_run = [&](uint16_t *row) {  // jq -> row[kRiceWinQ * lane ...], 16 bytes at a time
#pragma unroll
        for (int v = 0; v < kRiceWinQ / 8; v++) {
            uint4 u;
            u.x = (uint32_t)jq[8 * v] | ((uint32_t)jq[8 * v + 1] << 16);
            u.y = (uint32_t)jq[8 * v + 2] | ((uint32_t)jq[8 * v + 3] << 16);
            u.z = (uint32_t)jq[8 * v + 4] | ((uint32_t)jq[8 * v + 5] << 16);
            u.w = (uint32_t)jq[8 * v + 6] | ((uint32_t)jq[8 * v + 7] << 16);
            reinterpret_cast<uint4 *>(row + kRiceWinQ * lane)[v] = u;
        }
    };
    store_run(jt[0]);
#pragma unroll
    for (int k = 0; k < 5; k++) {
#pragma unroll
        for (int q = 0; q < kRiceWinQ; q++)
            jq[q] = *reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(jt[k]) + jq[q]);
        store_run(jt[k + 1]);
    }
}

typedef short dec_v2s16 __attribute__((ext_vector_type(2)));
__device__ inline int32_t dec_dot2(uint32_t a, uint32_t b, int32_t c) {  // v_dot2_i32_i16
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(dec_v2s16, a), __builtin_bit_cast(dec_v2s16, b), c, false);
}
constexpr int kPipeFallback = 1, kPipeDone = 2, kPipeRestore = 3, kPipeError = 4;
struct PipeInfo {
    int32_t state;       // 0 while parsing, then kPipe*
    int32_t progress;    // residuals published in resbuf (samples [o, progress) are ready)
    int32_t valid;       // producer's verdict at the end: 1 = frame ends at its CRC footer
    int32_t finished;    // producer done (valid final)
    int32_t crc_ok;      // OPT: the span's CRC-16 verifies (set before finished)
    int32_t o, shift, w, bs;
    int32_t cq[8];
    int32_t wu[8];
    // grid tables (one-partition Rice residuals): the producer publishes gstate = 1 with (gk1, gbase, glim), or -1;
    // wave 2 builds the tables of grid window j (bits gbase + kRiceWinBits j ...) into slot j & 1 and publishes
    // gready = j + 1; the producer publishes gused = the windows it has left behind, and gstop when it is done
    int32_t gstate, gready, gused, gstop;
    int32_t gk1;
    uint32_t gbase, glim;
};

__device__ inline void lds_publish(volatile int32_t *p, int32_t v) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's earlier LDS writes have landed
    *p = v;
}
__device__ inline int32_t lds_poll(volatile int32_t *p) { return *p; }

// OPT: the last work-group to finish (flags[8] counts them; re-armed to 0) copies the call's counters flags[0..7] to
// page-locked host memory, so the host reads them after its stream synchronisation without a device-to-host copy
// (system-scope fences: the work-group's output may be page-locked host memory, and the host takes hout[6] leaving -1
// as the decode's completion -- it is written last, after every other counter)
__device__ inline void pipe_wg_exit(int *flags, int64_t nframes, int *hout) {
    __threadfence_system();
    const int t = atomicAdd(&flags[8], 1);
    if (t == (int)nframes - 1) {
        flags[8] = 0;
        __threadfence();
        for (int k = 0; k < 8; k++)
            if (k != 6) hout[k] = __hip_atomic_load(&flags[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int h6 = __hip_atomic_load(&flags[6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence_system();
        __hip_atomic_store(&hout[6], h6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
    }
}
// OPT (small ranges, launched right after the selection): the optimistic form -- when the selection found exactly
// one candidate per frame and each stream's first at its first byte, frame i IS candidate i and its span ends at
// candidate i + 1 (or the stream end), so the span check and the chain are skipped: the consumer wave checks the
// span's CRC-16 over the staged bytes while the producer parses, and a frame counts (flags[7]) only when its CRC and
// its end both verify.  Anything else (a false sync, a frame the producer would hand to the one-lane decoder) sets
// flags[6], and the host runs the span check, chain and the non-optimistic decoder after all.
template <bool OPT = false>
__global__ void __launch_bounds__(192) k_decode_frames_pipe(const uint8_t *blob, const int64_t *soff, int ns,
                                                           const int64_t *poff, const int64_t *cpos,
                                                           const int64_t *ends, const int64_t *fbase,
                                                           const int64_t *frame_cand, int64_t nframes, int channels,
                                                           int stream_bps, int32_t *pcm, int blocksize, int *nvalid,
                                                           DecOut dout, const int *ncand = nullptr,
                                                           int *flags = nullptr, int *hout = nullptr) {
    __shared__ uint32_t stage[kDecStageWords + 2 * kRiceWinQ + 4];  // + the window step's look-ahead words
    __shared__ __attribute__((aligned(16))) int32_t resbuf[kDecResMax];
    __shared__ PipeInfo info;
    __shared__ __attribute__((aligned(16))) uint16_t ct4[OPT ? 4 : 1][256];  // slice-by-4 CRC-16 tables (OPT)
    // restored samples as int16 pairs + the producer's Rice-window jump tables (window + fixed points); a frame
    // that falls back to the one-lane decoder under a fused decode is decoded into `fb` instead (same bytes)
    union PipeU {
        struct {
            uint32_t xout[kDecResMax / 2];
            uint16_t jt[2][6][kJumpN];  // (the grid path's two slots; the partition-by-partition path slot 0)
        } p;
        int32_t fb[kDecResMax];
    };
    __shared__ __attribute__((aligned(16))) PipeU pu;
    uint32_t *xout = pu.p.xout;
    uint16_t(*jt)[kJumpN] = pu.p.jt[0];
    const int64_t fi = blockIdx.x;
    if (fi >= nframes) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t fpos, fend_known;
    int s;
    if constexpr (OPT) {
        int lo = 0, hi = ns - 1;  // stream of frame fi
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (fbase[mid] <= fi) lo = mid;
            else hi = mid - 1;
        }
        s = lo;
        bool okmap = *ncand == (int)nframes;
        fpos = okmap ? cpos[fi] : 0;
        fend_known = okmap ? (fi + 1 < fbase[s + 1] ? cpos[fi + 1] : soff[s + 1]) : 0;
        okmap = okmap && fpos >= soff[s] && (fi != fbase[s] || fpos == soff[s]) && fend_known > fpos &&
                fend_known <= soff[s + 1];
        if (!okmap) {
            if (threadIdx.x == 0) {
                atomicOr(&flags[6], 1);
                __threadfence();
            }
            __syncthreads();
            if (threadIdx.x == 64) pipe_wg_exit(flags, nframes, hout);
            return;
        }
        for (int k = threadIdx.x; k < 128; k += 128)
            reinterpret_cast<uint4 *>(&ct4[0][0])[k] = reinterpret_cast<const uint4 *>(&d_crc16x4[0][0])[k];
    } else {
        const int64_t ci = frame_cand[fi];
        if (ci < 0 || ends[ci] < 0) return;  // not on a verified chain (the host reports it)
        fpos = cpos[ci];
        fend_known = ends[ci];
        s = stream_of(soff, ns, fpos);
    }
    const int64_t send = soff[s + 1];
    const int64_t wb = fpos >> 2, we = (fend_known + 3) >> 2;
    const bool staged = we - wb <= kDecStageWords;
    if (staged)  // big-endian words: the scalar bit reader needs no byte swap
        stage_words<192, true>(stage, blob, wb, we - wb + 2 * kRiceWinQ + 4, send, (int)threadIdx.x);
    if (threadIdx.x == 0) {
        info.state = 0;
        info.progress = 0;
        info.finished = 0;
        info.valid = 0;
        info.crc_ok = 0;
        info.gstate = 0;
        info.gready = 0;
        info.gused = 0;
        info.gstop = 0;
    }
    __syncthreads();
    const int64_t nsamp = poff[s + 1] - poff[s];
    const int64_t kk = fi - fbase[s];
    const int64_t first = kk * blocksize;
    const int64_t obase = poff[s] + first;  // mono: sample i of the frame is element obase + i
    const bool fused = dout.out != nullptr;
    const float2 dnp = fused ? dout.dn[s] : make_float2(0.f, 0.f);
    auto put = [&](int i, int32_t v) {
        if (fused) dn_store(dout, obase + i, v, dnp);
        else pcm[obase + i] = v;
    };
    // after a one-lane fallback decode into pu.fb (fused decodes): the wave de-normalises the frame out of LDS
    auto flush_fb = [&]() {
        if (!fused) return;
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        const int n = (int)min<int64_t>(blocksize, nsamp - first);
        for (int i = lane; i < n; i += 64) dn_store(dout, obase + i, pu.fb[i], dnp);
    };
    volatile PipeInfo *vi = &info;
    if (wave == 0) {
        // ================= producer: parse + Rice decode (wave-uniform, scalar unit)
        // OPT: CRC-16 of the span [fpos, fend) over the staged big-endian words (bytes outside it zeroed: leading
        // zeros leave a CRC from 0 unchanged, trailing ones multiply it by x^8, invertible mod P) == 0 -- computed by
        // this wave after its Rice windows (the consumer's restore is the decode's critical path)
        auto span_crc = [&]() {
            if constexpr (OPT) {
                const int nw = (int)(we - wb), cw = (nw + 63) / 64;
                const int a = min(nw, lane * cw), b = min(nw, a + cw);
                uint32_t c = 0;
                for (int k = a; k < b; k++) {
                    const int64_t byte0 = 4 * (wb + k);
                    const int lo = (int)min<int64_t>(4, max<int64_t>(0, fpos - byte0));
                    const int hi = (int)min<int64_t>(4, max<int64_t>(0, fend_known - byte0));
                    const uint32_t m1 = lo >= 4 ? 0u : (0xFFFFFFFFu >> (8 * lo));
                    const uint32_t m2 = hi <= 0 ? 0u : (0xFFFFFFFFu << (8 * (4 - hi)));
                    const uint32_t w = stage[k] & m1 & m2;
                    c = (uint32_t)ct4[3][((c >> 8) ^ (w >> 24)) & 0xFF] ^ ct4[2][((c & 0xFF) ^ ((w >> 16) & 0xFF)) & 0xFF] ^
                        ct4[1][(w >> 8) & 0xFF] ^ ct4[0][w & 0xFF];
                }
                c = crc_xpow(c, 4u * (uint32_t)(nw - b));
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) c ^= (uint32_t)__shfl_xor((int)c, o);
                if (lane == 0) info.crc_ok = c == 0;
            }
        };
        auto finish = [&](int st, int valid) {
            if (lane == 0) lds_publish(&vi->gstate, -1);  // (every early end: the grid builder leaves)
            if (st == kPipeDone) span_crc();
            // OPT: a CONSTANT / VERBATIM frame's samples were stored by this wave; the consumer's exit (and the last
            // work-group's completion word the host takes as the decode's end) must not pass them, and a fence
            // orders only the executing wave's own stores: release them at system scope before publishing
            if constexpr (OPT) __threadfence_system();
            if (lane == 0) {
                info.valid = valid;
                lds_publish(&vi->finished, 1);
                if (st) lds_publish(&vi->state, st);
            }
        };
        if (OPT && !staged) {  // (the one-lane decoder needs the verified chain)
            if (lane == 0) {
                atomicOr(&flags[6], 1);
                __threadfence();
            }
            finish(kPipeError, 0);
            return;
        }
        if (!staged) {
            finish(kPipeFallback, 0);
            if (lane == 0)
                decode_one_frame(blob, blob, 0, soff, ns, poff, cpos, ends, fbase, frame_cand, fi, channels,
                                 stream_bps, pcm, blocksize, nvalid, resbuf, nullptr, fused ? pu.fb : nullptr);
            flush_fb();
            return;
        }
        const FrameHdr cd = parse_header(blob, fpos, send, channels, stream_bps);
        if (!cd.ok || cd.frame_no != kk || cd.bs > blocksize || first + cd.bs > nsamp) {
            finish(kPipeError, 0);
            return;
        }
        const int bs = __builtin_amdgcn_readfirstlane(cd.bs);
        const uint32_t lim = (uint32_t)((fend_known - 4 * wb) * 8);
        WaveBits br;
        br.init(stage, (uint32_t)(we - wb + 3), (uint32_t)((fpos + cd.hdr_len - 4 * wb) * 8), lane);
        br.bits(1);
        const int t = (int)br.bits(6);
        int w = 0;
        if (br.bits(1)) {
            uint32_t q;
            if (!br.unary(q, lim)) { finish(kPipeError, 0); return; }
            w = (int)q + 1;
        }
        const int sbps = __builtin_amdgcn_readfirstlane(cd.bps) - w;
        auto fallback = [&]() {
            if (OPT) {
                if (lane == 0) {
                    atomicOr(&flags[6], 1);
                    __threadfence();
                }
                finish(kPipeError, 0);
                return;
            }
            finish(kPipeFallback, 0);
            for (int64_t k = lane; k < we - wb + 4; k += 64) stage[k] = __builtin_bswap32(stage[k]);  // back to LE
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
            if (lane == 0)
                decode_one_frame(blob, reinterpret_cast<const uint8_t *>(stage), wb * 4, soff, ns, poff, cpos, ends,
                                 fbase, frame_cand, fi, channels, stream_bps, pcm, blocksize, nvalid, resbuf, stage,
                                 fused ? pu.fb : nullptr);
            flush_fb();
        };
        if (cd.bps > 16 || sbps <= 0) { fallback(); return; }
        auto end_ok = [&]() { return (int64_t)((br.pos() + 7) >> 3) + 4 * wb + 2 == fend_known; };
        if (t == 0) {  // CONSTANT
            const int32_t v = br.sbits(sbps);
            for (int i = lane; i < bs; i += 64) put(i, (int32_t)((uint32_t)v << w));
            const int ok = end_ok();
            if (!OPT && ok && lane == 0) atomicAdd(nvalid, 1);
            finish(kPipeDone, ok);
            return;
        }
        if (t == 1) {  // VERBATIM: fixed-width samples, so sample i sits at bit P0 + i * sbps -- lane-parallel
            // (the scalar reader took one dependent read per sample: a tile holding one VERBATIM frame took ~0.3 ms
            // longer than the others, the C5 p90)
            const uint32_t P0 = br.pos(), Pe = P0 + (uint32_t)bs * (uint32_t)sbps;
            if (Pe > lim) { finish(kPipeError, 0); return; }
            for (int i = lane; i < bs; i += 64) {
                const uint32_t b = P0 + (uint32_t)i * (uint32_t)sbps, wi = b >> 5, sh = b & 31u;
                const uint32_t hi = stage[wi], lo = stage[wi + 1];
                const uint32_t v = sh ? __builtin_amdgcn_alignbit(hi, lo, 32u - sh) : hi;
                const int32_t x = (int32_t)v >> (32 - sbps);
                put(i, (int32_t)((uint32_t)x << w));
            }
            br.seek(Pe);
            const int ok = end_ok();
            if (!OPT && ok && lane == 0) atomicAdd(nvalid, 1);
            finish(kPipeDone, ok);
            return;
        }
        if (!((t >= 8 && t <= 12) || (t >= 32 && t <= 39))) { fallback(); return; }
        const bool lpc = t >= 32;
        const int o = lpc ? t - 31 : t - 8;
        if (o > bs) { finish(kPipeError, 0); return; }
        int32_t wu[8], cq[8];
#pragma unroll
        for (int m = 0; m < 8; m++) {
            wu[m] = 0;
            cq[m] = 0;
        }
#pragma unroll
        for (int m = 0; m < 8; m++)
            if (m < o) wu[m] = br.sbits(sbps);
        int shift = 0, prec = 3;
        if (lpc) {
            prec = (int)br.bits(4) + 1;
            if (prec == 16) { finish(kPipeError, 0); return; }
            shift = br.sbits(5);
            if (shift < 0) { finish(kPipeError, 0); return; }
#pragma unroll
            for (int m = 0; m < 8; m++)
                if (m < o) cq[m] = br.sbits(prec);
        } else {
            if (o >= 1) cq[0] = o == 1 ? 1 : o == 2 ? 2 : o == 3 ? 3 : 4;
            if (o >= 2) cq[1] = o == 2 ? -1 : o == 3 ? -3 : -6;
            if (o >= 3) cq[2] = o == 3 ? 1 : 4;
            if (o >= 4) cq[3] = -1;
        }
        int lg = 0;
        while ((1 << lg) < o) lg++;
        // 16-bit samples and coefficients for the v_dot2 restore, 32-bit-safe prediction
        if (!(sbps <= 16 && prec <= 16 && prec + sbps + lg <= 31)) { fallback(); return; }
        const int method = (int)br.bits(2);
        if (method > 1) { finish(kPipeError, 0); return; }
        const int po = (int)br.bits(4);
        if ((bs >> po) < o || (bs & ((1 << po) - 1))) { finish(kPipeError, 0); return; }
        if (lane == 0) {
            info.o = o;
            info.shift = shift;
            info.w = w;
            info.bs = bs;
#pragma unroll
            for (int m = 0; m < 8; m++) {
                info.cq[m] = cq[m];
                info.wu[m] = wu[m];
            }
            lds_publish(&vi->state, kPipeRestore);
        }
        const int pb = method == 0 ? 4 : 5, esc = (1 << pb) - 1;
        const int psz = bs >> po;
        int i = o;
        bool bad = false;
        uint32_t P = br.pos();  // stage bit of the next field
        auto publish = [&]() {
            if (lane == 0) lds_publish(&vi->progress, i);
        };
        // ---- one-partition residuals (C4: 97 % of the frames): the Rice parameter is the frame's, so the windows'
        //      jump tables do not depend on where the chain enters them -- wave 2 builds them on a fixed bit grid
        //      (window j = bits base + kRiceWinBits j ..), two windows ahead of this wave, which only walks the chain
        //      (round 6: the table levels were ~half of each window's dependent LDS round trips)
        bool grid = false;
        if (po == 0) {
            br.seek(P);
            const int kp = (int)br.bits(pb);
            if (kp != esc) {
                grid = true;
                const uint32_t base = br.pos();
                if (lane == 0) {
                    info.gk1 = kp + 1;
                    info.gbase = base;
                    info.glim = lim;
                    lds_publish(&vi->gstate, 1);
                }
                uint32_t Pg = base;
                int left = bs - o, jdone = 0;
                while (left > 0) {
                    if (Pg > lim) {
                        bad = true;
                        break;
                    }
                    const uint32_t rel = Pg - base;
                    const int j = (int)(rel / (uint32_t)kRiceWinBits), e = (int)(rel % (uint32_t)kRiceWinBits);
                    if (j > jdone) {  // windows < j are left behind: their slots may be rebuilt
                        jdone = j;
                        if (lane == 0) lds_publish(&vi->gused, j);
                    }
                    while (lds_poll(&vi->gready) <= j) __builtin_amdgcn_s_sleep(1);
                    __asm__ volatile("" ::: "memory");  // table reads stay behind the poll
                    const uint16_t(*tb)[kJumpN] = pu.p.jt[j & 1];
                    auto tb_at = [&](int k, int byteoff) -> int {
                        return *reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(tb[k]) + byteoff);
                    };
                    const uint32_t wbits = base + (uint32_t)j * (uint32_t)kRiceWinBits;
                    const int cap = left < 64 ? left : 64;
                    int posv = 2 * e;  // (byte offset) lane m: the m-th code from the entry point
#pragma unroll
                    for (int k = 0; k < 6; k++) {
                        const int nx = tb_at(k, posv);
                        posv = ((lane >> k) & 1) ? nx : posv;
                    }
                    const int nxt = tb_at(0, posv);
                    const uint64_t chain = __ballot(posv < 2 * kRiceWinBits && nxt != posv && lane < cap);
                    const int cnt = __builtin_popcountll(chain);
                    int cur;
                    bool lng = false;
                    if (cnt < cap) {  // stopped at a long code (inside the window) or past the window
                        cur = __builtin_amdgcn_readlane(posv, cnt) >> 1;
                        lng = cur < kRiceWinBits;
                    } else {
                        cur = __builtin_amdgcn_readlane(nxt, cnt - 1) >> 1;
                    }
                    {
                        const uint32_t bc = wbits + (uint32_t)(posv >> 1), wc = bc >> 5;
                        const uint32_t sft = bc & 31u, x0 = stage[wc], x1 = stage[wc + 1], x2 = stage[wc + 2];
                        const uint32_t hi = sft ? __builtin_amdgcn_alignbit(x0, x1, 32u - sft) : x0;
                        const uint32_t lo = sft ? __builtin_amdgcn_alignbit(x1, x2, 32u - sft) : x1;
                        const uint64_t win = ((uint64_t)hi << 32) | lo;
                        const int z = win ? __builtin_clzll(win) : 64;
                        const uint32_t low = kp ? (uint32_t)((win << (z + 1)) >> (64 - kp)) : 0u;
                        const uint32_t u = ((uint32_t)z << kp) | low;
                        if (lane < cnt) resbuf[i + lane] = (int32_t)(((u >> 1) ^ (uint32_t)(-(int32_t)(u & 1))) << shift);
                    }
                    const int i0 = i;
                    i += cnt;
                    left -= cnt;
                    Pg = wbits + (uint32_t)cur;
                    if (lng) {  // a long unary run: one code through the scalar reader
                        br.seek(Pg);
                        uint32_t q;
                        if (!br.unary(q, lim)) {
                            bad = true;
                            break;
                        }
                        const uint32_t uu = (q << kp) | br.bits(kp);
                        if (lane == 0) resbuf[i] = (int32_t)(((uu >> 1) ^ (uint32_t)(-(int32_t)(uu & 1))) << shift);
                        i++;
                        left--;
                        Pg = br.pos();
                    }
                    if ((i0 >> 6) != (i >> 6) || left == 0) publish();  // per 64-sample group (and the end)
                }
                P = Pg;
                if (lane == 0) lds_publish(&vi->gstop, 1);
            }
        }
        if (!grid && lane == 0) lds_publish(&vi->gstate, -1);
#pragma unroll
        for (int k = 0; k < 6; k++) {  // jump-table entries past the window are fixed points
            jt[k][kRiceWinBits + lane] = (uint16_t)(2 * (kRiceWinBits + lane));
            jt[k][kRiceWinBits + 64 + lane] = (uint16_t)(2 * (kRiceWinBits + 64 + lane));
        }
        for (int p = 0; p < (1 << po) && !bad && !grid; p++) {
            br.seek(P);
            const int kp = (int)br.bits(pb);
            int left = psz - (p == 0 ? o : 0);
            if (kp == esc) {  // escaped partition: fixed-width residuals (rare; lane 0 stores them)
                const int nb = (int)br.bits(5);
                for (int j = 0; j < left; j++, i++) {
                    const int32_t r = nb ? br.sbits(nb) : 0;
                    if (lane == 0) resbuf[i] = (int32_t)((uint32_t)r << shift);
                }
                P = br.pos();
                publish();
                continue;
            }
            P = br.pos();
            const int k1 = kp + 1;
            // Window step over kRiceWinBits = 1024 bits: lane j decodes the lengths of the Rice codes that would
            // start at bits P + 16j + t (t < kRiceWinQ, from big-endian stage words); the chain of actual code starts
            // through them is resolved by pointer jumping over LDS tables (lane m lands on the m-th start in six reads, no
            // per-code scalar loop); lane m then decodes the value of the code at that start and the window's residuals
            // leave in one contiguous LDS store.  A 1024-bit window holds ~64 codes (the lane
            // cap) of a 15-bit/sample frame: measured per tile 0.221 / 0.204 / 0.192 ms at 512 / 768 / 1024 bits.
            while (left > 0) {
                if (P > lim) {
                    bad = true;
                    break;
                }
                auto window64 = [&](uint32_t x0, uint32_t x1, uint32_t x2, uint32_t sft) -> uint64_t {
                    const uint32_t hi = sft ? __builtin_amdgcn_alignbit(x0, x1, 32u - sft) : x0;
                    const uint32_t lo = sft ? __builtin_amdgcn_alignbit(x1, x2, 32u - sft) : x1;
                    return ((uint64_t)hi << 32) | lo;
                };
                // lane j owns the kRiceWinQ consecutive candidates c = kRiceWinQ * j + t (bits P + c): their 64-bit
                // windows all lie in four stage words, and the lane's jump-table entries are one contiguous run
                // (16-byte LDS stores)
                const uint32_t b = P + (uint32_t)(kRiceWinQ * lane), wi = b >> 5, sh = b & 31u;
                const uint64_t wA = ((uint64_t)stage[wi] << 32) | stage[wi + 1];
                const uint64_t wB = ((uint64_t)stage[wi + 2] << 32) | stage[wi + 3];
                // chain by pointer jumping: jt[k][c] = the code start 2^k codes after candidate c (absorbing at a
                // long code and past the window), so lane m finds the m-th code start in six dependent LDS reads;
                // the values are decoded after it, only at the chain's code starts.  Entries hold BYTE offsets into a
                // row (2 c), so a lookup's address is the entry itself plus the row's immediate offset (no scaling)
                const int cap = left < 64 ? left : 64;
                int jq[kRiceWinQ];
                {
                    // the lane's 64 bits from its first candidate; candidate t's code ends k1 bits after the first set
                    // bit at or after t: those first-set positions by a backward select chain over the top 16 bits
                    // (one 64-bit clz for the rest) instead of a shift + clz per candidate.  A code whose stop bit
                    // lies past these 64 bits is left absorbing (the chain's long-code path decodes it).
                    const uint64_t X = sh ? (wA << sh) | (wB >> (64u - sh)) : wA;
                    const uint64_t X16 = X << 16;
                    int f = (X16 ? __builtin_clzll(X16) : 64) + 16;  // 80: no set bit in [16, 64)
                    const uint32_t top = (uint32_t)(X >> 48);
                    const int c0 = kRiceWinQ * lane;
#pragma unroll
                    for (int t = kRiceWinQ - 1; t >= 0; t--) {
                        f = ((top >> (15 - t)) & 1u) ? t : f;
                        jq[t] = 2 * (f + k1 - t <= 64 ? c0 + f + k1 : c0 + t);
                    }
                }
                auto store_run = [&](uint16_t *row) {  // jq -> row[kRiceWinQ * lane ...], 16 bytes at a time
#pragma unroll
                    for (int v = 0; v < kRiceWinQ / 8; v++) {
                        uint4 u;
                        u.x = (uint32_t)jq[8 * v] | ((uint32_t)jq[8 * v + 1] << 16);
                        u.y = (uint32_t)jq[8 * v + 2] | ((uint32_t)jq[8 * v + 3] << 16);
                        u.z = (uint32_t)jq[8 * v + 4] | ((uint32_t)jq[8 * v + 5] << 16);
                        u.w = (uint32_t)jq[8 * v + 6] | ((uint32_t)jq[8 * v + 7] << 16);
                        reinterpret_cast<uint4 *>(row + kRiceWinQ * lane)[v] = u;
                    }
                };
                store_run(jt[0]);
#pragma unroll
                for (int k = 0; k < 5; k++) {
#pragma unroll
                    for (int q = 0; q < kRiceWinQ; q++)
                        jq[q] = *reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(jt[k]) + jq[q]);
                    store_run(jt[k + 1]);
                }
                auto jt_at = [&](int k, int byteoff) -> int {
                    return *reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(jt[k]) + byteoff);
                };
                int posv = 0;  // (byte offset)
#pragma unroll
                for (int k = 0; k < 6; k++) {
                    const int nx = jt_at(k, posv);
                    posv = ((lane >> k) & 1) ? nx : posv;
                }
                const int nxt = jt_at(0, posv);
                const uint64_t chain = __ballot(posv < 2 * kRiceWinBits && nxt != posv && lane < cap);  // lanes 0..cnt-1
                const int cnt = __builtin_popcountll(chain);
                int cur;
                bool lng = false;
                if (cnt < cap) {  // stopped at a long code (inside the window) or past the window
                    cur = __builtin_amdgcn_readlane(posv, cnt) >> 1;
                    lng = cur < kRiceWinBits;
                } else {
                    cur = __builtin_amdgcn_readlane(nxt, cnt - 1) >> 1;
                }
                {
                    const uint32_t bc = P + (uint32_t)(posv >> 1), wc = bc >> 5;  // lane m: the m-th code of the window
                    const uint64_t win = window64(stage[wc], stage[wc + 1], stage[wc + 2], bc & 31u);
                    const int z = win ? __builtin_clzll(win) : 64;
                    const uint32_t low = kp ? (uint32_t)((win << (z + 1)) >> (64 - kp)) : 0u;
                    const uint32_t u = ((uint32_t)z << kp) | low;
                    if (lane < cnt) resbuf[i + lane] = (int32_t)(((u >> 1) ^ (uint32_t)(-(int32_t)(u & 1))) << shift);
                }
                const int i0 = i;
                i += cnt;
                left -= cnt;
                P += (uint32_t)cur;
                if (lng) {  // a long unary run: one code through the scalar reader
                    br.seek(P);
                    uint32_t q;
                    if (!br.unary(q, lim)) {
                        bad = true;
                        break;
                    }
                    const uint32_t uu = (q << kp) | br.bits(kp);
                    if (lane == 0) resbuf[i] = (int32_t)(((uu >> 1) ^ (uint32_t)(-(int32_t)(uu & 1))) << shift);
                    i++;
                    left--;
                    P = br.pos();
                }
                if ((i0 >> 6) != (i >> 6) || left == 0) publish();  // per 64-sample group (and partition end)
            }
        }
        br.seek(P);  // the frame's end check reads br.pos()
        const int ok = !bad && end_ok();
        if (lane == 0) lds_publish(&vi->progress, bad ? -1 : bs);
        span_crc();
        if (lane == 0) {
            info.valid = ok;
            lds_publish(&vi->finished, 1);
        }
        return;
    }
    if (wave == 2) {
        // ================= grid table builder (one-partition residuals, see the producer)
        int gs;
        while ((gs = lds_poll(&vi->gstate)) == 0) __builtin_amdgcn_s_sleep(1);
        if (gs < 0) return;
        __asm__ volatile("" ::: "memory");
        const int k1 = vi->gk1;
        const uint32_t base = vi->gbase, glim = vi->glim;
#pragma unroll
        for (int sl = 0; sl < 2; sl++)
#pragma unroll
            for (int k = 0; k < 6; k++) {  // entries past the window are fixed points
                pu.p.jt[sl][k][kRiceWinBits + lane] = (uint16_t)(2 * (kRiceWinBits + lane));
                pu.p.jt[sl][k][kRiceWinBits + 64 + lane] = (uint16_t)(2 * (kRiceWinBits + 64 + lane));
            }
        for (int j = 0;; j++) {
            const uint32_t B = base + (uint32_t)j * (uint32_t)kRiceWinBits;
            if (B > glim) break;  // (the producer stops at glim)
            if (j >= 2)  // slot j & 1 held window j - 2: the producer has entered window j - 1
                while (lds_poll(&vi->gused) < j - 1 && !lds_poll(&vi->gstop)) __builtin_amdgcn_s_sleep(1);
            if (lds_poll(&vi->gstop)) break;
            __asm__ volatile("" ::: "memory");
            rice_window_tables(stage, B, k1, pu.p.jt[j & 1], lane);
            if (lane == 0) lds_publish(&vi->gready, j + 1);
        }
        return;
    }
    // ================= consumer (wave 1): LPC / FIXED restore behind the producer
    int st;
    while ((st = lds_poll(&vi->state)) == 0) __builtin_amdgcn_s_sleep(1);
    if (st != kPipeRestore) {  // handled by the producer
        if constexpr (OPT) {
            while (lds_poll(&vi->finished) == 0) __builtin_amdgcn_s_sleep(1);
            __asm__ volatile("" ::: "memory");
            if (st == kPipeDone && info.valid && info.crc_ok && lane == 0) atomicAdd(&flags[7], 1);
            if (lane == 0) pipe_wg_exit(flags, nframes, hout);
        }
        return;
    }
    const int o = info.o, shift = info.shift, w = info.w, bs = info.bs;
    // coefficient pairs C[k] = (c[2k+1] << 16 | c[2k] & 0xffff): dot2 with history pair H[k] = (x[i-2k-2], x[i-2k-1])
    uint32_t C[4], H[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; k++) C[k] = ((uint32_t)info.cq[2 * k + 1] << 16) | ((uint32_t)info.cq[2 * k] & 0xFFFFu);
    // warm-up samples: x[0..o-1]; H after them holds x[o-8..o-1]
    int32_t wu[8];
#pragma unroll
    for (int m = 0; m < 8; m++) wu[m] = info.wu[m];
#pragma unroll
    for (int m = 0; m < 8; m++)
        if (m < o) {
            H[3] = __builtin_amdgcn_alignbit(H[3], H[2], 16);
            H[2] = __builtin_amdgcn_alignbit(H[2], H[1], 16);
            H[1] = __builtin_amdgcn_alignbit(H[1], H[0], 16);
            H[0] = (H[0] << 16) | ((uint32_t)wu[m] & 0xFFFFu);
        }
#pragma unroll
    for (int m = 0; m < 8; m++)
        if (m < o && lane == 0) reinterpret_cast<int16_t *>(xout)[m] = (int16_t)wu[m];
    int avail = 0;
    bool failed = false;
    // one sample of the recurrence: x = r + (sum q.x >> shift), the four dot2 over (newest, older) pairs with the
    // oldest pairs first so only the last one waits on x[i-1]; the history pairs then shift by one sample
    // (residuals arrive pre-shifted, R = r << shift: x = (R + sum q.x) >> shift, exact in wrapping int32 for
    // shift <= 15 and a 16-bit x)
    auto restore = [&](int32_t R, int i, bool odd) {
        int32_t pred = dec_dot2(H[3], C[3], R);
        pred = dec_dot2(H[2], C[2], pred);
        pred = dec_dot2(H[1], C[1], pred);
        pred = dec_dot2(H[0], C[0], pred);
        const int32_t x = pred >> shift;
        H[3] = __builtin_amdgcn_alignbit(H[3], H[2], 16);
        H[2] = __builtin_amdgcn_alignbit(H[2], H[1], 16);
        H[1] = __builtin_amdgcn_alignbit(H[1], H[0], 16);
        H[0] = __builtin_amdgcn_perm(H[0], (uint32_t)x, 0x05040100u);  // (H0 << 16) | (x & 0xffff)
        if (odd) xout[i >> 1] = __builtin_amdgcn_alignbit(H[0], H[0], 16);  // (x[i] << 16) | x[i-1]
    };
    // wait until the producer has published residuals up to `need` (it publishes per 64-sample group, at
    // partition ends and bs at the end; -1 on a bad frame)
    auto wait_for = [&](int need) -> bool {
        if (avail >= need) return true;
        int pg;
        while ((pg = lds_poll(&vi->progress)) < need && pg >= 0) __builtin_amdgcn_s_sleep(1);
        __asm__ volatile("" ::: "memory");  // resbuf reads stay behind the poll
        if (pg < 0) return false;
        avail = pg;
        return true;
    };
    // per-sample path with run-time lane selects: the head up to the first 64-sample boundary and any tail
    auto generic = [&](int lo, int hi) {
        uint32_t vr = 0;
        for (int i = lo; i < hi; i++) {
            if (i == lo || (i & 63) == 0) {
                if (!wait_for(min((i & ~63) + 64, bs))) {
                    failed = true;
                    return;
                }
                vr = (uint32_t)resbuf[(i & ~63) + lane];
            }
            restore(__builtin_amdgcn_readlane((int)vr, i & 63), i, (i & 1) != 0);
        }
    };
    const int head = min(bs, (o + 63) & ~63);
    generic(o, head);
    int i = head;
    // whole 64-sample groups, fully unrolled, two samples per step on pair-aligned history: Q[m] = (x[2m+1] << 16 |
    // x[2m] & 0xffff), the output layout, in a four-register ring renamed by the unroll (no per-sample shifting of the
    // history).  x[2m] = r + (sum_k dot2(Q[m-1-k], C'[k]) >> shift), C'[k] = (q[2k] << 16 | q[2k+1]); x[2m+1] adds
    // q[0] x[2m] to dot2s of the same pairs against D'[k] = (q[2k+1] << 16 | q[2k+2]).  Residual j of the group by
    // v_readlane with an immediate lane index.  (Per sample ~8.5 instructions instead of ~12: the lone consumer wave
    // issues one every ~8 cycles.)  Round 6: taking the newest pair's two samples off the dot2 (24-bit multiply-adds,
    // four dependent operations per pair instead of six) is not faster: tools/micro/restore_chain.hip 25.6 (this
    // form) / 27.9 / 26.9 ns per sample, C5 decode_frames 0.104 ms either way (one box, one call).
    // OPT, de-normalised 1- / 2-byte output: each restored 64-sample group leaves (one 2-byte store per lane) while the
    // next group is restored, instead of all 4096 samples after the restore; a declined frame is decoded again by the
    // non-optimistic path, which rewrites its output
    const int dt = fused ? dout.dtype : -1;
    const bool dfast = (dt == FRS_DT_I16 || dt == FRS_DT_U16 || dt == FRS_DT_U8) && dout.shift == 0 &&
                       (obase & 7) == 0 && (bs & 7) == 0;
    const bool early = OPT && dfast;
    const float dnx = dnp.x * (1.0f / 65536.0f);
    auto dn1 = [&](int32_t x) -> uint32_t {  // (dn_bits_t's exact rewrite of ((x / 32768 + 1) / 2) * rng + mn)
        const float a = __fadd_rn(__fmul_rn((float)((int32_t)((uint32_t)x << w) + 32768), dnx), dnp.y);
        return (uint32_t)(int32_t)rintf(a);
    };
    int stored = 0;  // samples [0, stored) already stored (wave-uniform)
    if (!failed && i + 64 <= bs) {
        auto pk = [](int32_t hi, int32_t lo) { return ((uint32_t)hi << 16) | ((uint32_t)lo & 0xFFFFu); };
        const int32_t q0 = info.cq[0];
        uint32_t Ce[4], Co[4], Qr[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            Ce[k] = pk(info.cq[2 * k], info.cq[2 * k + 1]);
            Co[k] = pk(info.cq[2 * k + 1], k < 3 ? info.cq[2 * k + 2] : 0);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // the head's pairs are in xout
#pragma unroll
        for (int k = 0; k < 4; k++) Qr[3 - k] = i ? xout[(i >> 1) - 1 - k] : 0u;  // Qr[3] = Q[m-1] .. Qr[0] = Q[m-4]
        for (; i + 64 <= bs; i += 64) {
            if (!wait_for(i + 64)) {
                failed = true;
                break;
            }
            int4 rr = make_int4(0, 0, 0, 0);
            const int4 *rp = reinterpret_cast<const int4 *>(&resbuf[i]);  // (base pointers: immediate ds offsets)
            uint32_t *xp = xout + (i >> 1);
            // the group's 64 (pre-shifted) residuals read up front, every lane the same 16 bytes per read: they
            // arrive in VGPRs and seed the dot2 accumulators (no per-sample v_readlane + v_mov).  Round 6: reading
            // four at a time every second pair put an LDS round trip (s_waitcnt lgkmcnt(0)) on the lone wave's chain
            // every 4 samples -- tools/micro/restore_chain.hip 25.6 -> 19.7 ns per sample, C5 decode_frames 104.4 ->
            // 102.7 us: the restore (~80 us a frame) now runs behind the producer's Rice windows (a build with the
            // restore skipped: 95 vs 97.6 us into device memory)
            int4 rall[16];
#pragma unroll
            for (int j = 0; j < 16; j++) rall[j] = rp[j];
            // the previous 64 samples (the last group, or the head) leave after this group's restore: read now
            const bool st_now = early && i - stored >= 64;
            int32_t xprev = 0;
            if (st_now) xprev = reinterpret_cast<const int16_t *>(xout)[stored + lane];
#pragma unroll
            for (int p2 = 0; p2 < 32; p2++) {
                if (!(p2 & 1)) rr = rall[p2 >> 1];
                const int32_t Re = (p2 & 1) ? rr.z : rr.x, Ro = (p2 & 1) ? rr.w : rr.y;
                const uint32_t A = Qr[(p2 + 3) & 3], B = Qr[(p2 + 2) & 3], Cc = Qr[(p2 + 1) & 3], Dd = Qr[p2 & 3];
                int32_t pe = dec_dot2(Dd, Ce[3], Re);
                pe = dec_dot2(Cc, Ce[2], pe);
                pe = dec_dot2(B, Ce[1], pe);
                int32_t po = dec_dot2(Dd, Co[3], Ro);
                po = dec_dot2(Cc, Co[2], po);
                po = dec_dot2(B, Co[1], po);
                po = dec_dot2(A, Co[0], po);
                pe = dec_dot2(A, Ce[0], pe);
                const int32_t xe = pe >> shift;
                const int32_t xo = (__mul24(q0, xe) + po) >> shift;
                const uint32_t qn = __builtin_amdgcn_perm((uint32_t)xo, (uint32_t)xe, 0x05040100u);
                xp[p2] = qn;
                Qr[p2 & 3] = qn;
            }
            if (st_now) {
                const uint32_t ob = dn1(xprev);
                if (dt == FRS_DT_U8) static_cast<uint8_t *>(dout.out)[obase + stored + lane] = (uint8_t)ob;
                else static_cast<uint16_t *>(dout.out)[obase + stored + lane] = (uint16_t)ob;
                stored += 64;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) H[k] = __builtin_amdgcn_alignbit(Qr[3 - k], Qr[3 - k], 16);  // for the tail
    }
    if (!failed && i < bs) generic(i, bs);
    if (!failed && (bs & 1)) xout[bs >> 1] = H[0] & 0xFFFFu;
    while (lds_poll(&vi->finished) == 0) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    if (failed || !info.valid || (OPT && !info.crc_ok)) {
        if (OPT && lane == 0) pipe_wg_exit(flags, nframes, hout);
        return;
    }
    const int16_t *x16 = reinterpret_cast<const int16_t *>(xout);
    if (dfast) {
        // de-normalised 1- and 2-byte outputs: eight samples per lane and step, one 16-byte LDS read and one 16- (8-)
        // byte store (the per-sample loop issued 64 scattered 2-byte stores per lane: 13.6 of a frame's 137 us); the
        // groups stored during the restore are skipped
        const uint4 *x8 = reinterpret_cast<const uint4 *>(xout);
        for (int g = (stored >> 3) + lane; g < (bs >> 3); g += 64) {
            const uint4 v = x8[g];
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
            uint32_t ob[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int32_t x = (int32_t)(int16_t)(wv[j >> 1] >> (16 * (j & 1)));
                // (dn_bits_t's exact rewrite of ((x / 32768 + 1) / 2) * rng + mn)
                const float a = __fadd_rn(__fmul_rn((float)((int32_t)((uint32_t)x << w) + 32768), dnx), dnp.y);
                ob[j] = (uint32_t)(int32_t)rintf(a);
            }
            if (dt == FRS_DT_U8) {
                reinterpret_cast<uint2 *>(static_cast<uint8_t *>(dout.out) + obase)[g] =
                    make_uint2((ob[0] & 0xFF) | ((ob[1] & 0xFF) << 8) | ((ob[2] & 0xFF) << 16) | (ob[3] << 24),
                               (ob[4] & 0xFF) | ((ob[5] & 0xFF) << 8) | ((ob[6] & 0xFF) << 16) | (ob[7] << 24));
            } else {
                reinterpret_cast<uint4 *>(static_cast<uint16_t *>(dout.out) + obase)[g] =
                    make_uint4((ob[0] & 0xFFFF) | (ob[1] << 16), (ob[2] & 0xFFFF) | (ob[3] << 16),
                               (ob[4] & 0xFFFF) | (ob[5] << 16), (ob[6] & 0xFFFF) | (ob[7] << 16));
            }
        }
    } else {
        for (int i = lane; i < bs; i += 64) put(i, (int32_t)((uint32_t)(int32_t)x16[i] << w));
    }
    if (lane == 0) {
        atomicAdd(OPT ? &flags[7] : nvalid, 1);
        if (OPT) pipe_wg_exit(flags, nframes, hout);
    }
}

// One wave per frame: the frame's bytes are staged in LDS by the whole wave (coalesced dword loads), then lane 0
// decodes from LDS (bit refills are LDS reads instead of dependent global loads).  Frames larger than the stage
// are decoded straight from global memory.  Multi-channel and wide streams.  Under a fused decode the int32
// samples land in the `pcm` scratch first and the wave de-normalises the frame from there.
__device__ inline void wave_decode_frame(int64_t fi, uint32_t *stage, int32_t *resbuf, const uint8_t *blob,
                                         const int64_t *soff, int ns, const int64_t *poff, const int64_t *cpos,
                                         const int64_t *ends, const int64_t *fbase, const int64_t *frame_cand,
                                         int channels, int stream_bps, int32_t *pcm, int blocksize, int *nvalid,
                                         const DecOut &dout) {
    const int lane = threadIdx.x;
    const int64_t ci = frame_cand[fi];
    if (ci < 0 || ends[ci] < 0) return;  // (block-uniform) not on a verified chain (the host reports it)
    const int64_t fpos = cpos[ci], fend = ends[ci];
    const int s = stream_of(soff, ns, fpos);
    const int64_t send = soff[s + 1];
    const int64_t wb = fpos >> 2, we = (fend + 3) >> 2;
    const bool staged = we - wb <= kDecStageWords;
    __syncthreads();  // the stage's previous readers are done
    if (staged)
        for (int64_t k = lane; k < we - wb + 4; k += 64) stage[k] = load_word_guarded(blob, wb + k, send);
    __syncthreads();
    if (lane == 0) {
        if (staged)
            decode_one_frame(blob, reinterpret_cast<const uint8_t *>(stage), wb * 4, soff, ns, poff, cpos, ends, fbase,
                             frame_cand, fi, channels, stream_bps, pcm, blocksize, nvalid, resbuf, stage);
        else
            decode_one_frame(blob, blob, 0, soff, ns, poff, cpos, ends, fbase, frame_cand, fi, channels, stream_bps,
                             pcm, blocksize, nvalid, resbuf, nullptr);
    }
    if (dout.out == nullptr) return;
    __syncthreads();  // lane 0's global writes are visible to the work-group (one wave)
    const int64_t first = (fi - fbase[s]) * blocksize;
    const int64_t n = min<int64_t>(blocksize, poff[s + 1] - poff[s] - first) * channels;
    const int64_t e0 = (poff[s] + first) * channels;
    const float2 dnp = dout.dn[s];
    for (int64_t i = lane; i < n; i += 64) dn_store(dout, e0 + i, pcm[e0 + i], dnp);
}

__global__ void __launch_bounds__(64) k_decode_frames_wave(const uint8_t *blob, const int64_t *soff, int ns,
                                                          const int64_t *poff, const int64_t *cpos,
                                                          const int64_t *ends, const int64_t *fbase,
                                                          const int64_t *frame_cand, int64_t nframes, int channels,
                                                          int stream_bps, int32_t *pcm, int blocksize, int *nvalid,
                                                          DecOut dout) {
    __shared__ uint32_t stage[kDecStageWords + 4];
    __shared__ int32_t resbuf[kDecResMax];
    const int64_t fi = blockIdx.x;
    if (fi >= nframes) return;
    wave_decode_frame(fi, stage, resbuf, blob, soff, ns, poff, cpos, ends, fbase, frame_cand, channels, stream_bps,
                      pcm, blocksize, nvalid, dout);
}

// The frames the lane decoder queued (layouts it does not take), each by one wave; the grid strides over the
// device-side count, so no host sync separates the two launches.
__global__ void __launch_bounds__(64) k_decode_frames_wave_list(const uint8_t *blob, const int64_t *soff, int ns,
                                                               const int64_t *poff, const int64_t *cpos,
                                                               const int64_t *ends, const int64_t *fbase,
                                                               const int64_t *frame_cand, int channels, int stream_bps,
                                                               int32_t *pcm, int blocksize, int *nvalid, DecOut dout,
                                                               const int32_t *list, const int *count) {
    __shared__ uint32_t stage[kDecStageWords + 4];
    __shared__ int32_t resbuf[kDecResMax];
    const int nl = *count;
    for (int j = blockIdx.x; j < nl; j += gridDim.x)
        wave_decode_frame(list[j], stage, resbuf, blob, soff, ns, poff, cpos, ends, fbase, frame_cand, channels,
                          stream_bps, pcm, blocksize, nvalid, dout);
}

// ------------------------------------------------------------------ lane-per-frame decoder (batched decodes)
// Throughput form for decodes of many frames (a whole arena, FLAC -> TIFF of a large raster): one lane per frame,
// eight samples per step.  Each lane walks its own frame through a ring of big-endian dwords in LDS (RingReader:
// a code is read from a 32-bit window at the lane's bit position and consumed by an add; the ring is refilled once
// per step from 16-byte chunks whose loads were issued a chunk earlier).  Partition boundaries are consumed by
// conditional position steps, the LPC recurrence runs on an eight-register ring with compile-time slots (no
// register indexing), and each step's eight outputs leave in one vector store (8 to 32 bytes; scattered 2-byte
// stores from 64 lanes cost ~13x the bytes in partial-line writes).  The output kind is a template parameter, so
// the per-sample work has no dtype switch.  Taken: mono streams of <= 16-bit samples, FIXED / LPC (order <= 8,
// 32-bit-safe prediction), VERBATIM and CONSTANT subframes; an escaped partition or anything else sends the frame to
// k_decode_frames_wave_list (which rewrites all of its samples).  A frame counts as valid when its
// subframe ends exactly at the CRC-16 footer found by the span check.
constexpr int kOutPcm = 0, kOutI16 = 1, kOutU16 = 2, kOutU8 = 3, kOutAny = 4;
constexpr int kOutPlanar16 = 5;  // raw 16-bit PCM (the multi-channel planar scratch of >= 3 independent channels)
constexpr int kDecStageSlots = 8;  // 16-byte output groups staged per lane before a flush (one 128-byte line)

// Per-lane bit reader over a ring of kRingSlots big-endian dwords in LDS (column layout: slot s of a lane at
// col[64 s], so a wave's reads and writes of one slot each hit 64 distinct banks; slot kRingSlots repeats slot 0, so
// a two-dword window never wraps).  p is the next unread bit, counted from the first loaded chunk; a read is one
// ds_read2 of the dwords holding bits [p, p + 64) and one 64-bit shift, so consuming a code is an add to p -- no
// cache shifts and no queue bookkeeping per sample.  16-byte chunks enter the ring when it runs low (fill), each
// chunk's global load issued one chunk ahead.  (Measured, C4 batched decode: 8 ring slots with a refill every 4
// codes, i.e. 4 instead of 3 work-groups per CU, 3.20 -> 3.45 ms; every chunk also folded into the frame's CRC-16 as it
// enters the ring, slice-by-4 in LDS, so no separate span check: 3.20 -> 3.85 ms.)
constexpr int kRingSlots = 16;
struct RingReader {
    uint32_t *col;         // this lane's slot 0
    const uint8_t *abase;  // blob aligned down to 16 bytes; chunk q covers abase[q, q + 16)
    int64_t lead;          // blob - abase
    int64_t q0;            // aligned offset of the first chunk (bit 0 of p)
    int64_t next;          // aligned offset of the next chunk to load
    int64_t end;           // stream end (blob bytes)
    uint32_t p;            // next unread bit
    uint32_t wr;           // dwords written to the ring
    uint4 praw;            // the chunk loaded a fill ahead (raw little-endian)
    int pval;              // its bytes before the stream end
    bool bad;
    // The chunk at q, bytes at or past `end` counted in val.  Unconditional: a chunk past the end re-reads the
    // 16-byte-aligned chunk holding the last byte (never across a page) and is zeroed by the fill.
    __device__ inline uint4 fetch(int64_t q, int &val) const {
        const int64_t lastq = (end - 1 + lead) & ~(int64_t)15;
        val = (int)max<int64_t>(0, min<int64_t>(16, end - (q - lead)));
        return *reinterpret_cast<const uint4 *>(abase + (q <= lastq ? q : lastq));
    }
    __device__ inline void fill() {  // the prefetched chunk into the next four slots, the following chunk's load issued
        auto be = [&](uint32_t w, int d) -> uint32_t {  // dword d as big-endian, zero past pval
            const int nb = pval - 4 * d;
            return __builtin_bswap32(nb >= 4 ? w : nb <= 0 ? 0u : (w & ((1u << (8 * nb)) - 1u)));
        };
        const uint32_t d0 = be(praw.x, 0), d1 = be(praw.y, 1), d2 = be(praw.z, 2), d3 = be(praw.w, 3);
        const uint32_t s = wr & (kRingSlots - 1);
        uint32_t *a = col + (s << 6);
        a[0] = d0;
        a[64] = d1;
        a[128] = d2;
        a[192] = d3;
        if (s == 0) col[kRingSlots << 6] = d0;
        wr += 4;
        praw = fetch(next, pval);
        next += 16;
        if (next - lead > end + 64) bad = true;  // runaway walk (corrupt data)
    }
    // at least `need` unread dwords in the ring (fills leave at most need + 3, within the ring while need <= 13)
    __device__ inline void ahead(int need) {
        while ((int)(wr - (p >> 5)) < need && !bad) fill();
    }
    // a step's reads: up to eight codes of <= 32 bits read from windows at most 8 dwords on
    __device__ inline void refill() { ahead(9); }
    __device__ inline uint32_t window() const {  // bits [p, p + 32), MSB first (two dwords from p's in the ring)
        const uint32_t *a = col + (((p >> 5) & (kRingSlots - 1)) << 6);
        const uint64_t d = ((uint64_t)a[0] << 32) | a[64];
        return (uint32_t)((d << (p & 31)) >> 32);
    }
    __device__ inline uint32_t peek32() {
        ahead(2);
        return window();
    }
    __device__ inline void init(uint32_t *lane_col, const uint8_t *b, int64_t pos, int64_t e) {
        col = lane_col;
        end = e;
        lead = (int64_t)(reinterpret_cast<uintptr_t>(b) & 15);
        abase = b - lead;
        q0 = (pos + lead) & ~(int64_t)15;
        praw = fetch(q0, pval);
        next = q0 + 16;
        wr = 0;
        bad = false;
        p = (uint32_t)((pos + lead) & 15) * 8u;
        fill();
        fill();
    }
    __device__ inline uint32_t bits(int k) {  // 0 <= k <= 32
        const uint32_t w = peek32();
        p += (uint32_t)k;
        return k ? w >> (32 - k) : 0u;
    }
    __device__ inline int32_t sbits(int k) {
        const uint32_t v = bits(k);
        return (k == 0 || k == 32) ? (int32_t)v : ((int32_t)(v << (32 - k)) >> (32 - k));
    }
    __device__ inline uint32_t unary() {  // zeros before the next 1 (consumed)
        uint32_t q = 0, w;
        for (;;) {
            w = peek32();
            if (w != 0 || bad) break;
            q += 32;
            p += 32;
        }
        const uint32_t z = w ? (uint32_t)__builtin_clz(w) : 0u;
        p += z + 1;
        return q + z;
    }
    __device__ inline uint32_t rice(int k) {  // Rice code, parameter k <= 30
        const uint32_t q = unary();
        return (q << k) | bits(k);
    }
    __device__ inline int64_t pos() const {  // bit position of the next unread bit from the blob start
        return (q0 - lead) * 8 + (int64_t)p;
    }
};

// converter.py:88-110 value of one decoded sample as the bits of a <= 4-byte output element
template <int OUT>
__device__ inline uint32_t dn_bits_t(const DecOut &o, int32_t pcm, float2 p) {
    if constexpr (OUT == kOutPcm) {
        return (uint32_t)pcm;
    } else if constexpr (OUT == kOutPlanar16) {
        return (uint32_t)pcm & 0xFFFFu;
    } else {
        // ((v + 1) / 2) * rng + mn with v = h / 32768 (h = pcm >> shift, |h| < 2^24): (v + 1) / 2 = (h + 32768) 2^-16
        // exactly, and scaling rng by 2^-16 instead is exact too, so one product and one sum round as in the
        // reference's sequence; the rounded value is within the <= 16-bit output range, so an int32 conversion
        const float a = __fadd_rn(__fmul_rn((float)((pcm >> o.shift) + 32768), p.x * (1.0f / 65536.0f)), p.y);
        const int32_t r = (int32_t)rintf(a);
        if constexpr (OUT == kOutU8) return (uint32_t)(uint8_t)r;
        else return (uint32_t)(uint16_t)r;
    }
}

// Channel-planar int32 PCM of the multi-channel lane decoder -> the interleaved output (de-normalised when fused,
// int32 PCM otherwise).  One work-group per (frame, 256-sample chunk): its stream is found once (block-uniform), and
// each thread takes one sample position with all nch channels -- nch coalesced planar reads, nch adjacent output
// elements (a thread per output element, each locating its stream and frame by 64-bit division, was 4.6 ms for a
// 4-band 16384^2 stream: integer-divide bound).
// Two-channel streams (fchass != nullptr): the frame's channel assignment (written by the lane decoder) undoes
// libFLAC's stereo decorrelation here -- left-side R = L - S, right-side L = R + S, mid-side from (M << 1 | S & 1).
__global__ void __launch_bounds__(256) k_interleave_dn(const int32_t *planar, const int64_t *poff, const int64_t *fbase,
                                                      int ns, int nch, int blocksize, int32_t *pcm, DecOut dout,
                                                      const int8_t *fchass, int cpf, int planar16) {
    const int64_t fi = blockIdx.x / (unsigned)cpf;
    const int i = (int)(blockIdx.x - fi * cpf) * 256 + (int)threadIdx.x;  // sample position in the frame
    if (i >= blocksize) return;
    int lo = 0, hi = ns - 1;  // stream of frame fi (block-uniform)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (fbase[mid] <= fi) lo = mid;
        else hi = mid - 1;
    }
    const int64_t g = poff[lo] + (fi - fbase[lo]) * blocksize + i;  // sample index
    if (g >= poff[lo + 1]) return;
    int32_t x[8];
    if (planar16) {  // (>= 3 independent 16-bit channels: half the scratch bytes)
        const int16_t *src = reinterpret_cast<const int16_t *>(planar) + fi * nch * (int64_t)blocksize + i;
#pragma unroll
        for (int c = 0; c < 8; c++) x[c] = c < nch ? src[(int64_t)c * blocksize] : 0;
    } else {
        const int32_t *src = planar + fi * nch * (int64_t)blocksize + i;
#pragma unroll
        for (int c = 0; c < 8; c++) x[c] = c < nch ? src[(int64_t)c * blocksize] : 0;
    }
    if (fchass) {
        const int ca = fchass[fi];
        const int64_t a = x[0], sd = x[1];
        if (ca == 8) x[1] = (int32_t)(a - sd);
        else if (ca == 9) x[0] = (int32_t)(a + sd);
        else if (ca == 10) {
            const int64_t mid = (a * 2) | (sd & 1);
            x[0] = (int32_t)((mid + sd) >> 1);
            x[1] = (int32_t)((mid - sd) >> 1);
        }
    }
    if (dout.out && (dout.dtype == FRS_DT_I16 || dout.dtype == FRS_DT_U16) && !(nch & 1)) {
        // 16-bit outputs of an even channel count: the thread's nch elements in 4-byte (8-byte for 4 channels) stores
        uint32_t v[8];
#pragma unroll
        for (int c = 0; c < 8; c++) v[c] = c < nch ? dn_bits_t<kOutI16>(dout, x[c], dout.dn[lo]) : 0u;
        uint16_t *o = static_cast<uint16_t *>(dout.out) + g * nch;
        if (nch == 4) {
            *reinterpret_cast<uint2 *>(o) = make_uint2(v[0] | (v[1] << 16), v[2] | (v[3] << 16));
        } else {
#pragma unroll
            for (int c = 0; c < 8; c += 2)
                if (c < nch) *reinterpret_cast<uint32_t *>(o + c) = v[c] | (v[c + 1] << 16);
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < 8; c++) {
        if (c < nch) {
            if (dout.out) dn_store(dout, g * nch + c, x[c], dout.dn[lo]);
            else pcm[g * nch + c] = x[c];
        }
    }
}

// MC (multi-channel streams of >= 3 independent channels, and two-channel streams in any of the four assignments):
// the lane walks the frame's subframes in turn and writes them channel-planar as int32 PCM to `planar` (frame fi,
// channel c at (fi * nch + c) * blocksize); k_interleave_dn then interleaves (undoing the stereo decorrelation
// by fchass[fi]) and de-normalises.
template <int OUT, bool MC = false>
__global__ void __launch_bounds__(256) k_decode_frames_lane(const uint8_t *blob, const int64_t *soff, int ns,
                                                           const int64_t *poff, const int64_t *cpos,
                                                           const int64_t *ends, const int64_t *fbase,
                                                           const int64_t *frame_cand, int64_t nframes,
                                                           int stream_bps, int32_t *pcm, int blocksize, int *nvalid,
                                                           DecOut dout, int32_t *fb_list, int *fb_count,
                                                           int nch = 1, int32_t *planar = nullptr,
                                                           int8_t *fchass = nullptr) {
    static_assert(!MC || OUT == kOutPcm || OUT == kOutPlanar16, "channel-planar int32 / int16 output");
    constexpr int es = OUT == kOutPcm ? 4 : OUT == kOutU8 ? 1 : 2;  // kOutAny: per-sample dn_store
    // 1- and 2-byte outputs: a lane's aligned 8-sample groups are staged in LDS (slot-major: every ds op of the wave
    // is one contiguous 1 KB) and leave 8 groups at a time, i.e. a whole 128-byte line (64 B for bytes) as back-to-back
    // stores -- one 16-byte store per step to 64 different lines had the L2 write each line back several times
    // (PMC: 5x the output bytes written)
    constexpr bool kStage = OUT == kOutI16 || OUT == kOutU16 || OUT == kOutU8 || OUT == kOutPlanar16;
    __shared__ uint4 ostage[kStage ? 4 : 1][kStage ? kDecStageSlots : 1][kStage ? 64 : 1];
    __shared__ uint32_t ring[4][kRingSlots + 1][64];  // the lanes' bit readers
    const int64_t fi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint8_t *obytes = MC ? reinterpret_cast<uint8_t *>(planar)
                         : OUT == kOutPcm ? reinterpret_cast<uint8_t *>(pcm) : static_cast<uint8_t *>(dout.out);
    bool ok = false;
    if (fi < nframes) {
        const int64_t ci = frame_cand[fi];
        const int64_t fend = ci >= 0 ? ends[ci] : -1;
        if (fend >= 0) {
            const int64_t fpos = cpos[ci];
            const int s = stream_of(soff, ns, fpos);
            const int64_t send = soff[s + 1];
            const int64_t nsamp = poff[s + 1] - poff[s];
            const int64_t kk = fi - fbase[s];
            const int64_t first = kk * blocksize;
            const FrameHdr cd = parse_header(blob, fpos, send, MC ? nch : 1, stream_bps);
            // independent channels, or a two-channel frame in any assignment (k_interleave_dn undoes it)
            bool take_all = !MC || cd.chass == nch - 1 || (nch == 2 && cd.chass >= 8 && cd.chass <= 10);
            if (MC && fchass && cd.ok) fchass[fi] = (int8_t)cd.chass;
            if (cd.ok && cd.frame_no == kk && cd.bs <= blocksize && first + cd.bs <= nsamp && take_all) {
                const int bs = cd.bs;
                const float2 dnp = OUT != kOutPcm && OUT != kOutPlanar16 ? dout.dn[s] : make_float2(0.f, 0.f);
                RingReader br;
                br.init(&ring[threadIdx.x >> 6][0][threadIdx.x & 63], blob, fpos + cd.hdr_len, send);
                for (int chn = 0; chn < (MC ? nch : 1) && take_all; chn++) {
                const int64_t obase = MC ? (fi * nch + chn) * (int64_t)blocksize : poff[s] + first;
                br.bits(1);
                const int t = (int)br.bits(6);
                int w = 0;
                if (br.bits(1)) w = (int)br.unary() + 1;
                // the side signal of a two-channel frame carries one extra bit
                const bool side = MC && nch == 2 &&
                                  ((cd.chass == 8 && chn == 1) || (cd.chass == 9 && chn == 0) || (cd.chass == 10 && chn == 1));
                const int sbps = cd.bps - w + (side ? 1 : 0);
                int o = 0, shift = 0;
                bool take = cd.bps <= 16 && sbps > 0 && sbps <= 17;
                const bool raw = t == 1;  // VERBATIM: order 0, raw residuals
                if (t >= 8 && t <= 12) o = t - 8;
                else if (t >= 32 && t <= 39) o = t - 31;
                else if (t > 1) take = false;  // reserved: the wave decoder reports it
                int32_t cq[8], R[8];
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    cq[m] = 0;
                    R[m] = 0;
                }
                int32_t cval = 0;
                if (take && t == 0) cval = br.sbits(sbps);  // CONSTANT
#pragma unroll
                for (int m = 0; m < 8; m++)
                    if (take && m < o) R[m] = br.sbits(sbps);  // warm-up: ring slot m = sample m
                if (take && t >= 32) {
                    const int prec = (int)br.bits(4) + 1;
                    shift = br.sbits(5);
                    if (prec == 16 || shift < 0) take = false;
#pragma unroll
                    for (int m = 0; m < 8; m++)
                        if (m < o) cq[m] = br.sbits(prec);
                } else if (t >= 8 && t <= 12) {
                    cq[0] = o == 1 ? 1 : o == 2 ? 2 : o == 3 ? 3 : o == 4 ? 4 : 0;
                    cq[1] = o == 2 ? -1 : o == 3 ? -3 : o == 4 ? -6 : 0;
                    cq[2] = o == 3 ? 1 : o == 4 ? 4 : 0;
                    cq[3] = o == 4 ? -1 : 0;
                }
                // 32-bit prediction (__mul24 taps): |sum q.x| <= sum|q| 2^(sbps-1) must stay below 2^31
                uint32_t sumq = 0;
#pragma unroll
                for (int m = 0; m < 8; m++) sumq += (uint32_t)abs(cq[m]);
                if ((32 - __builtin_clz(sumq | 1u)) + sbps - 1 > 31) take = false;
                int pb = 4, esc = 15, psz = bs, part_end = bs, k = 0;
                if (take && t >= 8) {
                    const int method = (int)br.bits(2);
                    const int po = (int)br.bits(4);
                    if (method > 1 || (bs >> po) < o || (bs & ((1 << po) - 1))) {
                        take = false;  // malformed: the wave decoder reports it
                    } else {
                        pb = method == 0 ? 4 : 5;
                        esc = (1 << pb) - 1;
                        psz = bs >> po;
                        part_end = psz;
                        k = (int)br.bits(pb);
                        if (k == esc) take = false;  // escaped partition: the wave decoder
                    }
                }
                if (take) {
                    const bool vec = OUT != kOutAny && (obase & 7) == 0;  // 8-element groups aligned
                    const bool cst = t == 0;
                    int nst = 0;              // groups staged in this lane's row
                    uint8_t *rdst = nullptr;  // output address of the row's first group
                    uint4 *st = &ostage[kStage ? (threadIdx.x >> 6) : 0][0][0];  // [slot][lane]
                    const int ln = threadIdx.x & 63;
                    auto flush = [&]() {
                        if constexpr (kStage) {
#pragma unroll
                            for (int u = 0; u < kDecStageSlots; u++) {
                                if (u < nst) {
                                    const uint4 v = st[u * 64 + ln];
                                    if constexpr (es == 2) reinterpret_cast<uint4 *>(rdst)[u] = v;
                                    else reinterpret_cast<uint2 *>(rdst)[u] = make_uint2(v.x, v.y);
                                }
                            }
                            nst = 0;
                        }
                    };
                    for (int i0 = 0; i0 < bs && take; i0 += 8) {
                        br.refill();
                        uint32_t ob[8];
                        // the general per-sample body only where some lane needs it: warm-up samples (step 0), the
                        // block's end, a partition boundary of a Rice-coded subframe inside this step
                        const bool gen = i0 == 0 || i0 + 8 > bs || (!raw && !cst && part_end < i0 + 8);
                        if (!__ballot(gen)) {
                            // one code per sample: VERBATIM = sbps raw bits, Rice = unary run + stop bit + k low bits,
                            // CONSTANT = nothing read.  Read from a 32-bit window at p: the unary run (zeroed for
                            // VERBATIM / CONSTANT), then kk low bits; a Rice code longer than the window goes the
                            // general way (rare)
                            const uint32_t rmask = (raw || cst) ? 0u : ~0u, rbit = rmask & 1u;
                            const uint32_t kk = raw ? (uint32_t)sbps : cst ? 0u : (uint32_t)k;
#pragma unroll
                            for (int u = 0; u < 8; u++) {
                                const uint32_t win = br.window();
                                const uint32_t zr = (win ? (uint32_t)__builtin_clz(win) : 32u) & rmask;
                                const uint32_t used = zr + rbit + kk;
                                uint32_t v = (zr << k) | __builtin_amdgcn_ubfe(win, 32u - used, kk);
                                const bool longc = used > 32;
                                br.p += longc ? 0u : used;
                                if (__ballot(longc)) {  // (wave-uniform, rare)
                                    if (longc) v = br.rice(k);
                                    br.refill();
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
                        for (int u = 0; u < 8; u++) {
                            const int i = i0 + u;
                            int32_t x = cst ? cval : R[u];  // CONSTANT, or the warm-up sample (i < o)
                            if (!cst && i >= o && i < bs) {
                                // a partition boundary consumes the next Rice parameter (conditional shift)
                                const bool bnd = i == part_end && !raw;
                                const int kp = (int)(br.peek32() >> (32 - pb));
                                k = bnd ? kp : k;
                                const int adv = bnd ? pb : 0;
                                br.p += (uint32_t)adv;
                                part_end += bnd ? psz : 0;
                                if (bnd && k == esc) take = false;
                                int32_t r;
                                if (raw) {
                                    r = br.sbits(sbps);
                                } else {
                                    const uint32_t uu = br.rice(k);
                                    r = (int32_t)((uu >> 1) ^ (uint32_t)(-(int32_t)(uu & 1)));
                                }
                                int32_t pred = 0;
#pragma unroll
                                for (int m = 0; m < 8; m++) pred += __mul24(cq[m], R[(u + 7 - m) & 7]);
                                x = r + (pred >> shift);
                                R[u] = x;
                            }
                            const int32_t xo = (int32_t)((uint32_t)x << w);
                            if constexpr (OUT == kOutAny) {
                                if (i < bs) dn_store(dout, obase + i, xo, dnp);
                                ob[u] = 0;
                            } else {
                                ob[u] = dn_bits_t<OUT>(dout, xo, dnp);
                            }
                        }
                        if constexpr (OUT != kOutAny) {
                            const int nout = min(8, bs - i0);
                            uint8_t *dst = obytes + (obase + i0) * es;
                            if (vec && nout == 8) {
                                if constexpr (kStage) {
                                    if (nst == 0) rdst = dst;
                                    if constexpr (es == 2)
                                        st[nst * 64 + ln] = make_uint4(ob[0] | (ob[1] << 16), ob[2] | (ob[3] << 16),
                                                                 ob[4] | (ob[5] << 16), ob[6] | (ob[7] << 16));
                                    else
                                        st[nst * 64 + ln] = make_uint4(ob[0] | (ob[1] << 8) | (ob[2] << 16) | (ob[3] << 24),
                                                                 ob[4] | (ob[5] << 8) | (ob[6] << 16) | (ob[7] << 24), 0u,
                                                                 0u);
                                    if (++nst == kDecStageSlots) flush();
                                } else if constexpr (es == 2) {
                                    *reinterpret_cast<uint4 *>(dst) =
                                        make_uint4(ob[0] | (ob[1] << 16), ob[2] | (ob[3] << 16), ob[4] | (ob[5] << 16),
                                                   ob[6] | (ob[7] << 16));
                                } else if constexpr (es == 1) {
                                    *reinterpret_cast<uint2 *>(dst) =
                                        make_uint2(ob[0] | (ob[1] << 8) | (ob[2] << 16) | (ob[3] << 24),
                                                   ob[4] | (ob[5] << 8) | (ob[6] << 16) | (ob[7] << 24));
                                } else {
                                    reinterpret_cast<uint4 *>(dst)[0] = make_uint4(ob[0], ob[1], ob[2], ob[3]);
                                    reinterpret_cast<uint4 *>(dst)[1] = make_uint4(ob[4], ob[5], ob[6], ob[7]);
                                }
                            } else {
#pragma unroll
                                for (int u = 0; u < 8; u++) {
                                    if (u < nout) {
                                        if constexpr (es == 4) reinterpret_cast<uint32_t *>(dst)[u] = ob[u];
                                        else if constexpr (es == 2) reinterpret_cast<uint16_t *>(dst)[u] = (uint16_t)ob[u];
                                        else dst[u] = (uint8_t)ob[u];
                                    }
                                }
                            }
                        }
                        if (br.bad) break;
                    }
                    flush();
                }
                take_all = take_all && take;
                }  // channels
                ok = take_all && !br.bad && ((br.pos() + 7) >> 3) + 2 == fend;
                if (!take_all) fb_list[atomicAdd(fb_count, 1)] = (int32_t)fi;
            }
        }
    }
    const uint64_t m = __ballot(ok);
    if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(__ballot(1))) atomicAdd(nvalid, __builtin_popcountll(m));
}

// converter.py:88-110 (fp32, round half to even) after the pyflac/soundfile WAV round trip.
template <typename O>
__global__ void k_denormalize(const int32_t *pcm, int64_t n, int shift, float rng, float fmn, int is_float, O *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t p16 = pcm[i] >> shift;  // 32-bit streams: libsndfile int -> short keeps the high half
    const float v = (float)((double)p16 / 32768.0);
    if (is_float) {
        out[i] = (O)v;
        return;
    }
    float a = __fadd_rn(v, 1.0f);
    a = __fdiv_rn(a, 2.0f);
    a = __fmul_rn(a, rng);
    a = __fadd_rn(a, fmn);
    const float r = rintf(a);
    out[i] = (O)(int64_t)r;
}

static bool g_dec_tables[64];
constexpr int64_t kLaneMinFrames = 4096;
constexpr int64_t kSelOnePassBlocks = 256;  // up to 16 MB: the one-pass selection (latency: C5 queries)  // below: the pipelined decoder (C5 queries decode 64 frames)

int decode_job(frs_ctx *ctx, const uint8_t *blob_dev, int64_t blob_bytes, const int64_t *stream_off,
               int32_t nstreams, int32_t channels, int32_t bps, int32_t blocksize, int32_t *pcm_dev,
               const int64_t *pcm_off, const double *dmin, const double *dmax, int32_t out_dtype, void *out_dev) {
    hipStream_t st = ctx->stream;
    if (const int rc = check_unsynced(ctx)) return rc;
    if (!g_dec_tables[ctx->device]) {
        uint8_t t8[256];
        uint16_t t16[256];
        for (int i = 0; i < 256; i++) {
            uint8_t c = (uint8_t)i;
            for (int k = 0; k < 8; k++) c = (c & 0x80) ? (uint8_t)((c << 1) ^ 0x07) : (uint8_t)(c << 1);
            t8[i] = c;
            uint16_t d = (uint16_t)(i << 8);
            for (int k = 0; k < 8; k++) d = (d & 0x8000) ? (uint16_t)((d << 1) ^ 0x8005) : (uint16_t)(d << 1);
            t16[i] = d;
        }
        FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(d_crc8), t8, sizeof(t8), 0, hipMemcpyHostToDevice, st));
        FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(d_crc16), t16, sizeof(t16), 0, hipMemcpyHostToDevice, st));
        static uint16_t t16x4[4][256];
        for (int i = 0; i < 256; i++) {
            uint16_t c = t16[i];
            t16x4[0][i] = c;
            for (int j = 1; j < 4; j++) {
                c = (uint16_t)(((c << 8) & 0xFFFF) ^ t16[c >> 8]);
                t16x4[j][i] = c;
            }
        }
        FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(d_crc16x4), t16x4, sizeof(t16x4), 0, hipMemcpyHostToDevice, st));
        auto mulmod = [](uint32_t a, uint32_t b) {
            uint32_t r = 0;
            for (int i = 15; i >= 0; i--) {
                r <<= 1;
                if (r & 0x10000u) r ^= 0x18005u;
                if ((b >> i) & 1u) r ^= a;
            }
            return r;
        };
        static uint16_t lo[256], hi[4096];
        uint32_t pw = 1;
        for (int m = 0; m < 256; m++) {
            lo[m] = (uint16_t)pw;
            pw = mulmod(pw, 0x100);
        }
        const uint32_t step = pw;  // x^(8*256)
        pw = 1;
        for (int m = 0; m < 4096; m++) {
            hi[m] = (uint16_t)pw;
            pw = mulmod(pw, step);
        }
        // prefix-CRC selection tables: slice-by-16, x^(8 * 1024), x^(8 * 16 * 2^i) as byte-split multipliers
        static uint16_t sct[kSelCrcTab];
        {
            uint16_t *T = sct, *MK = sct + 16 * 256, *ML = sct + 18 * 256;
            for (int i = 0; i < 256; i++) {
                uint16_t c = t16[i];
                T[i] = c;
                for (int j = 1; j < 16; j++) {
                    c = (uint16_t)(((c << 8) & 0xFFFF) ^ t16[c >> 8]);
                    T[256 * j + i] = c;
                }
            }
            auto xpow8 = [&](uint64_t m) {  // x^(8m) mod P
                uint32_t r = 1, b = 0x100;
                while (m) {
                    if (m & 1) r = mulmod(r, b);
                    b = mulmod(b, b);
                    m >>= 1;
                }
                return r;
            };
            auto split = [&](uint16_t *M, uint32_t K) {
                for (int v = 0; v < 256; v++) {
                    M[v] = (uint16_t)mulmod((uint32_t)v << 8, K);
                    M[256 + v] = (uint16_t)mulmod((uint32_t)v, K);
                }
            };
            split(MK, xpow8(1024));
            for (int i = 0; i < 6; i++) split(ML + 512 * i, xpow8(16u << i));
        }
        FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(d_selcrc_tab), sct, sizeof(sct), 0, hipMemcpyHostToDevice, st));
        FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(d_xpow_lo), lo, sizeof(lo), 0, hipMemcpyHostToDevice, st));
        FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(d_xpow_hi), hi, sizeof(hi), 0, hipMemcpyHostToDevice, st));
        FRS_HIP(hipStreamSynchronize(st));
        g_dec_tables[ctx->device] = true;
    }
    if (blob_bytes <= 0 || nstreams <= 0) return FRS_OK;
    const bool fused = out_dev != nullptr;
    std::vector<int64_t> fbase(nstreams + 1, 0);
    for (int s = 0; s < nstreams; s++) fbase[s + 1] = fbase[s] + (pcm_off[s + 1] - pcm_off[s] + blocksize - 1) / blocksize;
    const int64_t frames = fbase[nstreams];
    if (frames == 0) return FRS_OK;
    const int64_t max_frame = (int64_t)blocksize * channels * 5 + 4096;
    // FRS_FORCE_GENERIC (tests): every frame through the one-lane wave decoder
    const bool pipe = channels == 1 && bps <= 16 && blocksize <= kDecResMax && !ctx->force_generic;
    // many mono frames: the lane-per-frame throughput decoder (the pipelined one is latency-optimised: ~2 work-groups
    // per CU at 62 KB of LDS each); FRS_DECODE_LANE=0/1 overrides for tests
    bool lane = pipe && frames >= kLaneMinFrames;
    if (ctx->decode_lane >= 0) lane = pipe && ctx->decode_lane == 1;
    // multi-channel streams (>= 3 independent channels, 16-bit): the lane decoder walks each frame's subframes into a
    // channel-planar int32 scratch, k_interleave_dn interleaves (and de-normalises); the wave decoder takes the rest
    const bool mcl = channels >= 2 && channels <= 8 && bps <= 16 && blocksize <= kDecResMax && !ctx->force_generic &&
                     frames >= 64 && ctx->decode_lane != 0;
    const int64_t nsamp_all = pcm_off[nstreams] - pcm_off[0];
    const int64_t planar_words = mcl ? frames * channels * (int64_t)blocksize : 0;
    if (fused && (!pipe || lane)) {  // the wave decoder de-normalises out of an int32 scratch
        if (!pcm_dev) {
            FRS_HIP(ctx->dec_pcm.ensure((size_t)std::max(nsamp_all * channels, planar_words) * 4 + 16));
            pcm_dev = ctx->dec_pcm.as<int32_t>() - pcm_off[0] * channels;
        }
    }
    if (mcl && !fused) FRS_HIP(ctx->dec_pcm.ensure((size_t)planar_words * 4 + 16));
    // (the planar scratch is consumed by k_interleave_dn before the fallback decoder reuses dec_pcm)
    // Candidate capacity: every true frame plus false syncs (a sync pattern with a CRC-8-correct header inside
    // frame data, ~1e-7 per byte) with a wide margin; a crafted stream with more is rejected (nothing is written
    // past the cap).  Indices stay below 2^31.
    const int64_t cand_cap = std::min<int64_t>(2 * frames + blob_bytes / 1024 + 4096, (int64_t)0x7FFFFFF0);
    const int64_t lead_bytes = blob_bytes + (int64_t)(reinterpret_cast<uintptr_t>(blob_dev) & 15);
    const int64_t kSmallBytes = (int64_t)kSelStepsSmall * 1024 * (kSelThreads / 64);
    const bool sel_small = (lead_bytes + kSmallBytes - 1) / kSmallBytes <= kSelOnePassBlocks;
    const int64_t sel_bytes = sel_small ? kSmallBytes : kSelBytes;
    const int64_t nblocks = (lead_bytes + sel_bytes - 1) / sel_bytes;
    if (nblocks > (int64_t)0xFFFFFFFF) {
        ctx->err = "decode range too large";
        return FRS_E_UNSUPPORTED;
    }
    FRS_HIP(ctx->dec_cand.ensure(sizeof(int64_t) * 2 * (size_t)cand_cap));
    FRS_HIP(ctx->dec_next.ensure(sizeof(int32_t) * (size_t)cand_cap + 64));
    if (!ctx->dec_count.ptr) {  // counters + the selection ticket: zeroed once, re-armed by the kernel
        FRS_HIP(ctx->dec_count.ensure(64));
        FRS_HIP(hipMemsetAsync(ctx->dec_count.ptr, 0, ctx->dec_count.bytes, st));
    }
    {
        // a grown buffer may come back at the same address with stale words (possibly of the current epoch), and an
        // epoch that wraps could match an old word: zero the status words in both cases
        const size_t before = ctx->dec_status.bytes;
        FRS_HIP(ctx->dec_status.ensure(sizeof(uint64_t) * (size_t)std::min<int64_t>(nblocks, kSelOnePassBlocks)));
        bool wrap = false;
        if (++ctx->dec_epoch >= (1u << 24)) {
            ctx->dec_epoch = 1;
            wrap = true;
        }
        if (ctx->dec_status.bytes != before || wrap)
            FRS_HIP(hipMemsetAsync(ctx->dec_status.ptr, 0, ctx->dec_status.bytes, st));
    }
    // per-call tables through the context's pinned staging in one DMA copy: stream_off | fbase | pcm_off | the
    // fused decode's per-stream (float32(max - min), float32(min)) pairs; the result counters come back after them
    const size_t tab = sizeof(int64_t) * (size_t)(nstreams + 1);
    const size_t dn_bytes = fused ? sizeof(float2) * (size_t)nstreams : 0;
    FRS_HIP(ctx->dec_soff.ensure(3 * tab + dn_bytes + sizeof(int64_t) * frames + 64));
    FRS_HIP(ctx->pin.ensure(3 * tab + dn_bytes + 128));
    int64_t *htab = ctx->pin.at<int64_t>(0);
    memcpy(htab, stream_off, tab);
    memcpy(htab + (nstreams + 1), fbase.data(), tab);
    memcpy(htab + 2 * (nstreams + 1), pcm_off, tab);
    float2 *hdn = reinterpret_cast<float2 *>(htab + 3 * (nstreams + 1));
    if (fused)  // python-float arithmetic first (data_max - data_min in double), then NEP 50 casts to float32
        for (int s = 0; s < nstreams; s++) hdn[s] = make_float2((float)(dmax[s] - dmin[s]), (float)dmin[s]);
    // one stream through the one-pass selection (a bbox query): the tables ride in the selection kernel's arguments
    const bool tabs_by_arg = nstreams == 1 && nblocks <= kSelOnePassBlocks;
    SmallTabs stabs = {};
    if (tabs_by_arg) {
        memcpy(stabs.v, htab, 3 * tab + dn_bytes);  // 6 int64 + one float2
    } else {
        FRS_HIP(hipMemcpyAsync(ctx->dec_soff.ptr, htab, 3 * tab + dn_bytes, hipMemcpyHostToDevice, st));
    }
    int64_t *dsoff = ctx->dec_soff.as<int64_t>();
    int64_t *dfbase = dsoff + (nstreams + 1);
    int64_t *dpoff = dfbase + (nstreams + 1);
    const float2 *ddn = reinterpret_cast<const float2 *>(dpoff + (nstreams + 1));
    int64_t *dchain = reinterpret_cast<int64_t *>(
        (reinterpret_cast<uintptr_t>(dpoff + (nstreams + 1)) + dn_bytes + 7) & ~(uintptr_t)7);
    int *ncand = ctx->dec_count.as<int>();
    int *nvalid = ncand + 1;
    int *bad = ncand + 2;
    unsigned long long *ticket = reinterpret_cast<unsigned long long *>(ctx->dec_count.as<char>() + 16);
    int64_t *cpos = ctx->dec_cand.as<int64_t>();
    int64_t *ends = cpos + cand_cap;
    int32_t *nexti = ctx->dec_next.as<int32_t>();
    // multi-channel decodes of a large range (the two-pass selection): the span check from prefix CRCs the selection
    // folds (k_span_pcrc), within the x^(8m) table range.  Measured (round 5, MI355X): a 4-band 16384^2 stream (one
    // stream of 65536 32-KB frames: the lane span check has few, long spans) select + span 2.49 -> 1.94 ms; the C4
    // batched mono decode (6241 streams of 8-KB frames) 2.16 -> 3.21 ms (the selection's CRC fold costs more than the
    // reading span check it replaces: 1 LDS table lookup per byte either way, at lower occupancy), so mono keeps the
    // reading form.  Round 6 (both counts in the queue form): select + span 1.73 (reading) vs 1.84 ms (prefix) on C4,
    // the 4-band stream's decode 5.35 -> 4.91 ms.  FRS_SPAN_READ=1 / 2 forces the reading / prefix form (tests).
    const char *span_env = nblocks > kSelOnePassBlocks ? getenv("FRS_SPAN_READ") : nullptr;  // (no env walk per query)
    const int span_mode = span_env ? atoi(span_env) : 0;
    const bool pcrc_span = span_mode != 1 && (span_mode == 2 || mcl) && nblocks > kSelOnePassBlocks &&
                           (lane || !pipe) && max_frame < (int64_t)4096 * 256;
    uint32_t *BPv = nullptr;
    uint16_t *sbibv = nullptr, *pcrcv = nullptr;
    hipEvent_t ev;
    prof_begin(ctx, "decode", &ev);
    if (nblocks <= kSelOnePassBlocks) {
        if (sel_small)
            k_sync_select<kSelStepsSmall><<<(unsigned)nblocks, kSelThreads, 0, st>>>(
                blob_dev, blob_bytes, dsoff, nstreams, channels, bps, ctx->dec_status.as<uint64_t>(), ticket,
                ctx->dec_epoch, nblocks, cpos, cand_cap, ncand, tabs_by_arg ? dsoff : nullptr, stabs);
        else
            k_sync_select<kSelSteps><<<(unsigned)nblocks, kSelThreads, 0, st>>>(
                blob_dev, blob_bytes, dsoff, nstreams, channels, bps, ctx->dec_status.as<uint64_t>(), ticket,
                ctx->dec_epoch, nblocks, cpos, cand_cap, ncand, tabs_by_arg ? dsoff : nullptr, stabs);
    } else {
        // (its own buffer: the one-pass status words must keep their epoch tags)
        // [bcount int32 | bbase int64 | bpos: kSelBlkCap positions per block]
        FRS_HIP(ctx->dec_sel.ensure(sizeof(int64_t) * (size_t)(2 * nblocks + 4 + (int64_t)kSelBlkCap * nblocks)));
        int32_t *bcount = ctx->dec_sel.as<int32_t>();
        int64_t *bbase = ctx->dec_sel.as<int64_t>() + (nblocks + 1) / 2 + 1;
        int64_t *bpos = bbase + nblocks + 1;
        // blocks whose 64 KB lie inside the range take the unguarded instance; the last, partial block its own launch
        const int64_t nfull = std::min<int64_t>(nblocks, lead_bytes / kSelBytes);
        if (pcrc_span) {
            // [BP u32 (nblocks + 1) | bfirst u32 nblocks | bcrc u16 nblocks | bipc u16 32 nblocks | sbib u16 ns + 1 |
            //  pcrc u16 cand_cap]
            const size_t nb = (size_t)nblocks;
            const size_t bytes = 4 * (nb + 1) + 4 * nb + 2 * nb + 2 * kSelBlkCap * nb + 2 * ((size_t)nstreams + 1) +
                                 2 * (size_t)cand_cap + 64;
            FRS_HIP(ctx->dec_crc.ensure(bytes));
            BPv = ctx->dec_crc.as<uint32_t>();
            uint32_t *bfirst = BPv + nb + 1;
            uint16_t *bcrc = reinterpret_cast<uint16_t *>(bfirst + nb);
            uint16_t *bipc = bcrc + nb;
            sbibv = bipc + kSelBlkCap * nb;
            pcrcv = sbibv + nstreams + 1;
            const int lead = (int)(reinterpret_cast<uintptr_t>(blob_dev) & 15);
            FRS_HIP(hipMemsetAsync(bfirst, 0xFF, 4 * nb, st));
            k_bound_mark<<<(unsigned)((nstreams + 255) / 256), 256, 0, st>>>(dsoff, nstreams, lead, bfirst);
            if (nfull)
                k_sync_count<true, true><<<(unsigned)nfull, kSelThreads, 0, st>>>(
                    blob_dev, blob_bytes, dsoff, nstreams, channels, bps, bcount, bpos, bcrc, bipc, bfirst, sbibv, 0);
            if (nblocks > nfull)
                k_sync_count<true, false><<<(unsigned)(nblocks - nfull), kSelThreads, 0, st>>>(
                    blob_dev, blob_bytes, dsoff, nstreams, channels, bps, bcount, bpos, bcrc, bipc, bfirst, sbibv, nfull);
            k_sync_scan<<<1, 1024, 0, st>>>(bcount, bbase, nblocks, ncand, bcrc, BPv);
            k_sync_scatter<true><<<(unsigned)nblocks, kSelThreads, 0, st>>>(blob_dev, blob_bytes, dsoff, nstreams,
                                                                            channels, bps, bbase, cpos, cand_cap,
                                                                            bcount, bpos, pcrcv, BPv, bipc);
        } else {
            if (nfull)
                k_sync_count<false, true><<<(unsigned)nfull, kSelThreads, 0, st>>>(
                    blob_dev, blob_bytes, dsoff, nstreams, channels, bps, bcount, bpos, nullptr, nullptr, nullptr,
                    nullptr, 0);
            if (nblocks > nfull)
                k_sync_count<false, false><<<(unsigned)(nblocks - nfull), kSelThreads, 0, st>>>(
                    blob_dev, blob_bytes, dsoff, nstreams, channels, bps, bcount, bpos, nullptr, nullptr, nullptr,
                    nullptr, nfull);
            k_sync_scan<<<1, 1024, 0, st>>>(bcount, bbase, nblocks, ncand);
            k_sync_scatter<<<(unsigned)nblocks, kSelThreads, 0, st>>>(blob_dev, blob_bytes, dsoff, nstreams, channels,
                                                                      bps, bbase, cpos, cand_cap, bcount, bpos);
        }
    }
    prof_end(ctx, "decode", ev);
    DecOut dout;
    dout.out = out_dev;
    dout.dn = ddn;
    dout.dtype = out_dtype;
    dout.shift = bps > 16 ? 16 : 0;
    int *hv = reinterpret_cast<int *>(reinterpret_cast<char *>(htab) + ((3 * tab + dn_bytes + 15) & ~(size_t)15));
    // small mono ranges (C5 queries): the optimistic pipe decode first (no span check, no chain); only when it
    // declined (counts[6]: a false sync, a frame for the one-lane decoder) do the span check, chain and decode below
    // run, after one more host round trip.  FRS_PIPE_OPT=0 at context creation disables it (tests)
    const bool pipe_opt = pipe && !lane && max_frame < (int64_t)4096 * 256 && ctx->pipe_opt;
    if (pipe_opt) {
        // the last work-group copies the counters into hv (page-locked) itself: no device-to-host copy to wait for
        hv[6] = -1;
        prof_begin(ctx, "decode_frames", &ev);
        k_decode_frames_pipe<true><<<(unsigned)frames, 192, 0, st>>>(blob_dev, dsoff, nstreams, dpoff, cpos, ends,
                                                                     dfbase, dchain, frames, channels, bps, pcm_dev,
                                                                     blocksize, nvalid, dout, ncand, ncand, hv);
        prof_end(ctx, "decode_frames", ev);
        FRS_HIP(hipGetLastError());
        // completion = the last work-group's page-locked counters (hv[6] written last, after system-scope fences over
        // every work-group's output): polled here, a few microseconds before the stream's completion signal; bounded,
        // then the stream synchronisation decides.  FRS_C5_POLL=0: synchronise only
        static const bool poll = !(getenv("FRS_C5_POLL") && atoi(getenv("FRS_C5_POLL")) == 0);
        bool seen = false;
        if (poll && !ctx->prof) {
            const auto t0 = std::chrono::steady_clock::now();
            for (uint32_t k = 0;; k++) {
                if (__atomic_load_n(&hv[6], __ATOMIC_ACQUIRE) != -1) {
                    seen = true;
                    break;
                }
                if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
            }
        }
        if (!seen) FRS_HIP(hipStreamSynchronize(st));
        if (__atomic_load_n(&hv[6], __ATOMIC_ACQUIRE) == -1) {  // (not expected) the epilogue did not run: copy, re-arm
            FRS_HIP(hipMemcpyAsync(hv, ncand, sizeof(int) * 8, hipMemcpyDeviceToHost, st));
            FRS_HIP(hipMemsetAsync(ncand + 8, 0, sizeof(int), st));
            FRS_HIP(hipStreamSynchronize(st));
            if (hv[6] == 0) hv[6] = 1;  // decide by the full path
        }
        if (hv[6] == 0) {
            // the early completion covers output in page-locked host memory (the kernels' system-scope fences); a
            // device-memory output is complete in the stream's order only: synchronise for it
            if (seen) {
                if (out_dev && ctx->is_host_alloc(out_dev, 1)) ctx->unsynced = true;
                else FRS_HIP(hipStreamSynchronize(st));
            }
            prof_collect(ctx);
            if (hv[7] != frames) {
                ctx->err = "decoded " + std::to_string(hv[7]) + " valid frames, expected " + std::to_string(frames);
                return FRS_E_CORRUPT;
            }
            return FRS_OK;
        }
    }
    prof_begin(ctx, "decode_span", &ev);
    // launched before the host knows the candidate count (no mid-query sync): an upper-bound grid strides over
    // *ncand on the device; an overflowing selection makes every later kernel a no-op and is reported below
    if (pcrc_span) {
        k_span_pcrc<<<(unsigned)((std::min<int64_t>(cand_cap, 2 * frames + 256) + 255) / 256), 256, 0, st>>>(
            dsoff, nstreams, cpos, ncand, (int)cand_cap, max_frame, pcrcv, BPv, sbibv,
            (int)(reinterpret_cast<uintptr_t>(blob_dev) & 15), ends, nexti);
    } else if (lane || !pipe) {  // batched (or long multi-channel / 32-bit frames, which the wave form would walk on
                                 // one lane past its LDS stage): one lane per candidate, over an upper-bound grid
        k_span_crc_lane<<<(unsigned)((std::min<int64_t>(cand_cap, 2 * frames + 256) + 255) / 256), 256, 0, st>>>(
            blob_dev, dsoff, nstreams, cpos, ncand, (int)cand_cap, max_frame, ends, nexti);
    } else if (max_frame < (int64_t)4096 * 256) {  // x^(8m) table range of the wave CRC
        const int64_t grid = std::min<int64_t>(cand_cap, std::min<int64_t>(2 * frames + 256, (int64_t)ctx->num_cus * 64));
        k_span_crc_wave<<<(unsigned)grid, 64, 0, st>>>(blob_dev, dsoff, nstreams, cpos, ncand, (int)cand_cap,
                                                       max_frame, ends, nexti);
    } else {
        k_span_crc<<<(unsigned)((cand_cap + 63) / 64), 64, 0, st>>>(blob_dev, dsoff, nstreams, cpos, ncand,
                                                                    (int)cand_cap, max_frame, ends, nexti);
    }
    k_chain_lds<<<nstreams, nstreams == 1 ? 1024 : 64, 0, st>>>(dsoff, nstreams, cpos, ncand, (int)cand_cap, nexti,
                                                                 dfbase, dchain, bad);
    prof_end(ctx, "decode_span", ev);
    prof_begin(ctx, pipe_opt ? "decode_fallback" : "decode_frames", &ev);
    if (lane) {
        FRS_HIP(ctx->dec_fb.ensure(sizeof(int32_t) * (size_t)frames + 64));
        int32_t *fbl = ctx->dec_fb.as<int32_t>();
        int *fbc = ncand + 3;
        const unsigned lg = (unsigned)((frames + 255) / 256);
        // (experiment) FRS_DEC_LANE_LDS: dynamic LDS per work-group, i.e. a cap on the lane decoder's occupancy
        static const size_t lane_lds = getenv("FRS_DEC_LANE_LDS") ? (size_t)atol(getenv("FRS_DEC_LANE_LDS")) : 0;
        const int okind = !fused ? kOutPcm : out_dtype == FRS_DT_I16 ? kOutI16 : out_dtype == FRS_DT_U16 ? kOutU16
                                   : out_dtype == FRS_DT_U8 ? kOutU8 : kOutAny;
#define FRS_LANE(K) k_decode_frames_lane<K><<<lg, 256, lane_lds, st>>>(blob_dev, dsoff, nstreams, dpoff, cpos, ends, dfbase, \
                                                              dchain, frames, bps, pcm_dev, blocksize, nvalid, dout, fbl, fbc)
        switch (okind) {
        case kOutPcm: FRS_LANE(kOutPcm); break;
        case kOutI16: FRS_LANE(kOutI16); break;
        case kOutU16: FRS_LANE(kOutU16); break;
        case kOutU8: FRS_LANE(kOutU8); break;
        default: FRS_LANE(kOutAny); break;
        }
#undef FRS_LANE
        k_decode_frames_wave_list<<<(unsigned)std::min<int64_t>(frames, 4 * (int64_t)ctx->num_cus), 64, 0, st>>>(
            blob_dev, dsoff, nstreams, dpoff, cpos, ends, dfbase, dchain, channels, bps, pcm_dev, blocksize, nvalid,
            dout, fbl, fbc);
    } else if (mcl) {
        FRS_HIP(ctx->dec_fb.ensure(sizeof(int32_t) * (size_t)frames + 64));
        int32_t *fbl = ctx->dec_fb.as<int32_t>();
        int *fbc = ncand + 3;
        int32_t *planar = ctx->dec_pcm.as<int32_t>();
        int8_t *fchass = nullptr;
        if (channels == 2) {
            FRS_HIP(ctx->dec_chass.ensure((size_t)frames + 64));
            fchass = ctx->dec_chass.as<int8_t>();
        }
        const int planar16 = channels >= 3;  // independent channels of <= 16 bits (two: the side is 17 bits)
        if (planar16)
            k_decode_frames_lane<kOutPlanar16, true><<<(unsigned)((frames + 255) / 256), 256, 0, st>>>(
                blob_dev, dsoff, nstreams, dpoff, cpos, ends, dfbase, dchain, frames, bps, pcm_dev, blocksize, nvalid,
                dout, fbl, fbc, channels, planar, fchass);
        else
            k_decode_frames_lane<kOutPcm, true><<<(unsigned)((frames + 255) / 256), 256, 0, st>>>(
                blob_dev, dsoff, nstreams, dpoff, cpos, ends, dfbase, dchain, frames, bps, pcm_dev, blocksize, nvalid,
                dout, fbl, fbc, channels, planar, fchass);
        const int cpf = (blocksize + 255) / 256;
        k_interleave_dn<<<(unsigned)(frames * cpf), 256, 0, st>>>(planar, dpoff, dfbase, nstreams, channels, blocksize,
                                                                 pcm_dev, dout, fchass, cpf, planar16);
        k_decode_frames_wave_list<<<(unsigned)std::min<int64_t>(frames, 4 * (int64_t)ctx->num_cus), 64, 0, st>>>(
            blob_dev, dsoff, nstreams, dpoff, cpos, ends, dfbase, dchain, channels, bps, pcm_dev, blocksize, nvalid,
            dout, fbl, fbc);
    } else if (pipe) {
        k_decode_frames_pipe<<<(unsigned)frames, 192, 0, st>>>(blob_dev, dsoff, nstreams, dpoff, cpos, ends, dfbase,
                                                               dchain, frames, channels, bps, pcm_dev, blocksize, nvalid,
                                                               dout);
    } else
        k_decode_frames_wave<<<(unsigned)frames, 64, 0, st>>>(blob_dev, dsoff, nstreams, dpoff, cpos, ends, dfbase,
                                                              dchain, frames, channels, bps, pcm_dev, blocksize, nvalid,
                                                              dout);
    prof_end(ctx, pipe_opt ? "decode_fallback" : "decode_frames", ev);
    FRS_HIP(hipGetLastError());
    FRS_HIP(hipMemcpyAsync(hv, ncand, sizeof(int) * 8, hipMemcpyDeviceToHost, st));
    FRS_HIP(hipStreamSynchronize(st));
    prof_collect(ctx);
    if (ctx->prof && (lane || mcl)) {  // frames the lane decoder handed to the wave decoder (profile_avg_ms of this name)
        ProfEntry &e = ctx->prof_tab["lane_fallback_frames"];
        e.total_ms += hv[3];
        e.count += 1;
    }
    if ((int64_t)hv[0] > cand_cap) {
        ctx->err = "too many frame sync candidates (" + std::to_string(hv[0]) + " > " + std::to_string(cand_cap) +
                   "): not a FLAC stream of the expected layout";
        return FRS_E_CORRUPT;
    }
    const int valid = hv[1];
    if (hv[2] != 0 || valid != frames) {
        ctx->err = "decoded " + std::to_string(valid) + " valid frames, expected " + std::to_string(frames) +
                   (hv[2] ? " (broken frame chain)" : "");
        return FRS_E_CORRUPT;
    }
    return FRS_OK;
}

int denormalize_job(frs_ctx *ctx, const int32_t *pcm_dev, int64_t n, int pcm_bps, double dmin, double dmax,
                    int32_t out_dtype, void *out_dev) {
    hipStream_t st = ctx->stream;
    if (const int rc = check_unsynced(ctx)) return rc;
    // python-float arithmetic first (data_max - data_min in double), then NEP 50 casts to float32
    const float rng = (float)(dmax - dmin), fmn = (float)dmin;
    const int sh = pcm_bps > 16 ? 16 : 0;
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (n == 0) return FRS_OK;
    switch (out_dtype) {
    case FRS_DT_U8: k_denormalize<uint8_t><<<grid, 256, 0, st>>>(pcm_dev, n, sh, rng, fmn, 0, (uint8_t *)out_dev); break;
    case FRS_DT_U16: k_denormalize<uint16_t><<<grid, 256, 0, st>>>(pcm_dev, n, sh, rng, fmn, 0, (uint16_t *)out_dev); break;
    case FRS_DT_I16: k_denormalize<int16_t><<<grid, 256, 0, st>>>(pcm_dev, n, sh, rng, fmn, 0, (int16_t *)out_dev); break;
    case FRS_DT_I32: k_denormalize<int32_t><<<grid, 256, 0, st>>>(pcm_dev, n, sh, rng, fmn, 0, (int32_t *)out_dev); break;
    case FRS_DT_U32: k_denormalize<uint32_t><<<grid, 256, 0, st>>>(pcm_dev, n, sh, rng, fmn, 0, (uint32_t *)out_dev); break;
    case FRS_DT_F32: k_denormalize<float><<<grid, 256, 0, st>>>(pcm_dev, n, sh, rng, fmn, 1, (float *)out_dev); break;
    case FRS_DT_F64: k_denormalize<double><<<grid, 256, 0, st>>>(pcm_dev, n, sh, rng, fmn, 1, (double *)out_dev); break;
    default: ctx->err = "bad dtype"; return FRS_E_ARG;
    }
    FRS_HIP(hipGetLastError());
    return FRS_OK;
}

}  // namespace frs
