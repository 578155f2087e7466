// frs_common.h -- shared structs and device helpers of the gfx950 spatial-FLAC codec.
//
// Exactness rules (libFLAC 1.4.3 parity, see DESIGN.md "Numerics"):
//   * the whole library is compiled with -ffp-contract=off: libFLAC's x86-64 build has no FMA, so every
//     fp64 multiply/add/divide here is a separate correctly rounded IEEE operation;
//   * fma() is used only where a product is exact (float x float in double: autocorrelation), where it
//     equals the separate multiply + add bit for bit.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace frs {

constexpr int kMaxLpc = 8;
constexpr int kMaxChannels = 8;
constexpr int kMaxPartOrder = 5;   // level 5: max_residual_partition_order
constexpr int kMaxBlock = 4096;    // blocksize fixed by the reference (converter.py:205)

// Per-tile geometry (host-built).
struct TileGeom {
    int64_t r0, c0;      // pixel origin in the raster
    int32_t h, w;        // tile size (edge tiles truncated, cli.py:694-696)
    int64_t frame_base;  // index of the tile's first frame in the job's frame list
    int32_t nframes;
    int32_t partial;     // fast path: 1 + index of the tile's partial last frame among the job's partial frames
                         // (coded by the generic kernels beforehand), 0 when every frame is a full block
};

// Per-tile normalisation parameters (k_tile_stats).
struct TileNorm {
    int64_t imin, imax;  // integer min / max, or order-preserving bits of float min / max
    double dmin, dmax;   // float(np.min(tile)), float(np.max(tile))
    double den;          // (double)(dtype)(max - min)  -- numpy same-kind (wrapping) subtraction
    double rinv;         // RN(1/den) for the exact reciprocal division (fastdiv)
    int32_t has_range;   // max > min
    int32_t mode;        // kNorm*: how the fast kernels normalise this tile
};
constexpr int kNormLut = 0;      // pcm = lut[x - min] (R + 1 <= kLutCap entries, built once per tile)
constexpr int kNormFastDiv = 1;  // no wrap, den <= 65535: RN(2d/den) by reciprocal + 2 FMA (exhaustively exact)
constexpr int kNormSlow = 2;     // anything else (wrapping int16, 32-bit dtypes, floats): IEEE division
constexpr int kNormZero = 3;     // max == min: zeros
constexpr int kLutCap = 4096;    // LUT entries per tile

// Per-subframe decision inputs produced by the analysis kernel (lane = subframe).
struct SubAnalysis {
    int32_t n;           // samples in the block
    int32_t wasted;      // get_wasted_bits_
    int32_t flags;       // kFlag*
    int32_t fixed_order; // fixed predictor guess
    int32_t lpc_order, lpc_prec, lpc_shift;
    int32_t q[kMaxLpc];  // quantised LPC coefficients
    uint32_t fixed_tg;   // fast path: fixed-predictor total of the guessed order (samples 4..n-1, shifted by wasted)
    uint32_t fixed_t1;   // fast path: the order-1 total (constant test: libFLAC's fixed bits[1] == 0)
};
constexpr int kFlagConstant = 1;  // CONSTANT subframe (all samples equal and fixed bits[1] == 0)
constexpr int kFlagFixedOk = 2;   // fixed estimate < subframe bps -> evaluate FIXED
constexpr int kFlagLpcOk = 4;     // LPC estimate < subframe bps and quantisation succeeded
constexpr int kFlagZero = 8;      // every sample of the coded signal is 0 (k_zero_subframes: raw-frames tiles)

// Encode job parameters passed to kernels by value.
struct EncodeParams {
    int64_t row_stride, band_stride;
    int32_t band0, nch;
    int32_t blocksize;
    int32_t sample_rate;
    int32_t bps;          // stream bits per sample: 16 or 32
    int32_t scale_bits;   // 16 -> *32767, 24 -> *8388607 (converter.py:78-83)
    int32_t qlp_precision;
    int32_t slot_words;   // capacity of one frame slot in 32-bit words
    int64_t nframes;
    int32_t ntiles;
    int32_t norm_mode;    // 0 converter.py:56-86, 1 spatial_encoder.py:229-248
    int32_t vec_ok;       // alignment class of the row segments: 16, 8 or 4 bytes (vector loads), 0 = gather
    int32_t nvch;         // coded signals per frame: nch, or 4 for a two-channel stream (L, R, mid, side:
                          // libFLAC's exhaustive mid/side search, stream_encoder.c process_subframes_)
    int32_t max_lpc;      // max_lpc_order of the compression level (0 = fixed predictors only)
    int32_t max_po;       // max_residual_partition_order of the compression level
    int32_t ncand;        // LPC candidates per coded signal from k_analyze_lpc_hi (subdivide_tukey levels), 0 = the
                          // single tukey(0.5) candidate of the SubAnalysis
    int32_t loose_frames; // loose mid/side (levels 1 / 4 on two channels): frames per evaluation, 0 = exhaustive
};

// libFLAC compression-level table (docs/sonos-pyflac.txt:6926-6934): mid/side, loose mid/side, max LPC order, max
// residual partition order, apodization parts (1 = tukey(0.5); n = subdivide_tukey(n): levels 6, 7 -> 2, 8 -> 3)
struct LevelParams {
    int32_t mid_side, loose, max_lpc, max_po, parts;
};
__host__ __device__ inline LevelParams level_params(int level) {
    constexpr LevelParams t[9] = {{0, 0, 0, 3, 1}, {1, 1, 0, 3, 1}, {1, 0, 0, 3, 1}, {0, 0, 6, 4, 1}, {1, 1, 8, 4, 1},
                                  {1, 0, 8, 5, 1}, {1, 0, 8, 6, 2}, {1, 0, 12, 6, 2}, {1, 0, 12, 6, 3}};
    return t[level < 0 ? 0 : level > 8 ? 8 : level];
}
// windows of a subdivide_tukey(parts) apodization (stream_encoder.c process_subframe_ + set_next_subdivide_tukey):
// the full block, 2 partial windows at depth 2, then 2 b per depth b >= 3 (partials and their punch-outs)
__host__ __device__ inline int apod_windows(int parts) {
    int n = 1;
    for (int b = 2; b <= parts; b++) n += b == 2 ? 2 : 2 * b;
    return n;
}
constexpr int kMaxLpcHi = 12;  // max_lpc_order of levels 7 and 8
constexpr int kMaxCand = 9;    // windows of subdivide_tukey(3)
constexpr int kMaxPo = 6;      // max residual partition order (levels 6..8)
// one LPC candidate (one window of the apodization) of a coded signal: quantised predictor or ok = 0
struct LpcCand {
    int32_t order, prec, shift, ok;
    int32_t q[kMaxLpcHi];
};

__host__ __device__ inline int ilog2_u32(uint32_t v) { return 31 - __builtin_clz(v); }
__host__ __device__ inline int ilog2_u64(uint64_t v) { return 63 - __builtin_clzll(v); }

// numpy's float64 -> int32 cast as compiled on x86-64 (cvttsd2si): truncation, out of range or NaN
// gives INT32_MIN ("integer indefinite").  The gfx950 v_cvt_i32_f64 saturates instead, so guard it.
__device__ inline int32_t cast_f64_i32_x86(double v) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT32_MIN;
    return (int32_t)v;
}

// libm-compatible lround (half away from zero) without the floor(x+0.5) double rounding trap.
__device__ inline int64_t lround_exact(double e) {
    double r = trunc(e);
    double f = e - r;  // exact
    if (f >= 0.5) r += 1.0;
    else if (f <= -0.5) r -= 1.0;
    return (int64_t)r;
}

}  // namespace frs

