// frs_encode.hip -- gfx950 encode path: raster tiles -> libFLAC-1.4.3-level-5-identical FLAC frames.
//
// Reference path replaced (Youssef-Harby/flac-raster): cli.py:690-763 (create_streaming tile loop, band 1),
// converter.py:56-86 (normalise to int16), converter.py:185-216 (interleave + pyflac StreamEncoder ->
// libFLAC FLAC__stream_encoder_process_interleaved/finish at level 5, blocksize 4096).
//
// Kernels (one encode job = a set of tiles; every tile is one FLAC stream):
//   k_stats_init / k_tile_stats / k_tile_finalize   per-tile min/max (np.min/np.max) + normalisation params
//   k_analyze        lane = (frame, channel) subframe: wasted bits, fixed-predictor totals and the
//                    tukey(0.5)-windowed autocorrelation (fp64, libFLAC's per-lag sequential order),
//                    Levinson-Durbin, order guess, qlp quantisation        [fp64-VALU bound]
//   k_encode_frames  workgroup = frame: candidate residuals, partition sums, Rice parameters, choice,
//                    exact bit positions (block prefix scan) and LDS bit packing into a frame slot
//   k_scan_sizes     exclusive scan of frame sizes -> arena offsets (tiles are consecutive frame runs)
//   k_compact        workgroup = frame: CRC-16 (parallel GF(2) combine) + copy slot -> arena offset

#include <type_traits>

#include <cstring>
#include <unistd.h>

#include "frs_internal.h"

namespace frs {

// ------------------------------------------------------------------------------------------- dtypes
template <int DT> struct Elem;
template <> struct Elem<FRS_DT_U8> { using T = uint8_t; static constexpr bool is_float = false; };
template <> struct Elem<FRS_DT_U16> { using T = uint16_t; static constexpr bool is_float = false; };
template <> struct Elem<FRS_DT_I16> { using T = int16_t; static constexpr bool is_float = false; };
template <> struct Elem<FRS_DT_I32> { using T = int32_t; static constexpr bool is_float = false; };
template <> struct Elem<FRS_DT_U32> { using T = uint32_t; static constexpr bool is_float = false; };
template <> struct Elem<FRS_DT_F32> { using T = float; static constexpr bool is_float = true; };
template <> struct Elem<FRS_DT_F64> { using T = double; static constexpr bool is_float = true; };

// order-preserving int64 key of a double (for atomic min/max of float rasters)
__device__ inline int64_t f2key(double v) {
    int64_t b = __double_as_longlong(v);
    return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFll);
}
__host__ __device__ inline double key2f(int64_t k) {
    int64_t b = k >= 0 ? k : (k ^ 0x7FFFFFFFFFFFFFFFll);
    double d;
    memcpy(&d, &b, 8);
    return d;
}

template <int DT> __device__ inline int64_t elem_key(typename Elem<DT>::T v) {
    if constexpr (Elem<DT>::is_float) return f2key((double)v);
    else return (int64_t)v;
}

// converter.py:56-86 for one element.  numpy 2 (NEP 50): x - min and max - min are evaluated in the
// raster dtype (wrapping), promoted to float64 by 2.0*(...); the cast to int16/int32 truncates.
// spatial_encoder.py:229-248 then pyflac's astype(int32): float32 arithmetic, truncation to int32.
template <int DT> __device__ inline int32_t spatial_norm(typename Elem<DT>::T x) {
    if constexpr (DT == FRS_DT_U8) return cast_f64_i32_x86((double)__fdiv_rn(__fsub_rn((float)x, 127.5f), 127.5f));
    else if constexpr (DT == FRS_DT_U16) return cast_f64_i32_x86((double)__fdiv_rn(__fsub_rn((float)x, 32767.5f), 32767.5f));
    else if constexpr (DT == FRS_DT_I16) return cast_f64_i32_x86((double)__fdiv_rn((float)x, 32767.0f));
    else if constexpr (DT == FRS_DT_I32) return cast_f64_i32_x86((double)__fdiv_rn((float)x, 2147483647.0f));
    else if constexpr (DT == FRS_DT_F32) return cast_f64_i32_x86((double)fminf(fmaxf(x, -1.0f), 1.0f));
    else return 0;  // other dtypes are rejected by the host (pyflac would see a 64-bit itemsize)
}

template <int DT> struct Normalizer {
    using T = typename Elem<DT>::T;
    T mn;
    double den;
    double rinv;  // 1 / den for the fast exact division (tiles in kNormLut / kNormFastDiv mode)
    double scale;
    int has_range;
    int bps16;
    int spatial;
    int fastdiv;
    __device__ inline int32_t operator()(T x) const {
        if (spatial) return spatial_norm<DT>(x);
        if constexpr (DT == FRS_DT_F32) {
            float v = x * 8388607.0f;  // float data used as-is, float32 product (converter.py:61-64, 81)
            return cast_f64_i32_x86((double)v);
        } else if constexpr (DT == FRS_DT_F64) {
            return cast_f64_i32_x86(x * 8388607.0);
        } else {
            if (!has_range) return 0;
            T d = (T)((int64_t)x - (int64_t)mn);
            double v;
            if (fastdiv) {  // RN(2d / den) by reciprocal + two FMAs: exhaustively exact for d <= den <= 65535
                const double a = 2.0 * (double)d;
                const double q0 = a * rinv;
                v = fma(fma(-q0, den, a), rinv, q0) - 1.0;
            } else {
                v = (2.0 * (double)d) / den - 1.0;
            }
            v = v * scale;
            int32_t c = cast_f64_i32_x86(v);
            return bps16 ? (int32_t)(int16_t)c : c;
        }
    }
};

template <int DT> __device__ inline Normalizer<DT> make_norm(const TileNorm &tn, int scale_bits, int norm_mode) {
    Normalizer<DT> nz;
    nz.spatial = norm_mode == 1;
    using T = typename Elem<DT>::T;
    if constexpr (!Elem<DT>::is_float) nz.mn = (T)tn.imin;
    else nz.mn = (T)0;
    nz.den = tn.den;
    nz.rinv = tn.rinv;
    nz.fastdiv = tn.mode == kNormLut || tn.mode == kNormFastDiv;
    nz.scale = scale_bits == 16 ? 32767.0 : 8388607.0;
    nz.has_range = tn.has_range;
    nz.bps16 = scale_bits == 16;
    return nz;
}

// tile of frame f (binary search over frame_base)
__device__ inline int tile_of_frame(const TileGeom *tiles, int ntiles, int64_t f) {
    int lo = 0, hi = ntiles - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (tiles[mid].frame_base <= f) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// frame -> tile table for the fast kernels (one load instead of a binary search per frame)
__global__ void k_frame_tile(const TileGeom *tiles, int ntiles, int32_t *ftile) {
    const int t = blockIdx.x;
    if (t >= ntiles) return;
    const TileGeom g = tiles[t];
    for (int i = threadIdx.x; i < g.nframes; i += blockDim.x) ftile[g.frame_base + i] = t;
}

// ------------------------------------------------------------------------------------ tile stats
__global__ void k_stats_init(TileNorm *norms, int ntiles) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ntiles) {
        norms[t].imin = INT64_MAX;
        norms[t].imax = INT64_MIN;
    }
}

template <int DT>
__global__ void __launch_bounds__(256) k_tile_stats(const typename Elem<DT>::T *raster, EncodeParams P,
                                                   const TileGeom *tiles, TileNorm *norms, int splits) {
    const int t = blockIdx.y;
    const TileGeom g = tiles[t];
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    const int64_t rows = (int64_t)g.h * P.nch;
    for (int64_t rr = blockIdx.x; rr < rows; rr += splits) {
        const int ch = (int)(rr / g.h);
        const int64_t r = rr - (int64_t)ch * g.h;
        const typename Elem<DT>::T *row =
            raster + (int64_t)(P.band0 + ch) * P.band_stride + (g.r0 + r) * P.row_stride + g.c0;
        for (int c = threadIdx.x; c < g.w; c += blockDim.x) {
            int64_t k = elem_key<DT>(row[c]);
            lo = k < lo ? k : lo;
            hi = k > hi ? k : hi;
        }
    }
    // wave reduce then one atomic per wave
    for (int o = 32; o > 0; o >>= 1) {
        int64_t l2 = __shfl_xor(lo, o), h2 = __shfl_xor(hi, o);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin((long long *)&norms[t].imin, (long long)lo);
        atomicMax((long long *)&norms[t].imax, (long long)hi);
    }
}

// vectorised min/max for 8/16-bit integer rasters whose tile rows are 16-byte aligned runs: 16-B loads,
// packed 16-bit min/max (v_pk_min_i16 / v_pk_min_u16), 4 loads in flight per thread
typedef short v2i16 __attribute__((ext_vector_type(2)));
typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));
template <int DT>
__global__ void __launch_bounds__(256) k_tile_stats_vec(const typename Elem<DT>::T *raster, EncodeParams P,
                                                       const TileGeom *tiles, TileNorm *norms, int splits) {
    using T = typename Elem<DT>::T;
    static_assert(sizeof(T) <= 2, "16-bit or narrower");
    const int t = blockIdx.y;
    const TileGeom g = tiles[t];
    const int nvec = (int)((int64_t)g.w * sizeof(T) / 16);  // 16-B vectors per row
    const int64_t rows = (int64_t)g.h * P.nch;
    const int64_t r0 = rows * blockIdx.x / splits, r1 = rows * (blockIdx.x + 1) / splits;
    const int64_t total = (r1 - r0) * nvec;
    // packed accumulators: (lo, hi) halves; u8 values are widened into u16 lanes
    using V = std::conditional_t<std::is_signed_v<T>, v2i16, v2u16>;
    using E16 = std::conditional_t<std::is_signed_v<T>, short, unsigned short>;
    V vmin = (V)(std::is_signed_v<T> ? (E16)32767 : (E16)65535), vmax = (V)(std::is_signed_v<T> ? (E16)-32768 : (E16)0);
    auto fold = [&](uint32_t w) {
        if constexpr (sizeof(T) == 2) {
            const V v = __builtin_bit_cast(V, w);
            vmin = __builtin_elementwise_min(vmin, v);
            vmax = __builtin_elementwise_max(vmax, v);
        } else {
            const V a = __builtin_bit_cast(V, w & 0x00FF00FFu), b = __builtin_bit_cast(V, (w >> 8) & 0x00FF00FFu);
            vmin = __builtin_elementwise_min(vmin, __builtin_elementwise_min(a, b));
            vmax = __builtin_elementwise_max(vmax, __builtin_elementwise_max(a, b));
        }
    };
    auto addr = [&](int64_t idx) -> const uint4 * {
        const int64_t rr = r0 + idx / nvec;
        const int v = (int)(idx - (idx / nvec) * nvec);
        const int ch = (int)(rr / g.h);
        const int64_t r = rr - (int64_t)ch * g.h;
        return reinterpret_cast<const uint4 *>(raster + (int64_t)(P.band0 + ch) * P.band_stride +
                                               (g.r0 + r) * P.row_stride + g.c0) + v;
    };
    int64_t idx = threadIdx.x;
    for (; idx + 3 * 256 < total; idx += 4 * 256) {
        uint4 q[4];
#pragma unroll
        for (int u = 0; u < 4; u++) q[u] = *addr(idx + u * 256);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            fold(q[u].x);
            fold(q[u].y);
            fold(q[u].z);
            fold(q[u].w);
        }
    }
    for (; idx < total; idx += 256) {
        const uint4 q = *addr(idx);
        fold(q.x);
        fold(q.y);
        fold(q.z);
        fold(q.w);
    }
    int32_t lo = min((int32_t)vmin.x, (int32_t)vmin.y), hi = max((int32_t)vmax.x, (int32_t)vmax.y);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
    }
    if ((threadIdx.x & 63) == 0 && total > 0) {
        atomicMin((long long *)&norms[t].imin, (long long)lo);
        atomicMax((long long *)&norms[t].imax, (long long)hi);
    }
}

// normalisation parameters of a tile from its min/max (converter.py:88-110): data_min/data_max, the range in
// the dtype, and the fast-path mode (LUT / zeros / fast division / exact division)
template <int DT> __device__ inline void tile_norm_finalize(TileNorm &n, int norm_mode, int scale_bits) {
    using T = typename Elem<DT>::T;
    n.mode = kNormSlow;
    n.rinv = 0.0;
    if constexpr (Elem<DT>::is_float) {
        n.dmin = key2f(n.imin);
        n.dmax = key2f(n.imax);
        n.den = 0.0;
        n.has_range = n.dmax > n.dmin;
    } else {
        n.dmin = (double)n.imin;
        n.dmax = (double)n.imax;
        n.has_range = n.imax > n.imin;
        n.den = (double)(T)(n.imax - n.imin);  // data_max - data_min in the dtype (wraps for int16)
        const int64_t R = n.imax - n.imin;
        const bool nowrap = (int64_t)(T)R == R;  // x - min and max - min never wrap in the dtype
        if (norm_mode == 0 && scale_bits == 16) {
            if (!n.has_range) n.mode = kNormZero;
            else if (nowrap && R + 1 <= kLutCap) n.mode = kNormLut;
            else if (nowrap && R <= 65535) n.mode = kNormFastDiv;
            n.rinv = 1.0 / n.den;
        }
    }
}

template <int DT> __global__ void k_tile_finalize(TileNorm *norms, int ntiles, int norm_mode, int scale_bits) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    TileNorm n = norms[t];
    tile_norm_finalize<DT>(n, norm_mode, scale_bits);
    norms[t] = n;
}

// ------------------------------------------------------------------------------- LPC helpers (fp64)
// FLAC__lpc_compute_lp_coefficients (lpc.c): returns the number of orders computed (early stop on
// err == 0); err[i] = prediction error after order i+1.
template <int MAXO = kMaxLpc>
__device__ int levinson_errors(const double *autoc, int max_order, double *err) {
    double lpc[MAXO];
    double e = autoc[0];
    int done = max_order;
#pragma unroll
    for (int i = 0; i < MAXO; i++) {
        if (i < done) {
            double r = -autoc[i + 1];
#pragma unroll
            for (int j = 0; j < MAXO; j++)
                if (j < i) r -= lpc[j] * autoc[i - j];
            r /= e;
            lpc[i] = r;
#pragma unroll
            for (int j = 0; j < MAXO / 2; j++) {
                if (j < (i >> 1)) {
                    double tmp = lpc[j];
                    lpc[j] += r * lpc[i - 1 - j];
                    lpc[i - 1 - j] += r * tmp;
                }
            }
            if (i & 1) lpc[i >> 1] += lpc[i >> 1] * r;
            e *= (1.0 - r * r);
            err[i] = e;
            if (e == 0.0) done = i + 1;
        }
    }
    return done;
}

// same recursion, returns the predictor coefficients of order `order` as floats (lp_coeff[order-1])
template <int MAXO = kMaxLpc>
__device__ void levinson_coefs(const double *autoc, int order, float *lp) {
    double lpc[MAXO];
    double e = autoc[0];
#pragma unroll
    for (int i = 0; i < MAXO; i++) {
        if (i < order) {
            double r = -autoc[i + 1];
#pragma unroll
            for (int j = 0; j < MAXO; j++)
                if (j < i) r -= lpc[j] * autoc[i - j];
            r /= e;
            lpc[i] = r;
#pragma unroll
            for (int j = 0; j < MAXO / 2; j++) {
                if (j < (i >> 1)) {
                    double tmp = lpc[j];
                    lpc[j] += r * lpc[i - 1 - j];
                    lpc[i - 1 - j] += r * tmp;
                }
            }
            if (i & 1) lpc[i >> 1] += lpc[i >> 1] * r;
            e *= (1.0 - r * r);
        }
    }
#pragma unroll
    for (int j = 0; j < MAXO; j++) lp[j] = j < order ? (float)(-lpc[j]) : 0.0f;
}

// FLAC__lpc_compute_expected_bits_per_residual_sample_with_error_scale
__device__ inline double expected_bits(double lpc_error, double error_scale) {
    if (lpc_error > 0.0) {
        double b = 0.5 * log(error_scale * lpc_error) / M_LN2;
        return b >= 0.0 ? b : 0.0;
    } else if (lpc_error < 0.0) {
        return 1e32;
    }
    return 0.0;
}

// ------------------------------------------------------------------------------------ k_analyze
// One lane per subframe; lanes of a wave walk their blocks in lockstep so the window sample is uniform.
// The level-5 decisions of one subframe from its sums (stream_encoder.c process_subframe_ up to the encode):
// wasted bits, constant test, fixed-predictor guess (fixed.c, totals over samples 4..n-1), LPC order by expected
// bits, Levinson coefficients and their quantisation (lpc.c).  acc = windowed autocorrelation lags 0..8, t = fixed
// totals of orders 0..4, or_acc = OR of the samples, diff = OR of (x ^ x[0]).
// extra = 1 for the side signal of a two-channel stream (subframe_bps_mid_side[1] = bps - wasted + 1).
template <bool WIDE>
__device__ inline SubAnalysis generic_decide(const double *acc, const uint64_t *tt, uint64_t or_acc, uint64_t diff,
                                             int n, const EncodeParams &P, int extra = 0) {
    const uint64_t t0 = tt[0], t1 = tt[1], t2 = tt[2], t3 = tt[3], t4 = tt[4];
    SubAnalysis A;
    A.n = n;
    int w = 0;
    if (or_acc) w = __builtin_ctzll(or_acc);
    if (w > P.bps) w = P.bps;
    const int sbps = P.bps - w + extra;
    A.wasted = w;
    A.flags = 0;
    A.fixed_order = 0;
    A.lpc_order = 0;
    A.lpc_prec = 0;
    A.lpc_shift = 0;
#pragma unroll
    for (int j = 0; j < kMaxLpc; j++) A.q[j] = 0;

    if (n > 4) {
        // fixed predictor guess (FLAC__fixed_compute_best_predictor on the shifted signal)
        float fb[5];
        int guess;
        {
            const uint64_t T0 = t0 >> w, T1 = t1 >> w, T2 = t2 >> w, T3 = t3 >> w, T4 = t4 >> w;
            uint64_t m = T1 < T2 ? T1 : T2;
            m = m < T3 ? m : T3;
            m = m < T4 ? m : T4;
            if (T0 <= m) guess = 0;
            else {
                uint64_t m2_ = T2 < T3 ? T2 : T3;
                m2_ = m2_ < T4 ? m2_ : T4;
                if (T1 <= m2_) guess = 1;
                else if (T2 <= (T3 < T4 ? T3 : T4)) guess = 2;
                else if (T3 <= T4) guess = 3;
                else guess = 4;
            }
            const uint64_t Ts[5] = {T0, T1, T2, T3, T4};
            const double dn = (double)(n - 4);
#pragma unroll
            for (int k = 0; k < 5; k++)
                fb[k] = (float)(Ts[k] > 0 ? log(M_LN2 * (double)Ts[k] / dn) / M_LN2 : 0.0);
        }
        // 32-bit streams: constant / fixed decisions come from k_analyze_fixed_wide (limit_residual
        // estimator); a constant block there clears the LPC candidate again.
        if (!WIDE && fb[1] == 0.0f && diff == 0) {
            A.flags |= kFlagConstant;
        } else {
            A.fixed_order = guess;
            float fg = fb[0];
#pragma unroll
            for (int k = 1; k < 5; k++)
                if (k == guess) fg = fb[k];
            if (!(fg >= (float)sbps)) A.flags |= kFlagFixedOk;

            int max_order = P.max_lpc < n ? P.max_lpc : n - 1;  // level 5: kMaxLpc
            // autocorrelation of the shifted signal = autoc * 4^-w exactly (power-of-two scaling)
            double autoc[kMaxLpc + 1];
            const double sc = ldexp(1.0, -2 * w);
#pragma unroll
            for (int l = 0; l <= kMaxLpc; l++) autoc[l] = acc[l] * sc;
            if (max_order > 0 && autoc[0] != 0.0) {
                double err[kMaxLpc];
                const int mo = levinson_errors(autoc, max_order, err);
                // FLAC__lpc_compute_best_order with overhead = subframe_bps + qlp_coeff_precision
                const double es = 0.5 / (double)n;
                const int ovh = sbps + P.qlp_precision;
                int best = 0;
                double best_bits = (double)(unsigned)(-1);
#pragma unroll
                for (int i = 0; i < kMaxLpc; i++) {
                    if (i < mo) {
                        const int o = i + 1;
                        const double b = expected_bits(err[i], es) * (double)(n - o) + (double)(o * ovh);
                        if (b < best_bits) {
                            best = i;
                            best_bits = b;
                        }
                    }
                }
                const int o = best + 1;
                double eo = err[0];
#pragma unroll
                for (int i = 1; i < kMaxLpc; i++)
                    if (i == best) eo = err[i];
                const double lbits = expected_bits(eo, 0.5 / (double)(n - o));
                if (!(lbits >= (double)sbps)) {
                    int prec = P.qlp_precision;
                    if (sbps <= 17) {
                        const int lim = 32 - sbps - ilog2_u32((uint32_t)o);
                        prec = lim < prec ? lim : prec;
                    }
                    float lp[kMaxLpc];
                    levinson_coefs(autoc, o, lp);
                    // FLAC__lpc_quantize_coefficients
                    const int pm1 = prec - 1;
                    const int32_t qmax = (1 << pm1) - 1, qmin = -(1 << pm1);
                    double cmax = 0.0;
#pragma unroll
                    for (int j = 0; j < kMaxLpc; j++)
                        if (j < o) {
                            const double d = fabs((double)lp[j]);
                            if (d > cmax) cmax = d;
                        }
                    if (cmax > 0.0) {
                        const int log2cmax = ilogb(cmax);  // frexp exponent - 1
                        int shift = pm1 - log2cmax - 1;
                        bool ok = true;
                        if (shift > 15) shift = 15;
                        else if (shift < -16) ok = false;
                        if (ok) {
                            double error = 0.0;
                            if (shift >= 0) {
                                const float m = (float)(1 << shift);
#pragma unroll
                                for (int j = 0; j < kMaxLpc; j++)
                                    if (j < o) {
                                        error += (double)(lp[j] * m);
                                        int64_t qi = lround_exact(error);
                                        if (qi > qmax) qi = qmax;
                                        else if (qi < qmin) qi = qmin;
                                        error -= (double)qi;
                                        A.q[j] = (int32_t)qi;
                                    }
                            } else {
                                const float m = (float)(1 << (-shift));
#pragma unroll
                                for (int j = 0; j < kMaxLpc; j++)
                                    if (j < o) {
                                        error += (double)(lp[j] / m);
                                        int64_t qi = lround_exact(error);
                                        if (qi > qmax) qi = qmax;
                                        else if (qi < qmin) qi = qmin;
                                        error -= (double)qi;
                                        A.q[j] = (int32_t)qi;
                                    }
                                shift = 0;
                            }
                            A.lpc_order = o;
                            A.lpc_prec = prec;
                            A.lpc_shift = shift;
                            A.flags |= kFlagLpcOk;
                        }
                    }
                }
            }
        }
    }
    return A;
}

// Coded signal v of a frame at sample pointer p (band0's pixel): channel v when the stream is coded independently;
// for a two-channel stream's mid/side pass (ST) v = 0 left, 1 right, 2 mid = (L + R) >> 1, 3 side = L - R (one bit
// wider; 33 bits for a 32-bit stream: integer_signal_33bit_side), as FLAC__stream_encoder_process_interleaved
// forms them from the unshifted samples.
template <int DT, bool ST, typename XT>
__device__ inline XT coded_sample(const typename Elem<DT>::T *p, int64_t band_stride, const Normalizer<DT> &nz,
                                  int v) {
    if constexpr (!ST) {
        return (XT)nz(p[(int64_t)v * band_stride]);
    } else {
        if (v < 2) return (XT)nz(p[(int64_t)v * band_stride]);
        const int64_t a = nz(p[0]), b = nz(p[band_stride]);
        return v == 2 ? (XT)((a + b) >> 1) : (XT)(a - b);
    }
}

template <int DT, bool WIDE, bool ST = false>
__global__ void __launch_bounds__(128) k_analyze(const typename Elem<DT>::T *raster, EncodeParams P,
                                                const TileGeom *tiles, const TileNorm *norms,
                                                const float *__restrict__ window, SubAnalysis *out,
                                                const int64_t *__restrict__ flist, int64_t nlist,
                                                const uint8_t *__restrict__ skip = nullptr) {
    // flist: the frames to analyse (the fast path's partial last frames), nullptr = every frame of the job.
    // skip: subframes already analysed (k_zero_subframes), nullptr = none.
    // One lane per coded signal: (frame, channel), or (frame, L/R/M/S) for a two-channel stream (ST).
    using T = typename Elem<DT>::T;
    // sample type: 32 bits except the 33-bit side signal of a 32-bit stereo stream
    using XA = std::conditional_t<ST && WIDE, int64_t, int32_t>;
    using UA = std::make_unsigned_t<XA>;
    const int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nsub = (flist ? nlist : P.nframes) * P.nvch;
    const bool inrange = li < nsub;
    const int64_t fi = inrange ? li / P.nvch : 0;
    const int ch = inrange ? (int)(li - fi * P.nvch) : 0;
    const int64_t f = flist ? flist[fi] : fi;
    const int64_t sub = f * P.nvch + ch;
    const bool live = inrange && !(skip && skip[sub]);
    if (skip && __ballot(live) == 0) return;  // (wave-uniform: a wave of skipped subframes walks nothing)
    const int t = tile_of_frame(tiles, P.ntiles, f);
    const TileGeom g = tiles[t];
    const int64_t s0 = (f - g.frame_base) * P.blocksize;
    const int64_t tile_px = (int64_t)g.h * g.w;
    const int n = live ? (int)((tile_px - s0) < P.blocksize ? (tile_px - s0) : P.blocksize) : 0;
    const Normalizer<DT> nz = make_norm<DT>(norms[t], P.scale_bits, P.norm_mode);

    int64_t row = s0 / g.w;
    int col = (int)(s0 - row * g.w);
    const T *rowp = raster + (int64_t)(P.band0 + (ST ? 0 : ch)) * P.band_stride + (g.r0 + row) * P.row_stride + g.c0;

    UA or_acc = 0, diff = 0;
    XA x0 = 0;
    int32_t x1 = 0, p1 = 0, p2 = 0, p3 = 0;
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    double acc[kMaxLpc + 1];
#pragma unroll
    for (int l = 0; l <= kMaxLpc; l++) acc[l] = 0.0;
    double prev[8], cur[8];
#pragma unroll
    for (int j = 0; j < 8; j++) prev[j] = 0.0;

    const int nloop = P.blocksize;  // uniform trip count; lanes with shorter blocks are predicated off
    // raw sample i (< n) at the row cursor, which then advances
    auto fetch = [&](int i) -> T {
        T v = T(0);
        if (i < n) {
            v = rowp[col];
            if (++col == g.w) {
                col = 0;
                rowp += P.row_stride;
            }
        }
        return v;
    };
    // coded sample i (< n) of a stereo lane at the row cursor, which then advances
    auto fetch_st = [&](int i) -> XA {
        XA v = 0;
        if (i < n) {
            v = coded_sample<DT, true, XA>(rowp + col, P.band_stride, nz, ch);
            if (++col == g.w) {
                col = 0;
                rowp += P.row_stride;
            }
        }
        return v;
    };
    auto block8 = [&](int i0, const XA *xin) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int i = i0 + j;
            XA x = 0;
            if (i < n) {
                x = xin[j];
                if (i == 0) x0 = x;
                or_acc |= (UA)x;
                diff |= (UA)(x ^ x0);
                if constexpr (!WIDE) {
                    // 16-bit streams: |e_k| < 2^21 (17-bit side), totals over samples 4..n-1 (fixed.c, data+4)
                    const int32_t xs = (int32_t)x;
                    const int32_t e1 = xs - x1, e2 = e1 - p1, e3 = e2 - p2, e4 = e3 - p3;
                    if (i >= 4) {
                        t0 += (uint32_t)abs(xs);
                        t1 += (uint32_t)abs(e1);
                        t2 += (uint32_t)abs(e2);
                        t3 += (uint32_t)abs(e3);
                        t4 += (uint32_t)abs(e4);
                    }
                    p3 = e3;
                    p2 = e2;
                    p1 = e1;
                    x1 = xs;
                }
            }
            // inactive lanes have x == 0 -> contribute exact zeros; window index is wave-uniform
            cur[j] = (double)((float)x * window[i]);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
#pragma unroll
            for (int l = 0; l <= kMaxLpc; l++) {
                const double other = (j - l >= 0) ? cur[j - l] : prev[8 + j - l];
                acc[l] = fma(cur[j], other, acc[l]);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) prev[j] = cur[j];
    };
    for (int i0 = 0; i0 < nloop; i0 += 8) {
        XA xin[8];
        if constexpr (ST) {
#pragma unroll
            for (int j = 0; j < 8; j++) xin[j] = fetch_st(i0 + j);
        } else {
            T raw[8];
#pragma unroll
            for (int j = 0; j < 8; j++) raw[j] = fetch(i0 + j);
#pragma unroll
            for (int j = 0; j < 8; j++) xin[j] = (i0 + j < n) ? (XA)nz(raw[j]) : (XA)0;
        }
        block8(i0, xin);
    }
    if (!live) return;

    const uint64_t tt[5] = {t0, t1, t2, t3, t4};
    out[sub] = generic_decide<WIDE>(acc, tt, (uint64_t)or_acc, (uint64_t)diff, n, P, (ST && ch == 3) ? 1 : 0);
}

// One LPC candidate from a window's autocorrelation (of the wasted-bit-shifted signal): stream_encoder.c
// process_subframe_'s LPC branch for one apodization window without exhaustive or precision search --
// FLAC__lpc_compute_lp_coefficients, FLAC__lpc_compute_best_order (overhead subframe_bps + qlp precision), the
// expected-bits test against subframe_bps, the 32-bit-decode precision clamp, FLAC__lpc_quantize_coefficients.
template <int MAXO>
__device__ inline void lpc_candidate(const double *autoc, int max_order, int n, int sbps, const EncodeParams &P,
                                     LpcCand &c) {
    c.ok = 0;
    c.order = 0;
    c.prec = 0;
    c.shift = 0;
#pragma unroll
    for (int j = 0; j < kMaxLpcHi; j++) c.q[j] = 0;
    if (max_order <= 0 || autoc[0] == 0.0) return;
    double err[MAXO];
    const int mo = levinson_errors<MAXO>(autoc, max_order, err);
    const double es = 0.5 / (double)n;
    const int ovh = sbps + P.qlp_precision;
    int best = 0;
    double best_bits = (double)(unsigned)(-1);
#pragma unroll
    for (int i = 0; i < MAXO; i++) {
        if (i < mo) {
            const int o = i + 1;
            const double b = expected_bits(err[i], es) * (double)(n - o) + (double)(o * ovh);
            if (b < best_bits) {
                best = i;
                best_bits = b;
            }
        }
    }
    const int o = best + 1;
    double eo = err[0];
#pragma unroll
    for (int i = 1; i < MAXO; i++)
        if (i == best) eo = err[i];
    if (expected_bits(eo, 0.5 / (double)(n - o)) >= (double)sbps) return;
    int prec = P.qlp_precision;
    if (sbps <= 17) {
        const int lim = 32 - sbps - ilog2_u32((uint32_t)o);
        prec = lim < prec ? lim : prec;
    }
    float lp[MAXO];
    levinson_coefs<MAXO>(autoc, o, lp);
    const int pm1 = prec - 1;
    const int32_t qmax = (1 << pm1) - 1, qmin = -(1 << pm1);
    double cmax = 0.0;
#pragma unroll
    for (int j = 0; j < MAXO; j++)
        if (j < o) {
            const double d = fabs((double)lp[j]);
            if (d > cmax) cmax = d;
        }
    if (!(cmax > 0.0)) return;
    int shift = pm1 - ilogb(cmax) - 1;
    if (shift > 15) shift = 15;
    else if (shift < -16) return;
    double error = 0.0;
    const float m = (float)(1 << (shift >= 0 ? shift : -shift));
#pragma unroll
    for (int j = 0; j < MAXO; j++)
        if (j < o) {
            error += shift >= 0 ? (double)(lp[j] * m) : (double)(lp[j] / m);
            int64_t qi = lround_exact(error);
            if (qi > qmax) qi = qmax;
            else if (qi < qmin) qi = qmin;
            error -= (double)qi;
            c.q[j] = (int32_t)qi;
        }
    c.order = o;
    c.prec = prec;
    c.shift = shift >= 0 ? shift : 0;
    c.ok = 1;
}

// k_analyze_lpc_hi: the LPC candidates of the subdivide_tukey(parts) levels (6..8), one lane per coded signal (as
// k_analyze, which has produced the signal's wasted bits and fixed-predictor decisions with max_lpc 0).  libFLAC
// evaluates one LPC subframe per window of the apodization (stream_encoder.c process_subframe_ with
// set_next_subdivide_tukey): window 0 is the whole block under tukey(0.5 / parts); at depth b = 2 .. parts the block
// is cut into b parts (part j starts at (j n) / b), each windowed by the rising then the falling half of that window
// (lpc.c FLAC__lpc_window_data_partial, n / b / 2 samples each, autocorrelation over n / b samples); from depth 3
// every partial window is followed by its punch-out, whose autocorrelation is the whole block's minus the part's.
// Parts of n / b <= 32 samples are skipped.  Each window's autocorrelation is summed per lag in sample order (as
// FLAC__lpc_compute_autocorrelation), so the candidates match the oracle's (oracle/flac_oracle.c decide_subframe).
template <int DT, bool WIDE, bool ST = false>
__global__ void __launch_bounds__(128) k_analyze_lpc_hi(const typename Elem<DT>::T *raster, EncodeParams P,
                                                       const TileGeom *tiles, const TileNorm *norms,
                                                       const float *__restrict__ window, const SubAnalysis *ana,
                                                       LpcCand *cand, int parts) {
    using T = typename Elem<DT>::T;
    using XA = std::conditional_t<ST && WIDE, int64_t, int32_t>;
    const int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= P.nframes * P.nvch) return;
    const int64_t f = li / P.nvch;
    const int ch = (int)(li - f * P.nvch);
    const int t = tile_of_frame(tiles, P.ntiles, f);
    const TileGeom g = tiles[t];
    const int64_t s0 = (f - g.frame_base) * P.blocksize;
    const int64_t tile_px = (int64_t)g.h * g.w;
    const int n = (int)((tile_px - s0) < P.blocksize ? (tile_px - s0) : P.blocksize);
    const Normalizer<DT> nz = make_norm<DT>(norms[t], P.scale_bits, P.norm_mode);
    const SubAnalysis A = ana[li];
    LpcCand *out = cand + li * P.ncand;
    LpcCand none;
    none.ok = 0;
    none.order = none.prec = none.shift = 0;
#pragma unroll
    for (int j = 0; j < kMaxLpcHi; j++) none.q[j] = 0;
    for (int c = 0; c < P.ncand; c++) out[c] = none;
    const int w = A.wasted;
    const int sbps = P.bps - w + ((ST && ch == 3) ? 1 : 0);
    const int max_order = P.max_lpc < n ? P.max_lpc : n - 1;
    if (n <= 4 || (A.flags & kFlagConstant) || max_order <= 0) return;
    const double sc = ldexp(1.0, -2 * w);  // autocorrelation of the shifted signal (power-of-two scaling: exact)
    const T *band = raster + (int64_t)(P.band0 + (ST ? 0 : ch)) * P.band_stride + g.r0 * P.row_stride + g.c0;
    auto sample = [&](int i) -> XA {  // coded sample i of the frame (unshifted)
        const int64_t q = s0 + i, r = q / g.w;
        const T *pp = band + r * P.row_stride + (q - r * g.w);
        if constexpr (ST) return coded_sample<DT, true, XA>(pp, P.band_stride, nz, ch);
        else return (XA)nz(*pp);
    };
    // autocorrelation (lags 0..12, scaled) of `len` windowed samples from `start`: ps == 0 the whole block with
    // window[i], else a part with the rising half window[0, ps) then the falling half window[n - ps, n)
    auto autoc_of = [&](int start, int len, int ps, double *ac) {
        double h[kMaxLpcHi];
#pragma unroll
        for (int l = 0; l <= kMaxLpcHi; l++) ac[l] = 0.0;
#pragma unroll
        for (int l = 0; l < kMaxLpcHi; l++) h[l] = 0.0;
        for (int s = 0; s < len; s++) {
            const int wi = ps == 0 ? s : (s < ps ? s : n - 2 * ps + s);
            const double d = (double)((float)sample(start + s) * window[wi]);
            ac[0] = fma(d, d, ac[0]);
#pragma unroll
            for (int l = 1; l <= kMaxLpcHi; l++) ac[l] = fma(d, h[l - 1], ac[l]);
#pragma unroll
            for (int l = kMaxLpcHi - 1; l > 0; l--) h[l] = h[l - 1];
            h[0] = d;
        }
#pragma unroll
        for (int l = 0; l <= kMaxLpcHi; l++) ac[l] *= sc;
    };
    double root[kMaxLpcHi + 1], ac[kMaxLpcHi + 1];
    autoc_of(0, n, 0, root);
    LpcCand c;
    lpc_candidate<kMaxLpcHi>(root, max_order, n, sbps, P, c);
    out[0] = c;
    int k = 1;
    for (int b = 2; b <= parts; b++) {
        for (int j = 0; j < b; j++) {
            const bool skip = n / b <= 32;  // (FLAC__MAX_LPC_ORDER) too small a part to window
            if (!skip) {
                autoc_of((j * n) / b, 2 * (n / b / 2), n / b / 2, ac);
                lpc_candidate<kMaxLpcHi>(ac, max_order, n, sbps, P, c);
                out[k] = c;
            }
            k++;
            if (b >= 3) {
                if (!skip) {
                    // libFLAC 1.4.3 apply_apodization_: lags 0 .. max_order - 1 are root - partial, lag max_order keeps
                    // the partial window's value (its loop and autoc_root memcpy stop below max_order)
#pragma unroll
                    for (int l = 0; l < kMaxLpcHi; l++) ac[l] = l < max_order ? root[l] - ac[l] : ac[l];
                    lpc_candidate<kMaxLpcHi>(ac, max_order, n, sbps, P, c);
                    out[k] = c;
                }
                k++;
            }
        }
    }
}

// The fast path's partial last frames (n < blocksize, at most one per tile, 16-bit mono streams): one work-group per
// frame instead of one lane (k_analyze's lane walks 4096 samples with fp64 divisions: ~0.75 ms for any number of
// frames).  The frame is normalised and windowed in parallel into LDS; lag l of the autocorrelation is summed by
// thread l in libFLAC's sequential order (the same fma sequence as k_analyze's lane, so bit-identical); the fixed
// totals, the OR and the constant test are integer reductions (order-free); thread 0 makes the decisions.
constexpr int kPartThreads = 256;
template <int DT, bool ST = false>
__global__ void __launch_bounds__(kPartThreads) k_analyze_partial(const typename Elem<DT>::T *raster, EncodeParams P,
                                                                 const TileGeom *tiles, const TileNorm *norms,
                                                                 const float *__restrict__ window, SubAnalysis *out,
                                                                 const int64_t *__restrict__ flist) {
    using T = typename Elem<DT>::T;
    __shared__ int32_t xs[kMaxBlock];
    __shared__ double xw[kMaxBlock];
    __shared__ unsigned long long red_t[5];
    __shared__ uint32_t red_or, red_diff;
    __shared__ double red_acc[kMaxLpc + 1];
    const int64_t f = flist[blockIdx.x];
    const int t = tile_of_frame(tiles, P.ntiles, f);
    const TileGeom g = tiles[t];
    const int64_t s0 = (f - g.frame_base) * P.blocksize;
    const int64_t tile_px = (int64_t)g.h * g.w;
    const int n = (int)((tile_px - s0) < P.blocksize ? (tile_px - s0) : P.blocksize);
    const Normalizer<DT> nz = make_norm<DT>(norms[t], P.scale_bits, P.norm_mode);
    const int chn = blockIdx.y;  // channel (multi-channel jobs: grid.y = nch; a two-channel stream: L, R, M, S)
    const T *tb = raster + (int64_t)(P.band0 + (ST ? 0 : chn)) * P.band_stride + g.r0 * P.row_stride + g.c0;
    if (threadIdx.x < 5) red_t[threadIdx.x] = 0;
    if (threadIdx.x == 0) red_or = red_diff = 0;
    // 1. normalise + window (samples past n are zeros, as in k_analyze)
    for (int i = threadIdx.x; i < P.blocksize; i += kPartThreads) {
        int32_t x = 0;
        if (i < n) {
            const int64_t q = s0 + i, r = q / g.w;
            if constexpr (ST) x = coded_sample<DT, true, int32_t>(tb + r * P.row_stride + (q - r * g.w), P.band_stride, nz, chn);
            else x = nz(tb[r * P.row_stride + (q - r * g.w)]);
        }
        xs[i] = x;
        xw[i] = (double)((float)x * window[i]);
    }
    __syncthreads();
    // 2. integer reductions over the frame: OR (wasted bits), OR of x ^ x[0] (constant), fixed totals over 4..n-1
    const int32_t x0 = xs[0];
    uint32_t o = 0, d = 0;
    uint64_t tk[5] = {0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < n; i += kPartThreads) {
        const int32_t x = xs[i];
        o |= (uint32_t)x;
        d |= (uint32_t)(x ^ x0);
        if (i >= 4) {
            const int32_t a = xs[i - 1], b = xs[i - 2], c = xs[i - 3], e = xs[i - 4];
            const int32_t e1 = x - a, e2 = e1 - (a - b), e3 = e2 - ((a - b) - (b - c));
            const int32_t e4 = e3 - (((a - b) - (b - c)) - ((b - c) - (c - e)));
            tk[0] += (uint32_t)abs(x);
            tk[1] += (uint32_t)abs(e1);
            tk[2] += (uint32_t)abs(e2);
            tk[3] += (uint32_t)abs(e3);
            tk[4] += (uint32_t)abs(e4);
        }
    }
    atomicOr(&red_or, o);
    atomicOr(&red_diff, d);
#pragma unroll
    for (int k = 0; k < 5; k++) atomicAdd(&red_t[k], (unsigned long long)tk[k]);
    // 3. autocorrelation: lag l by thread l, i ascending (k_analyze's order)
    if (threadIdx.x <= kMaxLpc) {
        const int l = threadIdx.x;
        double a = 0.0;
        int i = 0;
        for (; i < kMaxLpc; i++) a = fma(xw[i], i >= l ? xw[i - l] : 0.0, a);
        // (LDS reads of later terms issue ahead of the fma chain)
#pragma unroll 16
        for (; i < P.blocksize; i++) a = fma(xw[i], xw[i - l], a);
        red_acc[l] = a;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double acc[kMaxLpc + 1];
#pragma unroll
        for (int l = 0; l <= kMaxLpc; l++) acc[l] = red_acc[l];
        const uint64_t tt[5] = {red_t[0], red_t[1], red_t[2], red_t[3], red_t[4]};
        out[f * P.nvch + chn] = generic_decide<false>(acc, tt, red_or, red_diff, n, P, (ST && chn == 3) ? 1 : 0);
    }
}

// libFLAC 1.4.3 FLAC__fixed_compute_best_predictor_limit_residual's choice from the totals tt / validity of orders
// 0..4 (CHECK_ORDER_IS_VALID: the estimate of a best-so-far order uses total_error_0, the others are 34.0f), then
// process_subframe_'s constant test (fixed bits[1] == 0 and `is_constant()`: every sample equal) and the FIXED
// estimate test against subframe_bps.  Updates A's fixed_order and kFlagConstant / kFlagFixedOk.
template <typename IsConstant>
__device__ inline void fixed_wide_decide(SubAnalysis &A, const uint64_t *tt, const bool *valid, int n, int sbps,
                                         IsConstant is_constant) {
    uint64_t smallest = UINT64_MAX;
    int order = 0;
    float fb[5];
    const double dn = (double)(n - 4);
#pragma unroll
    for (int k = 0; k < 5; k++) {
        if (valid[k] && tt[k] < smallest) {
            order = k;
            smallest = tt[k];
            fb[k] = (float)(tt[0] > 0 ? log(M_LN2 * (double)tt[0] / dn) / M_LN2 : 0.0);
        } else {
            fb[k] = 34.0f;
        }
    }
    int flags = A.flags & ~(kFlagConstant | kFlagFixedOk);
    const bool constant = fb[1] == 0.0f && is_constant();
    if (constant) {
        A.flags = (flags & ~kFlagLpcOk) | kFlagConstant;
    } else {
        A.fixed_order = order;
        float fg = fb[0];
#pragma unroll
        for (int k = 1; k < 5; k++)
            if (k == order) fg = fb[k];
        if (!(fg >= (float)sbps)) flags |= kFlagFixedOk;
        A.flags = flags;
    }
}

// 32-bit streams (bits_per_sample 24 -> pyflac bps 32) use libFLAC's limit_residual fixed estimator;
// it needs 64-bit errors and validity tracking, done in a separate exact pass per lane.
template <int DT, bool ST = false>
__global__ void __launch_bounds__(128) k_analyze_fixed_wide(const typename Elem<DT>::T *raster, EncodeParams P,
                                                           const TileGeom *tiles, const TileNorm *norms,
                                                           SubAnalysis *out, const uint8_t *__restrict__ skip = nullptr) {
    // ST: two-channel stream, lanes per (frame, L/R/M/S); the side signal has 33 bits
    // (FLAC__fixed_compute_best_predictor_limit_residual_33bit: the same arithmetic on int64 samples)
    // skip: subframes already analysed (k_zero_subframes)
    using T = typename Elem<DT>::T;
    const int64_t sub = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sub >= P.nframes * P.nvch) return;
    if (skip && skip[sub]) return;
    const int64_t f = sub / P.nvch;
    const int ch = (int)(sub - f * P.nvch);
    const int t = tile_of_frame(tiles, P.ntiles, f);
    const TileGeom g = tiles[t];
    const int64_t s0 = (f - g.frame_base) * P.blocksize;
    const int64_t tile_px = (int64_t)g.h * g.w;
    const int n = (int)((tile_px - s0) < P.blocksize ? (tile_px - s0) : P.blocksize);
    const Normalizer<DT> nz = make_norm<DT>(norms[t], P.scale_bits, P.norm_mode);
    SubAnalysis A = out[sub];
    if (n <= 4) return;
    const int w = A.wasted;
    const int sbps = P.bps - w + ((ST && ch == 3) ? 1 : 0);
    int64_t row = s0 / g.w;
    int col = (int)(s0 - row * g.w);
    const T *const tbase = raster + (int64_t)(P.band0 + (ST ? 0 : ch)) * P.band_stride;
    const T *rowp = tbase + (g.r0 + row) * P.row_stride + g.c0;
    auto next = [&]() -> int64_t {
        const int64_t x = coded_sample<DT, ST, int64_t>(rowp + col, P.band_stride, nz, ST ? ch : 0);
        if (++col == g.w) {
            col = 0;
            rowp += P.row_stride;
        }
        return x;
    };
    int64_t h1 = 0, h2 = 0, h3 = 0, h4 = 0;
    uint64_t tt[5] = {0, 0, 0, 0, 0};
    bool valid[5] = {true, true, true, true, true};
    for (int i = 0; i < n; i++) {
        const int64_t x = next() >> w;
        uint64_t e[5];
        e[0] = (uint64_t)(x < 0 ? -x : x);
        int64_t v;
        v = x - h1;
        e[1] = i >= 1 ? (uint64_t)(v < 0 ? -v : v) : 0;
        v = x - 2 * h1 + h2;
        e[2] = i >= 2 ? (uint64_t)(v < 0 ? -v : v) : 0;
        v = x - 3 * h1 + 3 * h2 - h3;
        e[3] = i >= 3 ? (uint64_t)(v < 0 ? -v : v) : 0;
        v = x - 4 * h1 + 6 * h2 - 4 * h3 + h4;
        e[4] = i >= 4 ? (uint64_t)(v < 0 ? -v : v) : 0;
#pragma unroll
        for (int k = 0; k < 5; k++) {
            tt[k] += e[k];
            if (e[k] > (uint64_t)INT32_MAX) valid[k] = false;
        }
        h4 = h3;
        h3 = h2;
        h2 = h1;
        h1 = x;
    }
    fixed_wide_decide(A, tt, valid, n, sbps, [&]() {
        // all samples equal?  (rare; re-walk)
        row = s0 / g.w;
        col = (int)(s0 - row * g.w);
        rowp = tbase + (g.r0 + row) * P.row_stride + g.c0;
        int64_t first = 0;
        for (int i = 0; i < n; i++) {
            const int64_t x = next();
            if (i == 0) first = x;
            else if (x != first) return false;
        }
        return true;
    });
    out[sub] = A;
}

// ------------------------------------------------------------------------------ k_encode_frames
constexpr int kEncThreads = 256;
constexpr int kBitWords = 4096 + 64;  // one 32-bit subframe (4096 x 32 bits) + headers + carry

__constant__ uint8_t c_crc8[256];
// 2^18 / (n - order) for the first Rice partition of partition order po (n = 4096 >> po), order 0..8 (libFLAC's
// parameter estimate; the other partitions divide by a power of two)
__constant__ uint32_t c_rice_div[6][9] = {
    {64, 64, 64, 64, 64, 64, 64, 64, 64},
    {128, 128, 128, 128, 128, 128, 128, 128, 128},
    {256, 256, 256, 256, 257, 257, 257, 257, 258},
    {512, 513, 514, 515, 516, 517, 518, 519, 520},
    {1024, 1028, 1032, 1036, 1040, 1044, 1048, 1052, 1057},
    {2048, 2064, 2080, 2097, 2114, 2131, 2148, 2166, 2184}};

struct RiceChoice {
    uint32_t bits;   // estimated residual bits (find_best_partition_order_)
    int order;       // partition order
    int rice2;
    uint8_t k[1 << kMaxPo];  // parameters
};

// set_partitioned_rice_ for every order in [0, max_po] from the max-order partition sums; returns best.
__device__ void rice_search(const uint64_t *sums_max, int max_po, int n, int pred_order, int rice_limit,
                            RiceChoice *rc) {
    uint64_t sums[2 << kMaxPo];
    const int parts = 1 << max_po;
    for (int p = 0; p < parts; p++) sums[p] = sums_max[p];
    int from = 0, to = parts, pp = parts;
    for (int po = max_po - 1; po >= 0; po--) {
        pp >>= 1;
        for (int i = 0; i < pp; i++) {
            sums[to++] = sums[from] + sums[from + 1];
            from += 2;
        }
    }
    uint32_t best_bits = 0;
    int sumoff = 0;
    for (int po = max_po; po >= 0; po--) {
        const int np = 1 << po;
        const uint32_t pbase = (uint32_t)(n >> po);
        const uint32_t div_base = 0x40000u / pbase;
        uint32_t bits = 2 + 4;
        uint8_t ks[1 << kMaxPo];
        bool ok = true;
        for (int p = 0; p < np; p++) {
            uint32_t ns = pbase, div = div_base;
            if (p == 0) {
                if (ns <= (uint32_t)pred_order) {
                    ok = false;
                    break;
                }
                ns -= (uint32_t)pred_order;
                div = 0x40000u / ns;
            }
            const uint64_t mean = sums[sumoff + p];
            uint32_t k;
            if (mean < 2 || (((mean - 1) * div) >> 18) == 0) k = 0;
            else k = (uint32_t)ilog2_u64(((mean - 1) * div) >> 18) + 1;
            if (k >= (uint32_t)rice_limit) k = (uint32_t)rice_limit - 1;
            uint64_t pb = 4 + (uint64_t)(1 + k) * ns + (k ? (mean >> (k - 1)) : (mean << 1)) - (ns >> 1);
            if (pb > 0xFFFFFFFFull) pb = 0xFFFFFFFFull;
            bits += (uint32_t)pb;
            ks[p] = (uint8_t)k;
        }
        if (!ok) break;
        sumoff += np;
        if (best_bits == 0 || bits < best_bits) {
            best_bits = bits;
            rc->order = po;
            for (int p = 0; p < np; p++) rc->k[p] = ks[p];
        }
    }
    rc->bits = best_bits;
    rc->rice2 = 0;
    for (int p = 0; p < (1 << rc->order); p++)
        if (rc->k[p] >= 15) rc->rice2 = 1;
}

// LDS bit writer: MSB-first bit positions relative to the word-aligned buffer base.
__device__ inline void put_bits(uint32_t *buf, uint64_t pos, uint32_t val, int nbits) {
    if (nbits <= 0) return;
    const uint32_t wi = (uint32_t)(pos >> 5);
    const int off = (int)(pos & 31);
    const uint64_t v = (uint64_t)val << (64 - off - nbits);
    atomicOr(&buf[wi], (uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)v;
    if (lo) atomicOr(&buf[wi + 1], lo);
}

__device__ inline uint32_t mask_bits(int64_t v, int n) { return n >= 32 ? (uint32_t)v : (uint32_t)v & ((1u << n) - 1u); }

// a signed sample of nbits <= 33 bits (the 33-bit side signal of a 32-bit stereo stream goes out as 1 + 32 bits)
__device__ inline void put_sample(uint32_t *buf, uint64_t pos, int64_t v, int nbits) {
    if (nbits > 32) {
        put_bits(buf, pos, (uint32_t)(v >> 32) & ((1u << (nbits - 32)) - 1u), nbits - 32);
        put_bits(buf, pos + (uint64_t)(nbits - 32), (uint32_t)v, 32);
    } else {
        put_bits(buf, pos, mask_bits(v, nbits), nbits);
    }
}

// LDS index of sample i in EncShared::xs: one pad word per 16 samples, so the 256 threads' contiguous 16-sample
// chunks start in distinct banks (unpadded, thread t's chunk starts at bank 16 t mod 32: 16-way conflicts)
__device__ inline int xsi(int i) { return i + (i >> 4); }

// XT = int64_t only for the 33-bit side signal of a 32-bit stereo stream (a VERBATIM 33-bit subframe is 4224 words)
template <typename XT> struct EncShared {
    static constexpr int kWords = sizeof(XT) == 8 ? 4096 + 192 : kBitWords;
    XT xs[kMaxBlock + kMaxBlock / 16];
    uint32_t bits[kWords];
    uint64_t psum[2][1 << kMaxPo];
    RiceChoice rc[2];
    RiceChoice rc_try;   // an LPC candidate under evaluation (subdivide_tukey levels: several per signal)
    LpcCand lsel;        // the chosen LPC candidate of the current signal
    uint32_t lpc_best;   // its estimated bits (0xFFFFFFFF: none)
    int lpc_bad;
    int choice;          // subframe type: 0 const, 1 verbatim, 2 fixed, 3 lpc
    uint32_t best;       // its estimated bits (process_subframe_'s best_bits)
    // two-channel streams: the decisions of L, R, mid, side and the chosen channel assignment
    int vtype[4];
    uint32_t vbits[4];
    RiceChoice vrc[4];
    LpcCand vl[4];
    int assign;          // FLAC__ChannelAssignment: 0 independent, 1 left-side, 2 right-side, 3 mid-side
};

// Frame header of a generic-path frame (RFC 9639 9.1; libFLAC FLAC__frame_add_header) into h: fixed blocksize,
// frame number fk (UTF-8), sample rate and bps codes, channel assignment code cac, CRC-8; returns its bytes
__device__ inline int generic_frame_header(uint8_t *h, int n, const EncodeParams &P, int cac, uint32_t fk) {
    int hb = 0;
    int bsc, bsx = 0;
    switch (n) {
    case 192: bsc = 1; break;
    case 576: bsc = 2; break;
    case 1152: bsc = 3; break;
    case 2304: bsc = 4; break;
    case 4608: bsc = 5; break;
    case 256: bsc = 8; break;
    case 512: bsc = 9; break;
    case 1024: bsc = 10; break;
    case 2048: bsc = 11; break;
    case 4096: bsc = 12; break;
    case 8192: bsc = 13; break;
    case 16384: bsc = 14; break;
    case 32768: bsc = 15; break;
    default: bsc = bsx = (n <= 256 ? 6 : 7); break;
    }
    int src, srx = 0;
    const int sr = P.sample_rate;
    switch (sr) {
    case 88200: src = 1; break;
    case 176400: src = 2; break;
    case 192000: src = 3; break;
    case 8000: src = 4; break;
    case 16000: src = 5; break;
    case 22050: src = 6; break;
    case 24000: src = 7; break;
    case 32000: src = 8; break;
    case 44100: src = 9; break;
    case 48000: src = 10; break;
    case 96000: src = 11; break;
    default:
        if (sr <= 255000 && sr % 1000 == 0) src = srx = 12;
        else if (sr % 10 == 0 && sr / 10 <= 65535) src = srx = 14;
        else src = srx = 13;
    }
    int bpc = P.bps == 8 ? 1 : P.bps == 12 ? 2 : P.bps == 16 ? 4 : P.bps == 20 ? 5 : P.bps == 24 ? 6 : P.bps == 32 ? 7 : 0;
    // channel assignment: nch - 1 (independent), 8 left-side, 9 right-side, 10 mid-side
    h[hb++] = 0xFF;
    h[hb++] = 0xF8;
    h[hb++] = (uint8_t)((bsc << 4) | src);
    h[hb++] = (uint8_t)((cac << 4) | (bpc << 1));
    const uint32_t v = fk;
    if (v < 0x80) h[hb++] = (uint8_t)v;
    else if (v < 0x800) { h[hb++] = (uint8_t)(0xC0 | (v >> 6)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    else if (v < 0x10000) { h[hb++] = (uint8_t)(0xE0 | (v >> 12)); h[hb++] = (uint8_t)(0x80 | ((v >> 6) & 0x3F)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    else if (v < 0x200000) { h[hb++] = (uint8_t)(0xF0 | (v >> 18)); h[hb++] = (uint8_t)(0x80 | ((v >> 12) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 6) & 0x3F)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    else if (v < 0x4000000) { h[hb++] = (uint8_t)(0xF8 | (v >> 24)); h[hb++] = (uint8_t)(0x80 | ((v >> 18) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 12) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 6) & 0x3F)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    else { h[hb++] = (uint8_t)(0xFC | (v >> 30)); h[hb++] = (uint8_t)(0x80 | ((v >> 24) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 18) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 12) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 6) & 0x3F)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    if (bsx == 6) h[hb++] = (uint8_t)(n - 1);
    else if (bsx == 7) { h[hb++] = (uint8_t)((n - 1) >> 8); h[hb++] = (uint8_t)(n - 1); }
    if (srx == 12) h[hb++] = (uint8_t)(sr / 1000);
    else if (srx == 13) { h[hb++] = (uint8_t)(sr >> 8); h[hb++] = (uint8_t)sr; }
    else if (srx == 14) { h[hb++] = (uint8_t)((sr / 10) >> 8); h[hb++] = (uint8_t)(sr / 10); }
    uint8_t c = 0;
    for (int i = 0; i < hb; i++) c = c_crc8[c ^ h[i]];
    h[hb++] = c;
    return hb;
}

// workgroup = frame.  ST: a two-channel stream -- the four signals L, R, M, S are evaluated (process_subframe_ each),
// the assignment with the fewest estimated bits wins (stream_encoder.c process_subframes_, do_mid_side_stereo &&
// !loose: independent, left-side, right-side, mid-side; a later one only if strictly smaller) and its two subframes
// are written.
// cand (subdivide_tukey levels): P.ncand LPC candidates per coded signal (k_analyze_lpc_hi), evaluated in window order
// (a later one only if strictly smaller).  Loose mid/side (P.loose_frames > 0, levels 1 / 4 on two channels): the
// assignment of a frame is the one chosen on its group's first frame (frame number within the stream a multiple of
// loose_frames) between independent and mid-side; loose_pass = 1 evaluates the group leaders (flist) and stores their
// choice in loose_assign[frame], loose_pass = 0 codes every frame with its leader's choice.
template <int DT, bool ST = false, typename XT = int32_t>
__global__ void __launch_bounds__(kEncThreads) k_encode_frames(const typename Elem<DT>::T *raster, EncodeParams P,
                                                             const TileGeom *tiles, const TileNorm *norms,
                                                             const SubAnalysis *ana, uint32_t *slots,
                                                             int64_t *frame_bytes, int *error_flag,
                                                             const int64_t *__restrict__ flist,
                                                             const LpcCand *__restrict__ cand = nullptr,
                                                             int8_t *loose_assign = nullptr, int loose_pass = 0) {
    // flist: frames to code (the fast path's partial last frames; slot / frame_bytes indexed by list position),
    // nullptr = frame blockIdx.x
    using T = typename Elem<DT>::T;
    using Sh = EncShared<XT>;
    constexpr int kWords = Sh::kWords;
    __shared__ Sh S;
    const int tid = threadIdx.x;
    const int64_t si = blockIdx.x;
    const int64_t f = flist ? flist[si] : si;
    const int t = tile_of_frame(tiles, P.ntiles, f);
    const TileGeom g = tiles[t];
    const int64_t fk = f - g.frame_base;  // frame number within the tile's stream
    const int64_t s0 = fk * P.blocksize;
    const int64_t tile_px = (int64_t)g.h * g.w;
    const int n = (int)((tile_px - s0) < P.blocksize ? (tile_px - s0) : P.blocksize);
    const Normalizer<DT> nz = make_norm<DT>(norms[t], P.scale_bits, P.norm_mode);
    uint32_t *slot = slots + (size_t)si * P.slot_words;
    const int rice_limit = P.bps > 16 ? 31 : 15;
    const int max_po_block = min(P.max_po, __builtin_ctz((unsigned)n));  // level 5: kMaxPartOrder
    const int chunk = (n + kEncThreads - 1) / kEncThreads;
    const int i_beg = tid * chunk, i_end = min(n, i_beg + chunk);
    if constexpr (!ST) {
        if (!flist && !cand && n > 4) {  // every subframe all-zero: k_zero_frames_emit writes this frame
            bool all0 = true;
            for (int c = 0; c < P.nch; c++) all0 = all0 && (ana[f * P.nvch + c].flags & kFlagZero);
            if (all0) return;
        }
    }

    for (int i = tid; i < kWords; i += kEncThreads) S.bits[i] = 0;
    __syncthreads();

    // ---- coded signal v (wasted bits w shifted out) into LDS, strided over threads: coalesced row segments
    auto load = [&](int v, int w) {
        const T *base = raster + (int64_t)(P.band0 + (ST ? 0 : v)) * P.band_stride + g.r0 * P.row_stride + g.c0;
        for (int i = tid; i < n; i += kEncThreads) {
            const int64_t p = s0 + i;
            const int64_t r = p / g.w;
            const int cc = (int)(p - r * g.w);
            S.xs[xsi(i)] = coded_sample<DT, ST, XT>(base + r * P.row_stride + cc, P.band_stride, nz, ST ? v : 0) >> w;
        }
        if (tid < (2 << kMaxPo)) S.psum[tid >> kMaxPo][tid & ((1 << kMaxPo) - 1)] = 0;
        if (tid == 0) S.lpc_bad = 0;
        __syncthreads();
    };
    // residual i of the FIXED (fixed == true) or LPC predictor (L) of order o
    auto resid = [&](const LpcCand &L, bool fixed, int o, int i) -> int64_t {
        int64_t r;
        if (fixed) {
            const int64_t x = S.xs[xsi(i)];
            switch (o) {
            case 0: r = x; break;
            case 1: r = x - S.xs[xsi(i - 1)]; break;
            case 2: r = x - 2 * (int64_t)S.xs[xsi(i - 1)] + S.xs[xsi(i - 2)]; break;
            case 3: r = x - 3 * (int64_t)S.xs[xsi(i - 1)] + 3 * (int64_t)S.xs[xsi(i - 2)] - S.xs[xsi(i - 3)]; break;
            default: r = x - 4 * (int64_t)S.xs[xsi(i - 1)] + 6 * (int64_t)S.xs[xsi(i - 2)] - 4 * (int64_t)S.xs[xsi(i - 3)] + S.xs[xsi(i - 4)]; break;
            }
        } else {
            int64_t s = 0;
            for (int j = 0; j < o; j++) s += (int64_t)L.q[j] * S.xs[xsi(i - 1 - j)];
            r = (int64_t)S.xs[xsi(i)] - (s >> L.shift);
        }
        return r;
    };
    auto max_po_for = [&](int o) {
        int m = max_po_block;
        while (m > 0 && (n >> m) <= o) m--;
        return m;
    };
    // ---- process_subframe_: candidate partition sums, Rice search, choice (VERBATIM, CONSTANT | FIXED, LPC; strict <)
    //      -> S.choice, S.best, S.rc, S.lsel.  LPC candidates: A's single one (tukey(0.5) levels) or the signal's
    //      P.ncand window candidates, each evaluated in turn and kept when strictly smaller than the best so far.
    auto decide = [&](const SubAnalysis &A, int extra, const LpcCand *cands) {
        const int w = A.wasted;
        const int sbps = P.bps - w + extra;
        const bool cand_fixed = n > 4 && !(A.flags & kFlagConstant) && (A.flags & kFlagFixedOk);
        LpcCand a1;  // the SubAnalysis' candidate as a candidate record
        a1.order = A.lpc_order;
        a1.prec = A.lpc_prec;
        a1.shift = A.lpc_shift;
        a1.ok = (A.flags & kFlagLpcOk) ? 1 : 0;
#pragma unroll
        for (int j = 0; j < kMaxLpcHi; j++) a1.q[j] = j < kMaxLpc ? A.q[j] : 0;
        const int nc = cands ? P.ncand : 1;
        const bool lpc_any = n > 4 && !(A.flags & kFlagConstant);
        if (tid == 0) S.lpc_best = 0xFFFFFFFFu;
        for (int c = 0; c < nc; c++) {
            const LpcCand L = cands ? cands[c] : a1;
            const bool do_fixed = c == 0 && cand_fixed;
            const bool do_lpc = lpc_any && L.ok;
            if (c > 0) {  // the previous candidate's sums have been read
                if (tid < (1 << kMaxPo)) S.psum[1][tid] = 0;
                if (tid == 0) S.lpc_bad = 0;
                __syncthreads();
            }
            const int mpo[2] = {max_po_for(A.fixed_order), max_po_for(L.order)};
            for (int cd = 0; cd < 2; cd++) {
                if (cd == 0 && !do_fixed) continue;
                if (cd == 1 && !do_lpc) continue;
                const int o = cd == 0 ? A.fixed_order : L.order;
                const int ps = n >> mpo[cd];
                int cur_p = -1;
                uint64_t acc = 0;
                for (int i = max(i_beg, o); i < i_end; i++) {
                    int64_t r = resid(L, cd == 0, o, i);
                    if (cd == 0) r = (int32_t)r;  // libFLAC stores fixed residuals as int32
                    else if (r <= INT32_MIN || r > INT32_MAX) S.lpc_bad = 1;
                    const int p = i / ps;
                    if (p != cur_p) {
                        if (cur_p >= 0) atomicAdd((unsigned long long *)&S.psum[cd][cur_p], (unsigned long long)acc);
                        cur_p = p;
                        acc = 0;
                    }
                    acc += (uint64_t)(r < 0 ? -r : r);
                }
                if (cur_p >= 0) atomicAdd((unsigned long long *)&S.psum[cd][cur_p], (unsigned long long)acc);
            }
            __syncthreads();
            if (tid == 0 && do_fixed) rice_search(S.psum[0], mpo[0], n, A.fixed_order, rice_limit, &S.rc[0]);
            if (tid == 64 && do_lpc && !S.lpc_bad) {
                rice_search(S.psum[1], mpo[1], n, L.order, rice_limit, &S.rc_try);
                uint32_t est = (uint32_t)(1 + 6 + 1 + w + 4 + 5 + sbps * L.order + L.prec * L.order);
                est = (S.rc_try.bits < 0xFFFFFFFFu - est) ? est + S.rc_try.bits : 0xFFFFFFFFu;
                if (est != 0 && est < S.lpc_best) {
                    S.lpc_best = est;
                    S.rc[1] = S.rc_try;
                    S.lsel = L;
                }
            }
            __syncthreads();
        }
        if (tid == 0) {
            uint32_t best = (uint32_t)(1 + 6 + 1 + w + n * sbps);
            int type = 1;
            if (n > 4) {
                if (A.flags & kFlagConstant) {
                    const uint32_t cb = (uint32_t)(1 + 6 + 1 + w + sbps);
                    if (cb < best) {
                        best = cb;
                        type = 0;
                    }
                } else {
                    if (cand_fixed) {
                        uint32_t est = (uint32_t)(1 + 6 + 1 + w + A.fixed_order * sbps);
                        est = (S.rc[0].bits < 0xFFFFFFFFu - est) ? est + S.rc[0].bits : 0xFFFFFFFFu;
                        if (est < best) {
                            best = est;
                            type = 2;
                        }
                    }
                    if (S.lpc_best != 0xFFFFFFFFu && S.lpc_best < best) {
                        best = S.lpc_best;
                        type = 3;
                    }
                }
            }
            S.choice = type;
            S.best = best;
        }
        __syncthreads();
    };

    if constexpr (ST) {
        // loose mid/side, coding pass: the group leader's assignment (and only that pair is evaluated)
        const bool loose = P.loose_frames > 0;
        int lead_ca = -1;
        if (loose && !loose_pass) lead_ca = loose_assign[f - (fk % P.loose_frames)];
        for (int v = 0; v < 4; v++) {
            if (lead_ca == 0 && v >= 2) continue;
            if (lead_ca == 3 && v < 2) continue;
            const SubAnalysis A = ana[f * 4 + v];
            load(v, A.wasted);
            decide(A, v == 3 ? 1 : 0, cand ? cand + (f * 4 + v) * P.ncand : nullptr);
            if (tid == 0) {
                S.vtype[v] = S.choice;
                S.vbits[v] = S.best;
                S.vrc[v] = S.rc[S.choice == 2 ? 0 : 1];
                S.vl[v] = S.lsel;
            }
            __syncthreads();
        }
        if (tid == 0) {
            const uint32_t bits[4] = {S.vbits[0] + S.vbits[1], S.vbits[0] + S.vbits[3], S.vbits[1] + S.vbits[3],
                                      S.vbits[2] + S.vbits[3]};
            int ca = 0;
            // strict <, in this order; loose mid/side weighs independent against mid-side only
            for (int k = loose ? 3 : 1; k < 4; k++)
                if (bits[k] < bits[ca]) ca = k;
            S.assign = lead_ca >= 0 ? lead_ca : ca;
            if (loose && loose_pass) loose_assign[f] = (int8_t)ca;
        }
        __syncthreads();
        if (loose && loose_pass) return;  // (leader pass: the choice only)
    }

    // ---- frame header (RFC 9639 9.1; libFLAC FLAC__frame_add_header), thread 0
    uint64_t fb = 0;  // frame bit cursor relative to S.bits word 0
    int64_t w0 = 0;   // global slot word index of S.bits[0]
    {
        __shared__ int hdr_bits;
        if (tid == 0) {
            uint8_t h[16];
            // channel assignment: nch - 1 (independent), 8 left-side, 9 right-side, 10 mid-side
            const int hb = generic_frame_header(h, n, P, ST ? (S.assign == 0 ? 1 : 7 + S.assign) : P.nch - 1,
                                                (uint32_t)fk);
            for (int i = 0; i < hb; i++) put_bits(S.bits, (uint64_t)i * 8, h[i], 8);
            hdr_bits = hb * 8;
        }
        __syncthreads();
        fb = (uint64_t)hdr_bits;
    }

    for (int c = 0; c < P.nch; c++) {
        // the signal coded as channel c: channel c, or for stereo (L, R) / (L, S) / (S, R) / (M, S)
        int v = c;
        if constexpr (ST) {
            const int ca = S.assign;
            v = ca == 0 ? c : ca == 1 ? (c == 0 ? 0 : 3) : ca == 2 ? (c == 0 ? 3 : 1) : (c == 0 ? 2 : 3);
        }
        const SubAnalysis A = ana[f * P.nvch + v];
        const int w = A.wasted;
        const int sbps = P.bps - w + ((ST && v == 3) ? 1 : 0);
        // an all-zero subframe (k_zero_subframes: raw-frames tiles) needs no sample load: the signal is zeros, and
        // decide() runs unchanged on them; its residual codes are written as runs below (WG-uniform)
        const bool zsub = !ST && (A.flags & kFlagZero) && !cand;
        if (zsub) {
            for (int i = tid; i < n; i += kEncThreads) S.xs[xsi(i)] = 0;
            if (tid < (2 << kMaxPo)) S.psum[tid >> kMaxPo][tid & ((1 << kMaxPo) - 1)] = 0;
            if (tid == 0) S.lpc_bad = 0;
            __syncthreads();
        } else {
            load(v, w);
        }
        int type;
        const RiceChoice *rcp;
        const LpcCand *lcp;
        if constexpr (ST) {
            type = S.vtype[v];
            rcp = &S.vrc[v];
            lcp = &S.vl[v];
        } else {
            decide(A, 0, cand ? cand + (f * P.nvch + v) * P.ncand : nullptr);
            type = S.choice;
            rcp = &S.rc[type == 2 ? 0 : 1];
            lcp = &S.lsel;
        }
        const LpcCand Lc = *lcp;

        // ---- emit the subframe bits at fb (relative to S.bits)
        const uint64_t sb = fb;
        uint64_t pos = sb;
        const int typecode = type == 0 ? 0 : type == 1 ? 1 : type == 2 ? 8 + A.fixed_order : 32 + Lc.order - 1;
        if (tid == 0) {
            put_bits(S.bits, pos, (uint32_t)(typecode << 1) | (w ? 1u : 0u), 8);
        }
        pos += 8;
        if (w) {
            if (tid == 0) put_bits(S.bits, pos + (uint64_t)(w - 1), 1, 1);
            pos += (uint64_t)w;
        }
        uint64_t sub_end;
        if (type == 0) {
            if (tid == 0) put_sample(S.bits, pos, S.xs[xsi(0)], sbps);
            sub_end = pos + (uint64_t)sbps;
        } else if (type == 1) {
            for (int i = tid; i < n; i += kEncThreads) put_sample(S.bits, pos + (uint64_t)i * sbps, S.xs[xsi(i)], sbps);
            sub_end = pos + (uint64_t)n * sbps;
        } else {
            const int o = type == 2 ? A.fixed_order : Lc.order;
            const RiceChoice &rc = *rcp;
            for (int i = tid; i < o; i++) put_sample(S.bits, pos + (uint64_t)i * sbps, S.xs[xsi(i)], sbps);
            pos += (uint64_t)o * sbps;
            if (type == 3) {
                if (tid == 0) {
                    put_bits(S.bits, pos, (uint32_t)(Lc.prec - 1), 4);
                    put_bits(S.bits, pos + 4, mask_bits(Lc.shift, 5), 5);
                }
                pos += 9;
                for (int j = tid; j < o; j += kEncThreads)
                    put_bits(S.bits, pos + (uint64_t)j * Lc.prec, mask_bits(Lc.q[j], Lc.prec), Lc.prec);
                pos += (uint64_t)o * Lc.prec;
            }
            if (tid == 0) {
                put_bits(S.bits, pos, (uint32_t)rc.rice2, 2);
                put_bits(S.bits, pos + 2, (uint32_t)rc.order, 4);
            }
            pos += 6;
            const int pbits = rc.rice2 ? 5 : 4;
            const int po = rc.order;
            const int ps = n >> po;
            bool k0 = zsub;
            for (int p = 0; p < (1 << po) && k0; p++) k0 = rc.k[p] == 0;
            if (k0) {
                // all residuals 0 with parameter 0 in every partition: each code is the single stop bit '1' and the
                // parameter fields are zeros, so partition p is one run of ones after its field
                for (int p = 0; p < (1 << po); p++) {
                    const uint64_t before = p ? (uint64_t)p * ps - o : 0;  // codes of the earlier partitions
                    const uint64_t a = pos + (uint64_t)pbits * (p + 1) + before;
                    const uint64_t b = a + (uint64_t)(ps - (p ? 0 : o));
                    for (uint64_t wd = (a >> 5) + tid; wd <= ((b - 1) >> 5) && b > a; wd += kEncThreads) {
                        const uint64_t lo = a > wd * 32 ? a : wd * 32, hi = b < wd * 32 + 32 ? b : wd * 32 + 32;
                        const uint32_t nb = (uint32_t)(hi - lo), sh = (uint32_t)(wd * 32 + 32 - hi);
                        atomicOr(&S.bits[wd], (nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u)) << sh);
                    }
                }
                sub_end = pos + (uint64_t)pbits * (1 << po) + (uint64_t)(n - o);
            } else {
            // per-thread code lengths of its chunk, then block exclusive scan
            uint64_t my = 0;
            for (int i = max(i_beg, o); i < i_end; i++) {
                const int32_t r32 = (int32_t)resid(Lc, type == 2, o, i);
                const uint32_t u = ((uint32_t)r32 << 1) ^ (uint32_t)(r32 >> 31);
                const int k = rc.k[i / ps];
                my += 1 + (uint64_t)k + (u >> k);
            }
            // block scan of my: wave inclusive scan with shuffles, then wave totals in LDS
            uint64_t incl = my;
            const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t y = __shfl_up(incl, d);
                if (lane >= d) incl += y;
            }
            __shared__ uint64_t wtot[kEncThreads / 64];
            if (lane == 63) wtot[wv] = incl;
            __syncthreads();
            uint64_t wbase = 0;
            for (int k = 0; k < wv; k++) wbase += wtot[k];
            const uint64_t excl = wbase + incl - my;
            uint64_t total = 0;
            for (int k = 0; k < kEncThreads / 64; k++) total += wtot[k];
            sub_end = pos + (uint64_t)pbits * (1 << po) + total;
            if (sub_end > (uint64_t)kWords * 32 - 64) {  // exact code longer than the LDS window
                if (tid == 0) atomicOr(error_flag, 2);
                return;  // uniform: every thread sees the same sub_end
            }
            // bit position of sample i = pos + pbits*(p_i + 1) + (sum of code lengths before i);
            // partition p's parameter field precedes its first code
            uint64_t run = excl;
            __shared__ uint64_t pstart[1 << kMaxPo];
            for (int i = max(i_beg, o); i < i_end; i++) {
                const int32_t r32 = (int32_t)resid(Lc, type == 2, o, i);
                const uint32_t u = ((uint32_t)r32 << 1) ^ (uint32_t)(r32 >> 31);
                const int p = i / ps;
                const int k = rc.k[p];
                const uint32_t q = u >> k;
                const int first_of_p = p == 0 ? o : p * ps;
                if (i == first_of_p) pstart[p] = run;  // codes before this partition
                const uint64_t at = pos + (uint64_t)pbits * (p + 1) + run + q;
                const uint32_t low = k ? (u & ((1u << k) - 1u)) : 0u;
                put_bits(S.bits, at, (1u << k) | low, k + 1);
                run += 1 + (uint64_t)k + q;
            }
            __syncthreads();
            for (int p = tid; p < (1 << po); p += kEncThreads)
                put_bits(S.bits, pos + (uint64_t)pbits * p + pstart[p], rc.k[p], pbits);
            }
        }
        __syncthreads();
        // ---- flush complete words of S.bits to the slot, keep the partial word
        {
            const uint64_t full = sub_end >> 5;
            if ((int64_t)(w0 + full) + 2 > P.slot_words) {
                if (tid == 0) atomicOr(error_flag, 1);
                return;
            }
            for (uint64_t i = tid; i < full; i += kEncThreads) slot[w0 + i] = __builtin_bswap32(S.bits[i]);
            __syncthreads();
            const uint32_t keep = S.bits[full];
            __syncthreads();
            for (int i = tid; i < kWords; i += kEncThreads) S.bits[i] = 0;
            __syncthreads();
            if (tid == 0) S.bits[0] = keep;
            __syncthreads();
            w0 += (int64_t)full;
            fb = sub_end - (full << 5);
        }
    }
    // ---- byte-align; the final partial word goes out whole (zero tail)
    const uint64_t bits_total = (uint64_t)w0 * 32 + fb;
    const uint64_t bytes = (bits_total + 7) >> 3;
    if (fb && tid == 0) slot[w0] = __builtin_bswap32(S.bits[0]);
    if (tid == 0) frame_bytes[si] = (int64_t)bytes + 2;  // + CRC-16 footer
}

// ------------------------------------------------------------------------------------ k_compact
__constant__ uint16_t c_crc16[256];
__constant__ uint16_t c_xpow8[40];  // x^(8 * 2^j) mod P, j = 0..39

__device__ inline uint32_t gf_mulmod(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 15; i >= 0; i--) {
        r <<= 1;
        if (r & 0x10000u) r ^= 0x18005u;
        if ((b >> i) & 1u) r ^= a;
    }
    return r;
}

__device__ inline uint32_t xpow8(uint64_t m) {  // x^(8m) mod P
    uint32_t r = 1;
    int j = 0;
    while (m) {
        if (m & 1) r = gf_mulmod(r, c_xpow8[j]);
        m >>= 1;
        j++;
    }
    return r;
}

constexpr int kFrameWordsV3 = 2176;  // 69632 bits >= worst exact frame (estimate < verbatim)
constexpr int kXpowBytes = kFrameWordsV3 * 4 + 64;  // multiple of 64 (LDS split tables)
__constant__ uint16_t c_crc16x8[16][256];           // T_k[v] = CRC-16 of byte v followed by k zero bytes
__device__ uint16_t g_xpow_bytes[kXpowBytes];      // x^(8m) mod P for m bytes
__device__ uint16_t g_xpow_8k[32];                  // x^(8 * 8192 q) mod P
// x^(8m) mod P for a byte count m: one table read below kXpowBytes, two reads and a multiply below 256 KiB (frames
// of up to 8 channels), the square-and-multiply loop beyond
__device__ inline uint32_t xpow_bytes(int64_t m) {
    if (m < kXpowBytes) return g_xpow_bytes[m];
    if (m < 32 * 8192) return gf_mulmod(g_xpow_bytes[m & 8191], g_xpow_8k[m >> 13]);
    return xpow8((uint64_t)m);
}

// CRC-16 (init 0) of bytes [0, L) of a 4-byte aligned frame image, by one 256-thread work-group: thread t folds a
// contiguous word range with slice-by-4 tables in LDS (T), shifts it to the end of the frame by x^(8m) (one
// multiply from the byte-power table; the square-and-multiply loop only past it) and the ranges are XOR-combined.
__device__ inline uint32_t wg_crc16(const uint8_t *src, int64_t L, const uint16_t (*T)[256], uint32_t *wc) {
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(src);
    const int64_t nw = L >> 2;
    const int64_t ch = (nw + 255) / 256;
    const int64_t w0 = min(nw, (int64_t)threadIdx.x * ch), w1 = min(nw, w0 + ch);
    uint32_t c = 0;
    for (int64_t i = w0; i < w1; i++) {
        const uint32_t v = sw[i];  // bytes b0..b3 = v & 0xFF .. v >> 24 (stream order)
        c = (uint32_t)T[3][((c >> 8) ^ v) & 0xFF] ^ T[2][((c & 0xFF) ^ (v >> 8)) & 0xFF] ^ T[1][(v >> 16) & 0xFF] ^
            T[0][v >> 24];
    }
    int64_t end = w1 << 2;
    const bool last = (nw == 0) ? threadIdx.x == 0 : (w1 == nw && w1 > w0);
    if (last) {  // the L & 3 tail bytes
        for (int64_t i = nw << 2; i < L; i++) c = ((c << 8) & 0xFFFFu) ^ T[0][((c >> 8) ^ src[i]) & 0xFF];
        end = L;
    }
    const int64_t m = L - end;
    if (c && m > 0) c = gf_mulmod(c, xpow_bytes(m));
    for (int o = 32; o > 0; o >>= 1) c ^= __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    return wc[0] ^ wc[1] ^ wc[2] ^ wc[3];
}

__device__ inline void wg_load_crc_tables(uint16_t (*T)[256]) {
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) (&T[0][0])[i] = (&c_crc16x8[0][0])[i];
    __syncthreads();
}

// Generic path: frame f's bytes move from its slot to the arena at frame_off[f] with the CRC-16 footer appended.
// The copy writes aligned 4-byte words assembled by v_alignbyte (byte stores only for the partial words at either
// end, which neighbouring frames share).
__global__ void __launch_bounds__(256) k_compact(const uint32_t *slots, int slot_words, const int64_t *frame_bytes,
                                                const int64_t *frame_off, int64_t nframes, uint8_t *arena) {
    __shared__ uint16_t T[4][256];
    __shared__ uint32_t wc[4];
    const int64_t f = blockIdx.x;
    if (f >= nframes) return;
    wg_load_crc_tables(T);
    const uint32_t *sw = slots + (size_t)f * slot_words;
    const uint8_t *src = reinterpret_cast<const uint8_t *>(sw);
    const int64_t S = frame_bytes[f];
    const int64_t L = S - 2;  // CRC covers everything before the footer
    uint8_t *dst = arena + frame_off[f];
    const int h = (int)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3);  // bytes before dst's first aligned word
    const int64_t hb = min((int64_t)h, L);
    if ((int64_t)threadIdx.x < hb) dst[threadIdx.x] = src[threadIdx.x];
    const int64_t nbw = (L - hb) >> 2;  // whole aligned destination words
    uint32_t *dw = reinterpret_cast<uint32_t *>(dst + hb);
    const int sh = (int)(hb & 3);
    const int64_t swords = slot_words;
    for (int64_t k = threadIdx.x; k < nbw; k += 256) {
        const int64_t sbyte = hb + 4 * k, si = sbyte >> 2;
        const uint32_t lo = sw[si], hi = (sh && si + 1 < swords) ? sw[si + 1] : 0u;
        dw[k] = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)sh);
    }
    for (int64_t i = hb + 4 * nbw + threadIdx.x; i < L; i += 256) dst[i] = src[i];
    const uint32_t crc = wg_crc16(src, L, T, wc);
    if (threadIdx.x == 0) {
        dst[L] = (uint8_t)(crc >> 8);
        dst[L + 1] = (uint8_t)crc;
    }
}

// Fast path: the partial last frames coded by k_encode_frames get their CRC-16 footer in place (slot bytes
// [0, S - 2) -> [S - 2, S)), so k_encode_v3 copies finished frames.
__global__ void __launch_bounds__(256) k_seal_partial(uint32_t *slots, int slot_words, const int64_t *frame_bytes,
                                                     int64_t nlist) {
    __shared__ uint16_t T[4][256];
    __shared__ uint32_t wc[4];
    const int64_t si = blockIdx.x;
    if (si >= nlist) return;
    wg_load_crc_tables(T);
    uint8_t *src = reinterpret_cast<uint8_t *>(slots + (size_t)si * slot_words);
    const int64_t L = frame_bytes[si] - 2;
    const uint32_t crc = wg_crc16(src, L, T, wc);
    if (threadIdx.x == 0) {
        src[L] = (uint8_t)(crc >> 8);
        src[L + 1] = (uint8_t)crc;
    }
}

// Exclusive scan of the generic path's frame sizes in one work-group: out[i] = sum(in[0..i)), out[n] = total.
// Thread t owns the contiguous run [t c, (t + 1) c); run totals are scanned through LDS by wave shuffles.
constexpr int kScanThreads = 1024;
__global__ void __launch_bounds__(kScanThreads) k_scan_sizes(const int64_t *in, int64_t *out, int64_t n) {
    __shared__ int64_t wsum[kScanThreads / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t c = (n + kScanThreads - 1) / kScanThreads;
    const int64_t a = min(n, (int64_t)t * c), b = min(n, a + c);
    int64_t run = 0;
    for (int64_t i = a; i < b; i++) run += in[i];
    int64_t x = run;  // inclusive scan of the run totals within the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int64_t base = 0, total = 0;
    for (int k = 0; k < kScanThreads / 64; k++) {
        base += k < wv ? wsum[k] : 0;
        total += wsum[k];
    }
    int64_t acc = base + x - run;
    for (int64_t i = a; i < b; i++) {
        out[i] = acc;
        acc += in[i];
    }
    if (t == 0) out[n] = total;
}

__global__ void k_gather_tile_off(const int64_t *frame_off, const TileGeom *tiles, int ntiles, int64_t total,
                                  int64_t *tile_off) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ntiles) tile_off[t] = frame_off[tiles[t].frame_base];
    if (t == ntiles) tile_off[t] = total;
}

// =================================================================================================
// FAST PATH (16-bit mono streams: create-streaming band-1 tiles, converter bps 16)
//   k_build_lut     per tile: pcm = lut[x - min] for x - min in [0, R] (exact double path, once per value)
//   k_analyze_v3    lane = frame; 64-sample chunks loaded as 8 x 16 B per lane (no L1 reuse needed),
//                   LUT normalisation, wave-uniform window from LDS, 9 fp64 FMA chains per lane
//   k_encode_v3     persistent WGs, wave = frame, 64 consecutive samples per lane held as packed int16
//                   pairs: fixed totals, v_dot2 residuals, partition sums by lane shuffles, Rice search,
//                   exact bit positions by one wave scan, size published before LDS bit packing,
//                   slice-by-4 CRC-16, decoupled look-back for the arena offset, 16-B aligned stores
// =================================================================================================

// exact converter.py normalisation of one element for the fast kernels (mode per tile)
template <int DT>
__device__ inline int32_t norm_fast(typename Elem<DT>::T x, const TileNorm &tn, const int16_t *lut) {
    if constexpr (Elem<DT>::is_float) {
        (void)tn; (void)lut;
        return 0;  // float rasters never take the fast path (32-bit streams)
    } else {
        const int64_t d = (int64_t)x - tn.imin;
        switch (tn.mode) {
        case kNormLut: return lut[d];
        case kNormZero: return 0;
        case kNormFastDiv: {
            const double a = (double)(2 * d);
            const double q0 = a * tn.rinv;
            const double r = fma(-q0, tn.den, a);
            const double q1 = fma(r, tn.rinv, q0);  // == RN(a / den): verified for every d <= den <= 65535
            const double v = (q1 - 1.0) * 32767.0;
            return (int32_t)(int16_t)cast_f64_i32_x86(v);
        }
        default: {
            using T = typename Elem<DT>::T;
            const T dd = (T)((int64_t)x - tn.imin);
            const double v = ((2.0 * (double)dd) / tn.den - 1.0) * 32767.0;
            return (int32_t)(int16_t)cast_f64_i32_x86(v);
        }
        }
    }
}

// normalise 64 elements of a chunk into int32 (mode is wave-uniform in the callers' common case; the
// switch sits outside the unrolled element loop so the loop body is branch-free)
template <int DT, int N> struct ChunkN;
template <int DT> using Chunk64 = ChunkN<DT, 64>;

// normalise the 64 elements of a chunk (mode is wave-uniform in the encode kernel; the switch sits
// outside the unrolled element loop so the loop body is branch-free).  emit(j, x) in order j = 0..63.
template <int DT, typename Fn>
__device__ inline void norm_chunk(const Chunk64<DT> &ch, const TileNorm &tn, const int16_t *lut, Fn &&emit) {
    switch (tn.mode) {
    case kNormLut: {
        const int32_t mn = (int32_t)tn.imin;
#pragma unroll
        for (int j = 0; j < 64; j++) emit(j, (int32_t)lut[(int32_t)ch.get(j) - mn]);
        break;
    }
    case kNormZero:
#pragma unroll
        for (int j = 0; j < 64; j++) emit(j, 0);
        break;
    case kNormFastDiv: {
        const int32_t mn = (int32_t)tn.imin;
        const double rinv = tn.rinv, den = tn.den;
#pragma unroll
        for (int j = 0; j < 64; j++) {
            const double a = (double)(2 * ((int32_t)ch.get(j) - mn));
            const double q0 = a * rinv;
            const double r = fma(-q0, den, a);
            const double q1 = fma(r, rinv, q0);
            emit(j, (int32_t)(int16_t)(int32_t)((q1 - 1.0) * 32767.0));
        }
        break;
    }
    default:  // kNormSlow: the exact IEEE division (norm_fast's last case, without its per-element mode switch)
#pragma unroll
        for (int j = 0; j < 64; j++) {
            using T = typename Elem<DT>::T;
            const T dd = (T)((int64_t)ch.get(j) - tn.imin);
            emit(j, (int32_t)(int16_t)cast_f64_i32_x86(((2.0 * (double)dd) / tn.den - 1.0) * 32767.0));
        }
        break;
    }
}

// LUT entry d = x - min of a kNormLut tile (exact double path: numpy 2.0*(x-min)/(max-min)-1.0, *32767)
template <int DT> __device__ inline int16_t lut_entry(const TileNorm &tn, int64_t d) {
    using T = typename Elem<DT>::T;
    const T dd = (T)d;
    const double v = ((2.0 * (double)dd) / tn.den - 1.0) * 32767.0;
    return (int16_t)cast_f64_i32_x86(v);
}

template <int DT>
__global__ void __launch_bounds__(256) k_build_lut(const TileNorm *norms, int16_t *luts) {
    const int t = blockIdx.x;
    const TileNorm tn = norms[t];
    if (tn.mode != kNormLut) return;
    const int64_t R = tn.imax - tn.imin;
    for (int64_t d = threadIdx.x; d <= R; d += blockDim.x) luts[(int64_t)t * kLutCap + d] = lut_entry<DT>(tn, d);
}

// n / d for n < 2^32 via a double reciprocal (inv = 1.0 / d): the estimate is off by at most one, fixed up
__device__ inline uint32_t udiv_inv(uint32_t n, uint32_t d, double inv) {
    uint32_t q = (uint32_t)((double)n * inv);
    const int64_t r = (int64_t)n - (int64_t)q * d;
    q = r < 0 ? q - 1 : (r >= (int64_t)d ? q + 1 : q);
    return q;
}

// N (32 or 64) consecutive elements of a frame, kept packed in 32-bit words (int16, N = 64: 32 words).
// vec: 16-byte loads of one row segment; otherwise an element gather with a row cursor.
template <int DT, int N> struct ChunkN {
    using T = typename Elem<DT>::T;
    static constexpr int kWords = (int)(N * sizeof(T) / 4);
    static_assert(kWords % 4 == 0, "chunk = whole 16-byte loads");
    uint32_t w[kWords];
    __device__ inline void unpack(T *out) const {
#pragma unroll
        for (int j = 0; j < N; j++) out[j] = get(j);
    }
    __device__ inline T get(int j) const {  // j must be a compile-time constant after unrolling
        if constexpr (sizeof(T) == 1) return (T)((w[j >> 2] >> (8 * (j & 3))) & 0xFFu);
        else if constexpr (sizeof(T) == 2) return (T)((w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
        else return __builtin_bit_cast(T, w[j]);
    }
    // 16-byte loads of one row segment (p 16-B aligned, the 64 elements inside one row)
    __device__ inline void load_vec(const T *p_) {
        const uint4 *p = reinterpret_cast<const uint4 *>(p_);
#pragma unroll
        for (int k = 0; k < kWords / 4; k++) {
            const uint4 v = p[k];
            w[4 * k] = v.x;
            w[4 * k + 1] = v.y;
            w[4 * k + 2] = v.z;
            w[4 * k + 3] = v.w;
        }
    }
    // element gather with a row cursor starting at (row, col): tiles whose width is not a multiple of the chunk
    // (edge tiles, odd tile sizes).  Fully unrolled: the cursor advances by per-lane selects, so all N loads issue
    // before the first wait; 16-bit samples land pairwise in the halves of one register (d16 / d16_hi loads).
    // The fast paths only load whole chunks of full frames (nvalid == N).
    __device__ inline void load_gather_unrolled(const T *base, int64_t row_stride, int width, int64_t row, int col,
                                                int nvalid) {
        (void)nvalid;
        const T *rp = base + row * row_stride;
        auto next = [&]() {
            if (++col == width) {
                col = 0;
                rp += row_stride;
            }
        };
        if constexpr (sizeof(T) == 2) {
            typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int k = 0; k < kWords; k++) {
                u16x2 pr;
                pr.x = __builtin_bit_cast(unsigned short, rp[col]);
                next();
                pr.y = __builtin_bit_cast(unsigned short, rp[col]);
                next();
                w[k] = __builtin_bit_cast(uint32_t, pr);
            }
        } else if constexpr (sizeof(T) == 4) {
#pragma unroll
            for (int k = 0; k < kWords; k++) {
                w[k] = __builtin_bit_cast(uint32_t, rp[col]);
                next();
            }
        } else {
#pragma unroll
            for (int k = 0; k < kWords; k++) {
                uint32_t v = 0;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    v |= (uint32_t)(uint8_t)rp[col] << (8 * b);
                    next();
                }
                w[k] = v;
            }
        }
    }
    // compact element gather (the encoder's: the unrolled form above costs it registers and scheduling freedom even
    // where no tile needs it -- C4's encode 4.2 -> 5.0 ms)
    __device__ inline void load_gather(const T *base, int64_t row_stride, int width, int64_t row, int col,
                                       int nvalid) {
#pragma unroll
        for (int k = 0; k < kWords; k++) w[k] = 0;
        const T *rp = base + row * row_stride;
        for (int j = 0; j < nvalid; j++) {
            uint32_t v;
            if constexpr (sizeof(T) == 4) v = __builtin_bit_cast(uint32_t, rp[col]);
            else v = (uint32_t)(std::make_unsigned_t<T>)rp[col];
#pragma unroll
            for (int k = 0; k < kWords; k++) {
                constexpr int per = 4 / (int)sizeof(T);
                if (k == j / per) {
                    const int sh = (int)(8 * sizeof(T)) * (j % per);
                    w[k] |= (sizeof(T) == 4) ? v : (v << sh);
                }
            }
            if (++col == width) {
                col = 0;
                rp += row_stride;
            }
        }
    }
    // 8- / 4-byte loads of one row segment (rows only 8- or 4-byte aligned, e.g. a 10980-sample int16 row)
    __device__ inline void load_vec8(const T *p_) {
        const uint2 *p = reinterpret_cast<const uint2 *>(p_);
#pragma unroll
        for (int k = 0; k < kWords / 2; k++) {
            const uint2 v = p[k];
            w[2 * k] = v.x;
            w[2 * k + 1] = v.y;
        }
    }
    __device__ inline void load_vec4(const T *p_) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(p_);
#pragma unroll
        for (int k = 0; k < kWords; k++) w[k] = p[k];
    }
    // vec = the row segments' alignment class (EncodeParams::vec_ok): 16, 8 or 4 bytes, 0 = element gather
    template <bool UNROLLED_GATHER = false>
    __device__ inline void load(const T *base, int64_t row_stride, int width, int64_t row, int col, int vec,
                                int nvalid) {
        const T *p = base + row * row_stride + col;
        if (vec == 16) load_vec(p);
        else if (vec == 8) load_vec8(p);
        else if (vec == 4) load_vec4(p);
        else if constexpr (UNROLLED_GATHER) load_gather_unrolled(base, row_stride, width, row, col, nvalid);
        else load_gather(base, row_stride, width, row, col, nvalid);
    }
};

// Raw-frames tiles (`convert --spatial`: 32-bit streams of pyflac's truncated floats): a DEM's samples
// normalise to 0 almost everywhere, and k_analyze / k_analyze_fixed_wide would still walk every such subframe one
// sample at a time on one lane.  One wave per coded signal (frame, channel) ORs its normalised samples instead (each
// lane 64 consecutive samples, vector loads when the tile width is a multiple of 64 and the rows are aligned); an
// all-zero subframe gets its SubAnalysis here -- the decisions those two kernels make on all-zero sums
// (generic_decide: no wasted bits, fixed guess 0, no LPC since autoc[0] == 0; the limit_residual estimator: order 0,
// bits 0), flagged kFlagZero -- and zero[sub] = 1 makes them skip it.
template <int DT>
__global__ void __launch_bounds__(256) k_zero_subframes(const typename Elem<DT>::T *raster, EncodeParams P,
                                                       const TileGeom *tiles, const TileNorm *norms, SubAnalysis *out,
                                                       uint8_t *zero) {
    using T = typename Elem<DT>::T;
    const int64_t sub = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (sub >= P.nframes * P.nvch) return;
    const int64_t f = sub / P.nvch;
    const int ch = (int)(sub - f * P.nvch);
    const int t = tile_of_frame(tiles, P.ntiles, f);
    const TileGeom g = tiles[t];
    const int64_t s0 = (f - g.frame_base) * P.blocksize;
    const int64_t tile_px = (int64_t)g.h * g.w;
    const int n = (int)((tile_px - s0) < P.blocksize ? (tile_px - s0) : P.blocksize);
    const Normalizer<DT> nz = make_norm<DT>(norms[t], P.scale_bits, P.norm_mode);
    const T *band = raster + (int64_t)(P.band0 + ch) * P.band_stride + g.r0 * P.row_stride + g.c0;
    uint32_t o = 0;
    for (int i0 = 64 * lane; i0 < n; i0 += 64 * 64) {  // (blocksize 4096: one pass)
        const int64_t q = s0 + i0, r = q / g.w;
        const int col = (int)(q - r * g.w);
        const int cnt = n - i0 < 64 ? n - i0 : 64;
        const int vec = (cnt == 64 && (g.w % 64) == 0) ? P.vec_ok : 0;
        if constexpr (sizeof(T) <= 4) {
            if (vec) {
                Chunk64<DT> chk;
                chk.load(band, P.row_stride, g.w, r, col, vec, 64);
#pragma unroll
                for (int j = 0; j < 64; j++) o |= (uint32_t)nz(chk.get(j));
                continue;
            }
        }
        int c = col;
        const T *rowp = band + r * P.row_stride;
        for (int j = 0; j < cnt; j++) {
            o |= (uint32_t)nz(rowp[c]);
            if (++c == g.w) {
                c = 0;
                rowp += P.row_stride;
            }
        }
    }
    const bool z = __ballot(o != 0) == 0;
    if (lane == 0) {
        zero[sub] = z ? 1 : 0;
        if (z) {
            double acc[kMaxLpc + 1];
#pragma unroll
            for (int l = 0; l <= kMaxLpc; l++) acc[l] = 0.0;
            const uint64_t tt[5] = {0, 0, 0, 0, 0};
            const bool valid[5] = {true, true, true, true, true};
            SubAnalysis A = generic_decide<true>(acc, tt, 0, 0, n, P, 0);
            if (n > 4) fixed_wide_decide(A, tt, valid, n, P.bps - A.wasted, []() { return true; });
            A.flags |= kFlagZero;
            out[sub] = A;
        }
    }
}

// A frame whose every subframe is all-zero (kFlagZero, more than 4 samples): what k_encode_frames writes for it,
// without its work-group per frame -- decide() on all-zero sums keeps FIXED order 0 (the verbatim, LPC and constant
// candidates are out: no LPC since autoc[0] == 0, and the limit_residual estimator's bits[1] is 34), and libFLAC's
// Rice estimate (set_partitioned_rice_) is 4 + ceil(ns / 2) bits per partition at parameter 0, so partition order 0
// wins.  Subframe: 8 header bits (0x10: FIXED, order 0, no wasted bits), RICE method and partition order (6 zero bits),
// the parameter 0 (4 bits), then n codes of the single stop bit '1'.  One wave per frame writes the frame's words to
// its slot (byte order, as k_encode_frames' flush) and its byte count incl. the CRC-16 footer (k_compact adds it).
__global__ void __launch_bounds__(256) k_zero_frames_emit(EncodeParams P, const TileGeom *tiles,
                                                         const SubAnalysis *ana, uint32_t *slots,
                                                         int64_t *frame_bytes) {
    const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (f >= P.nframes) return;
    bool all0 = true;
    for (int c = 0; c < P.nch; c++) all0 = all0 && (ana[f * P.nvch + c].flags & kFlagZero);
    const int t = tile_of_frame(tiles, P.ntiles, f);
    const TileGeom g = tiles[t];
    const int64_t fk = f - g.frame_base;
    const int64_t tile_px = (int64_t)g.h * g.w;
    const int n = (int)((tile_px - fk * P.blocksize) < P.blocksize ? (tile_px - fk * P.blocksize) : P.blocksize);
    if (!all0 || n <= 4) return;  // (k_encode_frames codes it)
    uint8_t h[16];
    const int hb = generic_frame_header(h, n, P, P.nch - 1, (uint32_t)fk);
    const uint32_t hbits = (uint32_t)hb * 8, sbits = 18u + (uint32_t)n;
    const uint32_t bits = hbits + (uint32_t)P.nch * sbits;
    const uint32_t nwords = (bits + 31) >> 5;
    uint32_t *slot = slots + (size_t)f * P.slot_words;
    for (uint32_t wi = (uint32_t)lane; wi < nwords; wi += 64) {
        uint32_t v = 0;  // MSB-first bits [32 wi, 32 wi + 32)
        for (int k = 0; k < 4; k++) {
            const uint32_t byte = 4 * wi + (uint32_t)k;
            if (byte < (uint32_t)hb) v |= (uint32_t)h[byte] << (24 - 8 * k);
        }
        for (int c = 0; c < P.nch; c++) {
            const uint32_t b0 = hbits + (uint32_t)c * sbits;
            // 0x10 at [b0, b0 + 8): its one bit at b0 + 3; ones at [b0 + 18, b0 + sbits)
            const uint32_t one = b0 + 3;
            if (one >= 32 * wi && one < 32 * wi + 32) v |= 0x80000000u >> (one - 32 * wi);
            const uint32_t a = b0 + 18, e = b0 + sbits;
            const uint32_t lo = a > 32 * wi ? a : 32 * wi, hi = e < 32 * wi + 32 ? e : 32 * wi + 32;
            if (hi > lo) {
                const uint32_t nb = hi - lo, sh = 32 * wi + 32 - hi;
                v |= (nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u)) << sh;
            }
        }
        slot[wi] = __builtin_bswap32(v);
    }
    if (lane == 0) frame_bytes[f] = (int64_t)((bits + 7) >> 3) + 2;
}

// normalise elements [8b, 8b + 8) of a chunk (b compile-time after unrolling)
template <int DT>
__device__ inline void norm_block8(const Chunk64<DT> &ch, int b, const TileNorm &tn, const int16_t *lut, int32_t *x) {
    switch (tn.mode) {
    case kNormLut: {
        const int32_t mn = (int32_t)tn.imin;
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = (int32_t)lut[(int32_t)ch.get(8 * b + j) - mn];
        break;
    }
    case kNormZero:
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = 0;
        break;
    case kNormFastDiv: {
        const int32_t mn = (int32_t)tn.imin;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const double a = (double)(2 * ((int32_t)ch.get(8 * b + j) - mn));
            const double q0 = a * tn.rinv;
            const double r = fma(-q0, tn.den, a);
            const double q1 = fma(r, tn.rinv, q0);
            x[j] = (int32_t)(int16_t)(int32_t)((q1 - 1.0) * 32767.0);
        }
        break;
    }
    default:
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = norm_fast<DT>(ch.get(8 * b + j), tn, lut);
        break;
    }
}

// wasted bits, LPC order choice (expected bits), Levinson coefficients and quantisation of one frame from its
// windowed autocorrelation sums (stream_encoder.c process_subframe_ / lpc.c)
__device__ inline SubAnalysis analysis_finish(const double *acc, uint32_t or_acc, int n, const EncodeParams &P,
                                              const uint32_t *ft, int extra = 0) {
    SubAnalysis A;
    A.n = n;
    int w = or_acc ? __builtin_ctz(or_acc) : 0;
    if (w > P.bps) w = P.bps;
    const int sbps = P.bps - w + extra;  // (extra = 1: a two-channel stream's side signal)
    A.wasted = w;
    A.flags = 0;
    {
        // fixed.c FLAC__fixed_compute_best_predictor on the shifted samples: every e_k is a multiple of 2^w, so the
        // shifted totals are the unshifted ones >> w exactly; first minimum under <= comparisons
        const uint32_t T0 = ft[0] >> w, T1 = ft[1] >> w, T2 = ft[2] >> w, T3 = ft[3] >> w, T4 = ft[4] >> w;
        int guess;
        if (T0 <= min(min(T1, T2), min(T3, T4))) guess = 0;
        else if (T1 <= min(min(T2, T3), T4)) guess = 1;
        else if (T2 <= min(T3, T4)) guess = 2;
        else if (T3 <= T4) guess = 3;
        else guess = 4;
        A.fixed_order = guess;
        A.fixed_tg = guess == 0 ? T0 : guess == 1 ? T1 : guess == 2 ? T2 : guess == 3 ? T3 : T4;
        A.fixed_t1 = T1;
    }
    A.lpc_order = 0;
    A.lpc_prec = 0;
    A.lpc_shift = 0;
#pragma unroll
    for (int j = 0; j < kMaxLpc; j++) A.q[j] = 0;
    int max_order = kMaxLpc < n ? kMaxLpc : n - 1;
    double autoc[kMaxLpc + 1];
    const double sc = ldexp(1.0, -2 * w);
#pragma unroll
    for (int l = 0; l <= kMaxLpc; l++) autoc[l] = acc[l] * sc;
    if (n > 4 && max_order > 0 && autoc[0] != 0.0) {
        double err[kMaxLpc];
        const int mo = levinson_errors(autoc, max_order, err);
        const double es = 0.5 / (double)n;
        const int ovh = sbps + P.qlp_precision;
        int best = 0;
        double best_bits = (double)(unsigned)(-1);
#pragma unroll
        for (int i = 0; i < kMaxLpc; i++) {
            if (i < mo) {
                const int o = i + 1;
                const double b = expected_bits(err[i], es) * (double)(n - o) + (double)(o * ovh);
                if (b < best_bits) {
                    best = i;
                    best_bits = b;
                }
            }
        }
        const int o = best + 1;
        double eo = err[0];
#pragma unroll
        for (int i = 1; i < kMaxLpc; i++)
            if (i == best) eo = err[i];
        const double lbits = expected_bits(eo, 0.5 / (double)(n - o));
        if (!(lbits >= (double)sbps)) {
            int prec = P.qlp_precision;
            if (sbps <= 17) {
                const int lim = 32 - sbps - ilog2_u32((uint32_t)o);
                prec = lim < prec ? lim : prec;
            }
            float lp[kMaxLpc];
            levinson_coefs(autoc, o, lp);
            const int pm1 = prec - 1;
            const int32_t qmax = (1 << pm1) - 1, qmin = -(1 << pm1);
            double cmax = 0.0;
#pragma unroll
            for (int j = 0; j < kMaxLpc; j++)
                if (j < o) {
                    const double dd = fabs((double)lp[j]);
                    if (dd > cmax) cmax = dd;
                }
            if (cmax > 0.0) {
                int shift = pm1 - ilogb(cmax) - 1;
                bool ok = true;
                if (shift > 15) shift = 15;
                else if (shift < -16) ok = false;
                if (ok) {
                    double error = 0.0;
                    if (shift >= 0) {
                        const float m = (float)(1 << shift);
#pragma unroll
                        for (int j = 0; j < kMaxLpc; j++)
                            if (j < o) {
                                error += (double)(lp[j] * m);
                                int64_t qi = lround_exact(error);
                                qi = qi > qmax ? qmax : (qi < qmin ? qmin : qi);
                                error -= (double)qi;
                                A.q[j] = (int32_t)qi;
                            }
                    } else {
                        const float m = (float)(1 << (-shift));
#pragma unroll
                        for (int j = 0; j < kMaxLpc; j++)
                            if (j < o) {
                                error += (double)(lp[j] / m);
                                int64_t qi = lround_exact(error);
                                qi = qi > qmax ? qmax : (qi < qmin ? qmin : qi);
                                error -= (double)qi;
                                A.q[j] = (int32_t)qi;
                            }
                        shift = 0;
                    }
                    A.lpc_order = o;
                    A.lpc_prec = prec;
                    A.lpc_shift = shift;
                    A.flags |= kFlagLpcOk;
                }
            }
        }
    }
    return A;
}

// ------------------------------------------------------------------------------ k_analyze_v3
// the prefetching analysis (PF) below this many 64-frame groups (waves) with fused stats: C3's 1024 tiles take it, C4's
// 6241 keep occupancy 4
constexpr int kPfMaxWaves = 1536;
// Lane = frame (libFLAC's sequential fp64 autocorrelation per lane), laid
// out for occupancy and memory-level parallelism: a wave takes up to 64 frames of ONE tile (host wave table),
// so the normaliser is wave-uniform and chosen once (LUT in LDS read by ds_read / zeros / fast division /
// exact division) instead of a per-sample switch; each lane loads its next 64 samples as one 128-byte line
// (8 x 16 B; 16 samples in the fp64-division class) and normalises them 8 at a time straight into doubles.
constexpr int kAnaKindLds = 0, kAnaKindZero = 1, kAnaKindFastDiv = 2, kAnaKindGeneric = 3;

template <int DT, int KIND>
__device__ inline int32_t ana_norm(typename Elem<DT>::T x, const TileNorm &tn, const int16_t *slut,
                                   const int16_t *glut) {
    if constexpr (KIND == kAnaKindLds) {
        return (int32_t)slut[(int32_t)x - (int32_t)tn.imin];
    } else if constexpr (KIND == kAnaKindZero) {
        return 0;
    } else if constexpr (KIND == kAnaKindFastDiv) {
        const double a = (double)(2 * ((int32_t)x - (int32_t)tn.imin));
        const double q0 = a * tn.rinv;
        const double r = fma(-q0, tn.den, a);
        const double q1 = fma(r, tn.rinv, q0);
        return (int32_t)(int16_t)(int32_t)((q1 - 1.0) * 32767.0);
    } else {
        return norm_fast<DT>(x, tn, glut);
    }
}

__device__ inline uint32_t ana_sad(uint32_t a, uint32_t b, uint32_t c) {  // |a - b| + c (v_sad_u32)
    uint32_t d;
    asm("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// ST: `base` is the left band and sig (0..3) the coded signal of a two-channel stream's mid/side pass: left, right,
// mid = (L + R) >> 1, side = L - R (converter.py:185-194 interleaves the bands; libFLAC process_subframes_ forms mid
// and side from the normalised samples)
// SIG >= 0 (ST): the signal fixed at compile time, so a wave loads and normalises only the bands it needs
// PF (small jobs, k_analyze_v3<..., PF>): the next chunk's loads are issued before the current chunk is summed
template <int DT, int KIND, int kAnaChunk, bool ST = false, int SIG = -1, bool PF = false>
__device__ inline void ana_autoc(const typename Elem<DT>::T *base, const EncodeParams &P, const TileGeom &g,
                                 int64_t s0, const TileNorm &tn, const int16_t *slut, const int16_t *glut,
                                 const float *__restrict__ swin, int vec, double *acc, uint32_t &or_acc, uint32_t *ft,
                                 int sig_rt = 0) {
    const int sig = SIG >= 0 ? SIG : sig_rt;
    using Ch = ChunkN<DT, kAnaChunk>;
    const uint32_t r0 = udiv_inv((uint32_t)s0, (uint32_t)g.w, 1.0 / (double)g.w);
    int64_t crow = r0;
    int ccol = (int)((uint32_t)s0 - r0 * (uint32_t)g.w);
    double prev[8];
#pragma unroll
    for (int j = 0; j < 8; j++) prev[j] = 0.0;
    // (the fixed-predictor totals of fixed.c are the encoder's: encode_frame_v4 forms them lane-parallel from the
    // samples it has loaded anyway, which takes ~12 integer ops per sample out of this fp64-bound pass)
    static_assert(!(PF && ST), "prefetch: single-band signals");
    Ch pf;  // PF: the chunk whose loads are in flight
    if constexpr (PF) {
        pf.template load<true>(base, P.row_stride, g.w, crow, ccol, vec, kAnaChunk);
        ccol += kAnaChunk;
        while (ccol >= g.w) {
            ccol -= g.w;
            crow++;
        }
    }
    for (int c = 0; c < kMaxBlock / kAnaChunk; c++) {
        const int i0 = c * kAnaChunk;
        Ch ch, ch1;
        if constexpr (PF) {
            ch = pf;
            if (c + 1 < kMaxBlock / kAnaChunk) pf.template load<true>(base, P.row_stride, g.w, crow, ccol, vec, kAnaChunk);
        } else {
            if (!ST || sig != 1) ch.template load<true>(base, P.row_stride, g.w, crow, ccol, vec, kAnaChunk);
            if (ST && sig >= 1) ch1.template load<true>(base + P.band_stride, P.row_stride, g.w, crow, ccol, vec, kAnaChunk);
        }
        ccol += kAnaChunk;
        while (ccol >= g.w) {
            ccol -= g.w;
            crow++;
        }
#pragma unroll
        for (int b = 0; b < kAnaChunk / 8; b++) {
            double cur[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                int32_t x;
                if constexpr (ST) {
                    const int32_t l = sig == 1 ? 0 : ana_norm<DT, KIND>(ch.get(8 * b + j), tn, slut, glut);
                    const int32_t r = sig == 0 ? 0 : ana_norm<DT, KIND>(ch1.get(8 * b + j), tn, slut, glut);
                    x = sig == 0 ? l : sig == 1 ? r : sig == 2 ? (l + r) >> 1 : l - r;
                } else {
                    x = ana_norm<DT, KIND>(ch.get(8 * b + j), tn, slut, glut);
                }
                or_acc |= (uint32_t)x;
                cur[j] = (double)((float)x * swin[i0 + 8 * b + j]);  // lpc.c window_data: float product
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
#pragma unroll
                for (int l = 0; l <= kMaxLpc; l++) acc[l] = fma(cur[j], (j - l >= 0) ? cur[j - l] : prev[8 + j - l], acc[l]);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) prev[j] = cur[j];
        }
    }
#pragma unroll
    for (int k = 0; k < 5; k++) ft[k] = 0;  // (unused: the encoder forms the fixed totals)
}

// min/max of a whole tile by one wave (16-bit samples, 16-B aligned rows): 16-B loads, kStatsLoads in flight per lane,
// packed 16-bit min/max; the tile's vectors are dealt out lane-major (vector i to lane i % 64), lanes past the
// end re-read vector 0.  Returns the keys (elem_key order) in lo/hi, wave-uniform.
constexpr int kStatsLoads = 16;
template <int DT>
__device__ inline void wave_tile_minmax(const typename Elem<DT>::T *base, int64_t row_stride, const TileGeom &g,
                                        int lane, int64_t &lo, int64_t &hi) {
    using T = typename Elem<DT>::T;
    static_assert(sizeof(T) == 2, "16-bit samples");
    using V = std::conditional_t<std::is_signed_v<T>, v2i16, v2u16>;
    using E16 = std::conditional_t<std::is_signed_v<T>, short, unsigned short>;
    V vmin = (V)(std::is_signed_v<T> ? (E16)32767 : (E16)65535), vmax = (V)(std::is_signed_v<T> ? (E16)-32768 : (E16)0);
    const int nvec = g.w / 8;  // 16-B vectors per row
    const int total = g.h * nvec;
    const int dq = 64 / nvec, dr = 64 - dq * nvec;  // advance of a lane's (row, vector) per 64 vectors
    int row = lane / nvec, v = lane - row * nvec;
    const char *b = reinterpret_cast<const char *>(base);
    const int64_t rs = row_stride * 2;
    const int iters = (total + 64 * kStatsLoads - 1) / (64 * kStatsLoads);
    for (int it = 0; it < iters; it++) {
        uint4 q[kStatsLoads];
#pragma unroll
        for (int u = 0; u < kStatsLoads; u++) {
            const bool ok = row < g.h;
            q[u] = *reinterpret_cast<const uint4 *>(b + (ok ? row * rs + v * 16 : 0));
            v += dr;
            row += dq;
            if (v >= nvec) {
                v -= nvec;
                row++;
            }
        }
#pragma unroll
        for (int u = 0; u < kStatsLoads; u++) {
            const uint32_t w4[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const V x = __builtin_bit_cast(V, w4[k]);
                vmin = __builtin_elementwise_min(vmin, x);
                vmax = __builtin_elementwise_max(vmax, x);
            }
        }
    }
    int32_t l = min((int32_t)vmin.x, (int32_t)vmin.y), h = max((int32_t)vmax.x, (int32_t)vmax.y);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        l = min(l, __shfl_xor(l, o));
        h = max(h, __shfl_xor(h, o));
    }
    lo = l;
    hi = h;
}

// Two launches of one kernel body keep the common case lean: SLOW = false takes the tiles normalised by LUT (or
// zeros) -- ~120 VGPRs, 4 waves/SIMD; SLOW = true takes the fast-division / exact-division tiles, whose fp64
// normalisation needs more registers.  A wave of the other class returns at once.
// STATS = true (SLOW = false, 16-bit samples, every tile one wave): the wave first computes its tile's min/max
// and normalisation parameters (k_tile_stats_vec + k_tile_finalize) and builds the tile's LUT (k_build_lut) in
// LDS and in global memory for the encoder -- the tile is read twice, but the separate stats pass and its
// launches are gone.  A slow-class tile only gets its parameters written here; the SLOW launch analyses it.
// PF (small fused-stats jobs: fewer 64-frame groups than about 1.5 waves per SIMD, e.g. C3's 1024 tiles): a lone wave
// per SIMD waits on each chunk's loads in turn, so the next chunk's loads are issued before the current one is
// summed.  136 instead of 127 VGPRs (occupancy 3 instead of 4): the large jobs (C4) keep the plain form.
template <int DT, bool SLOW, bool STATS = false, bool ST = false, bool PF = false>
__global__ void __launch_bounds__(256) k_analyze_v3(const typename Elem<DT>::T *raster, EncodeParams P,
                                                   const TileGeom *tiles, TileNorm *norms,
                                                   int16_t *luts, const float *__restrict__ window,
                                                   SubAnalysis *out, const int2 *__restrict__ wtab, int nwaves) {
    static_assert(!(SLOW && STATS), "stats are fused into the lean launch only");
    static_assert(!(PF && (SLOW || ST)), "prefetch: the lean mono / multi-channel launch");
    __shared__ int16_t slut[SLOW ? 1 : 4][SLOW ? 1 : kLutCap];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wv = blockIdx.x * 4 + wave;
    if (wv >= nwaves) return;
    const int2 wt = wtab[wv];  // (tile, first frame of the tile handled by this wave)
    const int t = wt.x, k0w = wt.y & 0xFFFFFF, chn = wt.y >> 24;  // (tile, first frame | channel << 24)
    const TileGeom g = tiles[t];
    // (ST: the left band; ana_autoc reads the right one at + band_stride)
    const typename Elem<DT>::T *base = raster + (int64_t)(P.band0 + (ST ? 0 : chn)) * P.band_stride +
                                       g.r0 * P.row_stride + g.c0;
    int16_t *glut = luts + (int64_t)t * kLutCap;
    TileNorm tn;
    if constexpr (STATS) {
        if constexpr (sizeof(typename Elem<DT>::T) == 2 && !Elem<DT>::is_float) {
            wave_tile_minmax<DT>(base, P.row_stride, g, lane, tn.imin, tn.imax);
            tile_norm_finalize<DT>(tn, P.norm_mode, P.scale_bits);
            if (lane == 0) norms[t] = tn;
        }
    } else {
        tn = norms[t];
    }
    const int mode = tn.mode;  // wave-uniform: one tile per wave
    const bool lean = mode == kNormLut || mode == kNormZero;
    if (lean == SLOW) return;
    const int nfull = g.nframes - (g.partial ? 1 : 0);  // a partial last frame is analysed by k_analyze
    if (nfull == 0) return;                              // (wave-uniform) only its stats were needed here
    const bool live = k0w + lane < nfull;
    const int64_t fk = live ? k0w + lane : nfull - 1;  // dead lanes re-read the tile's last full frame
    const int64_t f = g.frame_base + fk;
    const int64_t s0 = fk * P.blocksize;
    const int64_t tile_px = (int64_t)g.h * g.w;
    const int n = live ? (int)min((int64_t)P.blocksize, tile_px - s0) : 0;
    constexpr int kChunk = SLOW ? 16 : 64;  // samples per lane load (SLOW: fewer VGPRs beside the fp64 division)
    const int vec = (g.w % kChunk) == 0 ? P.vec_ok : 0;
    double acc[kMaxLpc + 1];
#pragma unroll
    for (int l = 0; l <= kMaxLpc; l++) acc[l] = 0.0;
    uint32_t or_acc = 0, ft[5];
    // ST: one specialisation per coded signal (left / right read one band, mid / side both, in half-size chunks):
    // the runtime-selected form kept both bands' chunks and normalisations live (242 VGPRs, 2 waves per SIMD)
#define FRS_ANA_SIG(KIND, SLUT)                                                                                           \
    do {                                                                                                                \
        if constexpr (ST) {                                                                                             \
            if (chn == 0)                                                                                               \
                ana_autoc<DT, KIND, kChunk, true, 0>(base, P, g, s0, tn, SLUT, glut, window, vec, acc, or_acc, ft);     \
            else if (chn == 1)                                                                                          \
                ana_autoc<DT, KIND, kChunk, true, 1>(base, P, g, s0, tn, SLUT, glut, window, vec, acc, or_acc, ft);     \
            else if (chn == 2)                                                                                          \
                ana_autoc<DT, KIND, kChunkMS, true, 2>(base, P, g, s0, tn, SLUT, glut, window, vec, acc, or_acc, ft);   \
            else                                                                                                        \
                ana_autoc<DT, KIND, kChunkMS, true, 3>(base, P, g, s0, tn, SLUT, glut, window, vec, acc, or_acc, ft);   \
        } else {                                                                                                        \
            ana_autoc<DT, KIND, kChunk, false, -1, PF>(base, P, g, s0, tn, SLUT, glut, window, vec, acc, or_acc, ft,  \
                                                       chn);                                                            \
        }                                                                                                               \
    } while (0)
    constexpr int kChunkMS = kChunk > 16 ? kChunk / 2 : kChunk;
    if constexpr (!SLOW) {
        int16_t *wl = slut[wave];
        if (mode == kNormLut) {
            const int64_t R = tn.imax - tn.imin;
            if constexpr (STATS) {
                for (int64_t d = lane; d <= R; d += 64) {
                    const int16_t e = lut_entry<DT>(tn, d);
                    wl[d] = e;
                    glut[d] = e;
                }
            } else {
                for (int64_t d = lane; d <= R; d += 64) wl[d] = glut[d];
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's LUT stores have landed (each wave reads only its own)
            __builtin_amdgcn_wave_barrier();
            FRS_ANA_SIG(kAnaKindLds, wl);
        } else {
            FRS_ANA_SIG(kAnaKindZero, wl);
        }
    } else {
        if (mode == kNormFastDiv)
            FRS_ANA_SIG(kAnaKindFastDiv, nullptr);
        else
            FRS_ANA_SIG(kAnaKindGeneric, nullptr);
    }
    if (!live) return;
    out[f * P.nvch + chn] = analysis_finish(acc, or_acc, n, P, ft, (ST && chn == 3) ? 1 : 0);
#undef FRS_ANA_SIG
}

// ---- wave helpers (64 lanes)
__device__ inline uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ inline uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ inline uint32_t wave_or_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
    return v;
}
// exclusive scan of a 64-bit per-lane value
__device__ inline uint64_t wave_excl_scan_u64(uint64_t v, int lane) {
    uint64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(incl, d);
        if (lane >= d) incl += y;
    }
    return incl - v;
}

// ---- cross-lane primitives without LDS round trips: DPP within rows of 16, permlane16/32_swap across
//      rows (gfx950).  Butterfly steps must be applied in order 1, 2, 4, 8, 16, 32 (the mirror patterns
//      pair whole sub-groups only once the lower steps have made each sub-group uniform).
template <int CTRL> __device__ inline uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int STEP> __device__ inline uint32_t bfly_partner(uint32_t v);
template <> __device__ inline uint32_t bfly_partner<1>(uint32_t v) { return dpp_mov<0xB1>(v); }   // quad_perm [1,0,3,2]
template <> __device__ inline uint32_t bfly_partner<2>(uint32_t v) { return dpp_mov<0x4E>(v); }   // quad_perm [2,3,0,1]
template <> __device__ inline uint32_t bfly_partner<4>(uint32_t v) { return dpp_mov<0x141>(v); }  // row_half_mirror
template <> __device__ inline uint32_t bfly_partner<8>(uint32_t v) { return dpp_mov<0x140>(v); }  // row_mirror
template <> __device__ inline uint32_t bfly_partner<16>(uint32_t v) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return p[0] ^ p[1] ^ v;  // one of p[0], p[1] is v itself, the other the partner row's value
}
template <> __device__ inline uint32_t bfly_partner<32>(uint32_t v) {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return p[0] ^ p[1] ^ v;
}
template <int STEP> __device__ inline uint64_t bfly_partner64(uint64_t v) {
    return ((uint64_t)bfly_partner<STEP>((uint32_t)(v >> 32)) << 32) | bfly_partner<STEP>((uint32_t)v);
}
__device__ inline uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ inline uint32_t dpp_wave_sum_u32(uint32_t v) {  // total, wave-uniform (SGPR)
    v += bfly_partner<1>(v);
    v += bfly_partner<2>(v);
    v += bfly_partner<4>(v);
    v += bfly_partner<8>(v);
    v += bfly_partner<16>(v);
    v += bfly_partner<32>(v);
    return uni(v);
}
// N independent wave sums advanced in lockstep (their DPP/permlane wait states overlap)
template <int N> __device__ inline void dpp_wave_sum_multi(const uint32_t *in, uint32_t *out) {
    uint32_t v[N];
#pragma unroll
    for (int i = 0; i < N; i++) v[i] = in[i];
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += bfly_partner<1>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += bfly_partner<2>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += bfly_partner<4>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += bfly_partner<8>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += bfly_partner<16>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += bfly_partner<32>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) out[i] = uni(v[i]);
}
__device__ inline uint64_t dpp_wave_sum_u64(uint64_t v) {
    v += bfly_partner64<1>(v);
    v += bfly_partner64<2>(v);
    v += bfly_partner64<4>(v);
    v += bfly_partner64<8>(v);
    v += bfly_partner64<16>(v);
    v += bfly_partner64<32>(v);
    return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}
__device__ inline uint32_t dpp_wave_or_u32(uint32_t v) {
    v |= bfly_partner<1>(v);
    v |= bfly_partner<2>(v);
    v |= bfly_partner<4>(v);
    v |= bfly_partner<8>(v);
    v |= bfly_partner<16>(v);
    v |= bfly_partner<32>(v);
    return uni(v);
}
__device__ inline uint32_t dpp_wave_max_u32(uint32_t v) {
    v = max(v, bfly_partner<1>(v));
    v = max(v, bfly_partner<2>(v));
    v = max(v, bfly_partner<4>(v));
    v = max(v, bfly_partner<8>(v));
    v = max(v, bfly_partner<16>(v));
    v = max(v, bfly_partner<32>(v));
    return uni(v);
}
__device__ inline uint32_t dpp_wave_xor_u32(uint32_t v) {
    v ^= bfly_partner<1>(v);
    v ^= bfly_partner<2>(v);
    v ^= bfly_partner<4>(v);
    v ^= bfly_partner<8>(v);
    v ^= bfly_partner<16>(v);
    v ^= bfly_partner<32>(v);
    return uni(v);
}
// inclusive prefix sum over the wave: row_shr 1/2/4/8 within rows, then row_bcast15 / row_bcast31
__device__ inline uint32_t dpp_incl_scan_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
}
// value of lane - 1 (lane 0: 0)
__device__ inline uint32_t dpp_wave_shr1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}

typedef short v2s16 __attribute__((ext_vector_type(2)));
__device__ inline int32_t dot2(uint32_t a, uint32_t b, int32_t c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s16, a), __builtin_bit_cast(v2s16, b), c, false);
}
__device__ inline uint32_t pack2(int32_t lo, int32_t hi) { return ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16); }

// residual of local sample index j (0..63) of this lane given even pairs E[] (E[m] = x[2m], x[2m+1]) and
// odd pairs O[] (O[m] = x[2m-1], x[2m]), each array holding 4 history pairs from the previous lane
// first (indices 0..3) then this lane's 32 pairs (4..35).  C[] = coefficient pairs (q1,q0),(q3,q2),...
// residual of local sample index j (0..63, compile-time) of this lane given the even pairs E[] (E[0..3]:
// the previous lane's last 8 samples, E[4 + m] = (x[2m], x[2m+1])).  C[] = (q1,q0),(q3,q2),(q5,q4),(q7,q6).
// Odd j uses odd-aligned pairs (x[j-2], x[j-1]) = perm(E[m], E[m-1]).
// first product of a residual chain as VOP3P with an inline-zero accumulator (v_dot2c would need a v_mov 0)
__device__ inline int32_t dot2_z(uint32_t a, uint32_t b) {
    int32_t d;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "v"(a), "v"(b));
    return d;
}

__device__ inline int32_t residual_at(const uint32_t *E, const uint32_t *C, int shift, int j, int32_t x) {
    int32_t s = 0;
    const int m = 4 + (j >> 1);
    if ((j & 1) == 0) {
        s = dot2_z(E[m - 1], C[0]);
        s = dot2(E[m - 2], C[1], s);
        s = dot2(E[m - 3], C[2], s);
        s = dot2(E[m - 4], C[3], s);
    } else {
        s = dot2_z(__builtin_amdgcn_perm(E[m], E[m - 1], 0x05040302u), C[0]);
        s = dot2(__builtin_amdgcn_perm(E[m - 1], E[m - 2], 0x05040302u), C[1], s);
        s = dot2(__builtin_amdgcn_perm(E[m - 2], E[m - 3], 0x05040302u), C[2], s);
        s = dot2(__builtin_amdgcn_perm(E[m - 3], E[m - 4], 0x05040302u), C[3], s);
    }
    return x - (s >> shift);
}

// residuals of samples 2m and 2m+1 of this lane with their v_dot2 chains interleaved (no dependent-dot
// wait states): the even sample uses aligned pairs E[], the odd one pairs re-aligned by v_perm
__device__ inline void residual_pair(const uint32_t *E, const uint32_t *C, int shift, int m, int32_t &re, int32_t &ro) {
    const int b = 4 + m;
    const uint32_t o0 = __builtin_amdgcn_perm(E[b], E[b - 1], 0x05040302u);
    const uint32_t o1 = __builtin_amdgcn_perm(E[b - 1], E[b - 2], 0x05040302u);
    const uint32_t o2 = __builtin_amdgcn_perm(E[b - 2], E[b - 3], 0x05040302u);
    const uint32_t o3 = __builtin_amdgcn_perm(E[b - 3], E[b - 4], 0x05040302u);
    int32_t se = dot2_z(E[b - 1], C[0]);
    int32_t so = dot2_z(o0, C[0]);
    se = dot2(E[b - 2], C[1], se);
    so = dot2(o1, C[1], so);
    se = dot2(E[b - 3], C[2], se);
    so = dot2(o2, C[2], so);
    se = dot2(E[b - 4], C[3], se);
    so = dot2(o3, C[3], so);
    const uint32_t v = E[b];
    re = (int32_t)(int16_t)(v & 0xFFFFu) - (se >> shift);
    ro = ((int32_t)v >> 16) - (so >> shift);
}

__device__ inline void lds_put_bits(uint32_t *buf, uint32_t pos, uint32_t val, int nbits) {
    const uint32_t wi = pos >> 5;
    const int off = (int)(pos & 31);
    const uint64_t v = (uint64_t)val << (64 - off - nbits);
    atomicOr(&buf[wi], (uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)v;
    if (lo) atomicOr(&buf[wi + 1], lo);
}

constexpr uint64_t kFlagAgg = 1ull << 62, kFlagIncl = 2ull << 62, kValMask = (1ull << 62) - 1;

// ------------------------------------------------------------------------------ k_encode_v3
// Persistent work-groups of 4 waves; a WG takes a ticket of 4 consecutive frames (wave = frame), so
// tickets are handed out in frame order and every look-back waits only on frames already owned by
// resident waves.  Frames on this path are always full 4096-sample blocks (host guarantees), so no
// per-sample validity predicates exist: only lane 0's first `order` (<= 8) samples are masked, by
// selects.  LPC residuals stay in registers between the partition-sum, code-length and packing passes;
// the fixed candidate's partition sums fall out of the fixed-predictor totals pass.

constexpr int kXpowHi = (kXpowBytes + 63) / 64;
constexpr int kBufWordsV3 = kFrameWordsV3 + 64;  // + the overflow row of the code writer (lds_put_left)
// a subframe slot (multi-channel streams): a frame's words, or the 17-bit VERBATIM side subframe (2177 words)
constexpr int kSubWords = kFrameWordsV3 + 4;
struct EncV3Shared {
    uint32_t bits[4][kBufWordsV3];
    int16_t lut[kLutCap];
    uint16_t crc8x[16][256];  // slice-by-16 tables (T_0..T_3 serve the slice-by-4 / byte steps)
    uint16_t xlo[64];       // x^(8m) mod P, m = 0..63
    uint16_t xhi[kXpowHi];  // x^(8*64*m) mod P
    uint8_t crc8[256];
    int ticket[2];
    int want[2];
    int lut_tile;
};
// lut_gather_pairs forms LUT byte addresses mod 2^16: the LUT (the only LDS object of k_encode_v3 is this struct)
// must end below 64 KiB
static_assert(offsetof(EncV3Shared, lut) + sizeof(int16_t) * kLutCap <= 65536, "LUT beyond 64 KiB of LDS");

// Bank-aware layout of a wave's frame buffer.  Word w of the frame lives at row (w mod C), column (w / C) of a
// 64-column matrix, C = ceil(words / 64) <= 34 chosen per frame: phys(w) = (w mod C) * 64 + w / C, so the LDS
// bank is the column.  Lane L's codes fill roughly column L, so the 64 lanes' concurrent bit-writer atomics
// land in distinct banks whatever each lane's progress (in the plain layout they hit banks
// (base_L + progress_L) mod 32: a birthday-problem 3-4 way conflict).  w / C = (w * ceil(2^20 / C)) >> 20,
// exact for w < 2400 and C <= 34 (checked exhaustively): full-rate 24-bit multiplies only (a 32-bit mulhi is a
// quarter-rate op, and the compiler widened it to a 64-bit product).
struct FbMap {
    uint32_t c, magic, k;  // C, ceil(2^20 / C), 64 C - 1
    __device__ inline uint32_t col(uint32_t w) const { return __umul24(w, magic) >> 20; }
    __device__ inline uint32_t operator()(uint32_t w) const {
        return (uint32_t)__mul24((int)col(w), -(int)k) + (w << 6);
    }
};
__device__ inline FbMap fb_map(uint32_t words) {  // words the frame may touch (<= kFrameWordsV3)
    const uint32_t c = max(1u, (words + 63) >> 6);
    return FbMap{c, ((1u << 20) + c - 1) / c, 64 * c - 1};
}
// The code writer (lds_put_left) ORs a straddling code's second word one row below its first (a ds offset),
// which is word w + 1 except when w is the last word of its column: that part lands in the column's overflow
// row C instead of row 0 of the next column.  fb_fold moves those words home (after the wave's writes landed).
__device__ inline void fb_fold(uint32_t *buf, const FbMap &M, int lane) {
    uint32_t *ovr = buf + (M.c << 6) + lane;
    const uint32_t v = *ovr;
    *ovr = 0;
    if (lane < 63 && v) atomicOr(buf + lane + 1, v);
}

// bit writer without branches: the (up to 32-bit) code at [pos, pos + nbits) straddles at most 2 words
__device__ inline void lds_put_bits2(uint32_t *buf, const FbMap &M, uint32_t pos, uint32_t val, int nbits) {
    const uint32_t wi = pos >> 5;
    const uint64_t v = (uint64_t)val << (64 - (int)(pos & 31) - nbits);
    atomicOr(&buf[M(wi)], (uint32_t)(v >> 32));
    atomicOr(&buf[M(wi + 1)], (uint32_t)v);
}

// opaque register barrier: stops the compiler from carrying 64 residuals across passes (CSE) and
// instead recomputes them from the 36 packed pairs
__device__ inline void reg_fence(uint32_t *E) {
#pragma unroll
    for (int m = 0; m < 36; m++) asm volatile("" : "+v"(E[m]));
}

// |a - b| + c on unsigned operands (v_sad_u32; the compiler does not form it from the pattern)
__device__ inline uint32_t sad_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// OR a left-aligned code (its first bit in bit 31) into the bit buffer at bit position pos.  The second word goes
// one row below the first (+256 B, the ds offset): word wi + 1, or the column's overflow row (fb_fold).
// nk4 = -4 (64 C - 1): byte address = buf + 256 wi + nk4 col(wi), one 24-bit multiply-add.
__device__ inline void lds_put_left(uint32_t *buf, const FbMap &M, int nk4, uint32_t pos, uint32_t codeL) {
    const uint32_t hi = __builtin_amdgcn_alignbit(0u, codeL, pos);  // codeL >> (pos & 31)
    const uint32_t lo = __builtin_amdgcn_alignbit(codeL, 0u, pos);  // codeL << (32 - (pos & 31)); 0 if aligned
    const uint32_t wi = pos >> 5;
    uint32_t *p = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(buf) + (wi << 8) +
                                               __mul24((int)M.col(wi), nk4));
    atomicOr(p, hi);
    atomicOr(p + 64, lo);
}

// LUT normalisation of 64 packed 16-bit samples straight into packed pairs (no wasted bits): both halves' LDS
// byte addresses by one packed 16-bit multiply-add (2 x + lutbase - 2 min, exact mod 2^16: the LUT lies below
// 64 KB of LDS), two ds_read_u16 and one v_lshl_or per pair.  (d16 / d16_hi loads into one register would save the
// v_lshl_or, but the second load of a pair must not issue before the first has landed.)
__device__ inline void lut_gather_pairs(const uint32_t *w, const int16_t *lut, int32_t imin, uint32_t *out) {
    const uint32_t lb = (uint32_t)reinterpret_cast<uintptr_t>(lut);  // low 32 bits of a flat LDS address
    const uint32_t c16 = (lb - 2u * (uint32_t)imin) & 0xFFFFu, cc = c16 | (c16 << 16), two = 0x00020002u;
    const char *lds0 = reinterpret_cast<const char *>(lut) - lb;  // LDS byte 0
#pragma unroll
    for (int m = 0; m < 32; m++) {
        uint32_t a;
        asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(a) : "v"(w[m]), "v"(two), "v"(cc));
        const uint32_t lo = *reinterpret_cast<const uint16_t *>(lds0 + (a & 0xFFFFu));
        const uint32_t hi = *reinterpret_cast<const uint16_t *>(lds0 + (a >> 16));
        out[m] = lo | (hi << 16);
    }
}

__device__ inline uint32_t zigzag(int32_t r) { return ((uint32_t)r << 1) ^ (uint32_t)(r >> 31); }

struct PendingFrame {  // a frame whose bytes sit in the wave's bit buffer, offset not yet resolved
    int64_t f = -1;
    uint64_t fbytes = 0;
    bool ok = true;
    FbMap map{1, 1u << 20, 63};  // the frame's buffer layout
};

__device__ inline void sample_rate_code(int sr, int &src, int &srx) {  // RFC 9639 9.1.2
    srx = 0;
    switch (sr) {
    case 88200: src = 1; break;
    case 176400: src = 2; break;
    case 192000: src = 3; break;
    case 8000: src = 4; break;
    case 16000: src = 5; break;
    case 22050: src = 6; break;
    case 24000: src = 7; break;
    case 32000: src = 8; break;
    case 44100: src = 9; break;
    case 48000: src = 10; break;
    case 96000: src = 11; break;
    default:
        if (sr <= 255000 && sr % 1000 == 0) src = srx = 12;
        else if (sr % 10 == 0 && sr / 10 <= 65535) src = srx = 14;
        else src = srx = 13;
    }
}

// bytes of a fixed-blocksize (4096) frame header incl. CRC-8: sync/codes (4) + UTF-8 frame number + rate ext
__device__ inline uint32_t frame_header_bytes(uint32_t v, int srx) {
    const uint32_t u = v < 0x80 ? 1 : v < 0x800 ? 2 : v < 0x10000 ? 3 : v < 0x200000 ? 4 : v < 0x4000000 ? 5 : 6;
    return 4 + u + (srx == 12 ? 1 : (srx == 13 || srx == 14) ? 2 : 0) + 1;
}

// Offset of a finished frame (decoupled look-back), inclusive publish, store of its bytes from the wave's
// bit buffer, and re-zeroing of that buffer.
// (forced inline: the inliner otherwise emitted real calls with scratch arguments)
__device__ __forceinline__ void resolve_and_store(const EncodeParams &P, PendingFrame &pf, uint32_t *fbuf, uint8_t *arena,
                                         int64_t arena_cap, int64_t *frame_off, uint64_t *status, int *err, int lane) {
    const int64_t f = pf.f;
    const uint64_t fbytes = pf.fbytes;
    const bool ok = pf.ok;
    const bool l0 = lane == 0;
    // ---- decoupled look-back for the exclusive prefix (kPer predecessors per lane and round)
    uint64_t prefix = 0;
    if (f > 0) {
        constexpr int kPer = 1;
        int64_t hi = f - 1;
        uint64_t accum = 0;
        long spins = 0;
        while (true) {
            uint64_t sv[kPer];
#pragma unroll
            for (int i = 0; i < kPer; i++) {
                const int64_t j = hi - (int64_t)(lane * kPer + i);
                sv[i] = kFlagIncl;  // before frame 0: inclusive 0
                if (j >= 0) sv[i] = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            int my_first = kPer;  // first inclusive entry of this lane (by distance)
#pragma unroll
            for (int i = kPer - 1; i >= 0; i--)
                if ((sv[i] >> 62) == 2) my_first = i;
            const uint64_t has = __ballot(my_first < kPer);
            const int fl = has ? __builtin_ctzll(has) : 64;  // lane holding the nearest inclusive
            const int first_i = fl < 64 ? __builtin_amdgcn_readlane(my_first, fl) : kPer;
            // entries at distance <= (fl, first_i) are needed
            bool missing = false;
            uint64_t mine = 0;
#pragma unroll
            for (int i = 0; i < kPer; i++) {
                const bool need = lane < fl || (lane == fl && i <= first_i);
                if (need) {
                    missing |= (sv[i] >> 62) == 0;
                    mine += sv[i] & kValMask;
                }
            }
            if (__ballot(missing)) {  // a needed predecessor has not published yet
                if (++spins > (1l << 22)) {
                    if (l0) atomicOr(err, 8);
                    break;
                }
                // back off: polling waves otherwise flood L2 with 64-lane status reads
                __builtin_amdgcn_s_setprio(0);  // a polling wave yields the arbiter while it sleeps
                if (spins < 4) __builtin_amdgcn_s_sleep(2);
                else if (spins < 16) __builtin_amdgcn_s_sleep(8);
                else __builtin_amdgcn_s_sleep(32);
                __builtin_amdgcn_s_setprio(2);
                continue;
            }
            accum += dpp_wave_sum_u64(mine);
            if (fl < 64) break;
            hi -= 64 * kPer;
        }
        prefix = accum;
    }
    if (l0) {
        if (f > 0)
            __hip_atomic_store(&status[f], kFlagIncl | (prefix + fbytes), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        frame_off[f] = (int64_t)prefix;
    }
    const FbMap M = pf.map;
    if ((int64_t)(prefix + fbytes) > arena_cap) {
        if (l0) atomicOr(err, 16);
    } else if (fbytes) {
        // ---- store [prefix, prefix + fbytes): bytes up to 16-B alignment, 16-B chunks, byte tail
        uint8_t *dst = arena + prefix;
        const uint32_t a0 = min((uint32_t)fbytes, (uint32_t)((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15));
        auto byte_at = [&](uint32_t b) -> uint8_t { return (uint8_t)(fbuf[M(b >> 2)] >> (24 - 8 * (b & 3))); };
        if ((uint32_t)lane < a0) dst[lane] = byte_at((uint32_t)lane);
        const uint32_t n16 = ((uint32_t)fbytes - a0) >> 4;
        const uint32_t r = a0 & 3, sb = a0 >> 2;
        uint4 *d16 = reinterpret_cast<uint4 *>(dst + a0);
        // 16-B chunk ci = words sb + 4 ci .. sb + 4 ci + 4.  Lane L takes the chunks of column L (ci = L C/4 + j),
        // so at each step the 64 lanes read one buffer row: consecutive banks
        auto chunk = [&](uint32_t ci) {
            const uint32_t wq = sb + 4 * ci;
            const uint32_t w0 = __builtin_bswap32(fbuf[M(wq)]), w1 = __builtin_bswap32(fbuf[M(wq + 1)]);
            const uint32_t w2 = __builtin_bswap32(fbuf[M(wq + 2)]), w3 = __builtin_bswap32(fbuf[M(wq + 3)]);
            const uint32_t w4 = __builtin_bswap32(fbuf[M(wq + 4)]);
            uint4 o4;
            o4.x = __builtin_amdgcn_alignbyte(w1, w0, r);
            o4.y = __builtin_amdgcn_alignbyte(w2, w1, r);
            o4.z = __builtin_amdgcn_alignbyte(w3, w2, r);
            o4.w = __builtin_amdgcn_alignbyte(w4, w3, r);
            d16[ci] = o4;
        };
        // the chunks whose first word lies in column L: at each step the lanes read rows within 3 of each
        // other in their own columns, i.e. distinct banks
        const uint32_t c0 = (uint32_t)lane * M.c, c1 = c0 + M.c;
        const uint32_t ci0 = c0 > sb ? (c0 - sb + 3) >> 2 : 0u, ci1 = c1 > sb ? min(n16, (c1 - sb + 3) >> 2) : 0u;
        // chunks before the column's last lie wholly in column L: rows r .. r + 4 at phys r * 64 + L
        if (ci0 < ci1) {
            const uint32_t *cp = fbuf + M(sb + 4 * ci0);
            for (uint32_t ci = ci0; ci + 1 < ci1; ci++, cp += 256) {
                const uint32_t w0 = __builtin_bswap32(cp[0]), w1 = __builtin_bswap32(cp[64]);
                const uint32_t w2 = __builtin_bswap32(cp[128]), w3 = __builtin_bswap32(cp[192]);
                const uint32_t w4 = __builtin_bswap32(cp[256]);
                uint4 o4;
                o4.x = __builtin_amdgcn_alignbyte(w1, w0, r);
                o4.y = __builtin_amdgcn_alignbyte(w2, w1, r);
                o4.z = __builtin_amdgcn_alignbyte(w3, w2, r);
                o4.w = __builtin_amdgcn_alignbyte(w4, w3, r);
                d16[ci] = o4;
            }
            chunk(ci1 - 1);
        }
        const uint32_t tb = a0 + 16 * n16 + (uint32_t)lane;
        if (tb < (uint32_t)fbytes) dst[tb] = byte_at(tb);
    }
    // leave the bit buffer zeroed for this wave's next frame (LDS ops of one wave complete in order): the C rows
    // of the frame's matrix, or the whole buffer after a failed frame
    if (ok) {
        for (uint32_t i = 0; i < M.c; i++) fbuf[(i << 6) | (uint32_t)lane] = 0;
    } else {
        for (uint32_t i = (uint32_t)lane; i < (uint32_t)kBufWordsV3; i += 64) fbuf[i] = 0;
    }
    pf.f = -1;
}

// fixed.c FLAC__fixed_compute_best_predictor, lane-parallel: this lane's sums of |e_k(i)|, k = 0..4, over its 64 samples
// (packed pairs E[4 + m], E[2..3] = the previous lane's last four samples), lane 0 from sample 4 (tk); and lane 0's
// terms at k <= i < 4 (hk: with tk, the fixed candidate's Rice sum from its warm-up on).  Differences are carried
// sign-flipped (y = e ^ 2^31) so |e_{k+1}| = v_sad_u32(y_k(i), y_k(i-1)) in one op.
__device__ inline void fixed_lane_totals(const uint32_t *E, bool l0, uint32_t *tk, uint32_t *hk) {
    constexpr uint32_t M = 0x80000000u;
    const int32_t h1 = (int32_t)E[3] >> 16, h2 = (int16_t)(E[3] & 0xFFFFu);
    const int32_t h3 = (int32_t)E[2] >> 16, h4 = (int16_t)(E[2] & 0xFFFFu);
    uint32_t p0 = (uint32_t)h1 ^ M, p1 = (uint32_t)(h1 - h2) ^ M, p2 = (uint32_t)((h1 - h2) - (h2 - h3)) ^ M;
    uint32_t p3 = (uint32_t)(((h1 - h2) - (h2 - h3)) - ((h2 - h3) - (h3 - h4))) ^ M;
    uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
#pragma unroll
    for (int k = 0; k < 5; k++) hk[k] = 0;
#pragma unroll
    for (int j = 0; j < 64; j++) {
        const uint32_t v = E[4 + (j >> 1)];
        const int32_t x = (j & 1) ? ((int32_t)v >> 16) : (int32_t)(int16_t)(v & 0xFFFFu);
        const uint32_t y0 = (uint32_t)x ^ M;
        const uint32_t y1 = (y0 - p0) ^ M, y2 = (y1 - p1) ^ M, y3 = (y2 - p2) ^ M;
        if (j < 4) {  // lane 0: not in the totals; its order-k terms from i = k are the Rice sum's
            hk[0] = sad_u32(y0, M, hk[0]);
            if (j >= 1) hk[1] = sad_u32(y0, p0, hk[1]);
            if (j >= 2) hk[2] = sad_u32(y1, p1, hk[2]);
            if (j >= 3) hk[3] = sad_u32(y2, p2, hk[3]);
            if (!l0) {
                t0 = sad_u32(y0, M, t0);
                t1 = sad_u32(y0, p0, t1);
                t2 = sad_u32(y1, p1, t2);
                t3 = sad_u32(y2, p2, t3);
                t4 = sad_u32(y3, p3, t4);
            }
        } else {
            t0 = sad_u32(y0, M, t0);
            t1 = sad_u32(y0, p0, t1);
            t2 = sad_u32(y1, p1, t2);
            t3 = sad_u32(y2, p2, t3);
            t4 = sad_u32(y3, p3, t4);
        }
        p0 = y0;
        p1 = y1;
        p2 = y2;
        p3 = y3;
    }
    tk[0] = t0, tk[1] = t1, tk[2] = t2, tk[3] = t3, tk[4] = t4;
}

// A lane's 64 consecutive samples of one coded signal, and the residual / fixed-predictor arithmetic on them.
// LanePairs (16-bit signals): E[4 + m] = (x[2m], x[2m+1]) as int16 pairs, E[0..3] = the previous lane's last 8
// samples (zeros on lane 0); LPC residuals by v_dot2 on packed pairs.  LaneWide (the 17-bit side signal of a
// two-channel stream, L - R): X[8 + j] = x[j] as int32, X[0..7] the previous lane's last 8; residuals by 24-bit
// multiply-adds (every sample and coefficient fits 24 bits; the sum stays below 2^31, libFLAC's 32-bit residual
// path: subframe bps + precision + log2(order) <= 32).
struct LanePairs {
    uint32_t E[36];
    struct Coefs {
        uint32_t C[4];
    };
    __device__ inline int32_t x(int j) const {
        const uint32_t v = E[4 + (j >> 1)];
        return (j & 1) ? ((int32_t)v >> 16) : (int32_t)(int16_t)(v & 0xFFFFu);
    }
    __device__ inline void history() {
#pragma unroll
        for (int m = 0; m < 4; m++) E[m] = dpp_wave_shr1(E[32 + m]);
        reg_fence(E);
    }
    __device__ inline void fence() { reg_fence(E); }
    __device__ inline void totals(bool l0, uint32_t *tk, uint32_t *hk) const { fixed_lane_totals(E, l0, tk, hk); }
    __device__ inline uint32_t diff_from_first() const {  // OR of (x ^ x[0]) over the lane (wave-uniform x[0])
        const uint32_t x0 = uni(E[4] & 0xFFFFu);
        const uint32_t xx = x0 | (x0 << 16);
        uint32_t diff = 0;
#pragma unroll
        for (int m = 4; m < 36; m++) diff |= E[m] ^ xx;
        return diff;
    }
    __device__ static inline Coefs coefs(const int32_t *q) {
        Coefs c;
#pragma unroll
        for (int k = 0; k < 4; k++) c.C[k] = pack2(q[2 * k + 1], q[2 * k]);
        return c;
    }
    __device__ inline void residuals(const Coefs &c, int shift, int m, int32_t &re, int32_t &ro) const {
        residual_pair(E, c.C, shift, m, re, ro);
    }
    __device__ inline uint32_t warm(int lane) const {  // lane i (< 8): lane 0's sample i (as unsigned bits)
        const int i = lane & 7;
        uint32_t w01 = (uint32_t)__builtin_amdgcn_readlane((int)E[4 + 0], 0);
        w01 = (i >> 1) == 1 ? (uint32_t)__builtin_amdgcn_readlane((int)E[4 + 1], 0) : w01;
        w01 = (i >> 1) == 2 ? (uint32_t)__builtin_amdgcn_readlane((int)E[4 + 2], 0) : w01;
        w01 = (i >> 1) == 3 ? (uint32_t)__builtin_amdgcn_readlane((int)E[4 + 3], 0) : w01;
        return (i & 1) ? (w01 >> 16) : (w01 & 0xFFFFu);
    }
};
struct LaneWide {
    int32_t X[72];
    struct Coefs {
        int32_t q[8];
    };
    __device__ inline int32_t x(int j) const { return X[8 + j]; }
    __device__ inline void history() {
#pragma unroll
        for (int m = 0; m < 8; m++) X[m] = (int32_t)dpp_wave_shr1((uint32_t)X[64 + m]);
        fence();
    }
    __device__ inline void fence() {
#pragma unroll
        for (int m = 0; m < 72; m++) asm volatile("" : "+v"(X[m]));
    }
    __device__ inline void totals(bool l0, uint32_t *tk, uint32_t *hk) const {
        constexpr uint32_t M = 0x80000000u;
        const int32_t h1 = X[7], h2 = X[6], h3 = X[5], h4 = X[4];
        uint32_t p0 = (uint32_t)h1 ^ M, p1 = (uint32_t)(h1 - h2) ^ M, p2 = (uint32_t)((h1 - h2) - (h2 - h3)) ^ M;
        uint32_t p3 = (uint32_t)(((h1 - h2) - (h2 - h3)) - ((h2 - h3) - (h3 - h4))) ^ M;
        uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) hk[k] = 0;
#pragma unroll
        for (int j = 0; j < 64; j++) {
            const uint32_t y0 = (uint32_t)X[8 + j] ^ M;
            const uint32_t y1 = (y0 - p0) ^ M, y2 = (y1 - p1) ^ M, y3 = (y2 - p2) ^ M;
            if (j < 4) {
                hk[0] = sad_u32(y0, M, hk[0]);
                if (j >= 1) hk[1] = sad_u32(y0, p0, hk[1]);
                if (j >= 2) hk[2] = sad_u32(y1, p1, hk[2]);
                if (j >= 3) hk[3] = sad_u32(y2, p2, hk[3]);
            }
            if (j >= 4 || !l0) {
                t0 = sad_u32(y0, M, t0);
                t1 = sad_u32(y0, p0, t1);
                t2 = sad_u32(y1, p1, t2);
                t3 = sad_u32(y2, p2, t3);
                t4 = sad_u32(y3, p3, t4);
            }
            p0 = y0, p1 = y1, p2 = y2, p3 = y3;
        }
        tk[0] = t0, tk[1] = t1, tk[2] = t2, tk[3] = t3, tk[4] = t4;
    }
    __device__ inline uint32_t diff_from_first() const {
        const uint32_t x0 = uni((uint32_t)X[8]);
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < 64; j++) diff |= (uint32_t)X[8 + j] ^ x0;
        return diff;
    }
    __device__ static inline Coefs coefs(const int32_t *q) {
        Coefs c;
#pragma unroll
        for (int k = 0; k < 8; k++) c.q[k] = q[k];
        return c;
    }
    __device__ inline void residuals(const Coefs &c, int shift, int m, int32_t &re, int32_t &ro) const {
        const int j = 8 + 2 * m;
        int32_t se = 0, so = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            se = __mul24(c.q[i], X[j - 1 - i]) + se;
            so = __mul24(c.q[i], X[j - i]) + so;
        }
        re = X[j] - (se >> shift);
        ro = X[j + 1] - (so >> shift);
    }
    __device__ inline uint32_t warm(int lane) const {
        const int i = lane & 7;
        uint32_t v = (uint32_t)__builtin_amdgcn_readlane(X[8], 0);
#pragma unroll
        for (int k = 1; k < 8; k++) v = i == k ? (uint32_t)__builtin_amdgcn_readlane(X[8 + k], 0) : v;
        return v;
    }
};

// libFLAC's set_partitioned_rice_ (stream_encoder.c) for the fixed and LPC candidates of a 4096-sample frame: orders
// 5..0, group sums merged by lane shuffles (the 32-bit form when every lane sum is below 2^24)
__device__ __forceinline__ void rice_candidates(uint32_t sf, uint32_t sl, int of, int ol, bool cand_fixed,
                                                bool cand_lpc, int lane, uint32_t &rb_f, int &po_f, int &k_f,
                                                uint32_t &rb_l, int &po_l, int &k_l) {
    constexpr int n = kMaxBlock;
    auto rice64 = [&](uint32_t lane_sum, int order, uint32_t &best_bits, int &best_po, int &my_k) {
        best_bits = 0;
        best_po = 0;
        my_k = 0;
        uint64_t gsum = (uint64_t)lane_sum;
        gsum += bfly_partner64<1>(gsum);
#pragma unroll
        for (int po = 5; po >= 0; po--) {
            if (po == 4) gsum += bfly_partner64<2>(gsum);
            if (po == 3) gsum += bfly_partner64<4>(gsum);
            if (po == 2) gsum += bfly_partner64<8>(gsum);
            if (po == 1) gsum += bfly_partner64<16>(gsum);
            if (po == 0) gsum += bfly_partner64<32>(gsum);
            const int lanes_per = 64 >> po;
            const uint32_t pbase = (uint32_t)(n >> po);
            const bool first = lane < lanes_per;
            const uint32_t ns = first ? pbase - (uint32_t)order : pbase;
            // 0x40000 / ns: a power of two for every partition but the first (scalar division for that one)
            const uint32_t div_first = uni(0x40000u / (pbase - (uint32_t)order));
            const uint32_t div = first ? div_first : (64u << po);
            const uint64_t prod = gsum >= 1 ? ((gsum - 1) * div) >> 18 : 0;
            uint32_t k = (gsum < 2 || prod == 0) ? 0u : (uint32_t)ilog2_u64(prod) + 1;
            if (k >= 15) k = 14;
            uint64_t pb = 4 + (uint64_t)(1 + k) * ns + (k ? (gsum >> (k - 1)) : (gsum << 1)) - (ns >> 1);
            if (pb > 0xFFFFFFFFull) pb = 0xFFFFFFFFull;
            const uint32_t contrib = ((lane & (lanes_per - 1)) == 0) ? (uint32_t)pb : 0u;
            const uint32_t bits = 6 + dpp_wave_sum_u32(contrib);
            if (best_bits == 0 || bits < best_bits) {
                best_bits = bits;
                best_po = po;
                my_k = (int)k;
            }
        }
    };
    // 32-bit form of the same search, exact when every lane sum is < 2^24 (group sums < 2^30), for NC candidates
    // at once.  Every lane computes the bits of ITS partition at every order (replicated over the partition's lanes);
    // an order's total then needs only the butterfly stages at or above its partition width (5, 4, 3, 2, 1 and 0 stages
    // for orders 5..0 instead of a full 6-stage wave sum per order), and the division by a non-first partition's size is
    // a shift (the first partition's 2^18 / (n - order) comes from a table); k ? s >> (k-1) : s << 1 == (2s) >> k.
    auto rice32m = [&](auto NCt, const uint32_t *sums, const int *ord, uint32_t *bb, int *bp, int *bk) {
        constexpr int NC = decltype(NCt)::value;
        uint32_t g[NC], V[NC][6], Kp[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) {
            g[c] = sums[c] + bfly_partner<1>(sums[c]);
            Kp[c] = 0;
        }
#pragma unroll
        for (int po = 5; po >= 0; po--) {
#pragma unroll
            for (int c = 0; c < NC; c++) {
                if (po == 4) g[c] += bfly_partner<2>(g[c]);
                if (po == 3) g[c] += bfly_partner<4>(g[c]);
                if (po == 2) g[c] += bfly_partner<8>(g[c]);
                if (po == 1) g[c] += bfly_partner<16>(g[c]);
                if (po == 0) g[c] += bfly_partner<32>(g[c]);
            }
            const int lanes_per = 64 >> po;
            const uint32_t pbase = (uint32_t)(n >> po);
            const bool first = lane < lanes_per;
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const uint32_t ns = first ? pbase - (uint32_t)ord[c] : pbase;
                const uint32_t div_first = c_rice_div[po][ord[c]];
                const uint32_t pf = (uint32_t)(((uint64_t)(g[c] - 1u) * div_first) >> 18);
                const uint32_t pr = (g[c] - 1u) >> (12 - po);
                const uint32_t prod = first ? pf : pr;
                uint32_t k = (g[c] < 2 || prod == 0) ? 0u : 32u - (uint32_t)__builtin_clz(prod);
                k = min(k, 14u);
                Kp[c] |= k << (4 * (5 - po));
                V[c][5 - po] = 4 + (1 + k) * ns + ((2 * g[c]) >> k) - (ns >> 1);
            }
        }
        // V[c][i] (order 5 - i) is uniform over partitions of 2^(i + 1) lanes: butterflies from that width up
#pragma unroll
        for (int c = 0; c < NC; c++) V[c][0] += bfly_partner<2>(V[c][0]);
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int i = 0; i <= 1; i++) V[c][i] += bfly_partner<4>(V[c][i]);
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int i = 0; i <= 2; i++) V[c][i] += bfly_partner<8>(V[c][i]);
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int i = 0; i <= 3; i++) V[c][i] += bfly_partner<16>(V[c][i]);
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int i = 0; i <= 4; i++) V[c][i] += bfly_partner<32>(V[c][i]);
#pragma unroll
        for (int c = 0; c < NC; c++) {
            uint32_t best_bits = 0;
            int best_i = 0;
#pragma unroll
            for (int i = 0; i < 6; i++) {  // orders 5 .. 0, strict <
                const uint32_t bits = 6 + uni(V[c][i]);
                if (best_bits == 0 || bits < best_bits) {
                    best_bits = bits;
                    best_i = i;
                }
            }
            bb[c] = best_bits;
            bp[c] = 5 - best_i;
            bk[c] = (int)((Kp[c] >> (4 * best_i)) & 15u);
        }
    };
    auto rice = [&](uint32_t lane_sum, int order, uint32_t &best_bits, int &best_po, int &my_k) {
        if (__ballot(lane_sum >= (1u << 24)) == 0) {
            const uint32_t sm[1] = {lane_sum};
            const int od[1] = {order};
            uint32_t b1[1];
            int p1[1], k1[1];
            rice32m(std::integral_constant<int, 1>{}, sm, od, b1, p1, k1);
            best_bits = b1[0], best_po = p1[0], my_k = k1[0];
        } else {
            rice64(lane_sum, order, best_bits, best_po, my_k);
        }
    };
    rb_f = rb_l = 0;
    po_f = po_l = k_f = k_l = 0;
    if (cand_fixed && cand_lpc && __ballot(sf >= (1u << 24) || sl >= (1u << 24)) == 0) {
        uint32_t bb[2];
        int bp[2], bk[2];
        const uint32_t sm[2] = {sf, sl};
        const int od[2] = {of, ol};
        rice32m(std::integral_constant<int, 2>{}, sm, od, bb, bp, bk);
        rb_f = bb[0], po_f = bp[0], k_f = bk[0];
        rb_l = bb[1], po_l = bp[1], k_l = bk[1];
    } else {
        if (cand_fixed) rice(sf, of, rb_f, po_f, k_f);
        if (cand_lpc) rice(sl, ol, rb_l, po_l, k_l);
    }
}

// ------------------------------------------------------------------------------ k_encode_v4 (lane-private segments)
// The v3 encoder needs every code's frame position before it packs (the look-back publishes sizes early), so it
// walks the residuals three times: |r| sums for the Rice search, exact code lengths, packing.  v4 packs each lane's
// 64 codes into a PRIVATE column of the wave's buffer (lane L's word i at i * 64 + L, the partition's 4-bit Rice
// parameter first when the lane starts a partition), so the code-length pass disappears: a lane's length is its
// write position at the end.  The frame is then assembled in place in a linear layout (word w at w): every lane
// reads its column into registers, the buffer is zeroed, and the lane ORs its segment in at its bit offset (one
// v_alignbit per word; words shared with a neighbour lane are OR-ed by both).  Header, warm-up and coefficient
// fields are OR-ed at their fixed positions, the CRC-16 is summed per lane over word ranges, and only then does the
// wave look back for its frame's byte offset and store the frame (one buffer per wave: the store is not deferred to
// the next frame, which leaves the assembly and CRC as the look-back's slack).  A lane whose segment outgrows its
// column (> kPrivBits, e.g. a residual spike in an otherwise smooth frame) makes the whole wave repack from its
// registers at the now known offsets (the v3 writer on the linear layout).
constexpr int kPrivRows = 34;                    // column rows holding a lane's codes; row 34 takes the last lo words
constexpr uint32_t kPrivBits = kPrivRows * 32;   // 1088 bits = 17 bits per sample
static_assert(kBufWordsV3 >= (kPrivRows + 1) * 64, "private rows + the spill row");
static_assert(kBufWordsV3 % 4 == 0, "b128 zeroing");

// zero the wave's whole buffer (kBufWordsV3 words) with 16-byte stores
__device__ inline void zero_wave_buf(uint32_t *buf, int lane) {
    uint4 *b4 = reinterpret_cast<uint4 *>(buf);
#pragma unroll
    for (int i = 0; i < (kBufWordsV3 / 4 + 63) / 64; i++) {
        const int c = lane + 64 * i;
        if (i < kBufWordsV3 / 256 || c < kBufWordsV3 / 4) b4[c] = make_uint4(0u, 0u, 0u, 0u);
    }
}

// CRC-16 of body bytes [0, body) of a frame in the column layout M: lane L takes column L (words L C .. L C + C - 1,
// so at each step the lanes read one row: consecutive banks) by slice-by-16, the lane holding the last whole word adds
// the tail bytes, and the lanes' values are combined with x^(8m) factors (m = bytes after the lane's range)
__device__ __forceinline__ uint32_t crc16_cols(const uint32_t *fbuf, const FbMap &M, uint32_t body, const EncV3Shared &S,
                                               int lane) {
    const uint32_t nfw = body >> 2, tail = body & 3;
    const uint32_t wb = min(nfw, (uint32_t)lane * M.c), we = min(nfw, wb + M.c);
    uint32_t c = 0;
    const uint32_t *colp = fbuf + lane;
    const uint16_t(*T)[256] = S.crc8x;
    uint32_t i = wb;
    for (; i + 3 < we; i += 4, colp += 256) {
        const uint32_t w0 = colp[0], w1 = colp[64], w2 = colp[128], w3 = colp[192];
        c = (uint32_t)T[15][((c >> 8) ^ (w0 >> 24)) & 0xFF] ^ T[14][((c & 0xFF) ^ (w0 >> 16)) & 0xFF] ^
            T[13][(w0 >> 8) & 0xFF] ^ T[12][w0 & 0xFF] ^ T[11][w1 >> 24] ^ T[10][(w1 >> 16) & 0xFF] ^
            T[9][(w1 >> 8) & 0xFF] ^ T[8][w1 & 0xFF] ^ T[7][w2 >> 24] ^ T[6][(w2 >> 16) & 0xFF] ^
            T[5][(w2 >> 8) & 0xFF] ^ T[4][w2 & 0xFF] ^ T[3][w3 >> 24] ^ T[2][(w3 >> 16) & 0xFF] ^
            T[1][(w3 >> 8) & 0xFF] ^ T[0][w3 & 0xFF];
    }
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
    uint32_t end = we * 4;
    if (lane == (int)M.col(nfw - 1)) {
        const uint32_t word = fbuf[M(nfw)];
        for (uint32_t b = 0; b < tail; b++) {
            const uint32_t byte = (word >> (24 - 8 * b)) & 0xFF;
            c = ((c << 8) & 0xFFFFu) ^ S.crc8x[0][((c >> 8) ^ byte) & 0xFF];
        }
        end += tail;
    }
    const uint32_t m = body - end;
    return dpp_wave_xor_u32(gf_mulmod(gf_mulmod(c, S.xlo[m & 63]), S.xhi[m >> 6]));
}

// ST: units of a two-channel stream's mid/side pass (chn 0..3 = left, right, mid, side; WIDE for the side signal).
template <int DT, bool SUB = false, bool ST = false, bool WIDE = false>
__device__ __forceinline__ void encode_frame_v4(const typename Elem<DT>::T *raster, const EncodeParams &P,
                                                const TileGeom *tiles, const TileNorm *norms,
                                                const SubAnalysis *ana, uint8_t *arena, int64_t arena_cap,
                                                int64_t *frame_off, uint64_t *status, int *err, EncV3Shared &S,
                                                int want, int64_t f, int lane, const int32_t *ftile,
                                                PendingFrame &prev, const uint4 *hdr_tab, int hdr_n,
                                                const uint32_t *pslots, const int64_t *pbytes, int chn = 0,
                                                uint32_t *sub_slots = nullptr, int32_t *sub_bits = nullptr,
                                                int32_t *sub_est = nullptr) {
    using T = typename Elem<DT>::T;
    using Lane = std::conditional_t<WIDE, LaneWide, LanePairs>;
    uint32_t *fbuf = S.bits[threadIdx.x >> 6];  // holds the pending frame `prev` (or zero) on entry
    const int t = ftile[f];
    const TileGeom g = tiles[t];
    const bool l0 = lane == 0;
    if (!SUB && g.partial && f - g.frame_base == g.nframes - 1) {
        // (wave-uniform) the tile's partial last frame: already coded and sealed by the generic kernels; it only joins
        // the look-back chain
        const int64_t si = g.partial - 1;
        const uint64_t nb = (uint64_t)pbytes[si];
        const uint32_t words = (uint32_t)((nb + 3) >> 2);
        const bool ok = words + 2 <= (uint32_t)kFrameWordsV3;
        if (!ok && l0) atomicOr(err, 2);
        const uint64_t fbytes = ok ? nb : 0;
        const FbMap M = fb_map(words + 1);
        __builtin_amdgcn_s_setprio(2);
        if (l0)
            __hip_atomic_store(&status[f], (f == 0 ? kFlagIncl : kFlagAgg) | fbytes, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);
        if (ok) {
            const uint32_t *src = pslots + (size_t)si * P.slot_words;
            for (uint32_t w = (uint32_t)lane; w < words; w += 64) fbuf[M(w)] = __builtin_bswap32(src[w]);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_setprio(0);
        prev.f = f, prev.fbytes = fbytes, prev.ok = ok, prev.map = M;
        return;
    }
    TileNorm tn = norms[t];
    // the WG's LDS LUT belongs to tile `want`; a frame of another tile takes the exact division instead
    if (t != want && tn.mode == kNormLut) tn.mode = kNormSlow;
    const int16_t *lut = S.lut;
    // issue priority: the work up to the size publish gates the successors' look-backs
    __builtin_amdgcn_s_setprio(2);
    const int64_t fk = f - g.frame_base;
    const int64_t s0 = fk * kMaxBlock;
    constexpr int n = kMaxBlock;
    const int64_t sub = SUB ? f * P.nvch + chn : f;
    const SubAnalysis A = ana[sub];
    const int w = A.wasted;
    const int sbps = 16 - w + ((ST && chn == 3) ? 1 : 0);
    // (ST mid / side: the left band; the right one at + band_stride)
    const T *base = raster + (int64_t)(P.band0 + ((ST && chn >= 2) ? 0 : chn)) * P.band_stride + g.r0 * P.row_stride +
                    g.c0;

    // ---- this lane's 64 samples of the coded signal, normalised and shifted (Lane: packed pairs, or int32 for the
    //      side signal), with the previous lane's last 8 samples
    auto load_lane = [&](Lane &Ls) __attribute__((always_inline)) {
        Chunk64<DT> ch;
        const uint32_t sl0 = (uint32_t)s0 + 64u * (uint32_t)lane;  // tile pixels < 2^31
        const uint32_t row = udiv_inv(sl0, (uint32_t)g.w, 1.0 / (double)g.w);
        const int col = (int)(sl0 - row * (uint32_t)g.w), vec = (g.w % 64) == 0 ? P.vec_ok : 0;
        ch.load(base, P.row_stride, g.w, row, col, vec, 64);
        const bool lutp = sizeof(T) == 2 && tn.mode == kNormLut && w == 0;  // (wave-uniform) the common case
        auto sx = [](uint32_t v, int h) -> int32_t { return h ? ((int32_t)v >> 16) : (int32_t)(int16_t)(v & 0xFFFFu); };
        if constexpr (WIDE) {  // side = L - R (17 bits)
            if (lutp) {
                uint32_t Lp[32], Rp[32];
                lut_gather_pairs(ch.w, lut, (int32_t)tn.imin, Lp);
                ch.load(base + P.band_stride, P.row_stride, g.w, row, col, vec, 64);
                lut_gather_pairs(ch.w, lut, (int32_t)tn.imin, Rp);
#pragma unroll
                for (int m = 0; m < 32; m++) {
                    Ls.X[8 + 2 * m] = sx(Lp[m], 0) - sx(Rp[m], 0);
                    Ls.X[9 + 2 * m] = sx(Lp[m], 1) - sx(Rp[m], 1);
                }
            } else {
                norm_chunk<DT>(ch, tn, lut, [&](int j, int32_t x) { Ls.X[8 + j] = x; });
                ch.load(base + P.band_stride, P.row_stride, g.w, row, col, vec, 64);
                norm_chunk<DT>(ch, tn, lut, [&](int j, int32_t x) { Ls.X[8 + j] = (Ls.X[8 + j] - x) >> w; });
            }
        } else {
            // packed pairs of the normalised samples (shifted right by sh)
            auto pairs = [&](uint32_t *dst, int sh) __attribute__((always_inline)) {
                if (lutp) {  // (w == 0)
                    lut_gather_pairs(ch.w, lut, (int32_t)tn.imin, dst);
                } else {
                    int32_t lo = 0;
                    norm_chunk<DT>(ch, tn, lut, [&](int j, int32_t x) {
                        if (j & 1) dst[j >> 1] = pack2(lo, x >> sh);
                        else lo = x >> sh;
                    });
                }
            };
            if (ST && chn == 2) {  // mid = (L + R) >> 1, then the wasted bits
                uint32_t Lp[32], Rp[32];
                pairs(Lp, 0);
                ch.load(base + P.band_stride, P.row_stride, g.w, row, col, vec, 64);
                pairs(Rp, 0);
#pragma unroll
                for (int m = 0; m < 32; m++)
                    Ls.E[4 + m] = pack2(((sx(Lp[m], 0) + sx(Rp[m], 0)) >> 1) >> w,
                                        ((sx(Lp[m], 1) + sx(Rp[m], 1)) >> 1) >> w);
            } else {
                pairs(Ls.E + 4, w);
            }
        }
        Ls.history();
    };
    Lane Ls;
    load_lane(Ls);

    // ---- candidates: the fixed order guess from the totals (fixed.c: first minimum under <=), its lane sum; the LPC
    //      lane |r| sum
    uint32_t tk[5], hk[5], Tt[5];
    Ls.totals(l0, tk, hk);
    dpp_wave_sum_multi<5>(tk, Tt);
    int guess;
    if (Tt[0] <= min(min(Tt[1], Tt[2]), min(Tt[3], Tt[4]))) guess = 0;
    else if (Tt[1] <= min(min(Tt[2], Tt[3]), Tt[4])) guess = 1;
    else if (Tt[2] <= min(Tt[3], Tt[4])) guess = 2;
    else if (Tt[3] <= Tt[4]) guess = 3;
    else guess = 4;
    const uint32_t tg = guess == 0 ? Tt[0] : guess == 1 ? Tt[1] : guess == 2 ? Tt[2] : guess == 3 ? Tt[3] : Tt[4];
    const double dn = (double)(n - 4);
    const float fb1 = (float)(Tt[1] > 0 ? log(M_LN2 * (double)Tt[1] / dn) / M_LN2 : 0.0);
    const float fbg = (float)(tg > 0 ? log(M_LN2 * (double)tg / dn) / M_LN2 : 0.0);
    bool constant = false;
    if (fb1 == 0.0f) {
        Ls.fence();
        constant = dpp_wave_or_u32(Ls.diff_from_first()) == 0;
    }
    const bool cand_fixed = !constant && !(fbg >= (float)sbps);
    const bool cand_lpc = !constant && (A.flags & kFlagLpcOk);
    const int of = guess, ol = A.lpc_order, lshift = A.lpc_shift;
    // the fixed candidate's lane sum of |e_of(i)|, lane 0 from i = of (the totals start at 4: lane 0 adds its i < 4)
    uint32_t sf = of == 0 ? tk[0] + (l0 ? hk[0] : 0u) : of == 1 ? tk[1] + (l0 ? hk[1] : 0u)
                : of == 2 ? tk[2] + (l0 ? hk[2] : 0u) : of == 3 ? tk[3] + (l0 ? hk[3] : 0u) : tk[4];
    const typename Lane::Coefs CL = Lane::coefs(A.q);
    uint32_t sl = 0;
    if (cand_lpc) {
#pragma unroll
        for (int m = 0; m < 32; m++) {
            if (m % 4 == 0 && m) asm volatile("" : "+v"(sl));
            int32_t re, ro;
            Ls.residuals(CL, lshift, m, re, ro);
            // |r| + sl in one v_sad_u32 on the sign-flipped residual
            const uint32_t se = sad_u32((uint32_t)re ^ 0x80000000u, 0x80000000u, sl);
            sl = (2 * m < kMaxLpc && l0 && 2 * m < ol) ? sl : se;
            const uint32_t so = sad_u32((uint32_t)ro ^ 0x80000000u, 0x80000000u, sl);
            sl = (2 * m + 1 < kMaxLpc && l0 && 2 * m + 1 < ol) ? sl : so;
        }
    }
    Ls.fence();
    uint32_t rb_f = 0, rb_l = 0;
    int po_f = 0, po_l = 0, k_f = 0, k_l = 0;
    rice_candidates(sf, sl, of, ol, cand_fixed, cand_lpc, lane, rb_f, po_f, k_f, rb_l, po_l, k_l);
    uint32_t best = (uint32_t)(1 + 6 + 1 + w + n * sbps);
    int type = 1;
    if (constant) {
        const uint32_t cb = (uint32_t)(1 + 6 + 1 + w + sbps);
        if (cb < best) { best = cb; type = 0; }
    } else {
        if (cand_fixed) {
            uint32_t est = (uint32_t)(1 + 6 + 1 + w + of * sbps);
            est = (rb_f < 0xFFFFFFFFu - est) ? est + rb_f : 0xFFFFFFFFu;
            if (est < best) { best = est; type = 2; }
        }
        if (cand_lpc) {
            uint32_t est = (uint32_t)(1 + 6 + 1 + w + 4 + 5 + sbps * ol + A.lpc_prec * ol);
            est = (rb_l < 0xFFFFFFFFu - est) ? est + rb_l : 0xFFFFFFFFu;
            if (est != 0 && est < best) { best = est; type = 3; }
        }
    }
    // lane i (< 8) of lane 0's warm-up sample i, lane 0's sample 0 (CONSTANT): taken now, the registers die below
    const uint32_t xi = Ls.warm(lane);
    // ---- field positions
    int src, srx;
    sample_rate_code(P.sample_rate, src, srx);
    const bool tab = !SUB && fk < hdr_n;
    uint4 hrow = make_uint4(0, 0, 0, 0);
    if (tab) hrow = hdr_tab[fk];
    const uint32_t hb = SUB ? 0u : tab ? (hrow.w & 0xFFu) : frame_header_bytes((uint32_t)fk, srx);
    const uint32_t hdr_bits = hb << 3;
    const uint32_t pos0 = hdr_bits + 8 + (uint32_t)w;  // after the subframe header
    uint32_t pos = pos0;
    uint32_t end_bits;
    bool ok = true;
    typename Lane::Coefs C;
    int shift = lshift, k = 0, lanes_per = 64, o = 0, po = 0;
    uint32_t run = 0;      // lane-private write position (bits)
    uint32_t seglen = 0;   // the lane's segment length (bits)
    bool over = false;     // (wave-uniform) a lane outgrew its column: repack at known offsets
    if (type == 0) {
        end_bits = pos + (uint32_t)sbps;
    } else if (type == 1) {
        end_bits = pos + (uint32_t)n * sbps;
    } else {
        o = type == 2 ? of : ol;
        po = type == 2 ? po_f : po_l;
        k = type == 2 ? k_f : k_l;
        lanes_per = 64 >> po;
        if (type == 2) {
            int32_t qf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (of == 1) qf[0] = 1;
            else if (of == 2) { qf[0] = 2; qf[1] = -1; }
            else if (of == 3) { qf[0] = 3; qf[1] = -3; qf[2] = 1; }
            else if (of == 4) { qf[0] = 4; qf[1] = -6; qf[2] = 4; qf[3] = -1; }
            C = Lane::coefs(qf);
            shift = 0;
        } else {
            C = CL;
        }
        pos += (uint32_t)o * sbps;
        if (type == 3) pos += 9 + (uint32_t)o * A.lpc_prec;
        pos += 6;  // RICE method + partition order; the partitions' parameters sit in their first lanes' segments
    }
    // ---- the previous frame of this wave: its successors have had this frame's loads, sums and Rice search to
    //      publish, so the look-back rarely waits; store it and free the buffer (zero after this)
    if constexpr (!SUB)
        if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);
    if (type >= 2) {
        // ---- private packing: the lane's codes into its column (hi word at row p >> 5, lo word one row below;
        //      rows clamped so an overflowing lane stays inside the buffer -- its frame is repacked below)
        uint32_t *pcol = fbuf + lane;
        if ((lane & (lanes_per - 1)) == 0) {
            run = 4;
            pcol[0] = (uint32_t)k << 28;
        }
        const uint32_t sh = 31u - (uint32_t)k, oneL = 0x80000000u, k1 = 1u + (uint32_t)k;
#pragma unroll
        for (int m = 0; m < 32; m++) {
            if (m % 4 == 0 && m) asm volatile("" : "+v"(run));
            int32_t re, ro;
            Ls.residuals(C, shift, m, re, ro);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int j = 2 * m + h;
                const uint32_t u = zigzag(h ? ro : re);
                uint32_t codeL = (u << sh) | oneL;
                uint32_t p = run + (u >> k);  // the code's stop bit (its unary zeros are the buffer's)
                const bool warm = j < kMaxLpc && l0 && j < o;  // (lane 0's warm-up samples: no code)
                if (warm) {
                    codeL = 0;
                    p = run;
                }
                uint32_t *a = pcol + (min(p >> 5, (uint32_t)(kPrivRows - 1)) << 6);
                atomicOr(a, __builtin_amdgcn_alignbit(0u, codeL, p));
                atomicOr(a + 64, __builtin_amdgcn_alignbit(codeL, 0u, p));
                run = warm ? run : p + k1;
            }
        }
        over = __ballot(run > kPrivBits) != 0;
        const uint32_t incl = dpp_incl_scan_u32(run);
        const uint64_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint64_t fin = (uint64_t)pos + total;
        end_bits = (uint32_t)fin;
        if (fin + 64 > (uint64_t)kFrameWordsV3 * 32) ok = false;
        seglen = run;
        run = incl - run;  // from here: the lane's exclusive offset within the residual section
    }
    if (!ok) {
        if (l0) atomicOr(err, 2);
        end_bits = 0;
    }
    const uint32_t body = (end_bits + 7) >> 3;  // bytes before the CRC-16 footer
    const uint64_t fbytes = ok ? (uint64_t)body + 2 : 0;
    if (!SUB && l0) {  // publish our aggregate
        const uint64_t v = (f == 0 ? kFlagIncl : kFlagAgg) | fbytes;
        __hip_atomic_store(&status[f], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (SUB && WIDE) {
        if (type == 1 && sbps == 17) {
            // 17-bit VERBATIM side subframe: 69640 bits, one word past the LDS frame buffer.  A lane's 64 samples are
            // 1088 bits = 34 words starting at subframe bit 8 + 1088 lane: packed in registers, stored to the slot
            uint32_t X[34];
#pragma unroll
            for (int i = 0; i < 34; i++) X[i] = 0;
#pragma unroll
            for (int j = 0; j < 64; j++) {
                const int b = 17 * j, wi = b >> 5, r = b & 31;
                const uint32_t v = (uint32_t)Ls.x(j) & 0x1FFFFu;
                if (r <= 15) X[wi] |= v << (15 - r);
                else {
                    X[wi] |= v >> (r - 15);
                    X[wi + 1] |= v << (47 - r);
                }
            }
            const uint32_t before = (uint32_t)__shfl_up((int)X[33], 1);  // the previous lane's last word
            uint32_t *dst = sub_slots + (size_t)sub * kSubWords + 34 * lane;
            dst[0] = ((l0 ? 0x02u : before) << 24) | (X[0] >> 8);  // (lane 0: the subframe header, VERBATIM)
#pragma unroll
            for (int i = 1; i < 34; i++) dst[i] = (X[i - 1] << 24) | (X[i] >> 8);
            if (lane == 63) dst[34] = X[33] << 24;
            if (l0) {
                sub_bits[sub] = (int32_t)end_bits;
                if (sub_est) sub_est[sub] = (int32_t)best;
            }
            return;  // (the LDS buffer was not touched: still zero)
        }
    }
    // ---- assembly into the v3 frame layout (word w at row w mod C, column w / C: the store and CRC read rows, the
    //      lanes' columns fall in distinct banks)
    const FbMap M = fb_map(((end_bits + 23) >> 5) + 2);  // words written: body, CRC-16 (byte aligned), one spare
    const int nk4 = -4 * (int)M.k;
    bool fold = false;  // (wave-uniform) the v3 writer ran: its overflow row needs folding
    // OR a lane's segment (registers Pv: MSB-first words from segment bit 0) in at frame bit `off`, `nwl` words: word
    // i at column c0 row r0 + i while that is inside the column, then column c0 + 1 from row 0 (two base addresses,
    // the row step is the ds offset); a lane spanning three columns (a frame far smaller than its largest segment)
    // maps every word exactly
    auto assemble = [&](const uint32_t *Pv, uint32_t off, uint32_t nwl) {
        const uint32_t r = off & 31u, w0 = off >> 5;
        const uint32_t c0 = M.col(w0), r0 = w0 - c0 * M.c, split = M.c - r0;
        uint32_t *A = fbuf + (r0 << 6) + c0;
        uint32_t *B = A + 1 - (int)(M.c << 6);
        const uint32_t nmax = dpp_wave_max_u32(nwl);
        if (__ballot(nwl > split + M.c) == 0) {
            // words past the lane's last are zeros (its column is zero past its length): no per-lane predicate, and
            // every address stays inside the wave's buffer (row <= 33 of column c0 + 1 <= 64)
#pragma unroll
            for (int i = 0; i <= kPrivRows; i++) {
                if (i % 8 == 0 && (uint32_t)i >= nmax) break;  // (wave-uniform, every 8 words)
                atomicOr(((uint32_t)i < split ? A : B) + 64 * i,
                         __builtin_amdgcn_alignbit(i ? Pv[i - 1] : 0u, Pv[i], r));
            }
        } else {
#pragma unroll
            for (int i = 0; i <= kPrivRows; i++)
                if ((uint32_t)i < nwl) atomicOr(fbuf + M(w0 + (uint32_t)i), __builtin_amdgcn_alignbit(i ? Pv[i - 1] : 0u, Pv[i], r));
        }
    };
    if (type >= 2) {
        uint32_t Pv[kPrivRows + 1];
        const uint32_t *pcol = fbuf + lane;
#pragma unroll
        for (int i = 0; i <= kPrivRows; i++) Pv[i] = pcol[i << 6];
        __builtin_amdgcn_s_waitcnt(0xC07F);  // every lane's column is in registers before the zeroing
        __builtin_amdgcn_wave_barrier();
        zero_wave_buf(fbuf, lane);
        if (ok && !over) {
            const uint32_t off = pos + run;
            assemble(Pv, off, ((off & 31u) + seglen + 31) >> 5);
        } else if (ok) {
            // a lane outgrew its column: the v3 writer at the known offsets, from the samples loaded again (rare: the
            // registers of the first load are free for the assembly)
            load_lane(Ls);
            uint32_t rp = pos + run;
            if ((lane & (lanes_per - 1)) == 0) {
                lds_put_bits2(fbuf, M, rp, (uint32_t)k, 4);
                rp += 4;
            }
            const uint32_t sh = 31u - (uint32_t)k, oneL = 0x80000000u;
#pragma unroll
            for (int m = 0; m < 32; m++) {
                int32_t re, ro;
                Ls.residuals(C, shift, m, re, ro);
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int j = 2 * m + h;
                    const uint32_t u = zigzag(h ? ro : re);
                    uint32_t q = u >> k, codeL = (u << sh) | oneL, adv = q + 1 + (uint32_t)k;
                    if (j < kMaxLpc && l0 && j < o) {
                        q = 0;
                        codeL = 0;
                        adv = 0;
                    }
                    lds_put_left(fbuf, M, nk4, rp + q, codeL);
                    rp += adv;
                }
            }
            fold = true;
        }
    } else if (type == 1) {
        if (!WIDE && w == 0) {
            // 16-bit VERBATIM: the lane's 64 samples are its 32 packed pairs (halves swapped to MSB-first order)
            uint32_t Pv[kPrivRows + 1];
#pragma unroll
            for (int m = 0; m < 32; m++) {
                if constexpr (!WIDE) Pv[m] = __builtin_amdgcn_alignbit(Ls.E[4 + m], Ls.E[4 + m], 16);
            }
#pragma unroll
            for (int m = 32; m <= kPrivRows; m++) Pv[m] = 0;
            const uint32_t off = pos + 1024u * (uint32_t)lane;
            assemble(Pv, off, ((off & 31u) + 1024u + 31) >> 5);
        } else {
            const uint32_t p0 = pos + (uint32_t)(64 * lane) * (uint32_t)sbps;
            const uint32_t shl = 32u - (uint32_t)sbps;
#pragma unroll
            for (int j = 0; j < 64; j++) lds_put_left(fbuf, M, nk4, p0 + (uint32_t)j * sbps, (uint32_t)Ls.x(j) << shl);
            fold = true;
        }
    }
    // ---- header, subframe header, warm-up, coefficients, partition order (fixed positions below pos)
    if (l0) {
        if (tab) {
            // 13 header bytes at most; the 4th word's low byte holds the length (byte 15: never a header byte)
            atomicOr(fbuf + M(0), hrow.x);
            atomicOr(fbuf + M(1), hrow.y);
            atomicOr(fbuf + M(2), hrow.z);
            atomicOr(fbuf + M(3), hrow.w & 0xFFFFFF00u);
        } else if (!SUB) {
            uint32_t hbits = 0, c8 = 0;
            auto put8 = [&](uint32_t b) {
                lds_put_bits2(fbuf, M, hbits, b, 8);
                c8 = S.crc8[c8 ^ b];
                hbits += 8;
            };
            const int sr = P.sample_rate;
            put8(0xFF);
            put8(0xF8);
            put8((uint32_t)((12 << 4) | src));  // block size code 12 = 4096
            put8((uint32_t)(4 << 1));           // mono, 16 bits
            const uint32_t v = (uint32_t)fk;    // UTF-8 coded frame number
            if (v < 0x80) put8(v);
            else if (v < 0x800) { put8(0xC0 | (v >> 6)); put8(0x80 | (v & 0x3F)); }
            else if (v < 0x10000) { put8(0xE0 | (v >> 12)); put8(0x80 | ((v >> 6) & 0x3F)); put8(0x80 | (v & 0x3F)); }
            else if (v < 0x200000) { put8(0xF0 | (v >> 18)); put8(0x80 | ((v >> 12) & 0x3F)); put8(0x80 | ((v >> 6) & 0x3F)); put8(0x80 | (v & 0x3F)); }
            else if (v < 0x4000000) { put8(0xF8 | (v >> 24)); put8(0x80 | ((v >> 18) & 0x3F)); put8(0x80 | ((v >> 12) & 0x3F)); put8(0x80 | ((v >> 6) & 0x3F)); put8(0x80 | (v & 0x3F)); }
            else { put8(0xFC | (v >> 30)); put8(0x80 | ((v >> 24) & 0x3F)); put8(0x80 | ((v >> 18) & 0x3F)); put8(0x80 | ((v >> 12) & 0x3F)); put8(0x80 | ((v >> 6) & 0x3F)); put8(0x80 | (v & 0x3F)); }
            if (srx == 12) put8((uint32_t)(sr / 1000));
            else if (srx == 13) { put8((uint32_t)(sr >> 8) & 0xFF); put8((uint32_t)sr & 0xFF); }
            else if (srx == 14) { put8((uint32_t)((sr / 10) >> 8) & 0xFF); put8((uint32_t)(sr / 10) & 0xFF); }
            put8(c8);  // CRC-8
        }
        const int typecode = type == 0 ? 0 : type == 1 ? 1 : type == 2 ? 8 + of : 32 + ol - 1;
        lds_put_bits2(fbuf, M, hdr_bits, (uint32_t)(typecode << 1) | (w ? 1u : 0u), 8);
        if (w) lds_put_bits2(fbuf, M, hdr_bits + 8 + (uint32_t)(w - 1), 1, 1);
        if (type == 0) lds_put_bits2(fbuf, M, pos0, xi & ((1u << sbps) - 1u), sbps);  // (lane 0: its sample 0)
        if (type >= 2) {
            uint32_t qq = pos0 + (uint32_t)o * sbps;
            if (type == 3) {
                lds_put_bits2(fbuf, M, qq, (uint32_t)(A.lpc_prec - 1), 4);
                lds_put_bits2(fbuf, M, qq + 4, (uint32_t)lshift & 31u, 5);
                qq += 9 + (uint32_t)o * A.lpc_prec;
            }
            lds_put_bits2(fbuf, M, qq, (uint32_t)po, 6);  // RICE (00) + partition order (4 bits)
        }
    }
    if (type >= 2) {
        // warm-up samples and quantised coefficients in parallel: lane i < o writes lane 0's sample i, lane 8 + i
        // (LPC) coefficient i
        const int i = lane & 7;
        const int32_t qi = ana[sub].q[i];  // (a lane-indexed load: a select chain over A.q costs registers)
        const bool warm = lane < 8 && i < o, coef = type == 3 && lane >= 8 && lane < 16 && i < o;
        if (warm) lds_put_bits2(fbuf, M, pos0 + (uint32_t)i * sbps, xi & ((1u << sbps) - 1u), sbps);
        if (coef)
            lds_put_bits2(fbuf, M, pos0 + (uint32_t)o * sbps + 9 + (uint32_t)i * A.lpc_prec,
                          (uint32_t)qi & ((1u << A.lpc_prec) - 1u), A.lpc_prec);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS atomics have landed
    __builtin_amdgcn_wave_barrier();
    if (fold) {  // (wave-uniform) the v3 writer's overflow row home
        fb_fold(fbuf, M, lane);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
    if constexpr (SUB) {
        // the subframe's words (bits past end_bits are zeros) to its slot, then re-zero the buffer
        if (ok) {
            uint32_t *dst = sub_slots + (size_t)sub * kSubWords;
            const uint32_t nw = (end_bits + 31) >> 5;
            for (uint32_t wi = (uint32_t)lane; wi < nw; wi += 64) dst[wi] = fbuf[M(wi)];
            for (uint32_t i = 0; i < M.c; i++) fbuf[(i << 6) | (uint32_t)lane] = 0;
        } else {
            zero_wave_buf(fbuf, lane);
        }
        if (l0) sub_bits[sub] = ok ? (int32_t)end_bits : -1;
        if (l0 && sub_est) sub_est[sub] = (int32_t)best;  // (a two-channel stream picks its assignment by these)
        (void)fbytes;
        return;
    }
    if (ok) {
        const uint32_t crc = crc16_cols(fbuf, M, body, S, lane);
        if (l0) lds_put_bits2(fbuf, M, body << 3, crc, 16);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
    prev.f = f, prev.fbytes = fbytes, prev.ok = ok, prev.map = M;
}

// SUB: the units are subframes -- (frame, channel) of a >= 3-channel stream, or of a two-channel stream's mid/side
// pass (ST): left, right, mid in one launch, the 17-bit side signals (WIDE) in another.
template <int DT, bool SUB = false, bool ST = false, bool WIDE = false>
// (3 waves per SIMD for mono / >= 3-channel 16-bit units; 2 for the two-channel launches: L/R/M need 195 VGPRs, the
// int32 side 256 -- capped from 262, a 32-byte spill: convert_2band encode 3.17 -> 2.78 ms against 1 wave per SIMD)
__global__ void __launch_bounds__(256, sizeof(typename Elem<DT>::T) <= 2 ? (ST ? 2 : 3) : 1) k_encode_v4(const typename Elem<DT>::T *raster, EncodeParams P,
                                                  const TileGeom *tiles, const TileNorm *norms, const int16_t *luts,
                                                  const SubAnalysis *ana, uint8_t *arena, int64_t arena_cap,
                                                  int64_t *frame_off, uint64_t *status, int *ticket_ctr, int *err,
                                                  const int32_t *__restrict__ ftile, const uint4 *__restrict__ hdr_tab,
                                                  int hdr_n, const uint32_t *__restrict__ pslots,
                                                  const int64_t *__restrict__ pbytes, uint32_t *sub_slots = nullptr,
                                                  int32_t *sub_bits = nullptr, int32_t *sub_est = nullptr) {
    __shared__ __attribute__((aligned(16))) EncV3Shared S;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) (&S.crc8x[0][0])[i] = (&c_crc16x8[0][0])[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) S.crc8[i] = c_crc8[i];
    for (int i = threadIdx.x; i < 64; i += blockDim.x) S.xlo[i] = g_xpow_bytes[i];
    for (int i = threadIdx.x; i < kXpowHi; i += blockDim.x) S.xhi[i] = g_xpow_bytes[64 * i];
    for (int i = threadIdx.x; i < 4 * kBufWordsV3; i += blockDim.x) (&S.bits[0][0])[i] = 0;
    if (threadIdx.x == 0) S.lut_tile = -1;
    PendingFrame prev;
    uint32_t *fbuf = S.bits[wave];
    // one barrier per ticket: the ticket and the tile it wants are double-buffered (slot = iteration & 1), so thread 0
    // may write the next ticket while slower waves still read this one; every wave still meets the others once per
    // ticket, after the atomic, so the LUT is never rewritten under a wave that encodes with it (round 6: encode
    // 3.88-3.89 -> 3.84 ms, step 5.27-5.29 -> 5.22-5.24 ms, three alternations on one box; tools/r6/enc_variants.py)
    int it = 0;
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
            const TileNorm tw = norms[want];
            if (tw.mode == kNormLut) {
                const int64_t R = min(tw.imax - tw.imin, (int64_t)kLutCap - 1);
                const int16_t *src = luts + (int64_t)want * kLutCap;
                for (int64_t d = threadIdx.x; d <= R; d += blockDim.x) S.lut[d] = src[d];
            }
            __syncthreads();
            if (threadIdx.x == 0) S.lut_tile = want;
        }
        if constexpr (SUB) {
            const int64_t v = fbase + wave;
            if (v < nunits) {
                const int64_t f = v / upf;
                const int chn = WIDE ? 3 : (int)(v - f * upf);
                const TileGeom g = tiles[ftile[f]];
                if (!(g.partial && f - g.frame_base == g.nframes - 1))
                    encode_frame_v4<DT, true, ST, WIDE>(raster, P, tiles, norms, ana, arena, arena_cap, frame_off,
                                                        status, err, S, want, f, lane, ftile, prev, hdr_tab, hdr_n,
                                                        pslots, pbytes, chn, sub_slots, sub_bits, sub_est);
            }
        } else {
            const int64_t f = fbase + wave;
            if (f < nunits)
                encode_frame_v4<DT>(raster, P, tiles, norms, ana, arena, arena_cap, frame_off, status, err, S, want, f,
                                    lane, ftile, prev, hdr_tab, hdr_n, pslots, pbytes);
        }
    }
    if constexpr (!SUB)
        if (prev.f >= 0) resolve_and_store(P, prev, fbuf, arena, arena_cap, frame_off, status, err, lane);
}

// ---------------------------------------------------------------- multi-channel streams (>= 3 channels, 16-bit)
// libFLAC codes the channels of a >= 3-channel frame independently (no stereo decorrelation), so the subframes are
// the fast encoder's units (k_encode_v3<DT, true>); a frame is then its header, the subframes' bit strings back to
// back, zero padding to a byte and the CRC-16.  k_mc_frame_bytes sizes the frames, k_scan_sizes places them and
// k_mc_assemble writes them (the tile's partial last frame comes sealed from the generic kernels).

// frame header of a full 4096-sample frame (RFC 9639 9.1, as k_encode_frames writes it); returns its bytes
// chcode: the channel assignment nibble (nch - 1 for independent channels; 8 / 9 / 10 left-side / right-side / mid-side)
__device__ inline int mc_frame_header(uint8_t *h, uint32_t v, int chcode, int sr) {
    int src, srx;
    sample_rate_code(sr, src, srx);
    int hb = 0;
    h[hb++] = 0xFF;
    h[hb++] = 0xF8;
    h[hb++] = (uint8_t)((12 << 4) | src);
    h[hb++] = (uint8_t)((chcode << 4) | (4 << 1));
    if (v < 0x80) h[hb++] = (uint8_t)v;
    else if (v < 0x800) { h[hb++] = (uint8_t)(0xC0 | (v >> 6)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    else if (v < 0x10000) { h[hb++] = (uint8_t)(0xE0 | (v >> 12)); h[hb++] = (uint8_t)(0x80 | ((v >> 6) & 0x3F)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    else if (v < 0x200000) { h[hb++] = (uint8_t)(0xF0 | (v >> 18)); h[hb++] = (uint8_t)(0x80 | ((v >> 12) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 6) & 0x3F)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    else if (v < 0x4000000) { h[hb++] = (uint8_t)(0xF8 | (v >> 24)); h[hb++] = (uint8_t)(0x80 | ((v >> 18) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 12) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 6) & 0x3F)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    else { h[hb++] = (uint8_t)(0xFC | (v >> 30)); h[hb++] = (uint8_t)(0x80 | ((v >> 24) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 18) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 12) & 0x3F)); h[hb++] = (uint8_t)(0x80 | ((v >> 6) & 0x3F)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
    if (srx == 12) h[hb++] = (uint8_t)(sr / 1000);
    else if (srx == 13) { h[hb++] = (uint8_t)(sr >> 8); h[hb++] = (uint8_t)sr; }
    else if (srx == 14) { h[hb++] = (uint8_t)((sr / 10) >> 8); h[hb++] = (uint8_t)(sr / 10); }
    uint8_t c = 0;
    for (int i = 0; i < hb; i++) c = c_crc8[c ^ h[i]];
    h[hb++] = c;
    return hb;
}

// A two-channel stream's frame (P.nvch == 4: L, R, M, S coded): libFLAC process_subframes_ keeps the assignment with
// the fewest estimated bits among independent (L, R), left-side (L, S), right-side (S, R), mid-side (M, S) -- in that
// order, a later one only when strictly smaller (stream_encoder.c; oracle orc_encode_frames_level).
__device__ inline int st_pick(const int32_t *est4) {
    const uint32_t e0 = (uint32_t)est4[0], e1 = (uint32_t)est4[1], e2 = (uint32_t)est4[2], e3 = (uint32_t)est4[3];
    const uint32_t bits[4] = {e0 + e1, e0 + e3, e1 + e3, e2 + e3};
    int ca = 0;
    for (int k = 1; k < 4; k++)
        if (bits[k] < bits[ca]) ca = k;
    return ca;
}
__device__ inline void st_subs(int ca, int &a, int &b) {  // coded signals of an assignment (left/right order)
    a = ca == 2 ? 3 : ca == 3 ? 2 : 0;
    b = ca == 0 ? 1 : ca == 2 ? 1 : 3;
}

__global__ void k_mc_frame_bytes(const EncodeParams P, const TileGeom *tiles, const int32_t *ftile,
                                 const int32_t *sub_bits, const int64_t *pbytes, int64_t *frame_bytes, int *err,
                                 const int32_t *sub_est = nullptr, int8_t *pick = nullptr) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= P.nframes) return;
    const TileGeom g = tiles[ftile[f]];
    const int64_t fk = f - g.frame_base;
    if (g.partial && fk == g.nframes - 1) {
        frame_bytes[f] = pbytes[g.partial - 1];
        return;
    }
    uint8_t h[16];
    const bool st = P.nvch == 4 && P.nch == 2;
    int chcode = P.nch - 1, sa = 0, sb = 1;
    if (st) {
        const int ca = st_pick(sub_est + f * 4);
        pick[f] = (int8_t)ca;
        chcode = ca == 0 ? 1 : 7 + ca;
        st_subs(ca, sa, sb);
    }
    int64_t bits = 8 * mc_frame_header(h, (uint32_t)fk, chcode, P.sample_rate);
    for (int c = 0; c < P.nch; c++) {
        const int32_t b = sub_bits[f * P.nvch + (st ? (c ? sb : sa) : c)];
        if (b < 0) atomicOr(err, 2);
        bits += b < 0 ? 0 : b;
    }
    frame_bytes[f] = ((bits + 7) >> 3) + 2;
}

// One work-group per frame: the frame image in LDS (big-endian bit order words), then its bytes to the arena.
// (Persistent work-groups looping over the frames measured slower: 2.20 vs 2.11 ms for a 4-band 16384^2 job.)  Only the frame's own words are zeroed; a subframe's interior words are
// plain stores (each is made of two of its source words), its first and last words -- shared with the header or the
// neighbouring subframe -- are ORed in.
__global__ void __launch_bounds__(256) k_mc_assemble(const EncodeParams P, const TileGeom *tiles, const int32_t *ftile,
                                                    const uint32_t *sub_slots, const int32_t *sub_bits,
                                                    const uint32_t *pslots, const int64_t *pbytes,
                                                    const int64_t *frame_off, uint8_t *arena,
                                                    const int8_t *pick = nullptr) {
    extern __shared__ uint32_t W[];  // nch * kFrameWordsV3 + 16 words
    __shared__ uint16_t T[4][256];
    __shared__ uint32_t wc[4];
    const int tid = threadIdx.x;
    const int64_t f = blockIdx.x;
    const TileGeom g = tiles[ftile[f]];
    const int64_t fk = f - g.frame_base;
    uint8_t *dst = arena + frame_off[f];
    if (g.partial && fk == g.nframes - 1) {  // sealed by the generic kernels: copy
        const int64_t si = g.partial - 1, nb = pbytes[si];
        const uint8_t *src = reinterpret_cast<const uint8_t *>(pslots + (size_t)si * P.slot_words);
        for (int64_t i = tid; i < nb; i += 256) dst[i] = src[i];
        return;
    }
    wg_load_crc_tables(T);
    uint8_t h[16];
    const bool st = P.nvch == 4 && P.nch == 2;  // two channels: the picked pair of L, R, M, S
    int chcode = P.nch - 1, sa = 0, sb = 1;
    if (st) {
        const int ca = pick[f];
        chcode = ca == 0 ? 1 : 7 + ca;
        st_subs(ca, sa, sb);
    }
    auto unit = [&](int c) -> int64_t { return f * P.nvch + (st ? (c ? sb : sa) : c); };
    const int hb = mc_frame_header(h, (uint32_t)fk, chcode, P.sample_rate);
    int64_t total = 8 * hb;
    for (int c = 0; c < P.nch; c++) total += max(0, sub_bits[unit(c)]);
    const int nwz = (int)(((total + 7) >> 3) + 2 + 3) / 4 + 1;  // words of body + CRC-16, one spare
    for (int i = tid; i < nwz; i += 256) W[i] = 0;
    __syncthreads();
    if (tid == 0)
        for (int i = 0; i < hb; i++) W[i >> 2] |= (uint32_t)h[i] << (24 - 8 * (i & 3));
    int64_t o = 8 * hb;
    for (int c = 0; c < P.nch; c++) {
        const int32_t nbits = sub_bits[unit(c)];
        const uint32_t *sw = sub_slots + (size_t)unit(c) * kSubWords;
        const int nw = (nbits + 31) >> 5, sh = (int)(o & 31);
        const int64_t w0 = o >> 5;
        const int64_t wl = (o + nbits - 1) >> 5;  // last destination word holding a bit of this subframe
        // destination word w0 + k (k = 0 .. wl - w0) = (sw[k] >> sh) | (sw[k - 1] << (32 - sh)); the loads of a
        // thread's (up to) 8 words issue together (one memory latency per 2048 words, not one per word)
        const int64_t span = nbits > 0 ? wl - w0 : -1;
        for (int64_t kb = 0; kb <= span; kb += 256 * 8) {
            uint32_t va[8], vb[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int64_t k = kb + 256 * u + tid;
                va[u] = (k <= span && k < nw) ? sw[k] : 0u;
                vb[u] = (k <= span && k > 0 && k - 1 < nw) ? sw[k - 1] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int64_t k = kb + 256 * u + tid;
                if (k > span) break;
                const uint32_t v = (va[u] >> sh) | (sh ? vb[u] << (32 - sh) : 0u);
                if (k == 0 || k == span) atomicOr(&W[w0 + k], v);
                else W[w0 + k] = v;
            }
        }
        o += nbits;
    }
    __syncthreads();
    const int64_t B = (o + 7) >> 3;  // body bytes (zero-padded)
    // CRC-16 over bytes [0, B): words hold bytes big-endian
    {
        const int64_t nw = B >> 2;
        const int64_t ch = (nw + 255) / 256;
        const int64_t a0 = min(nw, (int64_t)tid * ch), a1 = min(nw, a0 + ch);
        uint32_t c = 0;
        for (int64_t i = a0; i < a1; i++) {
            const uint32_t v = W[i];
            c = (uint32_t)T[3][((c >> 8) ^ (v >> 24)) & 0xFF] ^ T[2][((c & 0xFF) ^ (v >> 16)) & 0xFF] ^
                T[1][(v >> 8) & 0xFF] ^ T[0][v & 0xFF];
        }
        int64_t end = a1 << 2;
        const bool last = (nw == 0) ? tid == 0 : (a1 == nw && a1 > a0);
        if (last) {
            for (int64_t i = nw << 2; i < B; i++) {
                const uint32_t byte = (W[i >> 2] >> (24 - 8 * (i & 3))) & 0xFF;
                c = ((c << 8) & 0xFFFFu) ^ T[0][((c >> 8) ^ byte) & 0xFF];
            }
            end = B;
        }
        const int64_t m = B - end;
        if (c && m > 0) c = gf_mulmod(c, xpow_bytes(m));
        for (int d = 32; d > 0; d >>= 1) c ^= __shfl_xor(c, d);
        if ((tid & 63) == 0) wc[tid >> 6] = c;
        __syncthreads();
        const uint32_t crc = wc[0] ^ wc[1] ^ wc[2] ^ wc[3];
        if (tid == 0) {
            W[B >> 2] |= ((crc >> 8) & 0xFF) << (24 - 8 * (B & 3));
            W[(B + 1) >> 2] |= (crc & 0xFF) << (24 - 8 * ((B + 1) & 3));
        }
        __syncthreads();
    }
    // bytes [0, B + 2) to dst: aligned 4-byte stores assembled from byte-swapped words
    const int64_t S = B + 2;
    const int hh = (int)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3);
    const int64_t hbytes = min((int64_t)hh, S);
    auto byte_at = [&](int64_t i) -> uint8_t { return (uint8_t)(W[i >> 2] >> (24 - 8 * (i & 3))); };
    if (tid < hbytes) dst[tid] = byte_at(tid);
    const int64_t nbw = (S - hbytes) >> 2;
    uint32_t *dw = reinterpret_cast<uint32_t *>(dst + hbytes);
    const int sh = (int)(hbytes & 3);
    for (int64_t k = tid; k < nbw; k += 256) {
        const int64_t si = (hbytes + 4 * k) >> 2;
        const uint32_t lo = __builtin_bswap32(W[si]), hi = sh ? __builtin_bswap32(W[si + 1]) : 0u;
        dw[k] = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)sh);
    }
    for (int64_t i = hbytes + 4 * nbw + tid; i < S; i += 256) dst[i] = byte_at(i);
}

// results of the fast path packed for one D2H copy: tile offsets [ntiles + 1], (dmin, dmax) per tile, error flags
__global__ void k_fast_finish(const int64_t *frame_off, const uint64_t *status, const TileGeom *tiles,
                              const TileNorm *norms, const int *err_flag, int ntiles, int64_t nframes, int64_t *pack) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    double *mm = reinterpret_cast<double *>(pack + ntiles + 1);
    if (t < ntiles) {
        pack[t] = frame_off[tiles[t].frame_base];
        mm[2 * t] = norms[t].dmin;
        mm[2 * t + 1] = norms[t].dmax;
    }
    if (t == ntiles) {
        pack[t] = (int64_t)(status[nframes - 1] & kValMask);
        pack[3 * (int64_t)ntiles + 1] = *err_flag;
    }
}

// ------------------------------------------------------------------------------------- host side
static bool g_tables_ready[64];

static int upload_tables(frs_ctx *ctx) {
    if (g_tables_ready[ctx->device]) return FRS_OK;
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
    // x^(8*2^j) mod P by repeated squaring of x^8
    uint16_t xp[40];
    auto mulmod = [](uint32_t a, uint32_t b) {
        uint32_t r = 0;
        for (int i = 15; i >= 0; i--) {
            r <<= 1;
            if (r & 0x10000u) r ^= 0x18005u;
            if ((b >> i) & 1u) r ^= a;
        }
        return r;
    };
    uint32_t v = 0x100;  // x^8
    for (int j = 0; j < 40; j++) {
        xp[j] = (uint16_t)v;
        v = mulmod(v, v);
    }
    FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_crc8), t8, sizeof(t8), 0, hipMemcpyHostToDevice, ctx->stream));
    FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_crc16), t16, sizeof(t16), 0, hipMemcpyHostToDevice, ctx->stream));
    FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_xpow8), xp, sizeof(xp), 0, hipMemcpyHostToDevice, ctx->stream));
    // slice-by-16 tables: T_k[v] = T_{k-1}[v] advanced by one zero byte
    static uint16_t t4[16][256];
    static uint16_t xb[kXpowBytes];
    for (int i = 0; i < 256; i++) t4[0][i] = t16[i];
    for (int k = 1; k < 16; k++)
        for (int i = 0; i < 256; i++) {
            const uint16_t c = t4[k - 1][i];
            t4[k][i] = (uint16_t)(((c << 8) & 0xFFFF) ^ t16[c >> 8]);
        }
    uint32_t pw = 1;  // x^(8m) mod P
    for (int m = 0; m < kXpowBytes; m++) {
        xb[m] = (uint16_t)pw;
        pw = mulmod(pw, 0x100);
    }
    FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_crc16x8), t4, sizeof(t4), 0, hipMemcpyHostToDevice, ctx->stream));
    FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_xpow_bytes), xb, sizeof(xb), 0, hipMemcpyHostToDevice, ctx->stream));
    static uint16_t x8k[32];
    uint32_t x8192 = 1;  // x^(8 * 8192)
    for (int m = 0; m < 8192; m++) x8192 = mulmod(x8192, 0x100);
    uint32_t q = 1;
    for (int j = 0; j < 32; j++) {
        x8k[j] = (uint16_t)q;
        q = mulmod(q, x8192);
    }
    FRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_xpow_8k), x8k, sizeof(x8k), 0, hipMemcpyHostToDevice, ctx->stream));
    FRS_HIP(hipStreamSynchronize(ctx->stream));
    g_tables_ready[ctx->device] = true;
    return FRS_OK;
}

int dtype_size(int dt) {
    switch (dt) {
    case FRS_DT_U8: return 1;
    case FRS_DT_U16:
    case FRS_DT_I16: return 2;
    case FRS_DT_I32:
    case FRS_DT_U32:
    case FRS_DT_F32: return 4;
    case FRS_DT_F64: return 8;
    default: return 0;
    }
}

static int stream_bps_of(const frs_encode_desc *d) {
    // pyflac: bits_per_sample = itemsize * 8 of the sample array (sonos-pyflac.txt:1986-1992): int16 for
    // bps 16, int32 for bps 24 and float32 for the spatial encoder's normalisation
    return (d->norm_mode == 0 && d->bits_per_sample == 16) ? 16 : 32;
}

static int qlp_precision_for(int bps, int blocksize) {
    // stream_encoder.c init: qlp_coeff_precision == 0 (level 5) -> chosen by bps and blocksize
    if (bps < 16) return (2 + bps / 2) > 5 ? 2 + bps / 2 : 5;
    if (bps == 16) {
        if (blocksize <= 192) return 7;
        if (blocksize <= 384) return 8;
        if (blocksize <= 576) return 9;
        if (blocksize <= 1152) return 10;
        if (blocksize <= 2304) return 11;
        if (blocksize <= 4608) return 12;
        return 13;
    }
    if (blocksize <= 384) return 13;
    if (blocksize <= 1152) return 14;
    return 15;
}

static int64_t slot_words_for(const frs_encode_desc *d) {
    // verbatim bound of a frame + header + slack (the exact coder can exceed the estimate a little)
    const int64_t bps = stream_bps_of(d);
    // (+ one bit per sample for a two-channel stream's side signal)
    const int64_t bits = 16 * 8 + (int64_t)d->nbands * (16 + 32 + (int64_t)d->blocksize * bps) +
                         (d->nbands == 2 ? (int64_t)d->blocksize : 0) + 64;
    return (bits + 31) / 32 + (int64_t)d->blocksize / 8 + 64;
}

static void build_tiles(const frs_encode_desc *d, std::vector<TileGeom> &tiles, int64_t &nframes) {
    const int64_t tcols = (d->width + d->tile_w - 1) / d->tile_w;
    nframes = 0;
    tiles.clear();
    for (int64_t ti = d->tile_begin; ti < d->tile_end; ti++) {
        TileGeom g;
        const int64_t tr = ti / tcols, tc = ti % tcols;
        g.r0 = tr * d->tile_h;
        g.c0 = tc * d->tile_w;
        g.h = (int32_t)std::min<int64_t>(d->tile_h, d->height - g.r0);
        g.w = (int32_t)std::min<int64_t>(d->tile_w, d->width - g.c0);
        const int64_t px = (int64_t)g.h * g.w;
        g.nframes = (int32_t)((px + d->blocksize - 1) / d->blocksize);
        g.frame_base = nframes;
        g.partial = 0;
        nframes += g.nframes;
        tiles.push_back(g);
    }
}

int64_t arena_bound(const frs_encode_desc *d) {
    std::vector<TileGeom> tiles;
    int64_t nframes;
    build_tiles(d, tiles, nframes);
    return nframes * (slot_words_for(d) * 4) + 64;
}

constexpr int kFastDeclined = 1000;  // run_encode: the fast path hit a frame it cannot hold; rerun generic

template <int DT>
static int run_encode(frs_ctx *ctx, const frs_encode_desc *d, const void *raster_dev, void *arena_dev,
                      int64_t arena_cap, int64_t *tile_off, double *tile_min, double *tile_max, bool allow_fast) {
    using T = typename Elem<DT>::T;
    // job geometry cache (frs_ctx::geo_*): everything the tile table, partial marking and wave table depend on
    const std::vector<int64_t> key = {d->height, d->width, d->tile_h, d->tile_w, d->tile_begin, d->tile_end,
                                      d->blocksize, d->nbands, d->dtype, d->bits_per_sample, d->norm_mode,
                                      (allow_fast && !ctx->force_generic) ? 1 : 0, d->compression_level};
    const bool geo_hit = !ctx->geo_key.empty() && ctx->geo_key == key;
    std::vector<TileGeom> tiles_local;
    std::vector<TileGeom> &tiles = geo_hit ? ctx->geo_tiles : tiles_local;
    int64_t nframes = ctx->geo_nframes;
    if (!geo_hit) {
        ctx->geo_key.clear();  // the device copies are rewritten below; valid again once uploaded
        build_tiles(d, tiles, nframes);
    }
    const int ntiles = (int)tiles.size();
    if (ntiles == 0) {
        tile_off[0] = 0;
        return FRS_OK;
    }
    EncodeParams P;
    P.row_stride = d->row_stride;
    P.band_stride = d->band_stride;
    P.band0 = d->band0;
    P.nch = d->nbands;
    P.blocksize = d->blocksize;
    P.sample_rate = d->sample_rate;
    P.bps = stream_bps_of(d);
    P.scale_bits = d->bits_per_sample == 16 ? 16 : 24;
    P.qlp_precision = qlp_precision_for(P.bps, d->blocksize);
    P.slot_words = (int32_t)slot_words_for(d);
    P.nframes = nframes;
    P.ntiles = ntiles;
    P.norm_mode = d->norm_mode;
    P.vec_ok = 0;
    const LevelParams lv = level_params(d->compression_level);
    // two channels with mid/side (levels 2, 5): L, R, mid, side (exhaustive mid/side stereo)
    P.nvch = (P.nch == 2 && lv.mid_side) ? 4 : P.nch;
    P.max_lpc = lv.max_lpc;
    P.max_po = lv.max_po;
    P.ncand = lv.parts > 1 ? apod_windows(lv.parts) : 0;
    // loose mid/side (stream_encoder.c init): an evaluation every (uint32_t)(sample_rate * 0.4 / blocksize + 0.5) frames
    P.loose_frames = 0;
    if (P.nch == 2 && lv.mid_side && lv.loose) {
        P.loose_frames = (int32_t)(uint32_t)((double)d->sample_rate * 0.4 / (double)d->blocksize + 0.5);
        if (P.loose_frames == 0) P.loose_frames = 1;
    }
    const bool level5 = d->compression_level == 5;  // the fast kernels hard-code level 5's search

    int rc = upload_tables(ctx);
    if (rc) return rc;
    hipStream_t st = ctx->stream;
    FRS_HIP(ctx->tiles.ensure(sizeof(TileGeom) * ntiles));
    FRS_HIP(ctx->norms.ensure(sizeof(TileNorm) * ntiles));
    FRS_HIP(ctx->analysis.ensure(sizeof(SubAnalysis) * nframes * P.nvch));
    FRS_HIP(ctx->frame_bytes.ensure(sizeof(int64_t) * (nframes + 1) + 64));
    FRS_HIP(ctx->frame_off.ensure(sizeof(int64_t) * (nframes + 1)));
    FRS_HIP(ctx->tile_sizes.ensure(sizeof(int64_t) * (ntiles + 1) + 64));
    // pinned staging: tiles | wave table | packed results (the previous call has synchronised, so it is free)
    const size_t pin_tiles = 0, pin_wt = (sizeof(TileGeom) * ntiles + 255) & ~(size_t)255;
    const size_t wt_cap = (size_t)(nframes / 64 + ntiles + 1) * (size_t)std::max(1, (int)P.nvch);
    const size_t pin_res = (pin_wt + sizeof(int2) * wt_cap + 255) & ~(size_t)255;
    const size_t res_bytes = sizeof(int64_t) * (3 * (size_t)ntiles + 2);
    const size_t pin_pl = (pin_res + res_bytes + 255) & ~(size_t)255;  // partial-frame list of the fast path
    FRS_HIP(ctx->pin.ensure(pin_pl + sizeof(int64_t) * (size_t)ntiles));
    // fast path: mono 16-bit streams of 4096-sample blocks.  A tile whose pixel count is not a multiple of 4096
    // ends in a partial frame: those frames (at most one per tile) are coded by the generic kernels first and
    // the fast encoder copies them into the arena in stream order
    const bool fast = allow_fast && !ctx->force_generic && level5 && P.bps == 16 && P.nch == 1 && P.norm_mode == 0 &&
                      d->blocksize == 4096 && !Elem<DT>::is_float;
    // multi-channel streams of >= 3 channels (plain convert of a multi-band raster): libFLAC codes their channels
    // independently, so the fast kernels code the subframes and k_mc_assemble joins them.  Two channels (st2):
    // libFLAC's mid/side pass codes L, R, M and S (17 bits) as subframes and keeps the cheapest pair by their
    // estimates (k_mc_frame_bytes picks, k_mc_assemble joins)
    const bool st2 = allow_fast && !ctx->force_generic && level5 && P.bps == 16 && P.nch == 2 && P.nvch == 4 &&
                     P.norm_mode == 0 && d->blocksize == 4096 && !Elem<DT>::is_float;
    const bool mc = st2 || (allow_fast && !ctx->force_generic && level5 && P.bps == 16 && P.nch >= 3 && P.nch <= 8 &&
                            P.norm_mode == 0 && d->blocksize == 4096 && !Elem<DT>::is_float);
    int64_t npartial = 0;
    int64_t *hplist = ctx->pin.at<int64_t>(pin_pl);
    if (geo_hit) {
        npartial = (int64_t)ctx->geo_plist.size();
        if (npartial) memcpy(hplist, ctx->geo_plist.data(), sizeof(int64_t) * (size_t)npartial);
    } else if (fast || mc) {
        for (TileGeom &tg : tiles)
            if (((int64_t)tg.h * tg.w) % d->blocksize != 0) {
                hplist[npartial] = tg.frame_base + tg.nframes - 1;
                tg.partial = (int32_t)(++npartial);
            }
    }
    // device copies of the cached geometry still in place (a grown buffer is a new allocation)
    const bool dev_tiles = geo_hit && ctx->geo_ptrs[0] == ctx->tiles.ptr;
    if (ctx->window_bs != d->blocksize) {
        std::vector<float> win(d->blocksize, 1.0f);
        // FLAC__window_tukey(0.5) computed in double with the host libm cos, stored as float (window.c)
        const float p = 0.5f;
        const int L = d->blocksize;
        const int Np = (int)(p / 2.0f * (float)L) - 1;
        if (Np > 0)
            for (int k = 0; k <= Np; k++) {
                win[k] = (float)(0.5f - 0.5f * cos(M_PI * k / Np));
                win[L - Np - 1 + k] = (float)(0.5f - 0.5f * cos(M_PI * (k + Np) / Np));
            }
        FRS_HIP(ctx->window.ensure(sizeof(float) * L));
        FRS_HIP(hipMemcpyAsync(ctx->window.ptr, win.data(), sizeof(float) * L, hipMemcpyHostToDevice, st));
        FRS_HIP(hipStreamSynchronize(st));
        ctx->window_bs = d->blocksize;
    }
    if (!dev_tiles) {
        memcpy(ctx->pin.at<TileGeom>(pin_tiles), tiles.data(), sizeof(TileGeom) * ntiles);
        FRS_HIP(hipMemcpyAsync(ctx->tiles.ptr, ctx->pin.at<TileGeom>(pin_tiles), sizeof(TileGeom) * ntiles,
                               hipMemcpyHostToDevice, st));
    }
    int *err_flag = reinterpret_cast<int *>(ctx->frame_bytes.as<int64_t>() + nframes + 1);
    FRS_HIP(hipMemsetAsync(err_flag, 0, sizeof(int), st));

    const T *raster = reinterpret_cast<const T *>(raster_dev);
    TileGeom *dtiles = ctx->tiles.as<TileGeom>();
    TileNorm *dnorms = ctx->norms.as<TileNorm>();
    SubAnalysis *dana = ctx->analysis.as<SubAnalysis>();

    hipEvent_t ev;
    bool one_wave_tiles = true;
    for (const TileGeom &tg : tiles) one_wave_tiles = one_wave_tiles && tg.nframes <= 64;
    bool stats_vec = false;
    if constexpr (sizeof(T) <= 2 && !Elem<DT>::is_float) {
        const int64_t es = (int64_t)sizeof(T);
        const uintptr_t b = reinterpret_cast<uintptr_t>(raster_dev) + (uintptr_t)(d->band0 * d->band_stride * es);
        stats_vec = (b % 16 == 0) && ((d->row_stride * es) % 16 == 0) && ((d->band_stride * es) % 16 == 0) &&
                    ((d->tile_w * es) % 16 == 0) && ((d->width * es) % 16 == 0);
    }
    // Tile stats on the fast path (16-bit samples, 16-B aligned rows, one wave per tile): fused into the analysis
    // launch (k_analyze_v3<DT, false, true>: min/max, parameters and LUT per wave).  Otherwise the stats kernels
    // run before the analysis.
    const bool fuse_stats = fast && stats_vec && sizeof(T) == 2 && one_wave_tiles;
    // 1. tile stats
    if (!fuse_stats) {
        prof_begin(ctx, "stats", &ev);
        k_stats_init<<<(ntiles + 255) / 256, 256, 0, st>>>(dnorms, ntiles);
        if (stats_vec) {
            const int64_t es = (int64_t)sizeof(T);
            const int64_t px = (int64_t)d->tile_h * d->tile_w * d->nbands;
            // ~256 KB per work-group, at least ~2048 work-groups overall
            int splits = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)d->tile_h * d->nbands, px * es / (256 << 10)));
            while ((int64_t)splits * ntiles < 2048 && splits < d->tile_h * d->nbands) splits++;
            dim3 grid(splits, ntiles);
            if constexpr (sizeof(T) <= 2 && !Elem<DT>::is_float)
                k_tile_stats_vec<DT><<<grid, 256, 0, st>>>(raster, P, dtiles, dnorms, splits);
        } else {
            int64_t rows = (int64_t)d->tile_h * d->nbands;
            int splits = (int)std::min<int64_t>(rows, std::max<int64_t>(1, (int64_t)4096 / ntiles));
            if (splits < 1) splits = 1;
            dim3 grid(splits, ntiles);
            k_tile_stats<DT><<<grid, 256, 0, st>>>(raster, P, dtiles, dnorms, splits);
        }
        k_tile_finalize<DT><<<(ntiles + 255) / 256, 256, 0, st>>>(dnorms, ntiles, P.norm_mode, P.scale_bits);
        prof_end(ctx, "stats", ev);
    }
    if constexpr (!Elem<DT>::is_float) if (fast || mc) {
        const int es = (int)sizeof(T);
        // alignment class of the 64-sample row segments (tiles whose width is a multiple of 64): the widest of 16,
        // 8, 4 bytes dividing the band base, the row stride and the tile width in bytes
        const uintptr_t b0 = reinterpret_cast<uintptr_t>(raster_dev) + (size_t)d->band0 * d->band_stride * es;
        P.vec_ok = 0;
        for (int a : {16, 8, 4})
            if (P.vec_ok == 0 && (d->row_stride * es) % a == 0 && b0 % a == 0 && ((int64_t)d->tile_w * es) % a == 0)
                P.vec_ok = a;
        FRS_HIP(ctx->luts.ensure(sizeof(int16_t) * (size_t)kLutCap * ntiles));
        FRS_HIP(ctx->status.ensure(sizeof(uint64_t) * (nframes + 1) + 64));
        if (!fuse_stats) k_build_lut<DT><<<ntiles, 256, 0, st>>>(dnorms, ctx->luts.as<int16_t>());
        FRS_HIP(ctx->frame_tile.ensure(sizeof(int32_t) * nframes));
        if (!(dev_tiles && ctx->geo_ptrs[3] == ctx->frame_tile.ptr))
            k_frame_tile<<<ntiles, 64, 0, st>>>(dtiles, ntiles, ctx->frame_tile.as<int32_t>());
        {
            // wave table: (tile, first frame) per wave, up to 64 frames of one tile each
            int nwaves = ctx->geo_nwaves;
            if (!(dev_tiles && ctx->geo_ptrs[1] == ctx->wave_tab.ptr)) {
                int2 *wt = ctx->pin.at<int2>(pin_wt);
                nwaves = 0;
                for (int ti = 0; ti < ntiles; ti++)
                    for (int c = 0; c < P.nvch; c++)  // (tile, first frame | coded signal << 24)
                        for (int k0 = 0; k0 < tiles[ti].nframes; k0 += 64) wt[nwaves++] = make_int2(ti, k0 | (c << 24));
                FRS_HIP(ctx->wave_tab.ensure(sizeof(int2) * nwaves));
                FRS_HIP(hipMemcpyAsync(ctx->wave_tab.ptr, wt, sizeof(int2) * nwaves, hipMemcpyHostToDevice, st));
            }
            prof_begin(ctx, "analyze", &ev);
            const unsigned wgrid = (unsigned)((nwaves + 3) / 4);
            const int2 *wtab = ctx->wave_tab.as<int2>();
            // small jobs with fused stats (C3): the prefetching form (FRS_ANA_PF=0/1 forces either).  Measured (round 6,
            // one box): C3 analysis 0.348 -> 0.322 ms; the Sentinel-2 example's separate-stats launch 0.529 -> 0.620 ms
            // and C4 1.30 -> 1.31-1.33 ms, so those keep the plain form
            const char *pf_env = getenv("FRS_ANA_PF");
            const bool pf = !st2 && (pf_env ? atoi(pf_env) == 1 : fuse_stats && nwaves <= kPfMaxWaves);
            if (pf) {
                if (fuse_stats) {
                    if constexpr (sizeof(T) == 2)
                        k_analyze_v3<DT, false, true, false, true><<<wgrid, 256, 0, st>>>(
                            raster, P, dtiles, dnorms, ctx->luts.as<int16_t>(), ctx->window.as<float>(), dana, wtab, nwaves);
                } else {
                    k_analyze_v3<DT, false, false, false, true><<<wgrid, 256, 0, st>>>(
                        raster, P, dtiles, dnorms, ctx->luts.as<int16_t>(), ctx->window.as<float>(), dana, wtab, nwaves);
                }
            } else if (fuse_stats) {
                if constexpr (sizeof(T) == 2)
                    k_analyze_v3<DT, false, true><<<wgrid, 256, 0, st>>>(raster, P, dtiles, dnorms, ctx->luts.as<int16_t>(),
                                                                         ctx->window.as<float>(), dana, wtab, nwaves);
            } else if (st2) {
                k_analyze_v3<DT, false, false, true><<<wgrid, 256, 0, st>>>(raster, P, dtiles, dnorms,
                                                                             ctx->luts.as<int16_t>(),
                                                                             ctx->window.as<float>(), dana, wtab, nwaves);
            } else {
                k_analyze_v3<DT, false><<<wgrid, 256, 0, st>>>(raster, P, dtiles, dnorms, ctx->luts.as<int16_t>(),
                                                                ctx->window.as<float>(), dana, wtab, nwaves);
            }
            if (st2)
                k_analyze_v3<DT, true, false, true><<<wgrid, 256, 0, st>>>(raster, P, dtiles, dnorms,
                                                                            ctx->luts.as<int16_t>(),
                                                                            ctx->window.as<float>(), dana, wtab, nwaves);
            else
                k_analyze_v3<DT, true><<<wgrid, 256, 0, st>>>(raster, P, dtiles, dnorms, ctx->luts.as<int16_t>(),
                                                               ctx->window.as<float>(), dana, wtab, nwaves);
            prof_end(ctx, "analyze", ev);
            if (!geo_hit) {  // the geometry's device copies are (being) uploaded on this stream: cache them
                ctx->geo_tiles = tiles;
                ctx->geo_plist.assign(hplist, hplist + npartial);
                ctx->geo_nframes = nframes;
                ctx->geo_ptrs[2] = nullptr;  // the partial list goes up below
            }
            ctx->geo_nwaves = nwaves;
            ctx->geo_key = key;
            ctx->geo_ptrs[0] = ctx->tiles.ptr;
            ctx->geo_ptrs[1] = ctx->wave_tab.ptr;
            ctx->geo_ptrs[3] = ctx->frame_tile.ptr;
        }
        // partial last frames: generic analysis + frame coding into compact slots, CRC-16 sealed in place
        int64_t *dpbytes = ctx->frame_bytes.as<int64_t>();  // [npartial] (< nframes + 1: below err_flag)
        if (npartial > 0) {
            prof_begin(ctx, "partial", &ev);
            FRS_HIP(ctx->plist.ensure(sizeof(int64_t) * (size_t)npartial));
            if (!(dev_tiles && ctx->geo_ptrs[2] == ctx->plist.ptr))
                FRS_HIP(hipMemcpyAsync(ctx->plist.ptr, hplist, sizeof(int64_t) * (size_t)npartial,
                                       hipMemcpyHostToDevice, st));
            ctx->geo_ptrs[2] = ctx->plist.ptr;
            FRS_HIP(ctx->slots.ensure((size_t)npartial * P.slot_words * 4));
            const int64_t *dpl = ctx->plist.as<int64_t>();
            if (st2) {
                k_analyze_partial<DT, true><<<dim3((unsigned)npartial, 4u), kPartThreads, 0, st>>>(
                    raster, P, dtiles, dnorms, ctx->window.as<float>(), dana, dpl);
                k_encode_frames<DT, true><<<(unsigned)npartial, kEncThreads, 0, st>>>(
                    raster, P, dtiles, dnorms, dana, ctx->slots.as<uint32_t>(), dpbytes, err_flag, dpl, nullptr,
                    nullptr, 0);
            } else {
                k_analyze_partial<DT><<<dim3((unsigned)npartial, (unsigned)P.nch), kPartThreads, 0, st>>>(
                    raster, P, dtiles, dnorms, ctx->window.as<float>(), dana, dpl);
                k_encode_frames<DT><<<(unsigned)npartial, kEncThreads, 0, st>>>(raster, P, dtiles, dnorms, dana,
                                                                               ctx->slots.as<uint32_t>(), dpbytes,
                                                                               err_flag, dpl);
            }
            k_seal_partial<<<(unsigned)npartial, 256, 0, st>>>(ctx->slots.as<uint32_t>(), P.slot_words, dpbytes,
                                                               npartial);
            prof_end(ctx, "partial", ev);
        }
        uint64_t *dstatus = ctx->status.as<uint64_t>();
        int *ticket = reinterpret_cast<int *>(dstatus + nframes);
        if (mc) {
            const int64_t nsub = nframes * P.nvch;
            FRS_HIP(ctx->sub_slots.ensure(sizeof(uint32_t) * (size_t)nsub * kSubWords));
            FRS_HIP(ctx->sub_bits.ensure(sizeof(int32_t) * (size_t)nsub));
            FRS_HIP(ctx->mc_bytes.ensure(sizeof(int64_t) * (size_t)(nframes + 1)));
            FRS_HIP(hipMemsetAsync(ticket, 0, 2 * sizeof(int), st));
            uint32_t *dsub = ctx->sub_slots.as<uint32_t>();
            int32_t *dsbits = ctx->sub_bits.as<int32_t>();
            int64_t *dmcb = ctx->mc_bytes.as<int64_t>();
            int32_t *dsest = nullptr;
            int8_t *dpick = nullptr;
            if (st2) {
                FRS_HIP(ctx->sub_est.ensure(sizeof(int32_t) * (size_t)nsub));
                FRS_HIP(ctx->st_pick.ensure((size_t)nframes + 64));
                dsest = ctx->sub_est.as<int32_t>();
                dpick = ctx->st_pick.as<int8_t>();
            }
            prof_begin(ctx, "encode", &ev);
            // (one occupancy query per kernel instantiation; the same gfx950 target for every device)
            auto launch = [&](auto kern, int &nwg_max, int64_t units, int *tk) {
                if (nwg_max == 0) FRS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nwg_max, kern, 256, 0));
                int64_t grid = (int64_t)std::max(1, nwg_max) * ctx->num_cus;
                grid = std::min<int64_t>(grid, (units + 3) / 4);
                kern<<<(unsigned)grid, 256, 0, st>>>(
                    raster, P, dtiles, dnorms, ctx->luts.as<int16_t>(), dana, reinterpret_cast<uint8_t *>(arena_dev),
                    arena_cap, ctx->frame_off.as<int64_t>(), dstatus, tk, err_flag, ctx->frame_tile.as<int32_t>(),
                    ctx->hdr_tab.as<uint4>(), 0, ctx->slots.as<uint32_t>(), dpbytes, dsub, dsbits, dsest);
                return FRS_OK;
            };
            if (st2) {  // left, right, mid (16-bit) in one launch; the 17-bit side signals in another
                static int nwg_lrm = 0, nwg_side = 0;
                if (int rc2 = launch(k_encode_v4<DT, true, true, false>, nwg_lrm, nframes * 3, ticket)) return rc2;
                if (int rc2 = launch(k_encode_v4<DT, true, true, true>, nwg_side, nframes, ticket + 1)) return rc2;
            } else {
                static int nwg_mc = 0;
                if (int rc2 = launch(k_encode_v4<DT, true>, nwg_mc, nsub, ticket)) return rc2;
            }
            k_mc_frame_bytes<<<(unsigned)((nframes + 255) / 256), 256, 0, st>>>(P, dtiles, ctx->frame_tile.as<int32_t>(),
                                                                               dsbits, dpbytes, dmcb, err_flag, dsest,
                                                                               dpick);
            prof_end(ctx, "encode", ev);
            k_scan_sizes<<<1, kScanThreads, 0, st>>>(dmcb, ctx->frame_off.as<int64_t>(), nframes);
            int64_t total = 0;
            int errv = 0;
            FRS_HIP(hipMemcpyAsync(&total, ctx->frame_off.as<int64_t>() + nframes, sizeof(int64_t),
                                   hipMemcpyDeviceToHost, st));
            FRS_HIP(hipMemcpyAsync(&errv, err_flag, sizeof(int), hipMemcpyDeviceToHost, st));
            FRS_HIP(hipStreamSynchronize(st));
            if (errv) {
                ctx->err = "fast encode declined, flags " + std::to_string(errv);
                return kFastDeclined;
            }
            if (total > arena_cap) {
                tile_off[ntiles] = total;
                ctx->err = "arena too small";
                return FRS_E_NOSPACE;
            }
            const size_t mc_lds = sizeof(uint32_t) * (size_t)(P.nch * kFrameWordsV3 + 16);  // <= 70 KB (8 channels)
            FRS_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mc_assemble),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)mc_lds));
            prof_begin(ctx, "assemble", &ev);
            k_mc_assemble<<<(unsigned)nframes, 256, mc_lds, st>>>(
                P, dtiles, ctx->frame_tile.as<int32_t>(), dsub, dsbits, ctx->slots.as<uint32_t>(), dpbytes,
                ctx->frame_off.as<int64_t>(), reinterpret_cast<uint8_t *>(arena_dev), dpick);
            prof_end(ctx, "assemble", ev);
            k_gather_tile_off<<<(ntiles + 1 + 255) / 256, 256, 0, st>>>(ctx->frame_off.as<int64_t>(), dtiles, ntiles,
                                                                       total, ctx->tile_sizes.as<int64_t>());
            std::vector<TileNorm> hn(ntiles);
            FRS_HIP(hipMemcpyAsync(tile_off, ctx->tile_sizes.ptr, sizeof(int64_t) * (ntiles + 1), hipMemcpyDeviceToHost,
                                   st));
            FRS_HIP(hipMemcpyAsync(hn.data(), dnorms, sizeof(TileNorm) * ntiles, hipMemcpyDeviceToHost, st));
            FRS_HIP(hipStreamSynchronize(st));
            prof_collect(ctx);
            for (int t = 0; t < ntiles; t++) {
                tile_min[t] = hn[t].dmin;
                tile_max[t] = hn[t].dmax;
            }
            return FRS_OK;
        }
        FRS_HIP(hipMemsetAsync(dstatus, 0, sizeof(uint64_t) * (nframes + 1) + 64, st));  // + the ticket counters
        // frame-header table by frame number within a stream (fast path: mono, 16-bit, blocksize 4096)
        int hdr_n = 0;
        {
            int32_t maxf = 0;
            for (const TileGeom &tg : tiles) maxf = std::max(maxf, tg.nframes);
            hdr_n = std::min<int32_t>(maxf, 1 << 16);
            if (ctx->hdr_tab_n != hdr_n || ctx->hdr_tab_sr != d->sample_rate) {
                int src, srx = 0;
                const int sr = d->sample_rate;
                switch (sr) {
                case 88200: src = 1; break;
                case 176400: src = 2; break;
                case 192000: src = 3; break;
                case 8000: src = 4; break;
                case 16000: src = 5; break;
                case 22050: src = 6; break;
                case 24000: src = 7; break;
                case 32000: src = 8; break;
                case 44100: src = 9; break;
                case 48000: src = 10; break;
                case 96000: src = 11; break;
                default:
                    if (sr <= 255000 && sr % 1000 == 0) src = srx = 12;
                    else if (sr % 10 == 0 && sr / 10 <= 65535) src = srx = 14;
                    else src = srx = 13;
                }
                uint8_t c8t[256];
                for (int i = 0; i < 256; i++) {
                    uint8_t c = (uint8_t)i;
                    for (int k = 0; k < 8; k++) c = (c & 0x80) ? (uint8_t)((c << 1) ^ 0x07) : (uint8_t)(c << 1);
                    c8t[i] = c;
                }
                std::vector<uint32_t> tab((size_t)hdr_n * 4, 0);
                for (int fk = 0; fk < hdr_n; fk++) {
                    uint8_t h[16] = {0};
                    int hb = 0;
                    h[hb++] = 0xFF;
                    h[hb++] = 0xF8;
                    h[hb++] = (uint8_t)((12 << 4) | src);
                    h[hb++] = (uint8_t)(4 << 1);
                    const uint32_t v = (uint32_t)fk;
                    if (v < 0x80) h[hb++] = (uint8_t)v;
                    else if (v < 0x800) { h[hb++] = (uint8_t)(0xC0 | (v >> 6)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
                    else { h[hb++] = (uint8_t)(0xE0 | (v >> 12)); h[hb++] = (uint8_t)(0x80 | ((v >> 6) & 0x3F)); h[hb++] = (uint8_t)(0x80 | (v & 0x3F)); }
                    if (srx == 12) h[hb++] = (uint8_t)(sr / 1000);
                    else if (srx == 13) { h[hb++] = (uint8_t)(sr >> 8); h[hb++] = (uint8_t)sr; }
                    else if (srx == 14) { h[hb++] = (uint8_t)((sr / 10) >> 8); h[hb++] = (uint8_t)(sr / 10); }
                    uint8_t c = 0;
                    for (int i = 0; i < hb; i++) c = c8t[c ^ h[i]];
                    h[hb++] = c;
                    for (int w = 0; w < 4; w++)
                        tab[(size_t)fk * 4 + w] = ((uint32_t)h[4 * w] << 24) | ((uint32_t)h[4 * w + 1] << 16) |
                                                  ((uint32_t)h[4 * w + 2] << 8) | h[4 * w + 3];
                    tab[(size_t)fk * 4 + 3] = (tab[(size_t)fk * 4 + 3] & 0xFFFFFF00u) | (uint32_t)hb;
                }
                FRS_HIP(ctx->hdr_tab.ensure(sizeof(uint32_t) * tab.size() + 16));
                FRS_HIP(hipMemcpyAsync(ctx->hdr_tab.ptr, tab.data(), sizeof(uint32_t) * tab.size(),
                                       hipMemcpyHostToDevice, st));
                FRS_HIP(hipStreamSynchronize(st));
                ctx->hdr_tab_n = hdr_n;
                ctx->hdr_tab_sr = d->sample_rate;
            }
        }
        {
            static int nwg_max = 0;  // (per instantiation; the same gfx950 target for every device)
            if (nwg_max == 0) FRS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nwg_max, k_encode_v4<DT>, 256, 0));
            prof_begin(ctx, "encode", &ev);
            int64_t grid = (int64_t)std::max(1, nwg_max) * ctx->num_cus;
            grid = std::min<int64_t>(grid, (nframes + 3) / 4);
            k_encode_v4<DT><<<(unsigned)grid, 256, 0, st>>>(raster, P, dtiles, dnorms, ctx->luts.as<int16_t>(), dana,
                                                            reinterpret_cast<uint8_t *>(arena_dev), arena_cap,
                                                            ctx->frame_off.as<int64_t>(), dstatus, ticket, err_flag,
                                                            ctx->frame_tile.as<int32_t>(), ctx->hdr_tab.as<uint4>(),
                                                            hdr_n, ctx->slots.as<uint32_t>(), dpbytes);
            prof_end(ctx, "encode", ev);
        }
        FRS_HIP(ctx->host_pack.ensure(res_bytes));
        int64_t *dpack = ctx->host_pack.as<int64_t>();
        k_fast_finish<<<(ntiles + 1 + 255) / 256, 256, 0, st>>>(ctx->frame_off.as<int64_t>(), dstatus, dtiles, dnorms,
                                                               err_flag, ntiles, nframes, dpack);
        const int64_t *hpack = ctx->pin.at<int64_t>(pin_res);
        FRS_HIP(hipMemcpyAsync(ctx->pin.at<int64_t>(pin_res), dpack, res_bytes, hipMemcpyDeviceToHost, st));
        FRS_HIP(hipStreamSynchronize(st));
        prof_collect(ctx);
        memcpy(tile_off, hpack, sizeof(int64_t) * (ntiles + 1));
        const double *mm = reinterpret_cast<const double *>(hpack + ntiles + 1);
        for (int t = 0; t < ntiles; t++) {
            tile_min[t] = mm[2 * t];
            tile_max[t] = mm[2 * t + 1];
        }
        const int errv = (int)hpack[3 * (int64_t)ntiles + 1];
        if (errv & 16) {
            ctx->err = "arena too small";
            return FRS_E_NOSPACE;
        }
        if (errv) {  // a frame the fast kernels cannot hold (never seen: estimates stay below verbatim)
            ctx->err = "fast encode declined, flags " + std::to_string(errv);
            return kFastDeclined;
        }
        return FRS_OK;
    }
    FRS_HIP(ctx->slots.ensure((size_t)nframes * P.slot_words * 4));
    // 2. analysis (lane = coded signal: channel, or L/R/M/S of a two-channel stream).  subdivide_tukey levels: the
    //    fixed-predictor / wasted-bits analysis first (max_lpc 0), then the LPC candidates of every window
    const int64_t nsub = nframes * P.nvch;
    const bool stereo = P.nvch == 4 && P.nch == 2;
    const unsigned agrid = (unsigned)((nsub + 127) / 128);
    EncodeParams Pa = P;
    LpcCand *dcand = nullptr;
    if (P.ncand > 0) {
        Pa.max_lpc = 0;
        FRS_HIP(ctx->lpc_cand.ensure(sizeof(LpcCand) * (size_t)nsub * (size_t)P.ncand));
        dcand = ctx->lpc_cand.as<LpcCand>();
        if (ctx->window_hi_bs != d->blocksize || ctx->window_hi_parts != lv.parts) {
            // subdivide_tukey(parts): FLAC__stream_encoder_set_apodization stores p / parts, the window is
            // FLAC__window_tukey(p / parts) (float p = 0.5f)
            std::vector<float> win(d->blocksize, 1.0f);
            const float pw = 0.5f / (float)lv.parts;
            const int L = d->blocksize;
            const int Np = (int)(pw / 2.0f * (float)L) - 1;
            if (Np > 0)
                for (int k = 0; k <= Np; k++) {
                    win[k] = (float)(0.5f - 0.5f * cos(M_PI * k / Np));
                    win[L - Np - 1 + k] = (float)(0.5f - 0.5f * cos(M_PI * (k + Np) / Np));
                }
            FRS_HIP(ctx->window_hi.ensure(sizeof(float) * L));
            FRS_HIP(hipMemcpyAsync(ctx->window_hi.ptr, win.data(), sizeof(float) * L, hipMemcpyHostToDevice, st));
            FRS_HIP(hipStreamSynchronize(st));
            ctx->window_hi_bs = d->blocksize;
            ctx->window_hi_parts = lv.parts;
        }
    }
    prof_begin(ctx, "analyze", &ev);
    uint8_t *zero = nullptr;  // raw-frames tiles: all-zero subframe flags (k_zero_subframes)
    if (P.bps > 16) {
        if (stereo) {
            k_analyze<DT, true, true><<<agrid, 128, 0, st>>>(raster, Pa, dtiles, dnorms, ctx->window.as<float>(), dana,
                                                                nullptr, 0);
            k_analyze_fixed_wide<DT, true><<<agrid, 128, 0, st>>>(raster, Pa, dtiles, dnorms, dana);
            if (dcand)
                k_analyze_lpc_hi<DT, true, true><<<agrid, 128, 0, st>>>(raster, P, dtiles, dnorms,
                                                                        ctx->window_hi.as<float>(), dana, dcand, lv.parts);
        } else {
            // raw-frames tiles: all-zero subframes analysed by a coalesced pass, skipped by the lane walks
            if (!dcand) {
                FRS_HIP(ctx->zero_sub.ensure((size_t)nsub + 64));
                zero = ctx->zero_sub.as<uint8_t>();
                EncodeParams Pz = Pa;  // 64-sample row segments: the widest load every band's rows allow
                const int es = (int)sizeof(T);
                const uintptr_t b0 = reinterpret_cast<uintptr_t>(raster_dev) + (size_t)d->band0 * d->band_stride * es;
                Pz.vec_ok = 0;
                for (int a : {16, 8, 4})
                    if (Pz.vec_ok == 0 && (d->row_stride * es) % a == 0 && (d->band_stride * es) % a == 0 &&
                        b0 % a == 0 && ((int64_t)d->tile_w * es) % a == 0)
                        Pz.vec_ok = a;
                k_zero_subframes<DT><<<(unsigned)((nsub + 3) / 4), 256, 0, st>>>(raster, Pz, dtiles, dnorms, dana, zero);
            }
            k_analyze<DT, true><<<agrid, 128, 0, st>>>(raster, Pa, dtiles, dnorms, ctx->window.as<float>(), dana,
                                                         nullptr, 0, zero);
            k_analyze_fixed_wide<DT><<<agrid, 128, 0, st>>>(raster, Pa, dtiles, dnorms, dana, zero);
            if (dcand)
                k_analyze_lpc_hi<DT, true><<<agrid, 128, 0, st>>>(raster, P, dtiles, dnorms, ctx->window_hi.as<float>(),
                                                                  dana, dcand, lv.parts);
        }
    } else {
        if (stereo) {
            k_analyze<DT, false, true><<<agrid, 128, 0, st>>>(raster, Pa, dtiles, dnorms, ctx->window.as<float>(), dana,
                                                                 nullptr, 0);
            if (dcand)
                k_analyze_lpc_hi<DT, false, true><<<agrid, 128, 0, st>>>(raster, P, dtiles, dnorms,
                                                                         ctx->window_hi.as<float>(), dana, dcand,
                                                                         lv.parts);
        } else {
            k_analyze<DT, false><<<agrid, 128, 0, st>>>(raster, Pa, dtiles, dnorms, ctx->window.as<float>(), dana,
                                                          nullptr, 0);
            if (dcand)
                k_analyze_lpc_hi<DT, false><<<agrid, 128, 0, st>>>(raster, P, dtiles, dnorms, ctx->window_hi.as<float>(),
                                                                   dana, dcand, lv.parts);
        }
    }
    prof_end(ctx, "analyze", ev);
    // 3. encode frames into slots (loose mid/side: the group leaders' assignments first)
    prof_begin(ctx, "encode", &ev);
    uint32_t *dslots = ctx->slots.as<uint32_t>();
    int64_t *dfb = ctx->frame_bytes.as<int64_t>();
    int8_t *dloose = nullptr;
    if (stereo && P.loose_frames > 0) {
        std::vector<int64_t> leaders;
        for (const TileGeom &tg : tiles)
            for (int k = 0; k < tg.nframes; k += P.loose_frames) leaders.push_back(tg.frame_base + k);
        FRS_HIP(ctx->loose_assign.ensure(sizeof(int8_t) * (size_t)nframes + 64));
        FRS_HIP(ctx->loose_lead.ensure(sizeof(int64_t) * leaders.size()));
        FRS_HIP(hipMemcpyAsync(ctx->loose_lead.ptr, leaders.data(), sizeof(int64_t) * leaders.size(),
                               hipMemcpyHostToDevice, st));
        dloose = ctx->loose_assign.as<int8_t>();
        const int64_t *dlead = ctx->loose_lead.as<int64_t>();
        if (P.bps > 16)
            k_encode_frames<DT, true, int64_t><<<(unsigned)leaders.size(), kEncThreads, 0, st>>>(
                raster, P, dtiles, dnorms, dana, dslots, dfb, err_flag, dlead, dcand, dloose, 1);
        else
            k_encode_frames<DT, true><<<(unsigned)leaders.size(), kEncThreads, 0, st>>>(
                raster, P, dtiles, dnorms, dana, dslots, dfb, err_flag, dlead, dcand, dloose, 1);
        FRS_HIP(hipStreamSynchronize(st));  // (the leader list's host vector goes out of scope)
    }
    if (stereo && P.bps > 16)
        k_encode_frames<DT, true, int64_t><<<(unsigned)nframes, kEncThreads, 0, st>>>(raster, P, dtiles, dnorms, dana,
                                                                                     dslots, dfb, err_flag, nullptr,
                                                                                     dcand, dloose, 0);
    else if (stereo)
        k_encode_frames<DT, true><<<(unsigned)nframes, kEncThreads, 0, st>>>(raster, P, dtiles, dnorms, dana, dslots,
                                                                             dfb, err_flag, nullptr, dcand, dloose, 0);
    else
        k_encode_frames<DT><<<(unsigned)nframes, kEncThreads, 0, st>>>(raster, P, dtiles, dnorms, dana, dslots, dfb,
                                                                       err_flag, nullptr, dcand, nullptr, 0);
    if (zero)  // the all-zero frames k_encode_frames left
        k_zero_frames_emit<<<(unsigned)((nframes + 3) / 4), 256, 0, st>>>(P, dtiles, dana, dslots, dfb);
    prof_end(ctx, "encode", ev);
    // 4. offsets (frame_off[nframes] = total)
    k_scan_sizes<<<1, kScanThreads, 0, st>>>(ctx->frame_bytes.as<int64_t>(), ctx->frame_off.as<int64_t>(), nframes);
    int64_t total = 0;
    int errv = 0;
    FRS_HIP(hipMemcpyAsync(&total, ctx->frame_off.as<int64_t>() + nframes, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    FRS_HIP(hipMemcpyAsync(&errv, err_flag, sizeof(int), hipMemcpyDeviceToHost, st));
    FRS_HIP(hipStreamSynchronize(st));
    if (errv) {
        ctx->err = "frame exceeded its slot (pathological residuals), flag " + std::to_string(errv);
        return FRS_E_UNSUPPORTED;
    }
    if (total > arena_cap) {
        tile_off[ntiles] = total;
        ctx->err = "arena too small";
        return FRS_E_NOSPACE;
    }
    // 5. compact + CRC
    prof_begin(ctx, "compact", &ev);
    k_compact<<<(unsigned)nframes, 256, 0, st>>>(ctx->slots.as<uint32_t>(), P.slot_words, ctx->frame_bytes.as<int64_t>(),
                                                 ctx->frame_off.as<int64_t>(), nframes,
                                                 reinterpret_cast<uint8_t *>(arena_dev));
    prof_end(ctx, "compact", ev);
    k_gather_tile_off<<<(ntiles + 1 + 255) / 256, 256, 0, st>>>(ctx->frame_off.as<int64_t>(), dtiles, ntiles, total,
                                                               ctx->tile_sizes.as<int64_t>());
    std::vector<TileNorm> hn(ntiles);
    FRS_HIP(hipMemcpyAsync(tile_off, ctx->tile_sizes.ptr, sizeof(int64_t) * (ntiles + 1), hipMemcpyDeviceToHost, st));
    FRS_HIP(hipMemcpyAsync(hn.data(), dnorms, sizeof(TileNorm) * ntiles, hipMemcpyDeviceToHost, st));
    FRS_HIP(hipStreamSynchronize(st));
    prof_collect(ctx);
    for (int t = 0; t < ntiles; t++) {
        tile_min[t] = hn[t].dmin;
        tile_max[t] = hn[t].dmax;
    }
    return FRS_OK;
}

template <int DT>
static int run_encode_any(frs_ctx *ctx, const frs_encode_desc *d, const void *raster_dev, void *arena_dev,
                          int64_t arena_cap, int64_t *tile_off, double *tile_min, double *tile_max) {
    int rc = run_encode<DT>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max, true);
    if (rc == kFastDeclined) rc = run_encode<DT>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max, false);
    return rc;
}

int encode_job(frs_ctx *ctx, const frs_encode_desc *d, const void *raster_dev, void *arena_dev, int64_t arena_cap,
               int64_t *tile_off, double *tile_min, double *tile_max, int32_t *stream_bps) {
    if (stream_bps) *stream_bps = stream_bps_of(d);
    if (const int rc = check_unsynced(ctx)) return rc;
#ifdef FRS_PROBE_I16  // (register probes: tools/kernel_regs.py --probe compiles the int16 kernels only)
    return run_encode_any<FRS_DT_I16>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max);
#else
    switch (d->dtype) {
    case FRS_DT_U8: return run_encode_any<FRS_DT_U8>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max);
    case FRS_DT_U16: return run_encode_any<FRS_DT_U16>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max);
    case FRS_DT_I16: return run_encode_any<FRS_DT_I16>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max);
    case FRS_DT_I32: return run_encode_any<FRS_DT_I32>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max);
    case FRS_DT_U32: return run_encode_any<FRS_DT_U32>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max);
    case FRS_DT_F32: return run_encode_any<FRS_DT_F32>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max);
    case FRS_DT_F64: return run_encode_any<FRS_DT_F64>(ctx, d, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max);
    default: ctx->err = "bad dtype"; return FRS_E_ARG;
    }
#endif
}

}  // namespace frs
