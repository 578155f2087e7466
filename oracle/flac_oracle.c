/*
 * oracle/flac_oracle.c -- TEST INFRASTRUCTURE ONLY (parity oracle + timed CPU baseline).
 *
 * CPU restatement of the reference's hot path for checking the HIP product:
 *   - numpy normalisation     reference src/flac_raster/converter.py:56-86  (_normalize_to_audio)
 *   - numpy de-normalisation  reference src/flac_raster/converter.py:88-110 (_denormalize_from_audio)
 *   - FLAC level-5 encode     third-party libFLAC 1.4.3 (pyFLAC 3.0.0, pixi.lock:3445-3448;
 *                             version evidence docs/sonos-pyflac.txt:150), called from
 *                             reference converter.py:201-216 via pyflac encoder.py
 *                             (docs/sonos-pyflac.txt:1968-2001)
 *   - FLAC decode             libFLAC 1.4.3 decoder via pyflac (docs/sonos-pyflac.txt:1584-1640, 1809-1854)
 *
 * libFLAC itself is NOT in /root/reference (and not on disk), so this is a restatement of its
 * published algorithm (RFC 9639 bitstream + the libFLAC 1.4.3 encoder's decision procedure:
 * stream_encoder.c process_subframe_ / evaluate_*_subframe_ / find_best_partition_order_ /
 * set_partitioned_rice_, fixed.c, lpc.c, window.c).  It is PINNED by the reference's own
 * fixtures: test_data/sample_rgb.flac (48 16-bit level-5 subframes, byte-exact) and
 * test_data/sample_dem.flac (32-bit frames, byte-exact modulo the text tags) -- see
 * tests/test_oracle_golden.py.
 *
 * This file is never linked into, called by, or shipped as the product; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MAX_LPC 12  /* level 7/8 max_lpc_order (level 5: 8) */
#define ORC_MAX_FIXED 4
#define ORC_MAX_CH 8

/* ------------------------------------------------------------------ bit writer (MSB first) */
typedef struct {
    uint8_t *buf;
    int64_t cap;  /* bytes */
    int64_t bits; /* bits written */
    int overflow;
} bw_t;

static void bw_put(bw_t *w, uint64_t v, int n) {
    /* n <= 57 */
    for (int i = n - 1; i >= 0; i--) {
        int64_t byte = w->bits >> 3;
        if (byte >= w->cap) { w->overflow = 1; w->bits++; continue; }
        int bit = 7 - (int)(w->bits & 7);
        if (bit == 7) w->buf[byte] = 0;
        if ((v >> i) & 1) w->buf[byte] |= (uint8_t)(1u << bit);
        w->bits++;
    }
}
static void bw_put_zeros(bw_t *w, uint64_t n) {
    while (n >= 32) { bw_put(w, 0, 32); n -= 32; }
    if (n) bw_put(w, 0, (int)n);
}
static void bw_put_signed(bw_t *w, int64_t v, int n) {
    uint64_t m = (n >= 64) ? ~0ull : ((1ull << n) - 1);
    bw_put(w, (uint64_t)v & m, n);
}
static void bw_align(bw_t *w) {
    while (w->bits & 7) bw_put(w, 0, 1);
}

/* CRC-8 poly 0x07 and CRC-16 poly 0x8005, MSB first, init 0 (RFC 9639 9.1.8 / 9.3) */
static uint8_t crc8_tab[256];
static uint16_t crc16_tab[256];
static int crc_init_done = 0;
static void crc_init(void) {
    if (crc_init_done) return;
    for (int i = 0; i < 256; i++) {
        uint8_t c = (uint8_t)i;
        for (int k = 0; k < 8; k++) c = (c & 0x80) ? (uint8_t)((c << 1) ^ 0x07) : (uint8_t)(c << 1);
        crc8_tab[i] = c;
        uint16_t d = (uint16_t)(i << 8);
        for (int k = 0; k < 8; k++) d = (d & 0x8000) ? (uint16_t)((d << 1) ^ 0x8005) : (uint16_t)(d << 1);
        crc16_tab[i] = d;
    }
    crc_init_done = 1;
}
static uint8_t crc8(const uint8_t *p, int64_t n) {
    uint8_t c = 0;
    for (int64_t i = 0; i < n; i++) c = crc8_tab[c ^ p[i]];
    return c;
}
static uint16_t crc16(const uint8_t *p, int64_t n) {
    uint16_t c = 0;
    for (int64_t i = 0; i < n; i++) c = (uint16_t)((c << 8) ^ crc16_tab[(c >> 8) ^ p[i]]);
    return c;
}

static uint32_t ilog2_u64(uint64_t v) { /* floor(log2(v)), v > 0 */
    uint32_t l = 0;
    while (v >>= 1) l++;
    return l;
}

/* ------------------------------------------------------------------ window (libFLAC window.c tukey) */
/* tukey(p): Np = (int)(p/2*L) - 1; ends are Hann, computed in double, stored as float. */
void orc_window_tukey(float *w, int L, float p) {
    for (int i = 0; i < L; i++) w[i] = 1.0f;
    int Np = (int)(p / 2.0f * (float)L) - 1;
    if (Np > 0) {
        for (int n = 0; n <= Np; n++) {
            w[n] = (float)(0.5f - 0.5f * cos(M_PI * n / Np));
            w[L - Np - 1 + n] = (float)(0.5f - 0.5f * cos(M_PI * (n + Np) / Np));
        }
    }
}

/* ------------------------------------------------------------------ fixed predictor analysis */
/* libFLAC fixed.c FLAC__fixed_compute_best_predictor(_wide): data points at sample 4 of the block
 * (warm-up read through data[-1..-4]).  Totals in 64 bits (identical to the 32-bit variant when it
 * does not overflow, which libFLAC guarantees by choosing the variant by bps). */
static int fixed_best(const int64_t *data, int n, float bits[5]) {
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    for (int i = 0; i < n; i++) {
        int64_t x0 = data[i], x1 = data[i - 1], x2 = data[i - 2], x3 = data[i - 3], x4 = data[i - 4];
        int64_t e0 = x0, e1 = x0 - x1, e2 = x0 - 2 * x1 + x2, e3 = x0 - 3 * x1 + 3 * x2 - x3,
                e4 = x0 - 4 * x1 + 6 * x2 - 4 * x3 + x4;
        t0 += (uint64_t)(e0 < 0 ? -e0 : e0);
        t1 += (uint64_t)(e1 < 0 ? -e1 : e1);
        t2 += (uint64_t)(e2 < 0 ? -e2 : e2);
        t3 += (uint64_t)(e3 < 0 ? -e3 : e3);
        t4 += (uint64_t)(e4 < 0 ? -e4 : e4);
    }
    int order;
    uint64_t m;
    m = t1 < t2 ? t1 : t2; m = m < t3 ? m : t3; m = m < t4 ? m : t4;
    if (t0 <= m) order = 0;
    else {
        m = t2 < t3 ? t2 : t3; m = m < t4 ? m : t4;
        if (t1 <= m) order = 1;
        else if (t2 <= (t3 < t4 ? t3 : t4)) order = 2;
        else if (t3 <= t4) order = 3;
        else order = 4;
    }
    uint64_t t[5] = {t0, t1, t2, t3, t4};
    for (int k = 0; k < 5; k++)
        bits[k] = (float)((t[k] > 0) ? log(M_LN2 * (double)t[k] / (double)n) / M_LN2 : 0.0);
    return order;
}

/* libFLAC 1.4.3 FLAC__fixed_compute_best_predictor_limit_residual (used when subframe_bps >= 28,
 * i.e. our 32-bit streams; the _33bit twin for the side channel of a 32-bit stereo stream runs the same
 * arithmetic on int64 samples).  Includes its CHECK_ORDER_IS_VALID estimate quirk: the estimate for a
 * "best so far" order is computed from total_error_0, the others are set to 34.0f.  This quirk is
 * why an all-zero 32-bit block is coded FIXED order 0 instead of CONSTANT (pinned by
 * test_data/sample_dem.flac). */
static int fixed_best_limit_residual(const int64_t *data, int n, float bits[5]) {
    uint64_t t[5] = {0, 0, 0, 0, 0}, smallest = UINT64_MAX;
    int valid[5] = {1, 1, 1, 1, 1};
    int order = 0;
    for (int i = -4; i < n; i++) {
        int64_t x0 = data[i];
        uint64_t e[5];
        e[0] = (uint64_t)llabs(x0);
        e[1] = (i > -4) ? (uint64_t)llabs(x0 - data[i - 1]) : 0;
        e[2] = (i > -3) ? (uint64_t)llabs(x0 - 2 * data[i - 1] + data[i - 2]) : 0;
        e[3] = (i > -2) ? (uint64_t)llabs(x0 - 3 * data[i - 1] + 3 * data[i - 2] - data[i - 3]) : 0;
        e[4] = (i > -1) ? (uint64_t)llabs(x0 - 4 * data[i - 1] + 6 * data[i - 2] - 4 * data[i - 3] + data[i - 4]) : 0;
        for (int k = 0; k < 5; k++) {
            t[k] += e[k];
            if (e[k] > INT32_MAX) valid[k] = 0;
        }
    }
    for (int k = 0; k < 5; k++) {
        if (valid[k] && t[k] < smallest) {
            order = k;
            smallest = t[k];
            bits[k] = (float)((t[0] > 0) ? log(M_LN2 * (double)t[0] / (double)n) / M_LN2 : 0.0);
        } else {
            bits[k] = 34.0f;
        }
    }
    return order;
}

static const int fixed_coefs[5][4] = {{0, 0, 0, 0}, {1, 0, 0, 0}, {2, -1, 0, 0}, {3, -3, 1, 0}, {4, -6, 4, -1}};

/* ------------------------------------------------------------------ LPC (libFLAC lpc.c) */
static void autocorrelation(const float *d, int n, int lags, double *autoc) {
    /* sum in increasing sample order per lag (the product is exact in double) */
    for (int l = 0; l < lags; l++) {
        double acc = 0.0;
        for (int i = l; i < n; i++) acc += (double)d[i] * (double)d[i - l];
        autoc[l] = acc;
    }
}

/* FLAC__lpc_compute_lp_coefficients; returns possibly reduced max_order */
static int lp_coefficients(const double *autoc, int max_order, float lp[ORC_MAX_LPC][ORC_MAX_LPC], double *error) {
    double lpc[ORC_MAX_LPC];
    double err = autoc[0];
    for (int i = 0; i < max_order; i++) {
        double r = -autoc[i + 1];
        for (int j = 0; j < i; j++) r -= lpc[j] * autoc[i - j];
        r /= err;
        lpc[i] = r;
        int j;
        for (j = 0; j < (i >> 1); j++) {
            double tmp = lpc[j];
            lpc[j] += r * lpc[i - 1 - j];
            lpc[i - 1 - j] += r * tmp;
        }
        if (i & 1) lpc[j] += lpc[j] * r;
        err *= (1.0 - r * r);
        for (j = 0; j <= i; j++) lp[i][j] = (float)(-lpc[j]);
        error[i] = err;
        if (err == 0.0) return i + 1;
    }
    return max_order;
}

static double expected_bits_scaled(double lpc_error, double error_scale) {
    if (lpc_error > 0.0) {
        double bps = (double)0.5 * log(error_scale * lpc_error) / M_LN2;
        return bps >= 0.0 ? bps : 0.0;
    } else if (lpc_error < 0.0) {
        return 1e32;
    }
    return 0.0;
}

static int best_lpc_order(const double *err, int max_order, int total, int overhead) {
    double error_scale = 0.5 / (double)total;
    int best = 0;
    double best_bits = (unsigned)(-1);
    for (int i = 0, o = 1; i < max_order; i++, o++) {
        double b = expected_bits_scaled(err[i], error_scale) * (double)(total - o) + (double)(o * overhead);
        if (b < best_bits) { best = i; best_bits = b; }
    }
    return best + 1;
}

/* FLAC__lpc_quantize_coefficients; returns 0 ok */
static int quantize_coefs(const float *lp, int order, int precision, int32_t *q, int *shift) {
    precision--;
    int32_t qmax = 1 << precision, qmin = -qmax;
    qmax--;
    double cmax = 0.0;
    for (int i = 0; i < order; i++) {
        double d = fabs(lp[i]);
        if (d > cmax) cmax = d;
    }
    if (cmax <= 0.0) return 2;
    int log2cmax;
    (void)frexp(cmax, &log2cmax);
    log2cmax--;
    *shift = precision - log2cmax - 1;
    if (*shift > 15) *shift = 15;
    else if (*shift < -16) return 1;
    if (*shift >= 0) {
        double error = 0.0;
        for (int i = 0; i < order; i++) {
            error += lp[i] * (float)(1 << *shift);
            int32_t qi = (int32_t)lround(error);
            if (qi > qmax) qi = qmax; else if (qi < qmin) qi = qmin;
            error -= qi;
            q[i] = qi;
        }
    } else {
        int nshift = -(*shift);
        double error = 0.0;
        for (int i = 0; i < order; i++) {
            error += lp[i] / (float)(1 << nshift);
            int32_t qi = (int32_t)lround(error);
            if (qi > qmax) qi = qmax; else if (qi < qmin) qi = qmin;
            error -= qi;
            q[i] = qi;
        }
        *shift = 0;
    }
    return 0;
}

/* residual; returns 0 if a residual does not fit (libFLAC *_limit_residual returns false) */
static int lpc_residual(const int64_t *x, int n, const int32_t *q, int order, int shift, int32_t *res) {
    for (int i = order; i < n; i++) {
        int64_t s = 0;
        for (int j = 0; j < order; j++) s += (int64_t)q[j] * x[i - 1 - j];
        int64_t r = x[i] - (s >> shift);
        if (r <= INT32_MIN || r > INT32_MAX) return 0;
        res[i - order] = (int32_t)r;
    }
    return 1;
}

/* ------------------------------------------------------------------ partitioned rice (stream_encoder.c) */
typedef struct {
    int order;        /* partition order */
    int params[64];   /* rice parameters */
    int rice2;        /* RICE2 needed */
} rice_t;

static uint32_t find_best_partition(const int32_t *res, int pred_order, int blocksize, int bps,
                                    int rice_limit, int max_po, rice_t *best) {
    while (max_po > 0 && (blocksize >> max_po) <= pred_order) max_po--;
    int min_po = 0;
    /* partition sums at max order, merged downwards */
    uint64_t sums[128];
    int parts = 1 << max_po;
    int base = blocksize >> max_po;
    (void)bps;
    int idx = 0;
    for (int p = 0; p < parts; p++) {
        int n = base - (p == 0 ? pred_order : 0);
        uint64_t s = 0;
        for (int i = 0; i < n; i++) { int64_t r = res[idx + i]; s += (uint64_t)(r < 0 ? -r : r); }
        sums[p] = s;
        idx += n;
    }
    int from = 0, to = parts, pp = parts;
    for (int po = max_po - 1; po >= min_po; po--) {
        pp >>= 1;
        for (int i = 0; i < pp; i++) { sums[to++] = sums[from] + sums[from + 1]; from += 2; }
    }
    uint32_t best_bits = 0;
    int sumoff = 0;
    for (int po = max_po; po >= min_po; po--) {
        int np = 1 << po;
        uint32_t pbase = (uint32_t)(blocksize >> po);
        uint32_t div_base = 0x40000u / pbase;
        uint32_t bits = 2 + 4;
        int params[64];
        int ok = 1;
        for (int p = 0; p < np; p++) {
            uint32_t ns = pbase, div = div_base;
            if (p == 0) {
                if (ns <= (uint32_t)pred_order) { ok = 0; break; }
                ns -= (uint32_t)pred_order;
                div = 0x40000u / ns;
            }
            uint64_t mean = sums[sumoff + p];
            uint32_t k;
            if (mean < 2 || (((mean - 1) * div) >> 18) == 0) k = 0;
            else k = ilog2_u64(((mean - 1) * div) >> 18) + 1;
            if (k >= (uint32_t)rice_limit) k = (uint32_t)rice_limit - 1;
            uint64_t pb = 4 + (uint64_t)(1 + k) * ns + (k ? (mean >> (k - 1)) : (mean << 1)) - (ns >> 1);
            if (pb > UINT32_MAX) pb = UINT32_MAX;
            bits += (uint32_t)pb;
            params[p] = (int)k;
        }
        if (!ok) break;
        sumoff += np;
        if (best_bits == 0 || bits < best_bits) {
            best_bits = bits;
            best->order = po;
            memcpy(best->params, params, sizeof(int) * np);
        }
    }
    best->rice2 = 0;
    for (int p = 0; p < (1 << best->order); p++)
        if (best->params[p] >= 15) best->rice2 = 1;
    return best_bits;
}

/* ------------------------------------------------------------------ subframe decision */
enum { SF_CONSTANT = 0, SF_VERBATIM = 1, SF_FIXED = 2, SF_LPC = 3 };

typedef struct {
    int type, wasted, sbps;
    int order;           /* fixed / lpc order */
    int prec, shift;     /* lpc */
    int32_t q[ORC_MAX_LPC];
    rice_t rice;
    uint32_t est_bits;
} subframe_t;

/* process_subframe_ of libFLAC 1.4.3 at levels 0..5 (tukey(0.5), no exhaustive search, no escapes, no qlp
 * precision search; max_lpc_order 8 and partition orders 0..5 at level 5, the other levels' values from the
 * compression-level table, docs/sonos-pyflac.txt:6926-6931: max_lpc 0 = fixed predictors only).  x is modified in place by the wasted
 * bits shift (as get_wasted_bits_ does).  bps is the STREAM's bits per sample (it sets the RICE2 limit,
 * the qlp precision and the wasted-bits cap); extra = 1 for the side channel of process_subframes_'s
 * mid/side pass (subframe_bps_mid_side[1] = bps - w + 1), 0 otherwise.  Samples are int64 so the side
 * channel of a 32-bit stream (33 bits, integer_signal_33bit_side) takes the same code. */
/* libFLAC 1.4.3 lpc.c FLAC__lpc_window_data_partial: part c of a block cut into 1/b parts, windowed by the rising
 * half then the falling half of the full-length window (tukey(p / parts): its tapers fit the smallest part), a zero
 * after it (the autocorrelation reads blocksize / b samples) */
static void window_partial(const int64_t *x, const float *window, float *out, int data_len, int part_size,
                           int data_shift) {
    if (part_size + data_shift < data_len) {
        int i, j;
        for (i = 0; i < part_size; i++) out[i] = (float)x[data_shift + i] * window[i];
        i = i < data_len - part_size - data_shift ? i : data_len - part_size - data_shift;
        for (j = data_len - part_size; j < data_len; i++, j++) out[i] = (float)x[data_shift + i] * window[j];
        if (i < data_len) out[i] = 0.0f;
    }
}

/* stream_encoder.c set_next_subdivide_tukey: the (depth b, part c) after the current one of a subdivide_tukey(parts)
 * apodization (c even: partial window c / 2; c odd: the punch-out of part c / 2, i.e. the root window's
 * autocorrelation minus the partial one's; depth 2 has partial windows only).  Returns 0 when the apodization is
 * done. */
static int next_subdivide(int parts, int *b, int *c) {
    if (*b == 2) {
        if (*c == 0) *c = 2;
        else { *c = 0; (*b)++; }
    } else if (*c < 2 * *b - 1) {
        (*c)++;
    } else {
        *c = 0;
        (*b)++;
    }
    return *b <= parts;
}

static void decide_subframe(int64_t *x, int n, int bps, int extra, int cfg_blocksize, const float *window,
                            int32_t *scratch_res, float *scratch_d, subframe_t *sf, int cfg_max_lpc, int cfg_max_po,
                            int parts) {
    /* get_wasted_bits_ / get_wasted_bits_wide_ */
    int64_t orv = 0;
    for (int i = 0; i < n && !(orv & 1); i++) orv |= x[i];
    int w = 0;
    if (orv != 0) { while (!(orv & 1)) { orv >>= 1; w++; } }
    if (w) for (int i = 0; i < n; i++) x[i] >>= w;
    if (w > bps) w = bps;
    int sbps = bps - w + extra;
    sf->wasted = w;
    sf->sbps = sbps;
    const int rice_limit = bps > 16 ? 31 : 15;
    /* stream_encoder.c init, qlp_coeff_precision == 0 (level 5): by bps and the configured blocksize */
    int qlp_precision;
    if (bps < 16) qlp_precision = (2 + bps / 2) > 5 ? 2 + bps / 2 : 5;
    else if (bps == 16) qlp_precision = cfg_blocksize <= 192 ? 7 : cfg_blocksize <= 384 ? 8 : cfg_blocksize <= 576 ? 9 :
                                        cfg_blocksize <= 1152 ? 10 : cfg_blocksize <= 2304 ? 11 : cfg_blocksize <= 4608 ? 12 : 13;
    else qlp_precision = cfg_blocksize <= 384 ? 13 : cfg_blocksize <= 1152 ? 14 : 15;
    /* process_subframes_: max partition order from the (possibly short final) block size, capped at the level's
     * max_residual_partition_order */
    int max_po = 0;
    { int b = n; while (!(b & 1) && max_po < cfg_max_po) { max_po++; b >>= 1; } }

    /* verbatim baseline */
    sf->type = SF_VERBATIM;
    sf->est_bits = (uint32_t)(1 + 6 + 1 + w + n * sbps);
    if (n <= ORC_MAX_FIXED) return;

    float fbits[5];
    int guess;
    if (sbps < 28) guess = fixed_best(x + 4, n - 4, fbits);
    else guess = fixed_best_limit_residual(x + 4, n - 4, fbits);

    if (fbits[1] == 0.0f) {
        int constant = 1;
        for (int i = 1; i < n; i++) if (x[i] != x[0]) { constant = 0; break; }
        if (constant) {
            uint32_t cb = (uint32_t)(1 + 6 + 1 + w + sbps);
            if (cb < sf->est_bits) { sf->type = SF_CONSTANT; sf->est_bits = cb; }
            return;
        }
    }
    /* fixed */
    if (!(fbits[guess] >= (float)sbps)) {
        int o = guess;
        for (int i = o; i < n; i++) {
            int64_t p = 0;
            for (int j = 0; j < o; j++) p += (int64_t)fixed_coefs[o][j] * x[i - 1 - j];
            scratch_res[i - o] = (int32_t)(x[i] - p);
        }
        rice_t rc;
        uint32_t rb = find_best_partition(scratch_res, o, n, sbps, rice_limit, max_po, &rc);
        uint32_t est = (uint32_t)(1 + 6 + 1 + w + o * sbps);
        est = (rb < UINT32_MAX - est) ? est + rb : UINT32_MAX;
        if (est < sf->est_bits) {
            sf->type = SF_FIXED; sf->order = o; sf->rice = rc; sf->est_bits = est;
        }
    }
    /* lpc: one candidate per window of the apodization (tukey(0.5) at levels <= 5: one window; subdivide_tukey(parts)
     * at levels 6..8: the full block, then at depth b = 2 .. parts its b partial windows and, from depth 3, their
     * punch-outs), each LPC candidate replacing the best subframe when strictly smaller */
    const int cfg_order = cfg_max_lpc >= n ? n - 1 : cfg_max_lpc;
    if (cfg_order <= 0) return;
    double autoc[ORC_MAX_LPC + 1], autoc_root[ORC_MAX_LPC + 1];
    int b = 1, c = 0;
    for (int more = 1; more;) {
        int max_order = cfg_order;
        if (b == 1) {
            for (int i = 0; i < n; i++) scratch_d[i] = (float)x[i] * window[i];
            autocorrelation(scratch_d, n, max_order + 1, autoc);
            if (parts > 1) {
                memcpy(autoc_root, autoc, sizeof(double) * (size_t)(max_order + 1));
                b = 2;
                c = 0;
            } else {
                more = 0;
            }
        } else {
            if (n / b <= 32) {  /* (FLAC__MAX_LPC_ORDER) parts this small are not windowed */
                more = next_subdivide(parts, &b, &c);
                continue;
            }
            if (!(c % 2)) {
                window_partial(x, window, scratch_d, n, n / b / 2, (c / 2 * n) / b);
                autocorrelation(scratch_d, n / b, max_order + 1, autoc);
            } else {
                /* libFLAC 1.4.3 apply_apodization_ (stream_encoder.c): the punch-out subtracts (and autoc_root holds,
                 * by its memcpy) lags 0 .. max_order - 1 only; lag max_order keeps the partial window's value */
                for (int i = 0; i < max_order; i++) autoc[i] = autoc_root[i] - autoc[i];
            }
            more = next_subdivide(parts, &b, &c);
        }
        if (autoc[0] == 0.0) continue;
        float lp[ORC_MAX_LPC][ORC_MAX_LPC];
        double lerr[ORC_MAX_LPC];
        max_order = lp_coefficients(autoc, max_order, lp, lerr);
        int o = best_lpc_order(lerr, max_order, n, sbps + qlp_precision);
        double lbits = expected_bits_scaled(lerr[o - 1], 0.5 / (double)(n - o));
        if (lbits >= (double)sbps) continue;
        int prec = qlp_precision;
        if (sbps <= 17) {
            int lim = 32 - sbps - (int)ilog2_u64((uint64_t)o);
            if (lim < prec) prec = lim;
        }
        int32_t q[ORC_MAX_LPC];
        int shift;
        if (quantize_coefs(lp[o - 1], o, prec, q, &shift) != 0) continue;
        if (!lpc_residual(x, n, q, o, shift, scratch_res)) continue;
        rice_t rc;
        uint32_t rb = find_best_partition(scratch_res, o, n, sbps, rice_limit, max_po, &rc);
        uint32_t est = (uint32_t)(1 + 6 + 1 + w + 4 + 5 + sbps * o + prec * o);
        est = (rb < UINT32_MAX - est) ? est + rb : UINT32_MAX;
        if (est == 0) continue;
        if (est < sf->est_bits) {
            sf->type = SF_LPC; sf->order = o; sf->prec = prec; sf->shift = shift;
            memcpy(sf->q, q, sizeof(q)); sf->rice = rc; sf->est_bits = est;
        }
    }
}

static void write_residual(bw_t *bw, const int32_t *res, int n, int pred_order, const rice_t *rc) {
    int pbits = rc->rice2 ? 5 : 4;
    bw_put(bw, rc->rice2 ? 1 : 0, 2);
    bw_put(bw, (uint64_t)rc->order, 4);
    int parts = 1 << rc->order;
    int idx = 0;
    for (int p = 0; p < parts; p++) {
        int ns = (n >> rc->order) - (p == 0 ? pred_order : 0);
        int k = rc->params[p];
        bw_put(bw, (uint64_t)k, pbits);
        for (int i = 0; i < ns; i++) {
            int32_t r = res[idx + i];
            uint32_t u = ((uint32_t)r << 1) ^ (uint32_t)(r >> 31);
            bw_put_zeros(bw, u >> k);
            bw_put(bw, 1, 1);
            if (k) bw_put(bw, u & ((1u << k) - 1), k);
        }
        idx += ns;
    }
}

static void write_subframe(bw_t *bw, const int64_t *x, int n, const subframe_t *sf, int32_t *scratch_res) {
    int typebits;
    switch (sf->type) {
    case SF_CONSTANT: typebits = 0; break;
    case SF_VERBATIM: typebits = 1; break;
    case SF_FIXED: typebits = 8 + sf->order; break;
    default: typebits = 32 + sf->order - 1; break;
    }
    bw_put(bw, 0, 1);
    bw_put(bw, (uint64_t)typebits, 6);
    if (sf->wasted) {
        bw_put(bw, 1, 1);
        bw_put_zeros(bw, (uint64_t)(sf->wasted - 1));
        bw_put(bw, 1, 1);
    } else {
        bw_put(bw, 0, 1);
    }
    int sbps = sf->sbps;
    if (sf->type == SF_CONSTANT) {
        bw_put_signed(bw, x[0], sbps);
    } else if (sf->type == SF_VERBATIM) {
        for (int i = 0; i < n; i++) bw_put_signed(bw, x[i], sbps);
    } else if (sf->type == SF_FIXED) {
        int o = sf->order;
        for (int i = 0; i < o; i++) bw_put_signed(bw, x[i], sbps);
        for (int i = o; i < n; i++) {
            int64_t p = 0;
            for (int j = 0; j < o; j++) p += (int64_t)fixed_coefs[o][j] * x[i - 1 - j];
            scratch_res[i - o] = (int32_t)(x[i] - p);
        }
        write_residual(bw, scratch_res, n, o, &sf->rice);
    } else {
        int o = sf->order;
        for (int i = 0; i < o; i++) bw_put_signed(bw, x[i], sbps);
        bw_put(bw, (uint64_t)(sf->prec - 1), 4);
        bw_put_signed(bw, sf->shift, 5);
        for (int i = 0; i < o; i++) bw_put_signed(bw, sf->q[i], sf->prec);
        lpc_residual(x, n, sf->q, o, sf->shift, scratch_res);
        write_residual(bw, scratch_res, n, o, &sf->rice);
    }
}

/* ------------------------------------------------------------------ frame header (RFC 9639 9.1) */
static int bs_code(int bs, int *hint) {
    *hint = 0;
    switch (bs) {
    case 192: return 1;
    case 576: return 2;
    case 1152: return 3;
    case 2304: return 4;
    case 4608: return 5;
    case 256: return 8;
    case 512: return 9;
    case 1024: return 10;
    case 2048: return 11;
    case 4096: return 12;
    case 8192: return 13;
    case 16384: return 14;
    case 32768: return 15;
    default: *hint = bs <= 256 ? 6 : 7; return *hint;
    }
}
static int sr_code(int sr, int *hint) {
    *hint = 0;
    switch (sr) {
    case 88200: return 1;
    case 176400: return 2;
    case 192000: return 3;
    case 8000: return 4;
    case 16000: return 5;
    case 22050: return 6;
    case 24000: return 7;
    case 32000: return 8;
    case 44100: return 9;
    case 48000: return 10;
    case 96000: return 11;
    default:
        if (sr <= 255000 && sr % 1000 == 0) *hint = 12;
        else if (sr % 10 == 0 && sr / 10 <= 65535) *hint = 14;
        else *hint = 13;
        return *hint;
    }
}
static int bps_code(int bps) {
    switch (bps) {
    case 8: return 1;
    case 12: return 2;
    case 16: return 4;
    case 20: return 5;
    case 24: return 6;
    case 32: return 7;
    default: return 0;
    }
}

static void write_frame_header(bw_t *bw, int bs, int sr, int ch_assign, int bps, uint32_t frame_no) {
    int64_t start = bw->bits >> 3;
    int bsh, srh;
    int bc = bs_code(bs, &bsh), sc = sr_code(sr, &srh);
    bw_put(bw, 0x3FFE, 14);
    bw_put(bw, 0, 1);
    bw_put(bw, 0, 1); /* fixed blocksize */
    bw_put(bw, (uint64_t)bc, 4);
    bw_put(bw, (uint64_t)sc, 4);
    bw_put(bw, (uint64_t)ch_assign, 4); /* ch - 1 (independent) or 8/9/10 (left/right/mid-side) */
    bw_put(bw, (uint64_t)bps_code(bps), 3);
    bw_put(bw, 0, 1);
    /* UTF-8 coded frame number */
    uint32_t v = frame_no;
    if (v < 0x80) bw_put(bw, v, 8);
    else if (v < 0x800) { bw_put(bw, 0xC0 | (v >> 6), 8); bw_put(bw, 0x80 | (v & 0x3F), 8); }
    else if (v < 0x10000) { bw_put(bw, 0xE0 | (v >> 12), 8); bw_put(bw, 0x80 | ((v >> 6) & 0x3F), 8); bw_put(bw, 0x80 | (v & 0x3F), 8); }
    else if (v < 0x200000) { bw_put(bw, 0xF0 | (v >> 18), 8); bw_put(bw, 0x80 | ((v >> 12) & 0x3F), 8); bw_put(bw, 0x80 | ((v >> 6) & 0x3F), 8); bw_put(bw, 0x80 | (v & 0x3F), 8); }
    else if (v < 0x4000000) { bw_put(bw, 0xF8 | (v >> 24), 8); bw_put(bw, 0x80 | ((v >> 18) & 0x3F), 8); bw_put(bw, 0x80 | ((v >> 12) & 0x3F), 8); bw_put(bw, 0x80 | ((v >> 6) & 0x3F), 8); bw_put(bw, 0x80 | (v & 0x3F), 8); }
    else { bw_put(bw, 0xFC | (v >> 30), 8); bw_put(bw, 0x80 | ((v >> 24) & 0x3F), 8); bw_put(bw, 0x80 | ((v >> 18) & 0x3F), 8); bw_put(bw, 0x80 | ((v >> 12) & 0x3F), 8); bw_put(bw, 0x80 | ((v >> 6) & 0x3F), 8); bw_put(bw, 0x80 | (v & 0x3F), 8); }
    if (bsh == 6) bw_put(bw, (uint64_t)(bs - 1), 8);
    else if (bsh == 7) bw_put(bw, (uint64_t)(bs - 1), 16);
    if (srh == 12) bw_put(bw, (uint64_t)(sr / 1000), 8);
    else if (srh == 13) bw_put(bw, (uint64_t)sr, 16);
    else if (srh == 14) bw_put(bw, (uint64_t)(sr / 10), 16);
    int64_t end = bw->bits >> 3;
    bw_put(bw, crc8(bw->buf + start, end - start), 8);
}

/* ------------------------------------------------------------------ public oracle API */

/* Encode the FLAC frames (no stream header) of `nsamples` interleaved samples with `ch` channels,
 * exactly as libFLAC 1.4.3 at `level` does through FLAC__stream_encoder_process_interleaved + finish
 * (a final short block keeps the full-length window: resize_buffers_ only grows).
 *
 * Two channels: levels 2 and 5 set do_mid_side_stereo=true, loose_mid_side_stereo=false
 * (docs/sonos-pyflac.txt:6931), so process_subframes_ codes left, right, mid = (L+R)>>1 (bps) and
 * side = L-R (bps+1) and writes the assignment with the fewest estimated bits among independent,
 * left-side, right-side, mid-side (that order; a later one must be strictly smaller), header codes
 * 1/8/9/10 (docs/sonos-pyflac.txt:2571-2576), subframes (L,R), (L,S), (S,R), (M,S).
 * Returns bytes written, or -(bytes needed) on overflow (rough upper bound). */
int64_t orc_encode_frames_level(const int32_t *interleaved, int64_t nsamples, int ch, int bps, int sample_rate,
                                int blocksize, int level, uint8_t *out, int64_t cap) {
    crc_init();
    if (ch < 1 || ch > ORC_MAX_CH || blocksize < 16) return -1;
    /* compression-level table (docs/sonos-pyflac.txt:6926-6934): mid/side, loose mid/side, max LPC order, max
     * residual partition order, apodization (tukey(0.5) = 1 part; subdivide_tukey(2) at 6 and 7, (3) at 8) */
    static const int lvl_ms[9] = {0, 1, 1, 0, 1, 1, 1, 1, 1}, lvl_loose[9] = {0, 1, 0, 0, 1, 0, 0, 0, 0};
    static const int lvl_lpc[9] = {0, 0, 0, 6, 8, 8, 8, 12, 12}, lvl_po[9] = {3, 3, 3, 4, 4, 5, 6, 6, 6};
    static const int lvl_parts[9] = {1, 1, 1, 1, 1, 1, 2, 2, 3};
    if (level < 0 || level > 8) return -2;
    const int max_lpc = lvl_lpc[level], max_po = lvl_po[level], parts = lvl_parts[level];
    const int stereo = ch == 2 && lvl_ms[level];
    const int loose = stereo && lvl_loose[level];
    /* loose mid/side (stream_encoder.c init): a full independent-vs-mid/side evaluation every
     * (uint32_t)(sample_rate * 0.4 / blocksize + 0.5) frames (at least 1), the last choice kept in between */
    int loose_frames = (int)(uint32_t)((double)sample_rate * 0.4 / (double)blocksize + 0.5);
    if (loose_frames == 0) loose_frames = 1;
    int loose_count = 0, last_assign = 1;
    const int nv = stereo ? 4 : ch; /* coded signals: channels, or L, R, M, S */
    float *window = (float *)malloc(sizeof(float) * (size_t)blocksize);
    float *dbuf = (float *)malloc(sizeof(float) * (size_t)blocksize);
    int64_t *xbuf = (int64_t *)malloc(sizeof(int64_t) * (size_t)blocksize * (size_t)nv);
    int32_t *res = (int32_t *)malloc(sizeof(int32_t) * (size_t)blocksize);
    /* subdivide_tukey(parts): set_apodization stores p / parts (float), the window is tukey(p / parts) */
    orc_window_tukey(window, blocksize, 0.5f / (float)parts);
    bw_t bw = {out, cap, 0, 0};
    uint32_t frame_no = 0;
    subframe_t sf[ORC_MAX_CH];
    for (int64_t s0 = 0; s0 < nsamples; s0 += blocksize, frame_no++) {
        int n = (int)((nsamples - s0) < blocksize ? (nsamples - s0) : blocksize);
        int64_t fstart = bw.bits >> 3;
        for (int c = 0; c < ch; c++) {
            int64_t *x = xbuf + (size_t)c * blocksize;
            for (int i = 0; i < n; i++) x[i] = interleaved[(s0 + i) * ch + c];
        }
        if (stereo) {
            int64_t *l = xbuf, *r = xbuf + blocksize, *m = xbuf + 2 * (size_t)blocksize, *sd = xbuf + 3 * (size_t)blocksize;
            for (int i = 0; i < n; i++) { m[i] = (l[i] + r[i]) >> 1; sd[i] = l[i] - r[i]; }
        }
        /* process_frame_: which signals are coded (loose mid/side: both pairs on an evaluation frame, otherwise
         * only the pair of the last choice) */
        int do_ind = 1, do_ms = stereo;
        if (loose && loose_count > 0) {
            do_ind = last_assign == 1;
            do_ms = !do_ind;
        }
        for (int v = 0; v < nv; v++) {
            memset(&sf[v], 0, sizeof(sf[v]));
            if (stereo && ((v < 2 && !do_ind) || (v >= 2 && !do_ms))) continue;
            decide_subframe(xbuf + (size_t)v * blocksize, n, bps, stereo && v == 3, blocksize, window, res, dbuf, &sf[v],
                            max_lpc, max_po, parts);
        }
        int assign = ch - 1, pick[2] = {0, 1};
        if (stereo) {
            static const int picks[4][2] = {{0, 1}, {0, 3}, {3, 1}, {2, 3}};
            int ca = 0;
            if (loose && loose_count > 0) {
                ca = last_assign == 1 ? 0 : 3;
            } else {
                const uint32_t bits[4] = {sf[0].est_bits + sf[1].est_bits, sf[0].est_bits + sf[3].est_bits,
                                          sf[1].est_bits + sf[3].est_bits, sf[2].est_bits + sf[3].est_bits};
                /* strict <, in this order; loose mid/side considers independent and mid-side only */
                for (int k = loose ? 3 : 1; k < 4; k++) if (bits[k] < bits[ca]) ca = k;
            }
            assign = ca == 0 ? 1 : 7 + ca;
            pick[0] = picks[ca][0]; pick[1] = picks[ca][1];
            if (loose) {
                loose_count = loose_count + 1 >= loose_frames ? 0 : loose_count + 1;
                last_assign = assign;
            }
        }
        write_frame_header(&bw, n, sample_rate, assign, bps, frame_no);
        for (int c = 0; c < ch; c++) {
            int v = stereo ? pick[c] : c;
            write_subframe(&bw, xbuf + (size_t)v * blocksize, n, &sf[v], res);
        }
        bw_align(&bw);
        int64_t fend = bw.bits >> 3;
        if (!bw.overflow) {
            uint16_t c16 = crc16(bw.buf + fstart, fend - fstart);
            bw_put(&bw, c16, 16);
        } else {
            bw_put(&bw, 0, 16);
        }
    }
    free(window); free(dbuf); free(xbuf); free(res);
    if (bw.overflow) return -(bw.bits >> 3);
    return bw.bits >> 3;
}

/* level 5 (cli.py:733, converter.py:112 default) */
int64_t orc_encode_frames(const int32_t *interleaved, int64_t nsamples, int ch, int bps, int sample_rate,
                          int blocksize, uint8_t *out, int64_t cap) {
    return orc_encode_frames_level(interleaved, nsamples, ch, bps, sample_rate, blocksize, 5, out, cap);
}

/* Bare libFLAC stream header: "fLaC" + STREAMINFO (min/max framesize 0, total 0, MD5 0: pyflac's
 * StreamEncoder has no seek callback) + last VORBIS_COMMENT with the vendor string only.
 * Pinned by test_data/sample_rgb.flac bytes 0..85. Returns bytes (86). */
int64_t orc_stream_header(int ch, int bps, int sample_rate, int blocksize, uint8_t *out, int64_t cap) {
    static const char vendor[] = "reference libFLAC 1.4.3 20230623";
    if (cap < 86) return -86;
    bw_t bw = {out, cap, 0, 0};
    bw_put(&bw, 'f', 8); bw_put(&bw, 'L', 8); bw_put(&bw, 'a', 8); bw_put(&bw, 'C', 8);
    bw_put(&bw, 0, 1); bw_put(&bw, 0, 7); bw_put(&bw, 34, 24);
    bw_put(&bw, (uint64_t)blocksize, 16); bw_put(&bw, (uint64_t)blocksize, 16);
    bw_put(&bw, 0, 24); bw_put(&bw, 0, 24);
    bw_put(&bw, (uint64_t)sample_rate, 20); bw_put(&bw, (uint64_t)(ch - 1), 3); bw_put(&bw, (uint64_t)(bps - 1), 5);
    bw_put(&bw, 0, 36);
    for (int i = 0; i < 16; i++) bw_put(&bw, 0, 8);
    int vlen = (int)strlen(vendor);
    bw_put(&bw, 1, 1); bw_put(&bw, 4, 7); bw_put(&bw, (uint64_t)(4 + vlen + 4), 24);
    bw_put(&bw, (uint64_t)(vlen & 0xFF), 8); bw_put(&bw, 0, 8); bw_put(&bw, 0, 8); bw_put(&bw, 0, 8);
    for (int i = 0; i < vlen; i++) bw_put(&bw, (uint8_t)vendor[i], 8);
    bw_put(&bw, 0, 32);
    return bw.bits >> 3;
}

/* ------------------------------------------------------------------ normalisation (numpy semantics) */
/* dtype codes shared with the product ABI: 1=u8 2=u16 3=i16 4=i32 5=u32 6=f32 7=f64 */
static int64_t ld_i(const void *p, int dtype, int64_t i) {
    switch (dtype) {
    case 1: return ((const uint8_t *)p)[i];
    case 2: return ((const uint16_t *)p)[i];
    case 3: return ((const int16_t *)p)[i];
    case 4: return ((const int32_t *)p)[i];
    default: return ((const uint32_t *)p)[i];
    }
}
/* wrap an integer to the input dtype (numpy 2 same-kind arithmetic, NEP 50) */
static int64_t wrap_dt(int64_t v, int dtype) {
    switch (dtype) {
    case 1: return (uint8_t)v;
    case 2: return (uint16_t)v;
    case 3: return (int16_t)v;
    case 4: return (int32_t)v;
    default: return (uint32_t)v;
    }
}
/* numpy's float64 -> int16 / int32 cast as compiled on x86-64 (cvttsd2si; out-of-range -> INT_MIN
 * pattern, then the low bits for int16).  NaN never occurs for integer inputs. */
static int32_t cast_f64_i32(double v) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT32_MIN;
    return (int32_t)v;
}

/* converter.py:56-86.  min/max over the whole array (np.min/np.max), outputs int32 samples that are
 * int16-valued for bps 16.  Returns stream bps (16 or 32, pyflac: itemsize*8, encoder.py:1986-1992). */
int orc_normalize(const void *src, int dtype, int64_t n, int bits_per_sample, double *out_min, double *out_max,
                  int32_t *dst) {
    if (dtype == 6 || dtype == 7) {
        /* float data is used as-is (converter.py:61-64), then * 8388607 (bps 24) in the input float type */
        double mn = INFINITY, mx = -INFINITY;
        for (int64_t i = 0; i < n; i++) {
            double v = dtype == 6 ? (double)((const float *)src)[i] : ((const double *)src)[i];
            if (v < mn) mn = v;
            if (v > mx) mx = v;
        }
        *out_min = mn; *out_max = mx;
        for (int64_t i = 0; i < n; i++) {
            if (dtype == 6) {
                float v = ((const float *)src)[i] * 8388607.0f;
                dst[i] = cast_f64_i32((double)v);
            } else {
                dst[i] = cast_f64_i32(((const double *)src)[i] * 8388607.0);
            }
        }
        return 32;
    }
    int64_t mn = ld_i(src, dtype, 0), mx = mn;
    for (int64_t i = 1; i < n; i++) {
        int64_t v = ld_i(src, dtype, i);
        if (v < mn) mn = v;
        if (v > mx) mx = v;
    }
    *out_min = (double)mn; *out_max = (double)mx;
    double scale = bits_per_sample == 16 ? 32767.0 : (bits_per_sample == 24 ? 8388607.0 : 2147483647.0);
    if (!(mx > mn)) {
        for (int64_t i = 0; i < n; i++) dst[i] = 0;
        return bits_per_sample == 16 ? 16 : 32;
    }
    double den = (double)wrap_dt(mx - mn, dtype);
    for (int64_t i = 0; i < n; i++) {
        double d = (double)wrap_dt(ld_i(src, dtype, i) - mn, dtype);
        double v = ((2.0 * d) / den - 1.0) * scale;
        int32_t c = cast_f64_i32(v);
        dst[i] = bits_per_sample == 16 ? (int32_t)(int16_t)c : c;
    }
    return bits_per_sample == 16 ? 16 : 32;
}

/* spatial_encoder.py:229-248 then pyflac's samples.astype(np.int32) (sonos-pyflac.txt:1994): float32 maths,
 * truncation.  Returns 0, or -1 for dtypes whose normalised array is float64 (pyflac then asks libFLAC for
 * 64-bit samples and fails). */
int orc_normalize_spatial(const void *src, int dtype, int64_t n, int32_t *dst) {
    for (int64_t i = 0; i < n; i++) {
        volatile float v;
        switch (dtype) {
        case 1: v = ((float)((const uint8_t *)src)[i] - 127.5f) / 127.5f; break;
        case 2: v = ((float)((const uint16_t *)src)[i] - 32767.5f) / 32767.5f; break;
        case 3: v = (float)((const int16_t *)src)[i] / 32767.0f; break;
        case 4: v = (float)((const int32_t *)src)[i] / 2147483647.0f; break;
        case 6: {
            float x = ((const float *)src)[i];
            v = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
            if (x != x) v = x;
            break;
        }
        default: return -1;
        }
        dst[i] = cast_f64_i32((double)v);
    }
    return 0;
}

/* converter.py:88-110 with the decode scaling of pyflac+soundfile (pcm/32768, docs/sonos-pyflac.txt:1629):
 * v = float32(pcm/32768); out = round_half_even(((v + 1)/2) * f32(max-min) + f32(min)), all fp32. */
static double rint_even(double v) { return nearbyint(v); }
void orc_denormalize_i16(const int32_t *pcm, int64_t n, int pcm_bps, double dmin, double dmax, int out_dtype,
                         void *out) {
    float rng = (float)(dmax - dmin), fmn = (float)dmin;
    for (int64_t i = 0; i < n; i++) {
        int32_t p16 = pcm_bps > 16 ? (pcm[i] >> 16) : pcm[i]; /* libsndfile int -> short for 32-bit streams */
        float v = (float)((double)p16 / 32768.0);
        volatile float a = v + 1.0f;
        volatile float b = a / 2.0f;
        volatile float c = b * rng;
        volatile float d = c + fmn;
        float r = (float)rint_even((double)d);
        switch (out_dtype) {
        case 1: ((uint8_t *)out)[i] = (uint8_t)(int64_t)r; break;
        case 2: ((uint16_t *)out)[i] = (uint16_t)(int64_t)r; break;
        case 3: ((int16_t *)out)[i] = (int16_t)(int64_t)r; break;
        case 4: ((int32_t *)out)[i] = (int32_t)(int64_t)r; break;
        case 5: ((uint32_t *)out)[i] = (uint32_t)(int64_t)r; break;
        case 6: ((float *)out)[i] = v; break;
        default: ((double *)out)[i] = (double)v; break;
        }
    }
}

/* ------------------------------------------------------------------ decoder (RFC 9639) */
typedef struct {
    const uint8_t *d;
    int64_t n;
    int64_t bit;
    int err;
} br_t;
static uint64_t br_u(br_t *b, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) {
        int64_t byte = b->bit >> 3;
        if (byte >= b->n) { b->err = 1; return 0; }
        v = (v << 1) | ((b->d[byte] >> (7 - (b->bit & 7))) & 1);
        b->bit++;
    }
    return v;
}
static int64_t br_s(br_t *b, int n) {
    uint64_t v = br_u(b, n);
    if (n && (v >> (n - 1))) v |= ~0ull << n;
    return (int64_t)v;
}
static uint32_t br_unary(br_t *b) {
    uint32_t q = 0;
    while (!b->err && br_u(b, 1) == 0) q++;
    return q;
}

/* Decode the frames that follow a stream header; returns samples per channel decoded, or <0 on error.
 * out: interleaved int32, capacity cap_samples per channel. */
static int64_t decode_frames_impl(const uint8_t *in, int64_t n, int ch, int bps, int32_t *out, int64_t cap_samples,
                                  int8_t *ca_out, int64_t ca_cap, int16_t *sf_out, int64_t sf_cap) {
    int64_t nsf = 0;
    crc_init();
    int64_t nfr = 0;
    br_t b = {in, n, 0, 0};
    int64_t total = 0;
    int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * 65536 * 8); /* int64: a 32-bit stream's side channel has 33 bits */
    while ((b.bit >> 3) + 2 <= n) {
        int64_t fstart = b.bit >> 3;
        if (br_u(&b, 14) != 0x3FFE) { free(tmp); return -2; }
        br_u(&b, 1); br_u(&b, 1);
        int bc = (int)br_u(&b, 4), sc = (int)br_u(&b, 4), ca = (int)br_u(&b, 4), ss = (int)br_u(&b, 3);
        br_u(&b, 1);
        uint32_t b0 = (uint32_t)br_u(&b, 8);
        int extra = 0;
        if (b0 & 0x80) { uint32_t m = 0x40; while (b0 & m) { extra++; m >>= 1; } }
        for (int i = 0; i < extra; i++) br_u(&b, 8);
        int bs;
        if (bc == 1) bs = 192;
        else if (bc >= 2 && bc <= 5) bs = 576 << (bc - 2);
        else if (bc == 6) bs = (int)br_u(&b, 8) + 1;
        else if (bc == 7) bs = (int)br_u(&b, 16) + 1;
        else if (bc >= 8) bs = 256 << (bc - 8);
        else { free(tmp); return -3; }
        if (sc == 12) br_u(&b, 8); else if (sc == 13 || sc == 14) br_u(&b, 16);
        int64_t hend = b.bit >> 3;
        uint8_t c8 = (uint8_t)br_u(&b, 8);
        if (c8 != crc8(in + fstart, hend - fstart)) { free(tmp); return -4; }
        int fbps = ss == 1 ? 8 : ss == 2 ? 12 : ss == 4 ? 16 : ss == 5 ? 20 : ss == 6 ? 24 : ss == 7 ? 32 : bps;
        if (ca_out && nfr < ca_cap) ca_out[nfr] = (int8_t)ca;
        nfr++;
        int nch = ca < 8 ? ca + 1 : 2;
        if (nch != ch || total + bs > cap_samples || bs > 65536) { free(tmp); return -5; }
        for (int c = 0; c < nch; c++) {
            int sbps = fbps;
            if ((ca == 8 && c == 1) || (ca == 9 && c == 0) || (ca == 10 && c == 1)) sbps++;
            int64_t *x = tmp + (size_t)c * 65536;
            br_u(&b, 1);
            int t = (int)br_u(&b, 6);
            if (sf_out && nsf < sf_cap) sf_out[nsf] = (int16_t)t;  /* + partition order << 8 for FIXED / LPC */
            int w = 0;
            if (br_u(&b, 1)) w = (int)br_unary(&b) + 1;
            sbps -= w;
            if (t == 0) {
                int64_t v = br_s(&b, sbps);
                for (int i = 0; i < bs; i++) x[i] = v;
            } else if (t == 1) {
                for (int i = 0; i < bs; i++) x[i] = br_s(&b, sbps);
            } else if ((t >= 8 && t <= 12) || t >= 32) {
                int lpc = t >= 32, o = lpc ? t - 31 : t - 8;
                int64_t q[32];
                int shift = 0, prec;
                for (int i = 0; i < o; i++) x[i] = br_s(&b, sbps);
                if (lpc) {
                    prec = (int)br_u(&b, 4) + 1;
                    shift = (int)br_s(&b, 5);
                    for (int i = 0; i < o; i++) q[i] = br_s(&b, prec);
                }
                int method = (int)br_u(&b, 2), po = (int)br_u(&b, 4);
                if (sf_out && nsf < sf_cap) sf_out[nsf] = (int16_t)(t | (po << 8));
                int pb = method == 0 ? 4 : 5, esc = (1 << pb) - 1;
                int idx = o;
                for (int p = 0; p < (1 << po); p++) {
                    int ns = (bs >> po) - (p == 0 ? o : 0);
                    int k = (int)br_u(&b, pb);
                    if (k == esc) {
                        int nb = (int)br_u(&b, 5);
                        for (int i = 0; i < ns; i++) x[idx + i] = nb ? br_s(&b, nb) : 0;
                    } else {
                        for (int i = 0; i < ns; i++) {
                            uint32_t qq = br_unary(&b);
                            uint32_t u = (qq << k) | (uint32_t)(k ? br_u(&b, k) : 0);
                            x[idx + i] = (int32_t)((u >> 1) ^ (uint32_t)-(int32_t)(u & 1));
                        }
                    }
                    idx += ns;
                }
                /* reconstruct */
                for (int i = o; i < bs; i++) {
                    int64_t pred = 0;
                    if (lpc) {
                        for (int j = 0; j < o; j++) pred += q[j] * x[i - 1 - j];
                        pred >>= shift;
                    } else {
                        for (int j = 0; j < o; j++) pred += (int64_t)fixed_coefs[o][j] * x[i - 1 - j];
                    }
                    x[i] = x[i] + pred;
                }
            } else {
                free(tmp);
                return -6;
            }
            if (w) for (int i = 0; i < bs; i++) x[i] = (int64_t)((uint64_t)x[i] << w);
            nsf++;
        }
        /* undo stereo decorrelation */
        if (ca >= 8) {
            int64_t *l = tmp, *r = tmp + 65536;
            for (int i = 0; i < bs; i++) {
                int64_t a = l[i], s = r[i];
                if (ca == 8) { r[i] = a - s; }
                else if (ca == 9) { l[i] = a + s; }
                else {
                    int64_t mid = (int64_t)((uint64_t)a << 1) | (s & 1);
                    l[i] = (mid + s) >> 1;
                    r[i] = (mid - s) >> 1;
                }
            }
        }
        while (b.bit & 7) br_u(&b, 1);
        int64_t fend = b.bit >> 3;
        uint16_t c16 = (uint16_t)br_u(&b, 16);
        if (b.err || c16 != crc16(in + fstart, fend - fstart)) { free(tmp); return -7; }
        for (int i = 0; i < bs; i++)
            for (int c = 0; c < nch; c++) out[(total + i) * nch + c] = (int32_t)tmp[(size_t)c * 65536 + i];
        total += bs;
    }
    free(tmp);
    return total;
}

int64_t orc_decode_frames(const uint8_t *in, int64_t n, int ch, int bps, int32_t *out, int64_t cap_samples) {
    return decode_frames_impl(in, n, ch, bps, out, cap_samples, NULL, 0, NULL, 0);
}

/* as orc_decode_frames, and every subframe's type code (| residual partition order << 8 for FIXED / LPC) into
 * sf_out, frame-major (test diagnostics: the compression level's predictor and partition limits) */
int64_t orc_decode_frames_sf(const uint8_t *in, int64_t n, int ch, int bps, int32_t *out, int64_t cap_samples,
                             int16_t *sf_out, int64_t sf_cap) {
    return decode_frames_impl(in, n, ch, bps, out, cap_samples, NULL, 0, sf_out, sf_cap);
}

/* as orc_decode_frames, and the channel assignment code of every frame into ca_out (test diagnostics) */
int64_t orc_decode_frames_ca(const uint8_t *in, int64_t n, int ch, int bps, int32_t *out, int64_t cap_samples,
                             int8_t *ca_out, int64_t ca_cap) {
    return decode_frames_impl(in, n, ch, bps, out, cap_samples, ca_out, ca_cap, NULL, 0);
}

/* ------------------------------------------------------------------ streaming tiler (cli.py:690-763) */
/* Encode the band-0 tiles of a row-major [H][W] raster (row stride in elements) into per-tile frame
 * payloads, as create-streaming does per tile (band 1 only, per-tile min/max, converter.py:152-197).
 * arena receives the tiles back-to-back; tile_off has ntiles+1 entries.  Tiles are independent and
 * encoded with OpenMP when available (CPU baseline).  Returns total bytes or <0. */
int64_t orc_encode_tiles(const void *raster, int dtype, int64_t H, int64_t W, int64_t row_stride, int tile,
                         int sample_rate, int blocksize, uint8_t *arena, int64_t arena_cap, int64_t *tile_off,
                         double *tile_min, double *tile_max, int nthreads) {
    int64_t tr = (H + tile - 1) / tile, tc = (W + tile - 1) / tile, nt = tr * tc;
    int esz = dtype == 1 ? 1 : (dtype == 2 || dtype == 3) ? 2 : (dtype == 7 ? 8 : 4);
    int bits = (dtype <= 3) ? 16 : 24;
    int64_t *sizes = (int64_t *)calloc((size_t)nt, sizeof(int64_t));
    uint8_t **bufs = (uint8_t **)calloc((size_t)nt, sizeof(uint8_t *));
    int fail = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t t = 0; t < nt; t++) {
        int64_t r0 = (t / tc) * tile, c0 = (t % tc) * tile;
        int64_t h = H - r0 < tile ? H - r0 : tile, w = W - c0 < tile ? W - c0 : tile;
        int64_t n = h * w;
        uint8_t *px = (uint8_t *)malloc((size_t)(n * esz));
        for (int64_t r = 0; r < h; r++)
            memcpy(px + r * w * esz, (const uint8_t *)raster + ((r0 + r) * row_stride + c0) * esz, (size_t)(w * esz));
        int32_t *pcm = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
        int sbps = orc_normalize(px, dtype, n, bits, &tile_min[t], &tile_max[t], pcm);
        int64_t cap = n * (sbps / 8) + (n / blocksize + 1) * 64 + 64;
        bufs[t] = (uint8_t *)malloc((size_t)cap);
        sizes[t] = orc_encode_frames(pcm, n, 1, sbps, sample_rate, blocksize, bufs[t], cap);
        if (sizes[t] < 0) fail = 1;
        free(px); free(pcm);
    }
    int64_t off = 0;
    for (int64_t t = 0; t < nt; t++) {
        tile_off[t] = off;
        if (!fail && arena && off + sizes[t] <= arena_cap) memcpy(arena + off, bufs[t], (size_t)sizes[t]);
        off += sizes[t] > 0 ? sizes[t] : 0;
        free(bufs[t]);
    }
    tile_off[nt] = off;
    free(sizes); free(bufs);
    if (fail) return -1;
    if (arena && off > arena_cap) return -off;
    return off;
}
