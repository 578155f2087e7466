// frs_abi.hip -- exported C-ABI (include/flac_raster_amd.h): contexts, argument checks, host staging,
// profiling.  The product has no CPU fallback: without a gfx950 device every entry point fails with
// FRS_E_NODEV and the Python host raises.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>

#include <vector>

#include "frs_internal.h"

namespace frs {

void prof_begin(frs_ctx *ctx, const char *name, hipEvent_t *start, hipStream_t s) {
    (void)name;
    *start = nullptr;
    if (!ctx->prof) return;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    hipEventRecord(e, s ? s : ctx->stream);
    *start = e;
}

void prof_end(frs_ctx *ctx, const char *name, hipEvent_t start, hipStream_t s) {
    if (!ctx->prof || !start) return;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    hipEventRecord(e, s ? s : ctx->stream);
    ctx->ev_pending.push_back({std::string(name), {start, e}});
}

void prof_collect(frs_ctx *ctx) {
    for (auto &p : ctx->ev_pending) {
        float ms = 0.f;
        hipEventSynchronize(p.second.second);
        if (hipEventElapsedTime(&ms, p.second.first, p.second.second) == hipSuccess) {
            ProfEntry &e = ctx->prof_tab[p.first];
            e.total_ms += ms;
            e.count += 1;
        }
        hipEventDestroy(p.second.first);
        hipEventDestroy(p.second.second);
    }
    ctx->ev_pending.clear();
}

}  // namespace frs

static bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

static int check_desc(frs_ctx *ctx, const frs_encode_desc *d) {
    if (!d) { ctx->err = "null desc"; return FRS_E_ARG; }
    if (d->height <= 0 || d->width <= 0 || d->tile_h <= 0 || d->tile_w <= 0) { ctx->err = "bad geometry"; return FRS_E_ARG; }
    if (d->row_stride < d->width) { ctx->err = "row_stride < width"; return FRS_E_ARG; }
    if (d->nbands < 1 || d->nbands > frs::kMaxChannels) { ctx->err = "nbands must be 1..8 (FLAC channels)"; return FRS_E_ARG; }
    if (frs::dtype_size(d->dtype) == 0) { ctx->err = "bad dtype"; return FRS_E_ARG; }
    if (d->blocksize != 4096) { ctx->err = "blocksize must be 4096 (converter.py:205)"; return FRS_E_UNSUPPORTED; }
    // levels 0..8 (docs/sonos-pyflac.txt:6926-6934): level 5 on the fast kernels, the others (subdivide_tukey windows at
    // 6..8, loose mid/side at 1 / 4 on two channels) on the generic kernels
    if (d->compression_level < 0 || d->compression_level > 8) { ctx->err = "compression level must be 0..8"; return FRS_E_ARG; }
    if (d->bits_per_sample != 16 && d->bits_per_sample != 24) { ctx->err = "bits_per_sample must be 16 or 24"; return FRS_E_ARG; }
    if (d->sample_rate <= 0 || d->sample_rate > 655350) { ctx->err = "bad sample rate"; return FRS_E_ARG; }
    if (d->norm_mode != 0 && d->norm_mode != 1) { ctx->err = "bad norm_mode"; return FRS_E_ARG; }
    if (d->norm_mode == 1 && !(d->dtype == FRS_DT_U8 || d->dtype == FRS_DT_U16 || d->dtype == FRS_DT_I16 ||
                               d->dtype == FRS_DT_I32 || d->dtype == FRS_DT_F32)) {
        ctx->err = "spatial (raw-frames) normalisation gives a 64-bit sample array for this dtype; pyflac rejects it";
        return FRS_E_UNSUPPORTED;
    }
    const int64_t tiles = ((d->height + d->tile_h - 1) / d->tile_h) * ((d->width + d->tile_w - 1) / d->tile_w);
    if (d->tile_begin < 0 || d->tile_end > tiles || d->tile_begin > d->tile_end) { ctx->err = "bad tile range"; return FRS_E_ARG; }
    if (d->nbands > 1 && d->band_stride < d->row_stride * d->height) { ctx->err = "band_stride too small"; return FRS_E_ARG; }
    return FRS_OK;
}

extern "C" {

int frs_abi_version(void) { return FRS_ABI_VERSION; }

int frs_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int k = 0;
    for (int i = 0; i < n; i++)
        if (is_gfx950(i)) k++;
    return k;
}

int frs_ctx_create(int device, frs_ctx **out) {
    if (!out) return FRS_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return FRS_E_NODEV;
    if (!is_gfx950(device)) return FRS_E_NODEV;
    frs_ctx *ctx = new frs_ctx();
    ctx->device = device;
    const char *fg = getenv("FRS_FORCE_GENERIC");
    ctx->force_generic = fg && fg[0] == '1';
    const char *dl = getenv("FRS_DECODE_LANE");
    ctx->decode_lane = dl ? (dl[0] == '1' ? 1 : 0) : -1;
    const char *po = getenv("FRS_PIPE_OPT");
    ctx->pipe_opt = !(po && atoi(po) == 0);
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return FRS_E_HIP;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        ctx->num_cus = cus;
    *out = ctx;
    return FRS_OK;
}

void frs_ctx_destroy(frs_ctx *ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    frs::prof_collect(ctx);
    DevBuf *bufs[] = {&ctx->tiles, &ctx->norms, &ctx->analysis, &ctx->slots, &ctx->frame_bytes, &ctx->frame_off,
                      &ctx->window, &ctx->tile_sizes, &ctx->luts, &ctx->status, &ctx->frame_tile, &ctx->hdr_tab, &ctx->wave_tab, &ctx->plist, &ctx->lpc_cand, &ctx->sub_est, &ctx->st_pick, &ctx->window_hi, &ctx->loose_assign, &ctx->loose_lead, &ctx->sub_slots, &ctx->sub_bits, &ctx->mc_bytes, &ctx->raster_stage, &ctx->arena_stage, &ctx->host_pack,
                      &ctx->dec_cand, &ctx->dec_count, &ctx->dec_pcm, &ctx->dec_soff, &ctx->dec_next, &ctx->dec_status, &ctx->dec_fb, &ctx->dec_sel, &ctx->dec_crc,
                      &ctx->dec_chass};
    for (DevBuf *b : bufs) b->release();
    ctx->pin.release();
    ctx->ring[0].release();
    ctx->ring[1].release();
    if (ctx->h2d_stream) hipStreamDestroy(ctx->h2d_stream);
    if (ctx->d2h_stream) hipStreamDestroy(ctx->d2h_stream);
    hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *frs_last_error(const frs_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void *frs_ctx_stream(frs_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int frs_profile_enable(frs_ctx *ctx, int on) {
    if (!ctx) return FRS_E_ARG;
    ctx->prof = on != 0;
    return FRS_OK;
}

double frs_profile_avg_ms(frs_ctx *ctx, const char *kernel) {
    if (!ctx || !kernel) return -1.0;
    auto it = ctx->prof_tab.find(kernel);
    if (it == ctx->prof_tab.end() || it->second.count == 0) return -1.0;
    return it->second.total_ms / it->second.count;
}

void frs_profile_reset(frs_ctx *ctx) {
    if (ctx) ctx->prof_tab.clear();
}

int64_t frs_encode_arena_bound(const frs_encode_desc *desc) {
    if (!desc) return -1;
    return frs::arena_bound(desc);
}

int frs_encode_tiles_device(frs_ctx *ctx, const frs_encode_desc *desc, const void *raster_dev, void *arena_dev,
                            int64_t arena_cap, int64_t *tile_off, double *tile_min, double *tile_max,
                            int32_t *stream_bps) {
    if (!ctx) return FRS_E_ARG;
    int rc = check_desc(ctx, desc);
    if (rc) return rc;
    if (!raster_dev || !arena_dev || !tile_off || !tile_min || !tile_max) { ctx->err = "null pointer"; return FRS_E_ARG; }
    if (hipSetDevice(ctx->device) != hipSuccess) return FRS_E_HIP;
    return frs::encode_job(ctx, desc, raster_dev, arena_dev, arena_cap, tile_off, tile_min, tile_max, stream_bps);
}

}  // extern "C"

// memcpy by up to `nt` threads over contiguous ranges (host staging into pinned memory runs at a fraction of the
// memory bandwidth on one thread)
static void par_memcpy(void *dst, const void *src, size_t n, int nt) {
    if (n < ((size_t)8 << 20) || nt <= 1) {
        memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t c = ((n + nt - 1) / nt + 4095) & ~(size_t)4095;
    for (int i = 0; i < nt; i++) {
        const size_t a = std::min(n, (size_t)i * c), b = std::min(n, a + c);
        if (b > a)
            th.emplace_back([=] { memcpy(static_cast<char *>(dst) + a, static_cast<const char *>(src) + a, b - a); });
    }
    for (auto &t : th) t.join();
}

static int host_threads() {
    if (const char *e = getenv("FRS_HOST_THREADS")) return std::max(1, atoi(e));
    if (const char *e = getenv("OMP_NUM_THREADS")) return std::max(1, std::min(16, atoi(e)));
    return (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// Host-pointer encode of a single-band job (create-streaming band 1) in tile-row batches, so the PCIe transfers hide
// behind each other and behind the kernels: batch b + 1 is copied into a pinned ring slot by `nt` host threads and
// DMA'd on its own stream while batch b encodes on the context's stream, and batch b's frames go back on a third
// stream while batch b + 1 encodes.  Frames land in arena_host exactly as one whole-job encode would put them.
static int encode_tiles_batched(frs_ctx *ctx, const frs_encode_desc *desc, const uint8_t *src, size_t es,
                                uint8_t *arena_host, int64_t arena_cap, int64_t *tile_off, double *tile_min,
                                double *tile_max, int32_t *stream_bps, int64_t batch_rows) {
    const int64_t tcols = (desc->width + desc->tile_w - 1) / desc->tile_w;
    const int64_t t_lo = desc->tile_begin, t_hi = desc->tile_end;
    const int64_t row_bytes = desc->row_stride * (int64_t)es;
    const uint8_t *band = src + (size_t)desc->band0 * desc->band_stride * es;
    // device copy of the band rows the job touches, and one arena for the whole job
    const int64_t r_lo = (t_lo / tcols) * desc->tile_h;
    const int64_t r_hi = std::min<int64_t>(desc->height, ((t_hi - 1) / tcols + 1) * desc->tile_h);
    FRS_HIP(ctx->raster_stage.ensure((size_t)((r_hi - r_lo) * row_bytes)));
    const int64_t bound = frs::arena_bound(desc);
    FRS_HIP(ctx->arena_stage.ensure((size_t)bound));
    if (!ctx->h2d_stream) FRS_HIP(hipStreamCreateWithFlags(&ctx->h2d_stream, hipStreamNonBlocking));
    if (!ctx->d2h_stream) FRS_HIP(hipStreamCreateWithFlags(&ctx->d2h_stream, hipStreamNonBlocking));
    const size_t slot = (size_t)(batch_rows * desc->tile_h * row_bytes);
    FRS_HIP(ctx->ring[0].ensure(slot));
    FRS_HIP(ctx->ring[1].ensure(slot));
    // batches of whole tile rows (the first and last may be partial rows of the tile range)
    struct Batch { int64_t t0, t1, r0, r1; };
    std::vector<Batch> B;
    for (int64_t t = t_lo; t < t_hi;) {
        const int64_t tr = t / tcols;
        const int64_t t1 = std::min(t_hi, (tr + batch_rows) * tcols);
        const int64_t r0 = tr * desc->tile_h;
        const int64_t r1 = std::min<int64_t>(desc->height, ((t1 - 1) / tcols + 1) * desc->tile_h);
        B.push_back({t, t1, r0, r1});
        t = t1;
    }
    const int nt = host_threads();
    hipEvent_t up[2] = {nullptr, nullptr}, down = nullptr;
    // every exit below goes through the tail that drains the copy streams and destroys the events: a pending D2H
    // must not land in arena_host after the caller saw the error and freed it
    auto tail = [&](int rc_) -> int {
        if (ctx->h2d_stream) hipStreamSynchronize(ctx->h2d_stream);
        if (ctx->d2h_stream) hipStreamSynchronize(ctx->d2h_stream);
        for (auto &e : up)
            if (e) hipEventDestroy(e);
        if (down) hipEventDestroy(down);
        return rc_;
    };
    for (auto &e : up)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return tail(FRS_E_HIP);
    if (hipEventCreateWithFlags(&down, hipEventDisableTiming) != hipSuccess) return tail(FRS_E_HIP);
    const int rc = [&]() -> int {
    bool used[2] = {false, false};
    int rc = FRS_OK;
    // the raster's last row ends `width` elements after its start (a strided descriptor need not hold the stride's
    // padding after it): a batch that reaches the last row copies only that much of it
    const int64_t last_row_short = (desc->row_stride - desc->width) * (int64_t)es;
    auto stage = [&](size_t b) -> int {  // host copy into ring slot b % 2, then its DMA
        const int k = (int)(b & 1);
        if (used[k]) FRS_HIP(hipEventSynchronize(up[k]));  // the slot's previous DMA has drained
        const size_t n = (size_t)((B[b].r1 - B[b].r0) * row_bytes - (B[b].r1 == desc->height ? last_row_short : 0));
        par_memcpy(ctx->ring[k].ptr, band + (size_t)B[b].r0 * row_bytes, n, nt);
        FRS_HIP(hipMemcpyAsync(ctx->raster_stage.as<uint8_t>() + (size_t)(B[b].r0 - r_lo) * row_bytes, ctx->ring[k].ptr,
                               n, hipMemcpyHostToDevice, ctx->h2d_stream));
        FRS_HIP(hipEventRecord(up[k], ctx->h2d_stream));
        used[k] = true;
        return FRS_OK;
    };
    int64_t aoff = 0;
    if (B.size()) rc = stage(0);
    // the device raster view starts at row r_lo: tiles address rows relative to the descriptor's origin
    const uint8_t *dev_raster = ctx->raster_stage.as<uint8_t>() - (size_t)r_lo * row_bytes -
                                (size_t)desc->band0 * desc->band_stride * es;
    for (size_t b = 0; b < B.size() && rc == FRS_OK; b++) {
        // the next batch's host copy overlaps this batch's DMA (and the previous batch's D2H)
        if (b + 1 < B.size() && (rc = stage(b + 1)) != FRS_OK) break;
        FRS_HIP(hipStreamWaitEvent(ctx->stream, up[b & 1], 0));  // batch b's rows are on the device
        frs_encode_desc db = *desc;
        db.tile_begin = B[b].t0;
        db.tile_end = B[b].t1;
        const int64_t nbt = B[b].t1 - B[b].t0, i0 = B[b].t0 - t_lo;
        std::vector<int64_t> off(nbt + 1);
        rc = frs::encode_job(ctx, &db, dev_raster, ctx->arena_stage.as<uint8_t>() + aoff, bound - aoff, off.data(),
                             tile_min + i0, tile_max + i0, stream_bps);
        if (rc) break;
        const int64_t nbytes = off[nbt];
        if (aoff + nbytes > arena_cap) {
            tile_off[nbt + i0] = aoff + nbytes;
            ctx->err = "arena too small";
            rc = FRS_E_NOSPACE;
            break;
        }
        for (int64_t i = 0; i <= nbt; i++) tile_off[i0 + i] = aoff + off[i];
        FRS_HIP(hipEventRecord(down, ctx->stream));
        FRS_HIP(hipStreamWaitEvent(ctx->d2h_stream, down, 0));
        FRS_HIP(hipMemcpyAsync(arena_host + aoff, ctx->arena_stage.as<uint8_t>() + aoff, (size_t)nbytes,
                               hipMemcpyDeviceToHost, ctx->d2h_stream));
        aoff += nbytes;
    }
    return rc;
    }();
    return tail(rc);
}

extern "C" {

int frs_encode_tiles(frs_ctx *ctx, const frs_encode_desc *desc, const void *raster_host, uint8_t *arena_host,
                     int64_t arena_cap, int64_t *tile_off, double *tile_min, double *tile_max, int32_t *stream_bps) {
    if (!ctx) return FRS_E_ARG;
    int rc = check_desc(ctx, desc);
    if (rc) return rc;
    if (!raster_host || !arena_host || !tile_off) { ctx->err = "null pointer"; return FRS_E_ARG; }
    FRS_HIP(hipSetDevice(ctx->device));
    const int es = frs::dtype_size(desc->dtype);
    const int64_t nb = desc->nbands > 1 ? desc->band0 + desc->nbands : desc->band0 + 1;
    const int64_t elems = (nb - 1) * desc->band_stride + (desc->height - 1) * desc->row_stride + desc->width;
    const size_t rbytes = (size_t)elems * es;
    // large single-band jobs of several tile rows: batched, overlapped transfers (create-streaming band 1)
    const int64_t tcols = (desc->width + desc->tile_w - 1) / desc->tile_w;
    const int64_t trows = (desc->tile_end - 1) / tcols - desc->tile_begin / tcols + 1;
    const int64_t trow_bytes = (int64_t)desc->tile_h * desc->row_stride * es;
    if (desc->nbands == 1 && trows >= 4 && rbytes >= ((size_t)64 << 20)) {
        const int64_t batch_rows = std::max<int64_t>(1, std::min<int64_t>(trows / 4, ((int64_t)256 << 20) / trow_bytes));
        return encode_tiles_batched(ctx, desc, static_cast<const uint8_t *>(raster_host), (size_t)es, arena_host,
                                    arena_cap, tile_off, tile_min, tile_max, stream_bps, batch_rows);
    }
    FRS_HIP(ctx->raster_stage.ensure(rbytes));
    FRS_HIP(hipMemcpyAsync(ctx->raster_stage.ptr, raster_host, rbytes, hipMemcpyHostToDevice, ctx->stream));
    const int64_t bound = frs::arena_bound(desc);
    FRS_HIP(ctx->arena_stage.ensure((size_t)bound));
    const int64_t ntiles = desc->tile_end - desc->tile_begin;
    rc = frs::encode_job(ctx, desc, ctx->raster_stage.ptr, ctx->arena_stage.ptr, bound, tile_off, tile_min, tile_max,
                         stream_bps);
    if (rc) return rc;
    const int64_t total = tile_off[ntiles];
    if (total > arena_cap) {
        ctx->err = "arena too small";
        return FRS_E_NOSPACE;
    }
    FRS_HIP(hipMemcpyAsync(arena_host, ctx->arena_stage.ptr, (size_t)total, hipMemcpyDeviceToHost, ctx->stream));
    FRS_HIP(hipStreamSynchronize(ctx->stream));
    return FRS_OK;
}

}  // extern "C"

// argument checks shared by every decode entry point, before anything is sized or copied: the geometry ranges and
// non-decreasing stream / sample offsets (reversed offsets would make a negative byte count a huge size_t)
static int check_decode_args(frs_ctx *ctx, const int64_t *stream_off, const int64_t *pcm_off, int32_t nstreams,
                             int32_t channels, int32_t bps, int32_t blocksize) {
    if (!stream_off || !pcm_off || nstreams < 0 || channels < 1 || channels > 8 || blocksize < 16 ||
        blocksize > 65535 || bps < 4 || bps > 32) {
        ctx->err = "bad decode arguments";
        return FRS_E_ARG;
    }
    for (int s = 1; s <= nstreams; s++)
        if (stream_off[s] < stream_off[s - 1] || pcm_off[s] < pcm_off[s - 1]) {
            ctx->err = "stream and sample offsets must be non-decreasing";
            return FRS_E_ARG;
        }
    if (nstreams > 0 && (stream_off[0] < 0 || pcm_off[0] < 0)) {
        ctx->err = "negative stream or sample offset";
        return FRS_E_ARG;
    }
    return FRS_OK;
}

// shared argument checks and stream rebasing of the decode entry points: only [stream_off[0],
// stream_off[nstreams]) is scanned, so a tile query inside a large arena touches just its own bytes
static int decode_entry(frs_ctx *ctx, const uint8_t *blob_dev, const int64_t *stream_off, int32_t nstreams,
                        int32_t channels, int32_t bps, int32_t blocksize, int32_t *pcm_dev, const int64_t *pcm_off,
                        const double *dmin, const double *dmax, int32_t out_dtype, void *out_dev) {
    if (!blob_dev) {
        ctx->err = "bad decode arguments";
        return FRS_E_ARG;
    }
    if (int rc = check_decode_args(ctx, stream_off, pcm_off, nstreams, channels, bps, blocksize)) return rc;
    if (out_dev && (!dmin || !dmax || frs::dtype_size(out_dtype) == 0)) {
        ctx->err = "bad decode arguments (data_min/data_max/out dtype)";
        return FRS_E_ARG;
    }
    if (!out_dev && !pcm_dev) {
        ctx->err = "bad decode arguments (no output)";
        return FRS_E_ARG;
    }
    FRS_HIP(hipSetDevice(ctx->device));
    if (nstreams == 0) return FRS_OK;
    const int64_t base = stream_off[0];
    std::vector<int64_t> rel(nstreams + 1);
    for (int s = 0; s <= nstreams; s++) {
        rel[s] = stream_off[s] - base;
        if (s && (rel[s] < rel[s - 1] || pcm_off[s] < pcm_off[s - 1])) {
            ctx->err = "stream and sample offsets must be non-decreasing";
            return FRS_E_ARG;
        }
    }
    return frs::decode_job(ctx, blob_dev + base, rel[nstreams], rel.data(), nstreams, channels, bps, blocksize,
                           pcm_dev, pcm_off, dmin, dmax, out_dtype, out_dev);
}

extern "C" {

int frs_decode_frames_device(frs_ctx *ctx, const uint8_t *blob_dev, const int64_t *stream_off, int32_t nstreams,
                             int32_t channels, int32_t bps, int32_t blocksize, int32_t *pcm_dev, const int64_t *pcm_off) {
    if (!ctx) return FRS_E_ARG;
    if (!pcm_dev) { ctx->err = "bad decode arguments"; return FRS_E_ARG; }
    return decode_entry(ctx, blob_dev, stream_off, nstreams, channels, bps, blocksize, pcm_dev, pcm_off, nullptr,
                        nullptr, 0, nullptr);
}

int frs_decode_frames(frs_ctx *ctx, const uint8_t *blob_host, const int64_t *stream_off, int32_t nstreams,
                      int32_t channels, int32_t bps, int32_t blocksize, int32_t *pcm_host, const int64_t *pcm_off) {
    if (!ctx) return FRS_E_ARG;
    if (!blob_host || !pcm_host) { ctx->err = "bad decode arguments"; return FRS_E_ARG; }
    if (int rc = check_decode_args(ctx, stream_off, pcm_off, nstreams, channels, bps, blocksize)) return rc;
    FRS_HIP(hipSetDevice(ctx->device));
    const int64_t nbytes = nstreams ? stream_off[nstreams] : 0;
    const int64_t nsamp = nstreams ? pcm_off[nstreams] : 0;
    FRS_HIP(ctx->raster_stage.ensure((size_t)nbytes + 16));
    FRS_HIP(ctx->arena_stage.ensure((size_t)nsamp * channels * 4 + 16));
    FRS_HIP(hipMemcpyAsync(ctx->raster_stage.ptr, blob_host, (size_t)nbytes, hipMemcpyHostToDevice, ctx->stream));
    int rc = frs_decode_frames_device(ctx, ctx->raster_stage.as<uint8_t>(), stream_off, nstreams, channels, bps,
                                      blocksize, ctx->arena_stage.as<int32_t>(), pcm_off);
    if (rc) return rc;
    FRS_HIP(hipMemcpyAsync(pcm_host, ctx->arena_stage.ptr, (size_t)nsamp * channels * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRS_HIP(hipStreamSynchronize(ctx->stream));
    return FRS_OK;
}

int frs_decode_tiles_device(frs_ctx *ctx, const uint8_t *blob_dev, const int64_t *stream_off, int32_t nstreams,
                            int32_t channels, int32_t bps, int32_t blocksize, const int64_t *pcm_off,
                            const double *data_min, const double *data_max, int32_t out_dtype, void *out_dev) {
    if (!ctx) return FRS_E_ARG;
    if (!out_dev) { ctx->err = "bad decode arguments (no output)"; return FRS_E_ARG; }
    return decode_entry(ctx, blob_dev, stream_off, nstreams, channels, bps, blocksize, nullptr, pcm_off, data_min,
                        data_max, out_dtype, out_dev);
}

int frs_decode_tile_device(frs_ctx *ctx, const uint8_t *blob_dev, int64_t start, int64_t end, int64_t count,
                           int32_t channels, int32_t bps, int32_t blocksize, double data_min, double data_max,
                           int32_t out_dtype, void *out_dev) {
    const int64_t soff[2] = {start, end}, poff[2] = {0, count};
    return frs_decode_tiles_device(ctx, blob_dev, soff, 1, channels, bps, blocksize, poff, &data_min, &data_max,
                                   out_dtype, out_dev);
}

int frs_decode_tiles(frs_ctx *ctx, const uint8_t *blob_host, const int64_t *stream_off, int32_t nstreams,
                     int32_t channels, int32_t bps, int32_t blocksize, const int64_t *pcm_off, const double *data_min,
                     const double *data_max, int32_t out_dtype, void *out_host) {
    if (!ctx) return FRS_E_ARG;
    const int es = frs::dtype_size(out_dtype);
    if (!blob_host || !out_host || es == 0) {
        ctx->err = "bad decode arguments";
        return FRS_E_ARG;
    }
    if (int rc = check_decode_args(ctx, stream_off, pcm_off, nstreams, channels, bps, blocksize)) return rc;
    FRS_HIP(hipSetDevice(ctx->device));
    if (nstreams == 0) return FRS_OK;
    const int64_t nbytes = stream_off[nstreams] - stream_off[0];
    const int64_t nout = (pcm_off[nstreams] - pcm_off[0]) * channels;
    FRS_HIP(ctx->raster_stage.ensure((size_t)nbytes + 16));
    FRS_HIP(ctx->arena_stage.ensure((size_t)nout * es + 16));
    // small jobs (a tile query): both copies through the context's page-locked ring (a host memcpy plus a DMA beat
    // the driver's pageable path: ~5 GB/s for a 512 KB tile)
    const bool small = nbytes <= ((int64_t)32 << 20) && nout * es <= ((int64_t)32 << 20);
    if (small) {
        FRS_HIP(ctx->ring[0].ensure((size_t)nbytes + 16));
        FRS_HIP(ctx->ring[1].ensure((size_t)nout * es + 16));
        memcpy(ctx->ring[0].ptr, blob_host + stream_off[0], (size_t)nbytes);
        FRS_HIP(hipMemcpyAsync(ctx->raster_stage.ptr, ctx->ring[0].ptr, (size_t)nbytes, hipMemcpyHostToDevice,
                               ctx->stream));
    } else {
        FRS_HIP(hipMemcpyAsync(ctx->raster_stage.ptr, blob_host + stream_off[0], (size_t)nbytes, hipMemcpyHostToDevice,
                               ctx->stream));
    }
    // stream and sample offsets relative to the first stream: the device output is the staging buffer itself
    std::vector<int64_t> rel(nstreams + 1), prel(nstreams + 1);
    for (int s = 0; s <= nstreams; s++) {
        rel[s] = stream_off[s] - stream_off[0];
        prel[s] = pcm_off[s] - pcm_off[0];
    }
    int rc = decode_entry(ctx, ctx->raster_stage.as<uint8_t>(), rel.data(), nstreams, channels, bps, blocksize, nullptr,
                          prel.data(), data_min, data_max, out_dtype, ctx->arena_stage.ptr);
    if (rc) return rc;
    uint8_t *dst = static_cast<uint8_t *>(out_host) + pcm_off[0] * channels * es;
    if (small) {
        FRS_HIP(hipMemcpyAsync(ctx->ring[1].ptr, ctx->arena_stage.ptr, (size_t)nout * es, hipMemcpyDeviceToHost,
                               ctx->stream));
        FRS_HIP(hipStreamSynchronize(ctx->stream));
        memcpy(dst, ctx->ring[1].ptr, (size_t)nout * es);
        return FRS_OK;
    }
    FRS_HIP(hipMemcpyAsync(dst, ctx->arena_stage.ptr, (size_t)nout * es, hipMemcpyDeviceToHost, ctx->stream));
    FRS_HIP(hipStreamSynchronize(ctx->stream));
    return FRS_OK;
}

int frs_denormalize_device(frs_ctx *ctx, const int32_t *pcm_dev, int64_t n, int32_t pcm_bps, double data_min,
                           double data_max, int32_t out_dtype, void *out_dev) {
    if (!ctx) return FRS_E_ARG;
    if (!pcm_dev || !out_dev || n < 0) { ctx->err = "bad denormalize arguments"; return FRS_E_ARG; }
    FRS_HIP(hipSetDevice(ctx->device));
    return frs::denormalize_job(ctx, pcm_dev, n, pcm_bps, data_min, data_max, out_dtype, out_dev);
}

int frs_denormalize(frs_ctx *ctx, const int32_t *pcm_host, int64_t n, int32_t pcm_bps, double data_min,
                    double data_max, int32_t out_dtype, void *out_host) {
    if (!ctx) return FRS_E_ARG;
    const int es = frs::dtype_size(out_dtype);
    if (!pcm_host || !out_host || n < 0 || es == 0) { ctx->err = "bad denormalize arguments"; return FRS_E_ARG; }
    FRS_HIP(hipSetDevice(ctx->device));
    FRS_HIP(ctx->dec_pcm.ensure((size_t)n * 4 + 16));
    FRS_HIP(ctx->raster_stage.ensure((size_t)n * es + 16));
    FRS_HIP(hipMemcpyAsync(ctx->dec_pcm.ptr, pcm_host, (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
    int rc = frs::denormalize_job(ctx, ctx->dec_pcm.as<int32_t>(), n, pcm_bps, data_min, data_max, out_dtype,
                                  ctx->raster_stage.ptr);
    if (rc) return rc;
    FRS_HIP(hipMemcpyAsync(out_host, ctx->raster_stage.ptr, (size_t)n * es, hipMemcpyDeviceToHost, ctx->stream));
    FRS_HIP(hipStreamSynchronize(ctx->stream));
    return FRS_OK;
}

void *frs_dev_malloc(frs_ctx *ctx, int64_t bytes) {
    if (!ctx || bytes <= 0) return nullptr;
    if (hipSetDevice(ctx->device) != hipSuccess) return nullptr;
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, (size_t)bytes);
    if (e != hipSuccess) {
        ctx->err = std::string("hipMalloc: ") + hipGetErrorString(e);
        return nullptr;
    }
    return p;
}

void frs_dev_free(frs_ctx *ctx, void *ptr) {
    if (!ctx || !ptr) return;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    hipFree(ptr);
}

void *frs_host_malloc(frs_ctx *ctx, int64_t bytes) {
    if (!ctx || bytes <= 0) return nullptr;
    if (hipSetDevice(ctx->device) != hipSuccess) return nullptr;
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, (size_t)bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        ctx->err = std::string("hipHostMalloc: ") + hipGetErrorString(e);
        return nullptr;
    }
    ctx->host_allocs.emplace_back(reinterpret_cast<uintptr_t>(p), (size_t)bytes);
    return p;
}

void frs_host_free(frs_ctx *ctx, void *ptr) {
    if (!ptr) return;
    if (ctx) {
        hipSetDevice(ctx->device);
        hipDeviceSynchronize();  // (copies on the context's side streams may still read or write it)
        ctx->unsynced = false;
        for (size_t k = 0; k < ctx->host_allocs.size(); k++)
            if (ctx->host_allocs[k].first == reinterpret_cast<uintptr_t>(ptr)) {
                ctx->host_allocs.erase(ctx->host_allocs.begin() + (long)k);
                break;
            }
    }
    hipHostFree(ptr);  // (ctx may be null: a buffer that outlived its context; its streams are gone)
}

int frs_memcpy_h2d(frs_ctx *ctx, void *dst_dev, const void *src_host, int64_t bytes) {
    if (!ctx) return FRS_E_ARG;
    if (bytes <= 0) return FRS_OK;
    FRS_HIP(hipSetDevice(ctx->device));
    FRS_HIP(hipMemcpyAsync(dst_dev, src_host, (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
    FRS_HIP(hipStreamSynchronize(ctx->stream));
    return FRS_OK;
}

int frs_memcpy_d2h(frs_ctx *ctx, void *dst_host, const void *src_dev, int64_t bytes) {
    if (!ctx) return FRS_E_ARG;
    if (bytes <= 0) return FRS_OK;
    FRS_HIP(hipSetDevice(ctx->device));
    FRS_HIP(hipMemcpyAsync(dst_host, src_dev, (size_t)bytes, hipMemcpyDeviceToHost, ctx->stream));
    FRS_HIP(hipStreamSynchronize(ctx->stream));
    return FRS_OK;
}

int frs_ctx_sync(frs_ctx *ctx) {
    if (!ctx) return FRS_E_ARG;
    ctx->unsynced = false;
    FRS_HIP(hipStreamSynchronize(ctx->stream));
    return FRS_OK;
}

int frs_synth_raster_device(frs_ctx *ctx, int16_t *dev, int32_t bands, int64_t height, int64_t width, int64_t row0,
                            int64_t full_height, uint64_t seed) {
    if (!ctx || !dev || bands < 1 || height < 0 || width < 1 || row0 < 0 || row0 + height > full_height) {
        if (ctx) ctx->err = "bad synth arguments";
        return FRS_E_ARG;
    }
    FRS_HIP(hipSetDevice(ctx->device));
    return frs::synth_job(ctx, dev, bands, height, width, row0, full_height, seed);
}

}  // extern "C"
