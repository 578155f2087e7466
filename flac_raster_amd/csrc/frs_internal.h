// frs_internal.h -- host-side context, device buffers and launcher entry points.
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/flac_raster_amd.h"
#include "frs_common.h"

// Grow-only device buffer owned by a context.
struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        if (ptr) hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
        size_t want = need + need / 8 + 4096;
        hipError_t e = hipMalloc(&ptr, want);
        if (e == hipSuccess) bytes = want;
        return e;
    }
    void release() {
        if (ptr) hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    template <typename T> T *as() const { return reinterpret_cast<T *>(ptr); }
};

// pinned host staging (small per-call H2D tables and the packed D2H results of the fast encode path): one
// allocation reused across calls, so the copies are DMA transfers instead of staged pageable copies
struct HostPin {
    void *ptr = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        if (ptr) hipHostFree(ptr);
        ptr = nullptr;
        bytes = 0;
        size_t want = need + need / 8 + 4096;
        hipError_t e = hipHostMalloc(&ptr, want, hipHostMallocDefault);
        if (e == hipSuccess) bytes = want;
        return e;
    }
    void release() {
        if (ptr) hipHostFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    template <typename T> T *at(size_t off) const { return reinterpret_cast<T *>(static_cast<char *>(ptr) + off); }
};

struct ProfEntry {
    double total_ms = 0.0;
    int count = 0;
};

struct frs_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    std::string err;
    // encode scratch
    DevBuf tiles, norms, analysis, slots, frame_bytes, frame_off, window, tile_sizes, luts, status, frame_tile,
        hdr_tab, wave_tab, plist, sub_slots, sub_bits, mc_bytes;
    int hdr_tab_n = -1, hdr_tab_sr = -1;  // cached frame-header table (fast encode path)
    bool force_generic = false;  // testing: route every job through the generic kernels
    // host staging (pinned)
    DevBuf raster_stage, arena_stage;  // device copies for the host-pointer entry points
    HostPin pin;                       // pinned staging of the fast encode path (tiles, wave table, results)
    HostPin ring[2];                   // pinned upload ring of the batched host-pointer encode (frs_encode_tiles)
    hipStream_t h2d_stream = nullptr, d2h_stream = nullptr;  // its copy engines' streams (created on first use)
    DevBuf host_pack;                  // device side of the packed fast-path results
    // decode scratch
    DevBuf dec_cand, dec_count, dec_pcm, dec_soff, dec_next, dec_status, dec_fb, dec_sel, dec_chass, dec_crc;
    int decode_lane = -1;    // FRS_DECODE_LANE=0/1 (tests): force the pipelined / lane-per-frame decoder
    bool pipe_opt = true;    // FRS_PIPE_OPT=0 (tests): no optimistic small-range decode (read once, not per query)
    uint32_t dec_epoch = 0;  // call counter tagging the candidate selection's look-back words (24 bits, never 0)
    // profiling
    bool prof = false;
    std::map<std::string, ProfEntry> prof_tab;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> ev_pending;
    // cached window (blocksize)
    int window_bs = 0;
    // cached job geometry of the fast encode path: the tile table (partial frames marked), the analysis wave table,
    // the partial-frame list and frame -> tile map stay on the device while the descriptor's geometry repeats (a
    // bench or a server encoding same-shaped jobs skips their rebuild and uploads)
    std::vector<int64_t> geo_key;      // descriptor geometry the cache holds (empty: nothing cached)
    std::vector<frs::TileGeom> geo_tiles;  // host tile table, partial frames marked
    std::vector<int64_t> geo_plist;    // partial-frame list
    int64_t geo_nframes = 0;
    int geo_nwaves = 0;
    void *geo_ptrs[4] = {nullptr, nullptr, nullptr, nullptr};  // tiles, wave_tab, plist, frame_tile as uploaded
    // subdivide_tukey levels (6..8): LPC candidates per coded signal, the tukey(0.5 / parts) window; loose mid/side:
    // per-frame assignment of the group leaders and the leader frame list
    DevBuf lpc_cand, window_hi, loose_assign, loose_lead;
    int window_hi_bs = 0, window_hi_parts = 0;
    DevBuf sub_est, st_pick;  // two-channel fast path: subframe estimates (L, R, M, S), the assignment per frame
    DevBuf zero_sub;          // raw-frames tiles: all-zero subframe flags (k_zero_subframes)
    // page-locked host allocations of this context (frs_host_malloc): a C5 decode whose output lies in one returns
    // when the kernel's last work-group has published it, before the stream's completion signal (`unsynced` then
    // makes the next call check the stream for an asynchronous fault first)
    std::vector<std::pair<uintptr_t, size_t>> host_allocs;
    bool unsynced = false;
    bool is_host_alloc(const void *p, size_t n) const {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        for (const auto &r : host_allocs)
            if (a >= r.first && a + n <= r.first + r.second) return true;
        return false;
    }
};

#define FRS_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ctx->err = std::string(#call) + ": " + hipGetErrorString(e_);              \
            return FRS_E_HIP;                                                          \
        }                                                                              \
    } while (0)

namespace frs {
// A call after an early-returning C5 decode (frs_ctx::unsynced): a fault of that kernel surfaces here, in the next
// call on the context, instead of in some later unrelated HIP call.
inline int check_unsynced(frs_ctx *ctx) {
    if (!ctx->unsynced) return FRS_OK;
    ctx->unsynced = false;
    const hipError_t e = hipStreamQuery(ctx->stream);
    if (e != hipSuccess && e != hipErrorNotReady) {
        ctx->err = std::string("an earlier decode's kernel failed: ") + hipGetErrorString(e);
        return FRS_E_HIP;
    }
    return FRS_OK;
}
// Kernel timing helpers (no-ops unless ctx->prof).
void prof_begin(frs_ctx *ctx, const char *name, hipEvent_t *start, hipStream_t s = nullptr);
void prof_end(frs_ctx *ctx, const char *name, hipEvent_t start, hipStream_t s = nullptr);
void prof_collect(frs_ctx *ctx);

int encode_job(frs_ctx *ctx, const frs_encode_desc *d, const void *raster_dev, void *arena_dev, int64_t arena_cap,
               int64_t *tile_off, double *tile_min, double *tile_max, int32_t *stream_bps);
// Decode the frames of nstreams streams.  out_dev == nullptr: int32 PCM into pcm_dev.  Otherwise the samples are
// de-normalised in the decode kernels (converter.py:88-110) with per-stream dmin/dmax into out_dev (out_dtype),
// and pcm_dev is only an optional int32 scratch (multi-channel / wide streams).
int decode_job(frs_ctx *ctx, const uint8_t *blob_dev, int64_t blob_bytes, const int64_t *stream_off,
               int32_t nstreams, int32_t channels, int32_t bps, int32_t blocksize, int32_t *pcm_dev,
               const int64_t *pcm_off, const double *dmin = nullptr, const double *dmax = nullptr,
               int32_t out_dtype = 0, void *out_dev = nullptr);
int denormalize_job(frs_ctx *ctx, const int32_t *pcm_dev, int64_t n, int pcm_bps, double dmin, double dmax,
                    int32_t out_dtype, void *out_dev);
int64_t arena_bound(const frs_encode_desc *d);
int synth_job(frs_ctx *ctx, int16_t *dev, int bands, int64_t height, int64_t width, int64_t row0, int64_t full_height,
              uint64_t seed);
int dtype_size(int dt);
}  // namespace frs
