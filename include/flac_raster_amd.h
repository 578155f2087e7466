/*
 * flac_raster_amd.h -- C-ABI of the MI355X (gfx950) spatial-FLAC codec library
 *                      (libflac_raster_amd.so, built from the HIP sources in flac_raster_amd/csrc).
 *
 * This is the drop-in boundary for the reference's hot path.  In the reference
 * (Youssef-Harby/flac-raster @ 2025-07-25) that seam is Python -> pyFLAC 3.0.0 (cffi) -> libFLAC 1.4.3:
 *
 *   reference call site                                     replaced by
 *   ------------------------------------------------------  ------------------------------------------
 *   converter.py:56-86   _normalize_to_audio (numpy)        frs_encode_tiles*   (fused, on device)
 *   converter.py:185-194 band interleave/reshape            frs_encode_tiles*   (desc.nbands channels)
 *   converter.py:201-216 pyflac.StreamEncoder(...).process   frs_encode_tiles*   (whole tiles, no per-frame
 *                        + finish()  (sonos-pyflac.txt:        write callback; frames land in one arena)
 *                        1968-2014, 2175-2212; libFLAC
 *                        FLAC__stream_encoder_process_interleaved)
 *   cli.py:690-763       create_streaming per-tile loop     frs_encode_tiles*   (all tiles in one call)
 *   converter.py:241-242 pyflac.FileDecoder(path).process()  frs_decode_frames*  (batched frames -> int32)
 *                        (sonos-pyflac.txt:1584-1640, 1809-1854; libFLAC
 *                        FLAC__stream_decoder_process_until_end_of_stream)
 *   converter.py:88-110  _denormalize_from_audio (numpy)    frs_denormalize*
 *
 * Container bytes (STREAMINFO, VORBIS_COMMENT tags, PADDING, streaming index JSON) are built by the
 * Python host (flac_raster_amd/container.py): they are text/metadata, not data-parallel work.
 *
 * Conventions: plain C types only; every buffer is caller-allocated.  Functions ending in _device take
 * device pointers (hipMalloc memory of the context's device) and run on the context's HIP
 * stream; the others take host pointers and copy through the context's staging buffers.  All functions
 * return FRS_OK (0) or a negative frs_status; frs_last_error() gives the message.  A context is bound to
 * one device and must not be used from two host threads at once (one context per GPU / rank).
 */
#ifndef FLAC_RASTER_AMD_H
#define FLAC_RASTER_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FRS_ABI_VERSION 1

typedef struct frs_ctx frs_ctx;

/* element types (numpy dtype of the raster) */
enum frs_dtype {
    FRS_DT_U8 = 1,
    FRS_DT_U16 = 2,
    FRS_DT_I16 = 3,
    FRS_DT_I32 = 4,
    FRS_DT_U32 = 5,
    FRS_DT_F32 = 6,
    FRS_DT_F64 = 7
};

enum frs_status {
    FRS_OK = 0,
    FRS_E_ARG = -1,         /* bad argument */
    FRS_E_HIP = -2,         /* HIP runtime error */
    FRS_E_NOSPACE = -3,     /* output buffer too small; required size reported where documented */
    FRS_E_CORRUPT = -4,     /* undecodable FLAC data */
    FRS_E_UNSUPPORTED = -5, /* valid but not supported by this build */
    FRS_E_NODEV = -6        /* no gfx950 device */
};

/* Geometry of one encode job.  The raster is [nbands_total][height][width] elements with the given
 * strides (elements).  Tiles are tile_h x tile_w windows in row-major tile order (cli.py:691-692),
 * edge tiles truncated.  Each tile is one FLAC stream whose channels are `nbands` bands starting at
 * band `band0` (create-streaming: nbands = 1, band0 = 0 -- cli.py:699 reads band 1 only; plain convert:
 * one tile covering the raster with nbands = count, converter.py:185-189).  Only the tiles
 * [tile_begin, tile_end) of the row-major tile grid are encoded (multi-GPU sharding). */
typedef struct {
    int64_t height, width;      /* raster size in pixels */
    int64_t row_stride;         /* elements between rows */
    int64_t band_stride;        /* elements between bands */
    int32_t dtype;              /* enum frs_dtype */
    int32_t band0, nbands;      /* channels of each stream */
    int32_t tile_h, tile_w;     /* tile size in pixels */
    int32_t blocksize;          /* FLAC block size (4096, converter.py:205) */
    int32_t sample_rate;        /* STREAMINFO / frame header sample rate (converter.py:25-54) */
    int32_t bits_per_sample;    /* 16 or 24 from _calculate_audio_params (converter.py:29-37) */
    int32_t compression_level;  /* 0..8 (cli.py:36-37; create-streaming uses 5, cli.py:733); 6..8 with
                                   subdivide_tukey apodizations, 1 / 4 on two bands with loose mid/side */
    int32_t norm_mode;          /* FRS_NORM_CONVERTER or FRS_NORM_SPATIAL */
    int64_t tile_begin, tile_end;
} frs_encode_desc;

/* sample normalisation of an encode job */
enum frs_norm_mode {
    FRS_NORM_CONVERTER = 0, /* converter.py:56-86: min/max -> int16 (bps 16) or int32 x 8388607 (bps 24) */
    FRS_NORM_SPATIAL = 1    /* spatial_encoder.py:229-248: dtype-fixed float32 scaling, pyflac casts to int32
                               (32-bit stream, samples in {-1, 0, 1}: the lossy raw-frames format) */
};

int frs_abi_version(void);
/* number of usable gfx950 devices (0 when none) */
int frs_device_count(void);
int frs_ctx_create(int device, frs_ctx **out);
void frs_ctx_destroy(frs_ctx *ctx);
const char *frs_last_error(const frs_ctx *ctx);

/* Upper bound of the arena bytes frs_encode_tiles* can need for desc (all frames verbatim). */
int64_t frs_encode_arena_bound(const frs_encode_desc *desc);

/* Encode tiles [tile_begin, tile_end) into FLAC *frames* (no stream header), tile after tile, into
 * `arena` (device memory for _device).  On return (host arrays, one entry per encoded tile):
 *   tile_off[i]..tile_off[i+1]  arena byte range of tile i's frames   (tile_off has ntiles+1 entries)
 *   tile_min[i], tile_max[i]    float(np.min(tile)), float(np.max(tile)) over the tile's channels
 *                               (converter.py:152-153), used for the GEOSPATIAL_DATA_MIN/MAX tags
 *   *stream_bps                 bits per sample written in STREAMINFO (16 or 32, pyflac
 *                               encoder.py: itemsize*8, sonos-pyflac.txt:1986-1992)
 * Frames are bit-identical to libFLAC 1.4.3 level 5 fed through pyflac with blocksize `blocksize`.
 * FRS_E_NOSPACE: arena_cap too small; tile_off[ntiles] holds the bytes required. */
int frs_encode_tiles_device(frs_ctx *ctx, const frs_encode_desc *desc, const void *raster_dev, void *arena_dev,
                            int64_t arena_cap, int64_t *tile_off, double *tile_min, double *tile_max,
                            int32_t *stream_bps);
int frs_encode_tiles(frs_ctx *ctx, const frs_encode_desc *desc, const void *raster_host, uint8_t *arena_host,
                     int64_t arena_cap, int64_t *tile_off, double *tile_min, double *tile_max,
                     int32_t *stream_bps);

/* Decode the FLAC frames of `nstreams` streams.  Stream s occupies blob[stream_off[s], stream_off[s+1])
 * and must start at its first frame (the caller skips the metadata blocks; container.py parses them).
 * channels/bps describe every stream (STREAMINFO); samples are written interleaved as int32 at
 * pcm_out + pcm_off[s] * channels, pcm_off has nstreams+1 entries (per-stream sample counts known
 * from the tile windows).  Frames are located by sync code + CRC-8/CRC-16 and decoded in parallel: one lane per
 * frame for large calls (thousands of frames), two waves per frame (a Rice-decoding and a restoring wave) for a
 * single tile, one wave per frame for 32-bit / wide streams.  Ranges of any size are accepted (64-bit positions);
 * a stream with more sync-code
 * candidates than the capacity (2 x frames + bytes / 1024 + 4096) is rejected with FRS_E_CORRUPT before
 * anything is written past it. */
int frs_decode_frames_device(frs_ctx *ctx, const uint8_t *blob_dev, const int64_t *stream_off, int32_t nstreams,
                             int32_t channels, int32_t bps, int32_t blocksize, int32_t *pcm_dev,
                             const int64_t *pcm_off);
int frs_decode_frames(frs_ctx *ctx, const uint8_t *blob_host, const int64_t *stream_off, int32_t nstreams,
                      int32_t channels, int32_t bps, int32_t blocksize, int32_t *pcm_host, const int64_t *pcm_off);

/* Decode + de-normalise in one pass: replaces converter.py:241-282 as a whole (pyflac FileDecoder ->
 * soundfile PCM_16 WAV -> _denormalize_from_audio, sonos-pyflac.txt:1584-1640, converter.py:88-110) for
 * `nstreams` tiles at once.  Same stream layout as frs_decode_frames; stream s carries its own
 * GEOSPATIAL_DATA_MIN/MAX (data_min[s], data_max[s], converter.py:375-427) and its samples are written
 * interleaved as out_dtype at out + (pcm_off[s] + i) * channels + c -- the int32 PCM never reaches memory for
 * mono 16-bit streams (create-streaming tiles).  out_dev is device memory, or page-locked host memory from
 * frs_host_malloc: the kernels then store the result straight into host memory (no separate D2H copy; a C5 query
 * returns one tile this way).  On FRS_OK the result is complete and visible to the host: a device-memory out_dev
 * after the call has synchronised the context stream; page-locked host memory from frs_host_malloc as soon as the
 * kernels have published it (system-scope fences), possibly before the stream has retired -- a fault of those kernels
 * is then reported by the next call on the context.  Errors as frs_decode_frames. */
int frs_decode_tiles_device(frs_ctx *ctx, const uint8_t *blob_dev, const int64_t *stream_off, int32_t nstreams,
                            int32_t channels, int32_t bps, int32_t blocksize, const int64_t *pcm_off,
                            const double *data_min, const double *data_max, int32_t out_dtype, void *out_dev);
int frs_decode_tiles(frs_ctx *ctx, const uint8_t *blob_host, const int64_t *stream_off, int32_t nstreams,
                     int32_t channels, int32_t bps, int32_t blocksize, const int64_t *pcm_off, const double *data_min,
                     const double *data_max, int32_t out_dtype, void *out_host);
/* frs_decode_tiles_device for ONE tile -- the bbox query of cli.py:984-1023 (extract-streaming decodes the single
 * selected tile): its frames are blob_dev[start, end), `count` samples per channel, scalar arguments only (no
 * per-call tables for the binding to marshal on the latency path).  Errors as frs_decode_tiles_device. */
int frs_decode_tile_device(frs_ctx *ctx, const uint8_t *blob_dev, int64_t start, int64_t end, int64_t count,
                           int32_t channels, int32_t bps, int32_t blocksize, double data_min, double data_max,
                           int32_t out_dtype, void *out_dev);

/* converter.py:88-110 after pyflac+soundfile's WAV round trip (sonos-pyflac.txt:1629, 1827-1852): the
 * decoder's int32 samples go into a PCM_16 WAV (16-bit streams unchanged; 32-bit streams keep x >> 16,
 * libsndfile's int->short conversion) and are read back as float64 = pcm16/32768.  Then
 * out = round_half_even(((float32(v) + 1)/2) * float32(max-min) + float32(min)), all fp32 ops, cast to
 * out_dtype; for a float out_dtype float32(v) is written as-is.  pcm_bps = STREAMINFO bits per sample. */
int frs_denormalize_device(frs_ctx *ctx, const int32_t *pcm_dev, int64_t n, int32_t pcm_bps, double data_min,
                           double data_max, int32_t out_dtype, void *out_dev);
int frs_denormalize(frs_ctx *ctx, const int32_t *pcm_host, int64_t n, int32_t pcm_bps, double data_min,
                    double data_max, int32_t out_dtype, void *out_host);

/* Multi-GPU create-streaming (one process per GPU).  The reference's tile loop (cli.py:690-763) is
 * serial; here tiles shard by contiguous tile rows and the only exchange is an RCCL all-gather (xGMI) of per-tile
 * byte sizes, after which every rank writes its own tiles at their file offsets.  librccl.so is loaded at run
 * time; rank 0 calls frs_comm_unique_id and the host ships the FRS_COMM_ID_BYTES bytes to every rank (any
 * bootstrap: flac_raster_amd/distributed.py uses a TCP star), then each rank calls frs_comm_init with its context
 * (one GPU per rank).  frs_comm_allgather_i64: `count` int64 per rank, host in/out, result in rank order;
 * synchronous on the context's stream. */
typedef struct frs_comm frs_comm;
#define FRS_COMM_ID_BYTES 128
int frs_comm_unique_id(uint8_t *id_out);
int frs_comm_init(frs_ctx *ctx, const uint8_t *id, int32_t nranks, int32_t rank, frs_comm **out);
void frs_comm_destroy(frs_comm *comm);
int frs_comm_allgather_i64(frs_comm *comm, const int64_t *send_host, int64_t count, int64_t *recv_host);

/* Device memory helpers so hosts need no other GPU runtime binding (no PyTorch in the codec path). */
void *frs_dev_malloc(frs_ctx *ctx, int64_t bytes);
void frs_dev_free(frs_ctx *ctx, void *ptr);
/* Page-locked host memory: an arena_host given to frs_encode_tiles in such memory takes the frames back at DMA rate
 * (a fresh pageable buffer is page-faulted and pinned page by page during the copy).  create-streaming writes the
 * file straight from it (streaming.create_streaming_array). */
void *frs_host_malloc(frs_ctx *ctx, int64_t bytes);
void frs_host_free(frs_ctx *ctx, void *ptr);
int frs_memcpy_h2d(frs_ctx *ctx, void *dst_dev, const void *src_host, int64_t bytes);
int frs_memcpy_d2h(frs_ctx *ctx, void *dst_host, const void *src_dev, int64_t bytes);
int frs_ctx_sync(frs_ctx *ctx);

/* Benchmark input: fills a [bands][height][width] int16 raster in device memory with the survey's
 * synthetic multispectral DEM: band b = int16(1000 + 300 sin(X(0.5+0.3b)) cos(0.3Y)
 * + 150 sin(1.2X) sin(1.1Y) + 50 u), X,Y = linspace(0, 20) over the full raster width/height, u a
 * counter-based uniform [0,1) draw of (seed, b, y, x).  Rows [row0, row0+height) of a raster of
 * full_height rows are generated (multi-GPU slabs).  Parity never depends on this generator: tests
 * download what it produced and feed the same bytes to the oracle. */
int frs_synth_raster_device(frs_ctx *ctx, int16_t *dev, int32_t bands, int64_t height, int64_t width,
                            int64_t row0, int64_t full_height, uint64_t seed);

/* Stream of the context (hipStream_t as void*) so callers can order their own work / events with it. */
void *frs_ctx_stream(frs_ctx *ctx);
/* Average device time (ms) of the named kernel over the launches since the last reset, measured with
 * HIP events on the context stream (kernel: "encode" = the frame-encode kernel, "analyze", "stats",
 * "compact", "decode"); returns -1 when not recorded.  frs_profile_enable(ctx, 1) turns recording on. */
int frs_profile_enable(frs_ctx *ctx, int on);
double frs_profile_avg_ms(frs_ctx *ctx, const char *kernel);
void frs_profile_reset(frs_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* FLAC_RASTER_AMD_H */
