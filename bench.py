#!/usr/bin/env python3
"""bench.py -- create-streaming encode throughput on MI355X (BASELINE.json metric, config C4 + C5).

One step = one pass of the hot path over one batch of synthetic input: every band-1 tile of this rank's share of
the 40000 x 40000 x 4 int16 raster (tile 512, level 5, blocksize 4096) is encoded into FLAC frames in HBM (tile
min/max, analysis, frame coding, offsets, CRC), the per-tile sizes come back to the host and, for N > 1, are
all-gathered over RCCL (the codec library's frs_comm_*, xGMI) so every rank knows every tile's byte offset in the
streaming file.  The raster is generated on the device before timing (inputs resident in HBM); nothing is
cached between steps.

Strong scaling (BASELINE C4: ONE 40000^2 raster, tiles sharded over the GPUs): with N ranks the 79 tile rows are
split 10/10/.../9 and `value` is the whole raster's pixels / the max-over-ranks step time.

Also reported (DESIGN.md "Measurement"):
  roofline      dominant kernel's algorithmic bytes / its HIP-event-timed average duration vs 8 TB/s
  bbox_extract  C5: 1000 seed-7 bbox queries against the streaming data in HBM (selection + fused decode +
                de-normalisation stored straight into page-locked host memory); at N > 1 each rank answers the
                queries whose tile it holds
  (N = 1 only)  batched_decode (all 6241 tiles in one call), sentinel2 (10980^2 uint16 at tile 1024: partial
                frames on the fast path), end_to_end (create-streaming array -> .flac file, extract-streaming
                file -> tile), cpu_baseline (the oracle on bounded samples of the same workloads)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import workloads  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E peak 8.0 TB/s
# VALU issue peak: 1024 SIMDs x 2.4 GHz x 1/2 wave64 instruction per cycle (MI355X_MICROARCH.md: a wave64 VALU
# instruction issues over 2 cycles, 32 lanes/cycle; = the 157.3 TFLOPS FP32 vector peak / 128 FLOP)
VALU_PEAK_GINST_S = 1024 * 2.4 * 0.5
METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"] if (ROOT / "BASELINE.json").exists() else \
    "Mpixels/sec encode (create-streaming) + bbox-extract ms, 1/2/4/8 GPU; bit-exact vs ref"
# bench kernel name -> the leading template arguments of its C4 instance in a rocprofv3 summary.  A template that
# grows trailing parameters keeps matching (pmc_for takes the unique symbol that extends the prefix); a missing or
# ambiguous match is reported on stderr, and tests/test_bench_pmc.py checks every entry against the committed summary.
KERNEL_SYMBOL = {"encode": "frs::k_encode_v4<3, false", "analyze": "frs::k_analyze_v3<3, false, true"}
# the kernels one C4 step launches (once each): their counter bytes per launch add up to the step's HBM traffic
STEP_KERNELS = ("frs::k_analyze_v3<", "frs::k_encode_v4<", "frs::k_fast_finish")
# achievable HBM rate (MI355X_MICROARCH.md: a streaming read+write kernel sustains ~6.29 TB/s of the 8 TB/s peak)
HBM_ACHIEVABLE_GBS = 6290.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--height", type=int, default=40000, help="raster rows (C4: 40000), split over the ranks")
    ap.add_argument("--width", type=int, default=40000)
    ap.add_argument("--bands", type=int, default=4)
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--cpu-tiles", type=int, default=632, help="tiles in the CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the N = 1 extras (e2e, batched decode, ...)")
    ap.add_argument("--legs", default="", help="comma-separated N = 1 extras to run (default: all of them)")
    ap.add_argument("--queries", type=int, default=1000, help="C5 bbox-extract queries (0: skip)")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"),
                    help="tools/pmc_traffic.py output of a rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE pass of this bench")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher environment: start N local ranks of this script (one per GPU, the
    environment torchrun would set) BEFORE anything touches the GPU, and return the exit code of the group (the
    first failing rank's; the others are stopped then).  Rank 0 prints the JSON line."""
    from flac_raster_amd import launch
    return launch.run_ranks(args.gpus, [str(Path(__file__).resolve())] + sys.argv[1:], module=None)


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    from flac_raster_amd import _native, distributed

    rank, world, local_rank = distributed.env_rank_world()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    backend = os.environ.get("FRS_COMM_BACKEND", "rccl") if world > 1 else "none"
    if os.environ.get("FRS_BENCH_SELFTEST") == "1":  # CPU tests of the launch path: ranks, world, exchange
        comm = distributed.init_comm(None, "tcp") if world > 1 else None
        ranks = comm.allgather_i64(np.array([rank])) if comm is not None else np.array([0])
        if rank == 0:
            print(json.dumps({"metric": METRIC, "n_gpus": world, "ranks": [int(r) for r in ranks],
                              "config": {"parallelism": parallelism(world, backend)}}), flush=True)
        if comm is not None:
            comm.close()
        return
    # one rank per GPU; FRS_COMM_BACKEND=tcp (the host exchange) lets a rehearsal put several ranks on one GPU
    ndev = _native.device_count()
    if world > 1 and backend == "rccl" and world > ndev:
        print(f"bench.py: {world} ranks but {ndev} GPUs (one rank per GPU; FRS_COMM_BACKEND=tcp shares a GPU)",
              file=sys.stderr)
        sys.exit(2)
    ctx = _native.Context(local_rank % max(1, ndev))
    comm = distributed.init_comm(ctx, backend) if world > 1 else None

    T, W, H, B = args.tile, args.width, args.height, args.bands
    tcols, trows = (W + T - 1) // T, (H + T - 1) // T
    tr0, tr1 = distributed.shard_tile_rows(trows, world, rank)
    row0 = tr0 * T
    rows = min(tr1 * T, H) - row0
    counts = [(distributed.shard_tile_rows(trows, world, r)[1] - distributed.shard_tile_rows(trows, world, r)[0]) * tcols
              for r in range(world)]

    raster = ctx.alloc(max(1, B * rows * W * 2))
    if rows:
        ctx.synth_raster(raster, B, rows, W, row0=row0, full_height=H, seed=1234)
    desc = ctx.make_desc(max(rows, 1), W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100,
                         bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(desc))
    ctx.sync()

    ag_s = []  # per-step wall time of the size all-gather (N > 1)

    def step():
        off, mn, mx, _ = ctx.encode_tiles_device(raster.ptr, desc, arena) if rows else \
            (np.zeros(1, np.int64), np.zeros(0), np.zeros(0), 16)
        if comm is not None:  # spatial-index exchange: every rank's per-tile sizes -> global byte offsets (RCCL)
            t = time.perf_counter()
            distributed.all_gather_sizes(np.diff(off), counts, comm)
            ag_s.append(time.perf_counter() - t)
        return off, mn, mx

    for _ in range(args.warmup):
        off, mn, mx = step()

    def barrier():
        ctx.sync()
        if comm is not None:
            comm.barrier()
        ctx.sync()

    ctx.profile(True)
    ctx.profile_reset()
    barrier()
    ag_s.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        off, mn, mx = step()
    barrier()
    t1 = time.perf_counter()
    ctx.profile(False)
    elapsed = t1 - t0
    if comm is not None:
        elapsed = float(comm.allgather_i64(np.array([int(elapsed * 1e9)])).max()) * 1e-9
    total_px = H * W

    kernels = {k: ctx.profile_avg_ms(k) for k in ("stats", "analyze", "partial", "encode", "compact")}
    kernels = {k: v for k, v in kernels.items() if v > 0}
    comp_bytes = int(off[-1])
    px_rank = rows * W
    # algorithmic bytes per launch: stats reads 2 B/px; analyze reads 2 B/px (4 B/px when the tile
    # stats are fused into it: min/max pass + autocorrelation pass); encode reads 2 B/px and writes the frames;
    # compact reads + writes the frames.
    fused = "stats" not in kernels
    algo = {"stats": 2 * px_rank, "analyze": (4 if fused else 2) * px_rank, "encode": 2 * px_rank + comp_bytes,
            "compact": 2 * comp_bytes, "partial": 0}
    dom = max(kernels, key=lambda k: kernels[k]) if kernels else "encode"
    dom_ms = kernels.get(dom, float("nan"))
    achieved = algo.get(dom, 0) / (dom_ms * 1e-3) / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    value = total_px / (elapsed / args.steps) / 1e6

    result = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic (on-device DEM recipe of SURVEY.md 8d, seed 1234)",
        "config": {"workload": ("C4 " if (H, W, B, T) == (40000, 40000, 4, 512) else "") +
                   "create-streaming encode (band 1, device-resident) + C5 bbox extract",
                   "raster": f"{H}x{W}x{B} int16", "tile_size": T, "tiles": trows * tcols,
                   "tiles_rank0": int(counts[0]), "blocksize": 4096, "compression_level": 5,
                   "parallelism": parallelism(world, backend),
                   "compressed_bytes_rank0": comp_bytes},
        "kernels_ms": {k: round(v, 4) for k, v in kernels.items()},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic_for(args.traffic_json, dom, px_rank),
                     # the north-star figure: the band's 2 B/px read once per step against the HBM read peak
                     "step_read": {"bytes": 2 * px_rank, "achieved": round(2 * px_rank / (ms_per_step * 1e-3) / 1e9, 1),
                                   "frac": round(2 * px_rank / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
                     # the step's own traffic floor: algorithmic bytes (band read once + frames written once) at
                     # the achievable HBM rate (~1.0 ms on C4)
                     "step_floor": {"bytes": 2 * px_rank + comp_bytes,
                                    "ms": round((2 * px_rank + comp_bytes) / (HBM_ACHIEVABLE_GBS * 1e9) * 1e3, 3),
                                    "frac": round((2 * px_rank + comp_bytes) / (HBM_ACHIEVABLE_GBS * 1e9) * 1e3
                                                  / ms_per_step, 4)},
                     "step_traffic": step_traffic_for(args.traffic_json, px_rank, ms_per_step)},
    }
    if comm is not None:
        result["allgather_us"] = allgather_figures(comm, ag_s, np.diff(off), counts)
        result["config"]["compressed_bytes_total"] = int(comm.allgather_i64(np.array([comp_bytes])).sum())
    else:
        result["config"]["compressed_bytes_total"] = comp_bytes
    valu = pmc_for(args.traffic_json, dom, px_rank, "valu_insts")
    if valu:  # the integer encoder is issue-bound, not HBM-bound: its VALU instruction rate vs the issue peak
        rate = valu / (dom_ms * 1e-3) / 1e9
        result["roofline"]["issue"] = {"valu_insts": round(valu), "achieved": round(rate, 1),
                                       "peak": VALU_PEAK_GINST_S, "unit": "G wave-instr/s",
                                       "frac": round(rate / VALU_PEAK_GINST_S, 4)}

    progress(f"step {ms_per_step:.3f} ms")
    if args.queries > 0:
        progress("bbox_extract")
        bx = bbox_extract(ctx, comm, raster, arena, off, mn, mx, H, W, T, row0, counts, args.queries)
        if rank == 0:
            result["bbox_extract"] = bx
    if world == 1 and not args.no_extras:
        for name, leg in (("batched_decode", lambda: batched_decode(ctx, arena, off, mn, mx, rows, W, T)),
                          ("c3_streaming", lambda: c3_streaming(ctx)),
                          ("sentinel2", lambda: sentinel2(ctx)), ("convert_multiband", lambda: convert_multiband(ctx)),
                          ("convert_2band", lambda: convert_2band(ctx)), ("raw_frames", lambda: raw_frames(ctx)),
                          ("convert_level8", lambda: convert_level8(ctx)),
                          ("end_to_end", lambda: end_to_end(ctx, raster, arena, off, rows, W, T, args))):
            if args.legs and name not in args.legs.split(","):
                continue
            progress(name)
            result[name] = leg()
    if rank == 0 and world == 1 and not args.no_cpu:  # (the CPU baseline is an N = 1 figure)
        progress("cpu_baseline")
        result["cpu_baseline"] = cpu_baseline(ctx, raster, rows, W, T, off, arena, args)
    if rank == 0:
        print(json.dumps(result), flush=True)
    arena.close()
    raster.close()
    if comm is not None:
        comm.close()
    ctx.close()


def progress(what):
    """One stderr line per bench leg (a long default run keeps writing while it works)."""
    print(f"bench.py: {what} ({time.strftime('%H:%M:%S')})", file=sys.stderr, flush=True)


def allgather_figures(comm, ag_s, sizes, counts, reps=20):
    """The spatial-index exchange of the N > 1 step, reported apart from the encode.  in_step: the
    all-gather's wall time inside the timed steps, which includes waiting for the slowest rank's encode (skew);
    isolated: the same all-gather of the same sizes after a barrier, i.e. the exchange itself.  mean = the mean
    over steps, max = the slowest step, each then the max over ranks."""
    from flac_raster_amd import distributed
    iso = []
    for _ in range(reps):
        comm.barrier()
        t = time.perf_counter()
        distributed.all_gather_sizes(sizes, counts, comm)
        iso.append(time.perf_counter() - t)

    def stat(v):
        v = np.asarray(v if len(v) else [0.0]) * 1e6
        g = comm.allgather_i64(np.array([int(v.mean() * 1000), int(v.max() * 1000), int(np.median(v) * 1000)]))
        g = g.reshape(-1, 3) / 1000.0
        return {"mean": round(float(g[:, 0].max()), 1), "max": round(float(g[:, 1].max()), 1),
                "p50": round(float(g[:, 2].max()), 1)}
    return {"in_step": stat(ag_s), "isolated": stat(iso), "steps": len(ag_s), "isolated_reps": reps,
            "bytes_per_rank": int(8 * max(counts)), "backend": type(comm).__name__}


def parallelism(world: int, backend: str) -> str:
    if world == 1:
        return "single GPU (no exchange)"
    how = {"rccl": "RCCL all-gather over xGMI", "tcp": "host TCP all-gather"}.get(backend, backend)
    return f"tile rows sharded x{world} ({how} of tile sizes)"


def bbox_extract(ctx, comm, raster, arena, off, tmin, tmax, H, W, T, row0, counts, nq):
    """C5: `nq` bbox queries (workloads.c5_queries, seed 7) against the streaming data in HBM.  Per
    query: selection of the first intersecting tile (cli.py:976-987, grid-accelerated), fused decode +
    de-normalisation of that tile's frames stored straight into page-locked host memory.  With N ranks the index
    is replicated and a query is answered by the rank holding its tile.  The decoded tiles are spot-checked against the raster
    (the C4 round trip is lossless)."""
    from flac_raster_amd import distributed, streaming

    rank = comm.rank if comm is not None else 0
    first_tile = sum(counts[:rank])
    # global index (sizes of every rank's tiles) for the selection
    sizes = np.diff(off) if comm is None else distributed.all_gather_sizes(np.diff(off), counts, comm)
    index = workloads.streaming_index(H, W, T, sizes)
    queries = workloads.c5_queries(H, W, T, nq)
    mine = [q for q in queries
            if first_tile <= streaming.first_intersecting(index, q)["frame_id"] < first_tile + counts[rank]]
    # the decode kernels store the de-normalised tile straight into page-locked host memory (frs_host_malloc):
    # the query's result is host-resident when the call returns, with no separate D2H copy
    out = ctx.host_buffer(T * T * 2)
    host = out.array.view(np.int16)
    lat, checked, lossless = [], 0, True
    nwarm = min(10, len(mine))
    for k, bbox in enumerate(mine[:nwarm] + mine):  # untimed warm-up queries first
        t0 = time.perf_counter()
        f = streaming.first_intersecting(index, bbox)
        i = f["frame_id"] - first_tile
        n = f["window"]["width"] * f["window"]["height"]
        ctx.decode_tile_device(arena, off[i], off[i + 1], n, 1, 16, tmin[i], tmax[i], np.int16, out)
        dt = time.perf_counter() - t0
        if k >= nwarm:
            lat.append(dt)
        if k % 100 == 0:  # spot-check: decoded tile == raster window (band 1)
            wnd = f["window"]
            ref = np.empty((wnd["height"], W), dtype=np.int16)
            raster.download(wnd["height"] * W * 2, (wnd["row_off"] - row0) * W * 2,
                            out=ref.view(np.uint8).reshape(-1))
            got = host[:n].reshape(wnd["height"], wnd["width"])
            lossless &= bool(np.array_equal(got, ref[:, wnd["col_off"]:wnd["col_off"] + wnd["width"]]))
            checked += 1
    # kernel times from a separate profiled pass over the first 100 queries (the profile's events between the
    # kernels add ~10 us each to a query, so the timed pass above runs without them)
    ctx.profile(True)
    ctx.profile_reset()
    for bbox in mine[:100]:
        f = streaming.first_intersecting(index, bbox)
        i = f["frame_id"] - first_tile
        n = f["window"]["width"] * f["window"]["height"]
        ctx.decode_tile_device(arena, off[i], off[i + 1], n, 1, 16, tmin[i], tmax[i], np.int16, out)
    ctx.sync()
    ctx.profile(False)
    kern = {k: round(ctx.profile_avg_ms(k), 4) for k in ("decode", "decode_span", "decode_frames")}
    kern = {k: v for k, v in kern.items() if v >= 0}  # (the optimistic C5 decode skips the span check)
    out.close()
    ns = np.array([int(x * 1e9) for x in lat], dtype=np.int64)
    if comm is not None:  # gather every rank's latencies (padded with -1)
        m = int(comm.allgather_i64(np.array([len(ns)])).max())
        pad = np.full(max(m, 1), -1, dtype=np.int64)
        pad[:len(ns)] = ns
        ns = comm.allgather_i64(pad)
        ns = ns[ns >= 0]
        checked = int(comm.allgather_i64(np.array([checked])).sum())
        lossless = bool(comm.allgather_i64(np.array([int(lossless)])).min())
    ms = ns / 1e6
    return {"p50_ms": round(float(np.percentile(ms, 50)), 3), "p90_ms": round(float(np.percentile(ms, 90)), 3),
            "queries": int(len(ms)), "n_gpus": comm.world if comm is not None else 1,
            "path": "device-resident streaming data: select + fused decode/denormalise stored straight into "
                    "page-locked host memory (query -> rank holding the tile)", "kernels_ms_rank0": kern, "lossless_spot_checks": checked, "lossless": lossless}


def batched_decode(ctx, arena, off, tmin, tmax, rows, W, T):
    """Every tile of the C4 arena (3.1 GB of frames, 6241 streams) decoded + de-normalised in ONE call."""
    from flac_raster_amd import streaming
    counts = [w * h for (_, _, w, h) in streaming.tile_grid(rows, W, T)]
    out = ctx.alloc(rows * W * 2)
    ctx.decode_tiles_device(arena, off, counts, channels=1, bps=16, data_min=tmin, data_max=tmax, dtype=np.int16,
                            out=out)  # warm-up (buffers)
    ctx.profile(True)
    ctx.profile_reset()
    reps = 2
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.decode_tiles_device(arena, off, counts, channels=1, bps=16, data_min=tmin, data_max=tmax,
                                dtype=np.int16, out=out)
    ctx.sync()
    dt = (time.perf_counter() - t0) / reps
    ctx.profile(False)
    kern = {k: round(ctx.profile_avg_ms(k), 3) for k in ("decode", "decode_span", "decode_frames")}
    out.close()
    px = rows * W
    return {"tiles": len(counts), "ms": round(dt * 1e3, 2), "Mpixels_s": round(px / dt / 1e6, 1),
            "GB_s": round((int(off[-1]) + 2 * px) / dt / 1e9, 1), "kernels_ms": kern}


def c3_streaming(ctx, steps=10):
    """BASELINE config C3: create-streaming of a synthetic 16384 x 16384 x 4 int16 multispectral raster at tile 512
    (band 1, cli.py:699; 1024 tiles), device-resident, with the encoder's algorithmic-bytes roofline (the same
    recipe as the C4 line: 2 B/px read + the frames written, over the encoder's HIP-event time)."""
    H = W = 16384
    B, T = 4, 512
    buf = ctx.alloc(B * H * W * 2)
    ctx.synth_raster(buf, B, H, W, seed=1234)
    d = ctx.make_desc(H, W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(d))
    for _ in range(3):
        ctx.encode_tiles_device(buf.ptr, d, arena)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        off, _, _, _ = ctx.encode_tiles_device(buf.ptr, d, arena)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    ctx.profile(False)
    kern = {k: round(ctx.profile_avg_ms(k), 4) for k in ("stats", "analyze", "partial", "encode", "compact")}
    kern = {k: v for k, v in kern.items() if v > 0}
    comp = int(off[-1])
    enc_gbs = (2 * H * W + comp) / (kern["encode"] * 1e-3) / 1e9 if "encode" in kern else None
    arena.close()
    buf.close()
    return {"raster": f"{H}x{W}x{B} int16", "tile_size": T, "tiles": (H // T) * (W // T), "band": 1,
            "ms_per_step": round(dt * 1e3, 3), "Mpixels_s": round(H * W / dt / 1e6, 1), "compressed_bytes": comp,
            "kernels_ms": kern,
            "roofline": None if enc_gbs is None else {"kernel": "encode", "achieved": round(enc_gbs, 1),
                                                       "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                                       "frac": round(enc_gbs / HBM_PEAK_GBS, 4)}}


def sentinel2(ctx, steps=5):
    """The reference's own create-streaming example (FLAC-SPATIAL.md:82-88): a 10980 x 10980 uint16 band at tile
    1024 -- 121 tiles, the last 740 x 740 (partial last frames on the fast path), device-resident."""
    H = W = 10980
    T = 1024
    buf = ctx.alloc(H * W * 2)
    ctx.synth_raster(buf, 1, H, W, seed=4)  # values 500..1500: the same bytes read as uint16
    d = ctx.make_desc(H, W, np.uint16, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(d))
    ctx.encode_tiles_device(buf.ptr, d, arena)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.encode_tiles_device(buf.ptr, d, arena)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    ctx.profile(False)
    kern = {k: round(ctx.profile_avg_ms(k), 4) for k in ("stats", "analyze", "partial", "encode", "compact")}
    arena.close()
    buf.close()
    return {"raster": f"{H}x{W} uint16", "tile_size": T, "tiles": 121, "ms_per_step": round(dt * 1e3, 3),
            "Mpixels_s": round(H * W / dt / 1e6, 1), "fast_path": kern["partial"] > 0 and kern["compact"] < 0,
            "kernels_ms": {k: v for k, v in kern.items() if v > 0}}


def convert_multiband(ctx, steps=3):
    """Plain `convert` of a C3-shaped multispectral raster (16384 x 16384 x 4 int16, converter.py:185-216): ONE
    stream with the 4 bands interleaved, device-resident -- the multi-channel fast path (subframes by the fast
    encoder, frames joined by k_mc_assemble)."""
    B, H, W = 4, 16384, 16384
    buf = ctx.alloc(B * H * W * 2)
    ctx.synth_raster(buf, B, H, W, seed=5)
    d = ctx.make_desc(H, W, np.int16, nbands=B, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=16)
    arena = ctx.alloc(ctx.arena_bound(d))
    ctx.encode_tiles_device(buf.ptr, d, arena)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        off, _, _, _ = ctx.encode_tiles_device(buf.ptr, d, arena)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    ctx.profile(False)
    kern = {k: round(ctx.profile_avg_ms(k), 4) for k in ("stats", "analyze", "partial", "encode", "assemble", "compact")}
    # the mirror (flac_to_tiff, converter.py:241-282): the whole stream decoded + de-normalised in one call
    _, mn, mx, _ = ctx.encode_tiles_device(buf.ptr, d, arena)
    out = ctx.alloc(B * H * W * 2)
    dargs = (arena, np.array([0, off[-1]]), [H * W], B, 16, [mn[0]], [mx[0]], np.int16, out)
    ctx.decode_tiles_device(*dargs)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.decode_tiles_device(*dargs)
    ctx.sync()
    ddt = (time.perf_counter() - t0) / steps
    ctx.profile(False)
    dkern = {k: round(ctx.profile_avg_ms(k), 4) for k in ("decode", "decode_span", "decode_frames")}
    # lossless: the interleaved samples against the band-planar raster, band by band (host memory bounded)
    got = out.download(B * H * W * 2).view(np.int16).reshape(H * W, B)
    ref = buf.download(B * H * W * 2).view(np.int16).reshape(B, H * W)
    lossless = all(np.array_equal(got[:, b], ref[b]) for b in range(B))
    del got, ref
    out.close()
    arena.close()
    buf.close()
    return {"raster": f"{H}x{W}x{B} int16", "streams": 1, "channels": B, "ms_per_step": round(dt * 1e3, 3),
            "Mpixels_s": round(H * W / dt / 1e6, 1), "Msamples_s": round(B * H * W / dt / 1e6, 1),
            "compressed_bytes": int(off[-1]), "fast_path": kern["assemble"] > 0,
            "kernels_ms": {k: v for k, v in kern.items() if v > 0},
            "decode": {"ms": round(ddt * 1e3, 3), "Mpixels_s": round(H * W / ddt / 1e6, 1), "lossless": lossless,
                       "kernels_ms": {k: v for k, v in dkern.items() if v > 0}}}


def _timed_encode(ctx, buf, d, steps):
    """Device-resident encode of descriptor d: warm-up, then the mean of `steps` timed calls and the kernel times."""
    arena = ctx.alloc(ctx.arena_bound(d))
    ctx.encode_tiles_device(buf.ptr, d, arena)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        off, _, _, _ = ctx.encode_tiles_device(buf.ptr, d, arena)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    ctx.profile(False)
    kern = {k: round(ctx.profile_avg_ms(k), 4) for k in ("stats", "analyze", "partial", "encode", "assemble", "compact")}
    arena.close()
    return dt, int(off[-1]), {k: v for k, v in kern.items() if v > 0}


def convert_2band(ctx, steps=3):
    """Plain `convert` of a 16384 x 16384 x 2 int16 raster as ONE two-channel stream (converter.py:185-216): libFLAC
    level 5's exhaustive mid/side search (L, R, M, S coded per frame, the cheapest assignment kept), device-resident:
    the fast kernels (k_analyze_v3 of the four signals, k_encode_v4 of L/R/M as packed pairs and of the 17-bit side as
    int32, the assignment picked from the subframe estimates in k_mc_frame_bytes, k_mc_assemble)."""
    B, H, W = 2, 16384, 16384
    buf = ctx.alloc(B * H * W * 2)
    ctx.synth_raster(buf, B, H, W, seed=6)
    d = ctx.make_desc(H, W, np.int16, nbands=B, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=16)
    dt, nbytes, kern = _timed_encode(ctx, buf, d, steps)
    buf.close()
    return {"raster": f"{H}x{W}x{B} int16", "streams": 1, "channels": B, "ms_per_step": round(dt * 1e3, 3),
            "Mpixels_s": round(H * W / dt / 1e6, 1), "compressed_bytes": nbytes, "kernels_ms": kern,
            "path": ("generic kernels (k_analyze L/R/M/S + k_encode_frames, frame per work-group)" if "compact" in kern
                     else "fast two-channel kernels (wave per subframe; picks from the estimates; k_mc_assemble)")}


def raw_frames(ctx, steps=3):
    """`convert --spatial` (spatial_encoder.py:136-294, the C1 recipe) at C3 size: a 16384 x 16384 int16 band in 256 x
    256 tiles, each a 32-bit stream of the {-1, 0, 1} samples pyflac makes of the float normalisation -- the generic
    kernels (32-bit streams), device-resident."""
    H = W = 16384
    T = 256
    buf = ctx.alloc(H * W * 2)
    ctx.synth_raster(buf, 1, H, W, seed=7)
    d = ctx.make_desc(H, W, np.int16, tile_h=T, tile_w=T, sample_rate=44100, bits_per_sample=24, norm_mode=1)
    dt, nbytes, kern = _timed_encode(ctx, buf, d, steps)
    buf.close()
    return {"raster": f"{H}x{W} int16", "tile_size": T, "tiles": (H // T) * (W // T), "bps": 32,
            "ms_per_step": round(dt * 1e3, 3), "Mpixels_s": round(H * W / dt / 1e6, 1), "compressed_bytes": nbytes,
            "kernels_ms": kern, "path": "generic kernels (32-bit streams)"}


def convert_level8(ctx, steps=2):
    """`convert -c 8` of a 4096 x 4096 x 3 int16 raster (one 3-channel stream): subdivide_tukey(3) -- nine LPC
    windows per subframe, LPC order up to 12, partition order up to 6 -- on the generic kernels, device-resident."""
    B, H, W = 3, 4096, 4096
    buf = ctx.alloc(B * H * W * 2)
    ctx.synth_raster(buf, B, H, W, seed=8)
    d = ctx.make_desc(H, W, np.int16, nbands=B, tile_h=H, tile_w=W, sample_rate=44100, bits_per_sample=16,
                      compression_level=8)
    dt, nbytes, kern = _timed_encode(ctx, buf, d, steps)
    buf.close()
    return {"raster": f"{H}x{W}x{B} int16", "level": 8, "ms_per_step": round(dt * 1e3, 3),
            "Mpixels_s": round(H * W / dt / 1e6, 1), "compressed_bytes": nbytes, "kernels_ms": kern}


def end_to_end(ctx, raster, arena, off_dev, rows, W, T, args):
    """The user-visible path on C4, host memory in and out.
    create: streaming.create_streaming_array(band 1 in host memory) -> .flac file (H2D, encode, D2H, headers +
            index, parallel pwritev), best of 2 runs.
    extract: per query (the C5 queries): index already loaded (its load is reported once), selection, byte-range
            read of the tile from the file, tag parse, fused GPU decode + de-normalisation into host memory."""
    from flac_raster_amd import streaming
    band = np.empty((rows, W), dtype=np.int16)
    raster.download(rows * W * 2, 0, out=band.view(np.uint8).reshape(-1))
    tmpd = Path(os.environ.get("FRS_BENCH_TMP", tempfile.gettempdir()))
    out = tmpd / f"frs_bench_c4_{os.getpid()}.flac"
    res = {}
    try:
        runs = []
        for _ in range(3):  # each run writes a fresh file (no truncation of the previous run's pages)
            if out.exists():
                out.unlink()
            tm = {}
            streaming.create_streaming_array(band, workloads.transform(), workloads.CRS, out, T, ctx, tm)
            runs.append(tm)
        best = min(runs, key=lambda t: t["total_s"])
        res["create_streaming"] = {"Mpixels_s": round(rows * W / best["total_s"] / 1e6, 1),
                                   "seconds": {k: round(v, 4) for k, v in best.items()},
                                   "write_s_runs": [round(t["write_s"], 4) for t in runs],
                                   "file_bytes": out.stat().st_size, "dir": str(tmpd)}
        # extract-streaming on the file
        t0 = time.perf_counter()
        src = streaming.Source(out)
        n, index = streaming.read_index(src)
        load_ms = (time.perf_counter() - t0) * 1e3
        # the file's tiles hold the device-resident step's frames (after their headers): three spot checks
        same = True
        for i in (0, len(index["frames"]) // 2, len(index["frames"]) - 1):
            blob = streaming.fetch_tiles(src, [index["frames"][i]], n)[0]
            nb = int(off_dev[i + 1] - off_dev[i])
            same &= blob[-nb:] == arena.download(nb, int(off_dev[i])).tobytes()
        res["create_streaming"]["index_entries"] = len(index["frames"])
        res["create_streaming"]["frames_equal_device_step"] = bool(same)
        res["create_streaming_file"] = e2e_from_geotiff(ctx, raster, rows, W, T, tmpd, out)
        dec = streaming.TileDecoder(ctx)
        lat, lossless = [], True
        qs = workloads.c5_queries(rows, W, T, args.queries)
        for k, bbox in enumerate(qs[:10] + qs):
            t0 = time.perf_counter()
            f = streaming.first_intersecting(index, bbox)
            data = streaming.fetch_tiles(src, [f], n)[0]
            (arr, md), = dec.decode_streams([data])
            dt = time.perf_counter() - t0
            if k >= 10:
                lat.append(dt)
            if k % 100 == 0:
                w = f["window"]
                lossless &= bool(np.array_equal(arr[0], band[w["row_off"]:w["row_off"] + w["height"],
                                                             w["col_off"]:w["col_off"] + w["width"]]))
        ms = np.array(lat) * 1e3
        if len(lat):  # (--queries 0: no extract leg)
            res["extract_streaming"] = {"p50_ms": round(float(np.percentile(ms, 50)), 3),
                                        "p90_ms": round(float(np.percentile(ms, 90)), 3), "queries": len(lat),
                                        "index_load_ms": round(load_ms, 2), "lossless": lossless,
                                        "path": "file: select + range read + tag parse + fused GPU decode -> host array"}
        if not args.no_cpu and len(lat):
            res["cpu_baseline"] = e2e_cpu_baseline(band, out, index, n, T, qs)
    finally:
        if out.exists():
            out.unlink()
    return res


def e2e_from_geotiff(ctx, raster, rows, W, T, tmpd, array_out):
    """create-streaming from a GeoTIFF file, as the CLI runs it (cli.py:620-804): the C4 raster (all 4 bands) is
    written once as an uncompressed band-sequential BigTIFF, one strip per band; then streaming.create_streaming
    opens it (memory map, band 1 read in place), encodes and writes the .flac.  Best of 2 runs; the output must equal
    the array leg's file byte for byte."""
    from flac_raster_amd import geotiff, streaming
    B = int(raster.nbytes // (rows * W * 2))
    tif = tmpd / f"frs_bench_c4_{os.getpid()}.tif"
    out = tmpd / f"frs_bench_c4_file_{os.getpid()}.flac"
    try:
        host = np.empty((B, rows, W), dtype=np.int16)
        raster.download(B * rows * W * 2, 0, out=host.view(np.uint8).reshape(-1))
        t0 = time.perf_counter()
        geotiff.write(tif, host, workloads.transform(), int(workloads.CRS.split(":")[1]), planar=2,
                      rows_per_strip=rows)
        write_tif_s = time.perf_counter() - t0
        del host
        def leg(materialize):
            runs = []
            for _ in range(3):  # a fresh output file per run, as in the array leg
                if out.exists():
                    out.unlink()
                tm = {}
                streaming.create_streaming(tif, out, T, ctx, tm, materialize=materialize)
                runs.append(tm)
            return min(runs, key=lambda t: t["total_s"]), runs
        # explicit read first: the band read from the file into host memory, timed as read_s
        best_rd, runs_rd = leg(True)
        explicit = {"Mpixels_s": round(rows * W / best_rd["total_s"] / 1e6, 1),
                    "seconds": {k: round(v, 4) for k, v in best_rd.items()},
                    "read_GB_s": round(rows * W * 2 / best_rd["read_s"] / 1e9, 2)}
        best, runs = leg(False)

        def same_bytes(a, b):
            if a.stat().st_size != b.stat().st_size:
                return False
            x, y = np.memmap(a, dtype=np.uint8, mode="r"), np.memmap(b, dtype=np.uint8, mode="r")
            step = 256 << 20
            ok = all(np.array_equal(x[i:i + step], y[i:i + step]) for i in range(0, x.size, step))
            del x, y
            return ok
        return {"Mpixels_s": round(rows * W / best["total_s"] / 1e6, 1),
                "seconds": {k: round(v, 4) for k, v in best.items()},
                "write_s_runs": [round(t["write_s"], 4) for t in runs],
                "input": f"{B}x{rows}x{W} int16 GeoTIFF, uncompressed, band-sequential, {tif.stat().st_size} B "
                         f"(written once in {write_tif_s:.2f} s); band 1 encoded from the memory map (its pages "
                         "are read while the encode copies them: inside encode_s)",
                "explicit_read": explicit,
                "file_bytes": out.stat().st_size, "dir": str(tmpd),
                "equal_array_leg_file": bool(same_bytes(out, array_out))}
    finally:
        for p in (tif, out):
            if p.exists():
                p.unlink()


def e2e_cpu_baseline(band, out, index, n, T, qs):
    """The oracle pipeline (oracle/pipeline.py: the reference's per-tile create-streaming loop, restated, 1 thread) on
    the first tile rows (~632 tiles), byte-checked against the GPU file; and the oracle's extract (range read + tag
    parse + decode + de-normalise) on 50 of the same queries."""
    from flac_raster_amd import container, streaming
    from oracle import oracle as O, pipeline as P
    W = band.shape[1]
    tcols = (W + T - 1) // T
    h = min(8 * T, band.shape[0])
    t0 = time.perf_counter()
    ref = P.create_streaming(np.ascontiguousarray(band[:h]), list(workloads.transform()), workloads.CRS, T)
    dt = time.perf_counter() - t0
    js_len = int.from_bytes(ref[:4], "big")
    tiles_ref = ref[4 + js_len:]
    with open(out, "rb") as fh:
        fh.seek(4 + n)
        tiles_gpu = fh.read(len(tiles_ref))
    create = {"Mpixels_s": round(h * W / dt / 1e6, 2), "seconds": round(dt, 3), "cores": 1, "kind": "port",
              "sample": f"{(h // T) * tcols} tiles ({h}x{W} px): oracle/pipeline.py create_streaming (per-tile "
                        "plain convert + mutagen restatement, in memory)",
              "bit_exact_vs_gpu_file": tiles_ref == tiles_gpu}
    lat = []
    src = streaming.Source(out)
    for bbox in qs[:50]:
        t0 = time.perf_counter()
        f = streaming.first_intersecting(index, bbox)
        data = streaming.fetch_tiles(src, [f], n)[0]
        m = container.parse_metadata(data)
        md = container.read_raster_tags(m)
        pcm = O.decode_frames(data[m.audio_offset:], 1, 16, md["width"] * md["height"])
        O.denormalize_i16(pcm, md["data_min"], md["data_max"], np.int16)
        lat.append(time.perf_counter() - t0)
    ms = np.array(lat) * 1e3
    extract = {"p50_ms": round(float(np.percentile(ms, 50)), 3), "queries": len(lat), "cores": 1, "kind": "port",
               "sample": "50 C5 queries on the same file, oracle decode + de-normalisation"}
    return {"create_streaming": create, "extract_streaming": extract}


def loaded_lib_sha256() -> str:
    """sha256 of the codec library this process loads (FRS_LIB_PATH or the in-tree build)."""
    import hashlib
    from flac_raster_amd import _native
    p = Path(os.environ.get("FRS_LIB_PATH", str(_native.LIB_PATH)))
    return hashlib.sha256(p.read_bytes()).hexdigest()


def resolve_symbol(kernels, kernel):
    """The summary key of bench kernel `kernel`: the exact symbol, else the unique symbol extending its
    KERNEL_SYMBOL prefix by further template arguments (`<3, false` matches `<3, false, false, false>`, not
    `<3, falsey>`).  None when absent or ambiguous (two instances extend the prefix)."""
    want = KERNEL_SYMBOL.get(kernel, kernel)
    if want in kernels:
        return want
    hits = [k for k in kernels if k.startswith(want) and k[len(want):len(want) + 1] in (",", ">")]
    return hits[0] if len(hits) == 1 else None


def load_pmc(path, px):
    """A committed counter summary (tools/pmc_traffic.py) measured on this same workload (C4 slab of `px`
    pixels) AND this same library build (its sha256 stamp); None otherwise."""
    try:
        d = json.loads(Path(path).read_text())
    except (OSError, ValueError):
        return None
    if d.get("pixels_per_launch") not in (None, px):
        return None
    if d.get("lib_sha256") != loaded_lib_sha256():
        print(f"bench.py: {path} was measured on another library build: no counter figures", file=sys.stderr)
        return None
    return d


def pmc_for(path, kernel, px, field):
    """Per-launch PMC figure `field` of bench kernel `kernel` (see load_pmc); None otherwise.  A summary of this
    library whose symbols do not resolve is a bug (a renamed template): reported on stderr."""
    d = load_pmc(path, px)
    if d is None:
        return None
    kernels = d.get("kernels", {})
    sym = resolve_symbol(kernels, kernel)
    if sym is None:
        print(f"bench.py: no unique counter entry for {kernel!r} ({KERNEL_SYMBOL.get(kernel, kernel)}) in {path}",
              file=sys.stderr)
        return None
    return kernels[sym].get(field)


def step_traffic_for(path, px, ms_per_step):
    """HBM bytes one C4 step moves by the counters: the FETCH x2 + WRITE bytes per launch of every kernel the
    step launches (STEP_KERNELS), against the step time and the achievable HBM rate; None without a summary."""
    d = load_pmc(path, px)
    if d is None:
        return None
    parts = {k: v["bytes"] for k, v in d.get("kernels", {}).items()
             if "bytes" in v and any(k.startswith(p) for p in STEP_KERNELS)}
    if not parts:
        return None
    total = sum(parts.values())
    rate = total / (ms_per_step * 1e-3) / 1e9
    return {"bytes": round(total), "kernels": {k: round(v) for k, v in parts.items()},
            "achieved": round(rate, 1), "achievable": HBM_ACHIEVABLE_GBS,
            "frac_achievable": round(rate / HBM_ACHIEVABLE_GBS, 4), "frac_peak": round(rate / HBM_PEAK_GBS, 4)}


def traffic_for(path, kernel, px):
    """HBM bytes per launch of `kernel` (FETCH_SIZE x2 + WRITE_SIZE passes)."""
    b = pmc_for(path, kernel, px, "bytes")
    return None if b is None else round(b)


def cpu_baseline(ctx, raster, rows, W, T, off, arena, args):
    """Time the oracle on the first `cpu_tiles` tiles (whole tile rows) of the same raster bytes."""
    from oracle import oracle as O

    tcols = (W + T - 1) // T
    nrows_t = max(1, min((args.cpu_tiles + tcols - 1) // tcols, (rows + T - 1) // T))
    h = min(nrows_t * T, rows)
    band = np.empty((h, W), dtype=np.int16)
    raster.download(h * W * 2, 0, out=band.view(np.uint8).reshape(-1))
    t0 = time.perf_counter()
    o_arena, o_off, _, _ = O.encode_tiles(band, T, threads=args.cpu_threads)
    dt = time.perf_counter() - t0
    nt = len(o_off) - 1
    gpu = arena.download(int(off[nt]), 0)
    parity = bool(np.array_equal(o_off, off[: nt + 1]) and gpu.tobytes() == o_arena.tobytes())
    res = {"value": round(h * W / dt / 1e6, 2), "unit": "Mpixels/s", "cores": args.cpu_threads, "kind": "port",
           "sample": f"{nt} band-1 tiles ({h}x{W} px) of the benchmark raster, oracle/flac_oracle.c",
           "seconds": round(dt, 3), "bit_exact_vs_gpu": parity}
    # the same sample on the box's CPU share (OpenMP over tiles; OMP_NUM_THREADS is the share on the GPU box)
    mt = workloads.oracle_threads()
    if args.cpu_threads == 1 and mt > 1:
        t0 = time.perf_counter()
        m_arena, m_off, _, _ = O.encode_tiles(band, T, threads=mt)
        dt_mt = time.perf_counter() - t0
        res["multi_thread"] = {"value": round(h * W / dt_mt / 1e6, 2), "cores": mt, "seconds": round(dt_mt, 3),
                               "bit_exact_vs_gpu": bool(m_arena.tobytes() == o_arena.tobytes())}
    return res


if __name__ == "__main__":
    main()
