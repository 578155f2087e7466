#!/usr/bin/env python3
"""bench.py -- create-streaming encode throughput on MI355X (BASELINE.json metric, config C4).

One step = one pass of the hot path over one batch of synthetic input: every band-1 tile of this rank's
slab of a 40000 x 40000 x 4 int16 raster (tile 512, level 5, blocksize 4096) is encoded into FLAC frames
in HBM (tile min/max, analysis, frame coding, offsets, CRC), the per-tile sizes come back to the host and,
for N > 1, are all-gathered over RCCL so every rank knows every tile's byte offset in the streaming file.
The raster is generated on the device before timing (inputs resident in HBM); nothing is cached between
steps.

Weak scaling: with N ranks the raster is N*40000 rows tall and rank r encodes its contiguous run of tile
rows (~40000 rows, 6241 tiles at N=1), so per-GPU work is fixed.

Also reported (DESIGN.md "Measurement"):
  roofline      dominant kernel's algorithmic bytes / its HIP-event-timed average duration vs 8 TB/s
  cpu_baseline  the CPU oracle (C restatement, oracle/) on a bounded sample of the same tiles, rank 0,
                checked byte-for-byte against the GPU frames of those tiles
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E peak 8.0 TB/s
# VALU issue peak: 1024 SIMDs x 2.4 GHz x 1/2 wave64 instruction per cycle (MI355X_MICROARCH.md: a wave64 VALU
# instruction issues over 2 cycles, 32 lanes/cycle; = the 157.3 TFLOPS FP32 vector peak / 128 FLOP)
VALU_PEAK_GINST_S = 1024 * 2.4 * 0.5
METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"] if (ROOT / "BASELINE.json").exists() else \
    "Mpixels/sec encode (create-streaming) + bbox-extract ms, 1/2/4/8 GPU; bit-exact vs ref"
KERNEL_SYMBOL = {"encode": "frs::k_encode_v3<3>", "analyze": "frs::k_analyze_v3<3, false, true>",
                 "stats": "frs::k_tile_stats_vec<3>"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--height", type=int, default=40000, help="rows per rank (C4: 40000)")
    ap.add_argument("--width", type=int, default=40000)
    ap.add_argument("--bands", type=int, default=4)
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--cpu-tiles", type=int, default=632, help="tiles in the CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--queries", type=int, default=1000, help="C5 bbox-extract queries (0: skip)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"),
                    help="tools/pmc_traffic.py output of a rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE pass of this bench")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local_rank
    if world > 1:
        import torch
        import torch.distributed as tdist
        # one rank per GPU; on a box with fewer GPUs than ranks (rehearsal only) ranks share devices
        device = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        tdist.init_process_group(args.backend)  # "nccl" = RCCL over xGMI
        dist = tdist

    from flac_raster_amd import _native

    ctx = _native.Context(device)
    T = args.tile
    W = args.width
    full_h = args.height * world
    trows = (full_h + T - 1) // T
    tr0 = rank * trows // world
    tr1 = (rank + 1) * trows // world
    row0 = tr0 * T
    rows = min(tr1 * T, full_h) - row0
    B = args.bands

    raster = ctx.alloc(B * rows * W * 2)
    ctx.synth_raster(raster, B, rows, W, row0=row0, full_height=full_h, seed=1234)
    desc = ctx.make_desc(rows, W, np.int16, nbands=1, band0=0, tile_h=T, tile_w=T, sample_rate=44100,
                         bits_per_sample=16)
    ntiles = desc.tile_end - desc.tile_begin
    arena = ctx.alloc(ctx.arena_bound(desc))
    ctx.sync()

    coll = None
    if dist is not None:
        import torch
        coll = torch.device("cpu") if args.backend == "gloo" else torch.device(f"cuda:{device}")
        tcols = (W + T - 1) // T
        slot = (trows + world - 1) // world * tcols  # tiles of the largest slab

    def step():
        off, mn, mx, bps = ctx.encode_tiles_device(raster.ptr, desc, arena)
        if dist is not None:
            import torch
            # spatial-index exchange: every rank's per-tile byte sizes -> global byte offsets (RCCL all-gather)
            mine = torch.zeros(slot, dtype=torch.int64, device=coll)
            sz = torch.from_numpy(np.diff(off)).to(coll)
            mine[: sz.numel()] = sz
            gathered = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(gathered, mine)
            global_off = torch.cumsum(torch.cat(gathered), 0)  # padded slots hold 0 bytes
            if coll.type == "cuda":
                torch.cuda.synchronize()
            del global_off
        return off, mn, mx

    for _ in range(args.warmup):
        off, mn, mx = step()

    def barrier():
        if dist is not None:
            dist.barrier()
            import torch
            torch.cuda.synchronize()
        ctx.sync()

    ctx.profile(True)
    ctx.profile_reset()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        off, mn, mx = step()
    barrier()
    t1 = time.perf_counter()
    ctx.profile(False)
    elapsed = t1 - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        px = torch.tensor([rows * W], dtype=torch.int64, device=coll)
        dist.all_reduce(px)
        total_px = int(px.item())
    else:
        total_px = rows * W

    kernels = {k: ctx.profile_avg_ms(k) for k in ("stats", "analyze", "encode", "compact")}
    kernels = {k: v for k, v in kernels.items() if v > 0}
    comp_bytes = int(off[-1])
    px_rank = rows * W
    # algorithmic bytes per launch: stats reads 2 B/px; analyze reads 2 B/px (4 B/px when the tile
    # stats are fused into it: min/max pass + autocorrelation pass); encode reads 2 B/px and writes the frames;
    # compact reads + writes the frames.
    fused = "stats" not in kernels
    algo = {"stats": 2 * px_rank, "analyze": (4 if fused else 2) * px_rank, "encode": 2 * px_rank + comp_bytes,
            "compact": 2 * comp_bytes}
    dom = max((k for k in kernels if kernels[k] > 0), key=lambda k: kernels[k])
    dom_ms = kernels[dom]
    achieved = algo[dom] / (dom_ms * 1e-3) / 1e9
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
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic (on-device DEM recipe of SURVEY.md 8d, seed 1234)",
        "config": {"workload": ("C4 " if (args.height, W, B, T) == (40000, 40000, 4, 512) else "") +
                   "create-streaming encode (band 1, device-resident) + C5 bbox extract", "raster": f"{full_h}x{W}x{B} int16",
                   "tile_size": T, "tiles_per_rank": int(ntiles), "blocksize": 4096, "compression_level": 5,
                   "parallelism": f"tile-rows sharded x{world}", "compressed_bytes_rank0": comp_bytes},
        "kernels_ms": {k: round(v, 4) for k, v in kernels.items()},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic_for(args.traffic_json, dom, px_rank)},
    }
    valu = pmc_for(args.traffic_json, dom, px_rank, "valu_insts")
    if valu:  # the integer encoder is issue-bound, not HBM-bound: its VALU instruction rate vs the issue peak
        rate = valu / (dom_ms * 1e-3) / 1e9
        result["roofline"]["issue"] = {"valu_insts": round(valu), "achieved": round(rate, 1),
                                       "peak": VALU_PEAK_GINST_S, "unit": "G wave-instr/s",
                                       "frac": round(rate / VALU_PEAK_GINST_S, 4)}

    if rank == 0 and args.queries > 0:
        result["bbox_extract"] = bbox_extract(ctx, raster, arena, off, mn, mx, rows, W, T, args.queries)
    if rank == 0 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(ctx, raster, rows, W, T, off, arena, args)
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def bbox_extract(ctx, raster, arena, off, tmin, tmax, rows, W, T, nq):
    """C5: `nq` bbox queries against the streaming data this rank just encoded, device
    resident.  Query = uniform tile-aligned centre, side U[0.1, 2.0] * tile_size * pixel (10 m,
    from_origin(500000, 4000000, 10, 10)), clipped to the raster; end-to-end latency = selection (first
    intersecting tile, cli.py:976-987) + decode of that tile's frames + de-normalisation + copy of the
    tile to host memory.  The decoded tiles are checked against the raster (the C4 round trip is
    lossless)."""
    from flac_raster_amd import geotiff, streaming

    tr = geotiff.Affine(10.0, 0.0, 500000.0, 0.0, -10.0, 4000000.0)
    grid = streaming.tile_grid(rows, W, T)
    frames = []
    for i, (col, row, w, h) in enumerate(grid):
        _, bb = streaming.tile_transform_and_bbox(tr, col, row, w, h)
        frames.append({"frame_id": i, "bbox": bb, "window": {"col_off": col, "row_off": row, "width": w, "height": h},
                       "byte_offset": int(off[i]), "byte_size": int(off[i + 1] - off[i])})
    index = {"transform": list(tr) + [0.0, 0.0, 1.0], "width": W, "height": rows, "tile_size": T, "frames": frames}
    left, top = 500000.0, 4000000.0
    right, bottom = left + W * 10.0, top - rows * 10.0
    rng = np.random.default_rng(7)
    out = ctx.alloc(T * T * 2)
    host = np.empty(T * T, dtype=np.int16)
    lat = []
    checked, lossless = 0, True
    ctx.profile(True)
    for q in range(nq + 10):  # 10 untimed warm-up queries
        if q == 10:
            ctx.profile_reset()
        col, row, w, h = grid[int(rng.integers(len(grid)))]
        cx, cy = left + (col + w / 2) * 10.0, top - (row + h / 2) * 10.0
        half = rng.uniform(0.1, 2.0) * T * 10.0 / 2
        bbox = [max(left, cx - half), max(bottom, cy - half), min(right, cx + half), min(top, cy + half)]
        t0 = time.perf_counter()
        f = streaming.first_intersecting(index, bbox)
        i = f["frame_id"]
        n = f["window"]["width"] * f["window"]["height"]
        ctx.decode_tiles_device(arena, np.array([off[i], off[i + 1]], dtype=np.int64), [n], channels=1, bps=16,
                                data_min=[float(tmin[i])], data_max=[float(tmax[i])], dtype=np.int16, out=out)
        out.download(n * 2, 0, out=host[:n].view(np.uint8))
        dt = time.perf_counter() - t0
        if q >= 10:
            lat.append(dt)
        if q % 100 == 0:  # spot-check: decoded tile == raster window (band 1)
            wnd = f["window"]
            ref = np.empty((wnd["height"], W), dtype=np.int16)
            raster.download(wnd["height"] * W * 2, wnd["row_off"] * W * 2, out=ref.view(np.uint8).reshape(-1))
            got = host[:n].reshape(wnd["height"], wnd["width"])
            lossless &= bool(np.array_equal(got, ref[:, wnd["col_off"]:wnd["col_off"] + wnd["width"]]))
            checked += 1
    ctx.profile(False)
    kern = {k: round(ctx.profile_avg_ms(k), 4) for k in ("decode", "decode_span", "decode_frames")}
    out.close()
    ms = np.array(lat) * 1e3
    return {"p50_ms": round(float(np.percentile(ms, 50)), 3), "p90_ms": round(float(np.percentile(ms, 90)), 3),
            "queries": nq, "n_gpus": 1, "path": "device-resident streaming data: select + fused decode/denormalise + D2H",
            "kernels_ms": kern, "lossless_spot_checks": checked, "lossless": lossless}


def pmc_for(path, kernel, px, field):
    """Per-launch PMC figure `field` of `kernel` from a committed summary (tools/pmc_traffic.py) measured on this
    same workload (C4 slab of `px` pixels); None when absent or taken on another workload."""
    try:
        d = json.loads(Path(path).read_text())
    except (OSError, ValueError):
        return None
    if d.get("pixels_per_launch") not in (None, px):
        return None
    k = d.get("kernels", {}).get(KERNEL_SYMBOL.get(kernel, kernel))
    return None if k is None or field not in k else k[field]


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
    mt = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    if args.cpu_threads == 1 and mt > 1:
        t0 = time.perf_counter()
        m_arena, m_off, _, _ = O.encode_tiles(band, T, threads=mt)
        dt_mt = time.perf_counter() - t0
        res["multi_thread"] = {"value": round(h * W / dt_mt / 1e6, 2), "cores": mt, "seconds": round(dt_mt, 3),
                               "bit_exact_vs_gpu": bool(m_arena.tobytes() == o_arena.tobytes())}
    return res


if __name__ == "__main__":
    main()
