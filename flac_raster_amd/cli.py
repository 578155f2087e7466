"""flac-raster command line (reference cli.py:15-93, 620-804, 875-1039): convert, create-streaming,
extract-streaming -- same command names, options and defaults; every sample goes through the GPU codec."""
from __future__ import annotations

import json
import logging
from pathlib import Path
from typing import Optional

import typer

app = typer.Typer(name="flac-raster", add_completion=False,
                  help="Convert between TIFF raster and FLAC audio formats while preserving geospatial metadata "
                       "(MI355X codec)")
log = logging.getLogger("flac_raster")


@app.command()
def convert(
    input_file: Path = typer.Argument(..., help="Input file (TIFF or FLAC)"),
    output_file: Optional[Path] = typer.Option(None, "--output", "-o", help="Output file path"),
    compression_level: int = typer.Option(5, "--compression", "-c", min=0, max=8,
                                          help="FLAC compression level (0-8); the GPU encoder implements 0-5 "
                                               "(not 1/4 on two bands) and rejects the others"),
    force: bool = typer.Option(False, "--force", "-f", help="Overwrite existing output file"),
    verbose: bool = typer.Option(False, "--verbose", "-v", help="Enable verbose logging"),
    spatial_tiling: bool = typer.Option(False, "--spatial", "-s", help="Enable spatial tiling for HTTP range streaming"),
    tile_size: int = typer.Option(512, "--tile-size", help="Size of spatial tiles (default: 512x512)"),
):
    """Convert between TIFF and FLAC formats"""
    from .converter import RasterFLACConverter
    if verbose:
        logging.getLogger("flac_raster").setLevel(logging.DEBUG)
    if not input_file.exists():
        typer.echo(f"Error: Input file does not exist: {input_file}", err=True)
        raise typer.Exit(1)
    suf = input_file.suffix.lower()
    if suf in (".tif", ".tiff"):
        kind, out_suf = "tiff_to_flac", ".flac"
    elif suf == ".flac":
        kind, out_suf = "flac_to_tiff", ".tif"
    else:
        typer.echo(f"Error: Unsupported file format: {suf}", err=True)
        raise typer.Exit(1)
    output_file = output_file or input_file.with_suffix(out_suf)
    if output_file.exists() and not force:
        typer.echo(f"Error: Output file already exists: {output_file}", err=True)
        raise typer.Exit(1)
    try:
        conv = RasterFLACConverter()
        if kind == "tiff_to_flac":
            res = conv.tiff_to_flac(input_file, output_file, compression_level, spatial_tiling, tile_size)
            if spatial_tiling and res:
                typer.echo(f"Spatial index created with {len(res.frames)} tiles")
        else:
            conv.flac_to_tiff(input_file, output_file)
        typer.echo(f"SUCCESS: {output_file}")
    except Exception as e:  # reference: any error -> exit 1 (cli.py:90-93)
        log.exception("Conversion failed")
        typer.echo(f"Error during conversion: {e}", err=True)
        raise typer.Exit(1)


@app.command("create-streaming")
def create_streaming(
    input_file: Path = typer.Argument(..., help="Input TIFF file to convert"),
    output_file: Optional[Path] = typer.Option(None, "--output", "-o", help="Output streaming FLAC file"),
    tile_size: int = typer.Option(1024, "--tile-size", help="Size of streaming tiles (default: 1024x1024)"),
    force: bool = typer.Option(False, "--force", "-f", help="Overwrite existing output file"),
    gpus: int = typer.Option(1, "--gpus", help="Extension: shard the tiles over N local GPUs (one process each)"),
    distributed: bool = typer.Option(False, "--distributed",
                                     help="Extension: run as one rank of a launcher (RANK/WORLD_SIZE/LOCAL_RANK/"
                                          "MASTER_ADDR/MASTER_PORT in the environment)"),
):
    """Create Netflix-style streaming FLAC with self-contained tiles"""
    from . import streaming
    if not input_file.exists():
        typer.echo(f"Error: Input file does not exist: {input_file}", err=True)
        raise typer.Exit(1)
    if input_file.suffix.lower() not in (".tif", ".tiff"):
        typer.echo(f"Error: Input must be a TIFF file, got: {input_file.suffix}", err=True)
        raise typer.Exit(1)
    if output_file is None:
        output_file = input_file.with_suffix(".flac").with_name(input_file.stem + "_streaming.flac")
    if output_file.exists() and not force and not distributed:
        typer.echo(f"Error: Output file already exists: {output_file}", err=True)
        raise typer.Exit(1)
    if gpus > 1 and not distributed:
        from .launch import run_ranks
        argv = ["create-streaming", str(input_file), "--output", str(output_file), "--tile-size", str(tile_size),
                "--force", "--distributed"]
        rc = run_ranks(gpus, argv)
        if rc:
            typer.echo(f"Error creating streaming FLAC: a rank exited with {rc}", err=True)
            raise typer.Exit(1)
        typer.echo(f"SUCCESS: {output_file} ({gpus} GPUs)")
        return
    try:
        if distributed:
            from .distributed import create_streaming_distributed
            index = create_streaming_distributed(input_file, output_file, tile_size)
        else:
            index = streaming.create_streaming(input_file, output_file, tile_size)
        typer.echo(f"SUCCESS: {output_file} ({len(index['frames'])} tiles)")
    except Exception as e:
        log.exception("Streaming FLAC creation failed")
        typer.echo(f"Error creating streaming FLAC: {e}", err=True)
        raise typer.Exit(1)


@app.command("extract-streaming")
def extract_streaming(
    flac_url: str = typer.Argument(..., help="Streaming FLAC file (local path or HTTP URL)"),
    bbox: Optional[str] = typer.Option(None, "--bbox", "-b", help="Bounding box as 'xmin,ymin,xmax,ymax'"),
    tile_id: Optional[int] = typer.Option(None, "--tile-id", help="Extract specific tile by ID"),
    output: Path = typer.Option(..., "--output", "-o", help="Output TIFF file path"),
    center: bool = typer.Option(False, "--center", help="Extract center tile"),
    last: bool = typer.Option(False, "--last", help="Extract last tile"),
    mosaic: bool = typer.Option(False, "--mosaic", help="Extension: mosaic every tile intersecting --bbox"),
):
    """Extract tiles from Netflix-style streaming FLAC files"""
    from . import streaming
    coords = None
    if bbox:
        try:
            coords = [float(x.strip()) for x in bbox.split(",")]
            if len(coords) != 4:
                raise ValueError("Bbox must have exactly 4 coordinates")
        except (ValueError, IndexError) as e:
            typer.echo(f"Error: Invalid bbox format. Use 'xmin,ymin,xmax,ymax': {e}", err=True)
            raise typer.Exit(1)
    try:
        if mosaic and coords is not None:
            from . import geotiff
            arr, win, tr = streaming.extract_bbox_mosaic(flac_url, coords)
            n, index = streaming.read_index(flac_url)
            crs = index.get("crs")
            epsg = int(crs.split(":")[1]) if crs and crs.upper().startswith("EPSG:") else None
            geotiff.write(output, arr, transform=geotiff.Affine(*tr[:6]), epsg=epsg)
            typer.echo(f"SUCCESS: mosaic {win} -> {output}")
        else:
            f = streaming.extract_streaming(flac_url, output, bbox=coords, tile_id=tile_id, center=center, last=last)
            typer.echo(f"SUCCESS: Extracted tile {f['frame_id']} to {output}")
    except (KeyError, LookupError, ValueError) as e:
        typer.echo(f"Error: {e}", err=True)
        raise typer.Exit(1)
    except Exception as e:
        log.exception("Streaming extraction failed")
        typer.echo(f"Error during streaming extraction: {e}", err=True)
        raise typer.Exit(1)


def _bbox(text: str):
    coords = [float(x.strip()) for x in text.split(",")]
    if len(coords) != 4:
        raise ValueError("Bbox must have 4 coordinates")
    return coords


@app.command()
def info(file_path: str = typer.Argument(..., help="FLAC or TIFF file to inspect (local path or HTTP URL)")):
    """Display information about a FLAC or TIFF file"""  # reference cli.py:96-244
    from rich.console import Console
    con = Console()
    is_url = file_path.startswith(("http://", "https://"))
    if not is_url:
        p = Path(file_path)
        if not p.exists():
            con.print(f"[red]Error: File does not exist: {file_path}[/red]")
            raise typer.Exit(1)
        suffix = p.suffix.lower()
    else:
        from urllib.parse import urlparse
        suffix = Path(urlparse(file_path).path).suffix.lower()
    if suffix in (".tif", ".tiff"):
        from . import geotiff
        if is_url:
            con.print("[red]Error: URL-based TIFF inspection not supported yet[/red]")
            raise typer.Exit(1)
        r = geotiff.read(file_path)
        con.print("[cyan]TIFF Information:[/cyan]")
        con.print(f"  Dimensions: {r.width} x {r.height}")
        con.print(f"  Bands: {r.count}")
        con.print(f"  Data type: {r.dtype}")
        con.print(f"  CRS: {r.crs_string}")
        con.print(f"  Bounds: {r.bounds}")
        con.print(f"  File size: {Path(file_path).stat().st_size / 1024 / 1024:.2f} MB")
    elif suffix == ".flac":
        con.print("[cyan]FLAC Information:[/cyan]")
        if is_url:
            try:
                import requests
                from .spatial_encoder import SpatialFLACStreamer
                size = int(requests.head(file_path).headers.get("content-length", 0))
                con.print(f"  Remote file size: {size / 1024 / 1024:.2f} MB")
                st = SpatialFLACStreamer(file_path)
                con.print(f"  Spatial tiles: {len(st.spatial_index.frames)}")
                con.print(f"  Total indexed data: {st.spatial_index.total_bytes:,} bytes")
                con.print("\n[green]Spatial FLAC Metadata:[/green]")
                con.print("  Spatial format: Yes")
                con.print(f"  Total frames/tiles: {len(st.spatial_index.frames)}")
                con.print(f"  CRS: {st.spatial_index.crs}")
                con.print(f"  Transform: {st.spatial_index.transform}")
            except Exception as e:
                con.print(f"  [red]Error reading remote FLAC file: {e}[/red]")
            return
        from . import container
        buf = Path(file_path).read_bytes()
        meta = None
        try:
            import numpy as np
            from ._native import default_context
            meta = container.parse_metadata(buf)
            frames = np.frombuffer(buf, dtype=np.uint8)[meta.audio_offset:]
            md0 = container.read_raster_tags(meta)
            n = int(md0["width"]) * int(md0["height"]) if md0 else None
            if n is None:
                raise ValueError("sample count unknown without geospatial tags (STREAMINFO total is 0)")
            pcm = default_context().decode_frames_host(frames, [0, len(frames)], [n], channels=meta.channels,
                                                       bps=meta.bps, blocksize=meta.blocksize)
            con.print(f"  Sample rate: {meta.sample_rate} Hz")
            con.print(f"  Channels: {meta.channels}")
            con.print(f"  Audio shape: {pcm.shape}")
            con.print("  Data type: float64")
            con.print(f"  File size: {len(buf) / 1024 / 1024:.2f} MB")
        except Exception as e:
            con.print(f"  [red]Error reading FLAC file: {e}[/red]")
            con.print(f"  File size: {len(buf) / 1024 / 1024:.2f} MB")
        shown = False
        try:
            m = meta or container.parse_metadata(buf)
            if m.tag("GEOSPATIAL_CRS") is None:
                raise ValueError("No embedded metadata")
            con.print("\n[green]Embedded Geospatial Metadata:[/green]")
            g = lambda k: m.tag(k) if m.tag(k) is not None else "N/A"  # noqa: E731
            con.print(f"  Original dimensions: {g('GEOSPATIAL_WIDTH')} x {g('GEOSPATIAL_HEIGHT')}")
            con.print(f"  Original bands: {g('GEOSPATIAL_COUNT')}")
            con.print(f"  Original dtype: {g('GEOSPATIAL_DTYPE')}")
            con.print(f"  CRS: {g('GEOSPATIAL_CRS')}")
            con.print(f"  Data range: [{g('GEOSPATIAL_DATA_MIN')}, {g('GEOSPATIAL_DATA_MAX')}]")
            tiled = (m.tag("GEOSPATIAL_SPATIAL_TILING") or "false").lower() == "true"
            con.print(f"  Spatial tiling: {'Yes' if tiled else 'No'}")
            bs = m.tag("GEOSPATIAL_BOUNDS")
            if bs:
                b = json.loads(bs)
                if isinstance(b, dict):
                    b = [b["left"], b["bottom"], b["right"], b["top"]]
                con.print(f"  Bounds: ({b[0]:.6f}, {b[1]:.6f}, {b[2]:.6f}, {b[3]:.6f})")
            shown = True
        except Exception:
            side = Path(file_path).with_suffix(".json")
            if side.exists():
                mj = json.loads(side.read_text())
                con.print(f"\n[yellow]Raster Metadata (from {side.name}):[/yellow]")
                con.print(f"  Original dimensions: {mj['width']} x {mj['height']}")
                con.print(f"  Original bands: {mj['count']}")
                con.print(f"  Original dtype: {mj['dtype']}")
                con.print(f"  CRS: {mj.get('crs', 'None')}")
                if mj.get("bounds"):
                    b = mj["bounds"]
                    con.print(f"  Bounds: ({b['left']}, {b['bottom']}, {b['right']}, {b['top']})")
                shown = True
        if not shown:
            con.print("\n[yellow]No embedded or sidecar metadata found[/yellow]")
    else:
        con.print(f"[red]Error: Unsupported file format: {suffix}[/red]")
        raise typer.Exit(1)


@app.command()
def query(
    flac_file: str = typer.Argument(..., help="Spatial FLAC file to query (local path or HTTP URL)"),
    bbox: str = typer.Option(..., "--bbox", "-b", help="Bounding box as 'xmin,ymin,xmax,ymax'"),
    output: Optional[Path] = typer.Option(None, "--output", "-o", help="Output file for extracted data"),
    format: str = typer.Option("ranges", "--format", "-f", help="Output format: 'ranges' or 'data'"),
):
    """Query spatial FLAC file by bounding box for HTTP range streaming"""  # reference cli.py:293-406
    from rich.console import Console
    from rich.table import Table
    con = Console()
    is_url = flac_file.startswith(("http://", "https://"))
    if not is_url and not Path(flac_file).exists():
        con.print(f"[red]Error: FLAC file does not exist: {flac_file}[/red]")
        raise typer.Exit(1)
    try:
        coords = _bbox(bbox)
    except (ValueError, IndexError) as e:
        con.print(f"[red]Error: Invalid bbox format. Use 'xmin,ymin,xmax,ymax': {e}[/red]")
        raise typer.Exit(1)
    try:
        from .spatial_encoder import SpatialFLACStreamer
        st = SpatialFLACStreamer(flac_file)
        if format == "ranges":
            ranges = st.get_byte_ranges_for_bbox(tuple(coords))
            con.print(f"[green]Found {len(ranges)} byte ranges for bbox {bbox}[/green]")
            table = Table(title=f"HTTP Byte Ranges for {flac_file.split('/')[-1] if is_url else Path(flac_file).name}")
            for c in ("Range #", "Start Byte", "End Byte", "Size (bytes)", "HTTP Range Header"):
                table.add_column(c)
            total = 0
            for i, (a, b) in enumerate(ranges, 1):
                total += b - a + 1
                table.add_row(str(i), f"{a:,}", f"{b:,}", f"{b - a + 1:,}", f"bytes={a}-{b}")
            con.print(table)
            con.print(f"[bold]Total data to fetch: {total:,} bytes[/bold]")
            if output:
                data = {"bbox": coords, "total_ranges": len(ranges), "total_bytes": total,
                        "ranges": [{"start": a, "end": b, "size": b - a + 1} for a, b in ranges],
                        "http_headers": [f"bytes={a}-{b}" for a, b in ranges]}
                with open(output, "w") as fh:
                    json.dump(data, fh, indent=2)
                con.print(f"[green]Ranges saved to: {output}[/green]")
        elif format == "data":
            con.print(f"[cyan]Streaming data for bbox {bbox}...[/cyan]")
            data = st.stream_bbox_data(tuple(coords))
            con.print(f"[green]Extracted {len(data):,} bytes of FLAC data[/green]")
            if output:
                Path(output).write_bytes(data)
                con.print(f"[green]Data saved to: {output}[/green]")
            else:
                con.print("[yellow]Use --output to save extracted data to file[/yellow]")
        else:
            con.print(f"[red]Error: Unknown format '{format}'. Use 'ranges' or 'data'[/red]")
            raise typer.Exit(1)
    except typer.Exit:
        raise
    except FileNotFoundError as e:
        con.print(f"[red]Error: Spatial index not found. File may not have spatial tiling enabled: {e}[/red]")
        raise typer.Exit(1)
    except Exception as e:
        log.exception("Query failed")
        con.print(f"[red]Error during query: {e}[/red]")
        raise typer.Exit(1)


@app.command("spatial-info")
def spatial_info(flac_file: str = typer.Argument(..., help="Spatial FLAC file to analyze (local path or HTTP URL)")):
    """Show spatial index information for FLAC file"""  # reference cli.py:807-872
    from rich.console import Console
    from rich.table import Table
    con = Console()
    is_url = flac_file.startswith(("http://", "https://"))
    if not is_url and not Path(flac_file).exists():
        con.print(f"[red]Error: FLAC file does not exist: {flac_file}[/red]")
        raise typer.Exit(1)
    try:
        from .spatial_encoder import SpatialFLACStreamer
        idx = SpatialFLACStreamer(flac_file).spatial_index
        con.print(f"[green]Spatial FLAC File: {Path(flac_file).name if not is_url else flac_file}[/green]")
        con.print(f"CRS: {idx.crs}")
        con.print(f"Transform: {idx.transform}")
        con.print(f"Total frames/tiles: {len(idx.frames)}")
        table = Table(title="Spatial Frames")
        for c in ("Frame ID", "Bbox (xmin, ymin, xmax, ymax)", "Window (col, row, width, height)", "Byte Range",
                  "Size"):
            table.add_column(c)
        total = 0
        for f in idx.frames[:10]:
            table.add_row(str(f.frame_id), f"({f.bbox[0]:.6f}, {f.bbox[1]:.6f}, {f.bbox[2]:.6f}, {f.bbox[3]:.6f})",
                          f"({f.window.col_off}, {f.window.row_off}, {f.window.width}, {f.window.height})",
                          f"{f.byte_offset}-{f.byte_offset + f.byte_size - 1}", f"{f.byte_size:,} bytes")
            total += f.byte_size
        con.print(table)
        if len(idx.frames) > 10:
            con.print(f"[yellow]... and {len(idx.frames) - 10} more frames[/yellow]")
        con.print(f"[bold]Total indexed data: {total:,} bytes[/bold]")
    except FileNotFoundError as e:
        con.print(f"[red]Error: Spatial index not found. File may not have spatial tiling enabled: {e}[/red]")
        raise typer.Exit(1)
    except Exception as e:
        log.exception("Spatial info failed")
        con.print(f"[red]Error reading spatial info: {e}[/red]")
        raise typer.Exit(1)


def main():
    app()


if __name__ == "__main__":
    main()
