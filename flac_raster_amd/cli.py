"""flac-raster command line (reference cli.py:15-93, 620-804, 875-1039): convert, create-streaming,
extract-streaming -- same command names, options and defaults; every sample goes through the GPU codec."""
from __future__ import annotations

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
    compression_level: int = typer.Option(5, "--compression", "-c", min=0, max=8, help="FLAC compression level (0-8)"),
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
    if output_file.exists() and not force:
        typer.echo(f"Error: Output file already exists: {output_file}", err=True)
        raise typer.Exit(1)
    try:
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


def main():
    app()


if __name__ == "__main__":
    main()
