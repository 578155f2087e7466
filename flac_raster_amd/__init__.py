"""flac_raster_amd -- MI355X-native spatial-FLAC raster codec (drop-in for flac-raster's hot path).

Host side mirrors the reference Python API (src/flac_raster): RasterFLACConverter (converter.py),
SpatialFLACEncoder / SpatialIndex / SpatialFrame (spatial_encoder.py), and the create-streaming /
extract-streaming commands (cli.py).  All sample arithmetic runs in libflac_raster_amd.so (HIP, gfx950).
"""
__version__ = "0.1.0"
