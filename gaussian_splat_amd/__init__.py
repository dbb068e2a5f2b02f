"""gaussian_splat_amd — MI355X-native Gaussian-splat tile rasterizer.

Host mirror of nshelton/gaussian_splat's renderer API over libgsplat.so (HIP,
gfx950).  See DESIGN.md for the pipeline and INTEGRATION.md for the C-ABI.
"""
from .api import (InstancedSplatRenderer, Options, PLYLoader, Scene, ShardedGroup, TrackballCamera, default_camera,
                  look_at, perspective, radix_sort_pairs, RECORD_DTYPE, POINT_FLOATS)
from ._lib import GsError, lib

__all__ = ["InstancedSplatRenderer", "Options", "PLYLoader", "Scene", "ShardedGroup", "TrackballCamera", "default_camera",
           "look_at", "perspective", "radix_sort_pairs", "RECORD_DTYPE", "POINT_FLOATS", "GsError", "lib"]
