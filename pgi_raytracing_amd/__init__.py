"""pgi_raytracing_amd -- MI355X-native Whitted trace path of rddrdhd/PGI_RayTracing.

The product is ``lib/libpgrt.so`` (gfx950 HIP kernels behind the C ABI of include/pgrt.h);
this package is its Python host API (``raytracer``), the data layouts (``abi``) and host-side
scene setup (``scene``).
"""
from . import abi  # noqa: F401
from .scene import LightData, MaterialData, Scene, TextureData  # noqa: F401

__all__ = ["abi", "Scene", "TextureData", "MaterialData", "LightData"]
