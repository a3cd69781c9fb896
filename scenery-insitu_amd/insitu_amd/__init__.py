"""insitu_amd -- MI355X-native distributed VDI volume-rendering hot path of scenery-insitu.

The compute lives in libinsitu_hip.so (HIP kernels for gfx950 + RCCL); this package is the
Python host mirror of the reference's renderer API over that C ABI.
"""
from . import native, scene
from .renderer import DistributedVolumes, InSituContext

__all__ = ["native", "scene", "InSituContext", "DistributedVolumes"]
