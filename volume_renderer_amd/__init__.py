"""volume_renderer_amd -- MI355X-native drop-in for the ray-march path of raphiniert-com/volume_renderer.

The product is ``libvrhip.so`` (HIP kernels for gfx950 + the C-ABI of ``include/vrhip.h``).  This
package holds its ctypes binding and a Python mirror of the reference's MATLAB API
(``VolumeRender``, ``Volume``, ``LightSource``, ``StereoRenderMode``, the ``volumeRender``,
``HenyeyGreenstein`` and ``timestamp`` mex entry points).  Importing it loads the library and fails
loudly if it has not been built -- there is no CPU fallback.
"""
from ._lib import VrError, lib
from .mex import HenyeyGreenstein, set_clock, timestamp, volumeRender
from .volume import LightSource, Volume
from .volume_render import StereoRenderMode, VolumeRender

lib()  # fail at import time if libvrhip.so is missing

__all__ = ["VolumeRender", "Volume", "LightSource", "StereoRenderMode", "volumeRender", "HenyeyGreenstein",
           "timestamp", "set_clock", "VrError", "lib"]
