"""ctypes binding of libvrhip.so (the C-ABI of include/vrhip.h).

The shared object is built in-tree by ``volume_renderer_amd/csrc/Makefile`` (``__graft_entry__.build``).
There is no fallback: if the library is missing, importing the bindings raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_PATH = os.path.join(_HERE, "libvrhip.so")
LIB_PATH = os.environ.get("VR_LIB_PATH") or _DEFAULT_PATH  # override: A/B builds

VR_OK = 0
VR_HOST = 0
VR_DEVICE = 1


class VrVolume(ctypes.Structure):
    _fields_ = [("data", c_void_p), ("dims", c_uint64 * 3), ("last_update", c_uint64),
                ("location", c_int32), ("reserved", c_int32)]


class VrLight(ctypes.Structure):
    _fields_ = [("position", c_float * 3), ("color", c_float * 3)]


class VrRenderArgs(ctypes.Structure):
    _fields_ = [("lights", POINTER(VrLight)), ("num_lights", c_int64),
                ("illumination", POINTER(VrVolume)), ("factors", c_float * 3),
                ("element_size_um", c_float * 3), ("resolution", c_uint64 * 2),
                ("rotation_flipped", c_float * 9), ("props", c_float * 3),
                ("opacity_threshold", c_float), ("color", c_float * 3)]


class VrSlab(ctypes.Structure):
    _fields_ = [("depth", c_uint64), ("z_first", c_uint64), ("z0", ctypes.c_double), ("z1", ctypes.c_double),
                ("direction", c_int32), ("reserved", c_int32)]


class VrPartition(ctypes.Structure):
    _fields_ = [("block_cols", c_int32), ("part", c_int32), ("num_parts", c_int32),
                ("reserved", c_int32)]


class VrChannel(ctypes.Structure):
    _fields_ = [("handle", c_void_p), ("time_last_mem_sync", c_uint64),
                ("emission", POINTER(VrVolume)), ("reflection", POINTER(VrVolume)),
                ("absorption", POINTER(VrVolume)), ("dx", POINTER(VrVolume)), ("dy", POINTER(VrVolume)),
                ("dz", POINTER(VrVolume)), ("args", POINTER(VrRenderArgs))]


class VrError(RuntimeError):
    """A non-zero status from libvrhip; ``code`` is the vr_status value."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


_lib = None

# (name, restype, argtypes) for every symbol of include/vrhip.h
SIGNATURES = [
    ("vr_new", c_int, [POINTER(c_void_p)]),
    ("vr_new_multi", c_int, [POINTER(c_int32), c_int32, POINTER(c_void_p)]),
    ("vr_delete", c_int, [c_void_p]),
    ("vr_mem_info", c_int, [c_void_p, c_char_p, c_size_t]),
    ("vr_sync_volumes", c_int, [c_void_p, c_uint64, POINTER(VrVolume), POINTER(VrVolume), POINTER(VrVolume),
                                POINTER(VrVolume), POINTER(VrVolume), POINTER(VrVolume)]),
    ("vr_render", c_int, [c_void_p, POINTER(VrRenderArgs), c_void_p]),
    ("vr_render_stereo", c_int, [c_void_p, POINTER(VrRenderArgs), c_float, c_void_p, c_void_p]),
    ("vr_render_channels", c_int, [POINTER(VrChannel), c_int32, c_int32, c_float, c_void_p]),
    ("vr_render_channels_device", c_int, [POINTER(VrChannel), c_int32, c_int32, c_float, c_void_p, c_void_p]),
    ("vr_sum_channels_device", c_int, [c_void_p, c_int32, c_int32, c_uint64, c_void_p, c_void_p]),
    ("vr_henyey_greenstein", c_int, [c_uint32, c_float, c_void_p]),
    ("vr_timestamp", c_uint64, []),
    ("vr_render_device", c_int, [c_void_p, POINTER(VrRenderArgs), POINTER(VrPartition), c_void_p, c_void_p,
                                 c_void_p]),
    ("vr_render_stereo_device", c_int, [c_void_p, POINTER(VrRenderArgs), c_float, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    ("vr_partition_columns", c_int64, [c_int64, POINTER(VrPartition)]),
    ("vr_assemble_partitions", c_int, [c_void_p, c_int64, c_int64, c_int32, c_int32, c_int64, c_void_p,
                                       c_void_p]),
    ("vr_depth_lanes", c_int, [c_int64, c_int64]),
    ("vr_depth_lanes_tau", c_int, [c_int64, c_int64, ctypes.c_double]),
    ("vr_render_slab", c_int, [c_void_p, POINTER(VrRenderArgs), POINTER(VrSlab), POINTER(VrPartition), c_void_p,
                                c_void_p, c_void_p]),
    ("vr_slab_planes", c_int, [POINTER(c_uint64), POINTER(c_float), ctypes.c_double, ctypes.c_double,
                               POINTER(c_uint64), POINTER(c_uint64)]),
    ("vr_synth_shell_device", c_int, [c_void_p, c_uint64, c_void_p]),
    ("vr_synth_shell_planes_device", c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_void_p]),
    ("vr_gradient_device", c_int, [c_void_p, POINTER(c_uint64), c_void_p, c_void_p, c_void_p, c_void_p]),
    ("vr_henyey_greenstein_device", c_int, [c_uint32, c_float, c_void_p, c_void_p]),
    ("vr_normalize_device", c_int, [c_void_p, c_uint64, ctypes.c_double, ctypes.c_double, c_void_p, c_void_p]),
    ("vr_resize_device", c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64), c_void_p, c_void_p]),
    ("vr_resize_contributions", c_int, [c_uint64, c_uint64, POINTER(c_int32), c_void_p, c_void_p]),
    ("vr_debug_slot_transition", c_int, [POINTER(c_int32), c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                                         POINTER(c_int32), POINTER(c_int32)]),
    ("vr_last_error", c_char_p, []),
    ("vr_hip_errors", c_int64, [c_char_p, c_size_t]),
    ("vr_last_march_kernel", c_int, [c_char_p, c_size_t]),
    ("vr_set_option", c_int, [c_char_p, c_int64]),
    ("vr_version", c_char_p, []),
]


def lib():
    """Load libvrhip.so once; raise (never fall back) if it is absent."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: when PyTorch-ROCm is installed it carries its own
        # libamdhip64.so.7 / libhsa-runtime64.so.1; loading it first makes libvrhip bind to the
        # same copy (same SONAMEs), so torch tensors and libvrhip buffers share one device context.
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libvrhip.so not built at {LIB_PATH}: run __graft_entry__.build() "
                              "(make -C volume_renderer_amd/csrc)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            if LIB_PATH != _DEFAULT_PATH and not hasattr(handle, name):
                continue  # an A/B build of an earlier tree (VR_LIB_PATH) may predate a diagnostic entry
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc: int) -> None:
    if rc != VR_OK:
        msg = lib().vr_last_error().decode(errors="replace")
        raise VrError(rc, msg)


def hip_errors() -> tuple[int, list[str]]:
    """HIP errors the library handled or found pending at an API entry (vr_hip_errors): the count
    since load and the last log lines, newest last."""
    buf = ctypes.create_string_buffer(32 * 400)
    n = lib().vr_hip_errors(buf, len(buf))
    return int(n), [l for l in buf.value.decode(errors="replace").splitlines() if l]
