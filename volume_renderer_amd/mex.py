"""The three MEX entry points of the reference, re-exposed over libvrhip's C-ABI.

``volumeRender(cmd, ...)`` keeps the command protocol and the argument marshalling of
/root/reference/src/C/mex/render.cpp:50-278 (positional MATLAB arguments, same order, same
permutations -- done inside libvrhip exactly where the reference does them), ``HenyeyGreenstein``
mirrors /root/reference/src/C/mex/HenyeyGreenstein.cc:29-96 and ``timestamp`` mirrors
/root/reference/src/C/mex/timestamp.cpp:17-33.  MATLAB values map to Python as:
logical ``false`` -> ``False``; ``single``/``uint64`` arrays -> numpy arrays (column-major);
``Volume``/``LightSource`` objects -> the classes of this package.
"""
from __future__ import annotations

import ctypes
import warnings

import numpy as np

from . import _lib
from ._lib import VrLight, VrRenderArgs, VrVolume, check, lib

_clock = None


def set_clock(fn) -> None:
    """Replace the millisecond clock behind ``timestamp`` (tests use a deterministic counter;
    the reference's change tracking misses updates made within the same millisecond,
    SURVEY.md A.9).  ``None`` restores the real clock."""
    global _clock
    _clock = fn


def timestamp() -> np.uint64:
    """ms since the epoch, low 32 bits (timestamp.cpp stores it through an int*)."""
    if _clock is not None:
        return np.uint64(_clock())
    return np.uint64(lib().vr_timestamp())


def HenyeyGreenstein(n, g=0.8) -> np.ndarray:
    """N x N x N single LUT of the Henyey-Greenstein phase function (HenyeyGreenstein.cc)."""
    n = int(n)
    out = np.empty((n, n, n), dtype=np.float32, order="F")
    check(lib().vr_henyey_greenstein(ctypes.c_uint32(n), ctypes.c_float(g), out.ctypes.data_as(ctypes.c_void_p)))
    return out


def _is_false(x) -> bool:
    return isinstance(x, (bool, np.bool_)) and not bool(x)


def _matlab_dims(a: np.ndarray):
    """mxGetDimensions as the mex reads them: (d0, d1, d2) with d2 = 1 for 2-D data."""
    if a.ndim == 0:
        return (1, 1, 1)
    if a.ndim == 1:
        return (a.shape[0], 1, 1)
    if a.ndim == 2:
        return (a.shape[0], a.shape[1], 1)
    if a.ndim == 3:
        return tuple(a.shape)
    raise ValueError("volumes must have at most 3 dimensions")


class DeviceVolume:
    """A Volume whose Data already lives in HBM (e.g. a torch tensor on cuda): MATLAB-shaped dims
    (d0, d1, d2), column-major fp32 at device address `ptr`.  Synced device-to-device."""

    def __init__(self, ptr: int, dims, last_update=None, owner=None):
        self.ptr = int(ptr)
        d = tuple(int(x) for x in dims) + (1,) * (3 - len(dims))
        self.dims = d[:3]
        self.TimeLastUpdate = timestamp() if last_update is None else np.uint64(last_update)
        self.owner = owner  # keeps the backing allocation alive

    @classmethod
    def from_tensor(cls, t, dims=None, last_update=None):
        """`t` is a contiguous float32 cuda tensor holding the column-major data."""
        import torch
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise TypeError("DeviceVolume needs a contiguous float32 cuda tensor")
        dims = dims if dims is not None else tuple(reversed(t.shape))  # C-order (z,y,x) tensor -> (x,y,z)
        return cls(t.data_ptr(), dims, last_update, owner=t)

    def min(self):
        return 0.0


def _vr_volume(vol) -> VrVolume:
    """mxMake_volume (volumeRender.cpp:307-342): zero-copy view of Data + TimeLastUpdate."""
    v = VrVolume()
    if isinstance(vol, DeviceVolume):
        v.data = vol.ptr
        for i in range(3):
            v.dims[i] = vol.dims[i]
        v.last_update = int(vol.TimeLastUpdate)
        v.location = _lib.VR_DEVICE
        return v
    data = vol.Data
    if not (isinstance(data, np.ndarray) and data.dtype == np.float32 and
            (data.flags.f_contiguous or data.ndim <= 1)):
        raise TypeError("Volume.Data must be a column-major single array")
    v.data = data.ctypes.data if data.size else None
    d = _matlab_dims(data)
    for i in range(3):
        v.dims[i] = d[i]
    v.last_update = int(vol.TimeLastUpdate)
    v.location = _lib.VR_HOST
    return v


def _handle(h) -> ctypes.c_void_p:
    a = np.asarray(h)
    if a.size != 1 or a.dtype != np.uint64:
        raise _lib.VrError(_lib.VR_OK + 1, "Input must be a real uint64 scalar.")
    return ctypes.c_void_p(int(a.reshape(-1)[0]))


def _f32(x, n: int, name: str) -> np.ndarray:
    a = np.asarray(x, dtype=np.float32).reshape(-1, order="F")
    if a.size < n:
        raise ValueError(f"{name}: expected {n} values")
    return a


def render_args(lights_arg, illum_arg, factors, element_size_um, resolution, rotation_flipped, props,
                opacity_threshold, color):
    """Marshal the positional 'render' arguments (prhs[2..10], render.cpp:142-240) into the
    C-ABI struct.  Returns (VrRenderArgs, keep-alive list)."""
    ra = VrRenderArgs()
    keep = []
    if not (_is_false(lights_arg) or _is_false(illum_arg)):
        lights = list(lights_arg) if isinstance(lights_arg, (list, tuple, np.ndarray)) else [lights_arg]
        arr = (VrLight * max(len(lights), 1))()
        for i, ls in enumerate(lights):
            pos = _f32(ls.Position, 3, "Position")
            col = _f32(ls.Color, 3, "Color")
            for k in range(3):
                arr[i].position[k] = pos[k]
                arr[i].color[k] = col[k]
        illum = _vr_volume(illum_arg)
        keep += [arr, illum, getattr(illum_arg, "Data", None)]
        ra.lights = ctypes.cast(arr, ctypes.POINTER(VrLight))
        ra.num_lights = len(lights)
        ra.illumination = ctypes.pointer(illum)
    else:
        ra.num_lights = -1
        ra.illumination = None
    fac = _f32(factors, 3, "factors")
    es = _f32(element_size_um, 3, "ElementSizeUm")
    res = np.asarray(resolution).reshape(-1)
    rot = _f32(rotation_flipped, 9, "RotationMatrix")
    pr = _f32(props, 3, "props")
    thr = np.float32(np.asarray(opacity_threshold).reshape(-1)[0])
    col = _f32(color, 3, "Color")
    for k in range(3):
        ra.factors[k] = fac[k]
        ra.element_size_um[k] = es[k]
        ra.props[k] = pr[k]
        ra.color[k] = col[k]
    for k in range(9):
        ra.rotation_flipped[k] = rot[k]
    ra.resolution[0] = int(res[0])
    ra.resolution[1] = int(res[1])
    ra.opacity_threshold = thr
    return ra, keep


def partition(block_cols: int, part: int, num_parts: int) -> _lib.VrPartition:
    p = _lib.VrPartition()
    p.block_cols, p.part, p.num_parts = int(block_cols), int(part), int(num_parts)
    return p


def partition_columns(width: int, part) -> int:
    return int(lib().vr_partition_columns(int(width), ctypes.byref(part) if part is not None else None))


SLAB_PLANES = 10  # include/vrhip.h VR_SLAB_PLANES


def slab(depth: int, z_first: int, z0: float, z1: float, direction: int) -> _lib.VrSlab:
    """vr_slab: the synced emission volume holds planes [z_first, ...) of a volume of depth
    `depth`; the render owns the samples with z0 <= p.z * depth < z1; direction +1 / -1, or 0
    (both: the top slab's ascending launch, where the descending rays start)."""
    s = _lib.VrSlab()
    s.depth, s.z_first, s.z0, s.z1, s.direction = int(depth), int(z_first), float(z0), float(z1), int(direction)
    return s


def slab_planes(dims, element_size_um, z0: float, z1: float):
    """(first, count): the planes a slab owning [z0, z1) of a (d0, d1, D) volume must hold."""
    d = (ctypes.c_uint64 * 3)(*[int(x) for x in dims])
    es = (ctypes.c_float * 3)(*[float(x) for x in element_size_um])
    first, count = ctypes.c_uint64(0), ctypes.c_uint64(0)
    check(lib().vr_slab_planes(d, es, float(z0), float(z1), ctypes.byref(first), ctypes.byref(count)))
    return int(first.value), int(count.value)


def render_slab(handle, ra: VrRenderArgs, sl, d_state_in: int, d_state_out: int, stream: int = 0,
                part=None) -> None:
    """vr_render_slab: march this slab's samples of every ray (of the part's columns, if a
    partition is given); state = SLAB_PLANES planes of cols*H floats (colour, alpha, goes-on,
    and the resume point t, x, y, z, sample index of a ray that goes on)."""
    check(lib().vr_render_slab(_handle(handle), ctypes.byref(ra), ctypes.byref(sl),
                               ctypes.byref(part) if part is not None else None,
                               ctypes.c_void_p(int(d_state_in)) if d_state_in else None,
                               ctypes.c_void_p(int(d_state_out)), ctypes.c_void_p(int(stream))))


def depth_lanes(part_cols: int, height: int, texels_per_pixel=None) -> int:
    """Depth lanes the march uses for a launch of this shape on the current device (vr_depth_lanes;
    with texels_per_pixel, vr_depth_lanes_tau: the choice a render at that sampling density makes)."""
    if texels_per_pixel is None:
        return int(lib().vr_depth_lanes(int(part_cols), int(height)))
    return int(lib().vr_depth_lanes_tau(int(part_cols), int(height), float(texels_per_pixel)))


def render_device(handle, ra: VrRenderArgs, d_out: int, part=None, d_steps: int = 0, stream: int = 0) -> None:
    """'render' into device memory (vr_render_device): asynchronous on `stream`."""
    check(lib().vr_render_device(_handle(handle), ctypes.byref(ra), ctypes.byref(part) if part is not None else None,
                                 ctypes.c_void_p(int(d_out)), ctypes.c_void_p(int(d_steps)) if d_steps else None,
                                 ctypes.c_void_p(int(stream)) if stream else None))


def render_stereo_device(handle, ra: VrRenderArgs, base: float, d_left: int, d_right: int, d_steps: int = 0,
                         stream: int = 0) -> None:
    """Both eyes of a stereo pair into device memory in one launch (vr_render_stereo_device): the
    left eye (camera offset -base) to d_left, the right (+base) to d_right; ra.props[0] is ignored."""
    check(lib().vr_render_stereo_device(_handle(handle), ctypes.byref(ra), ctypes.c_float(base),
                                        ctypes.c_void_p(int(d_left)), ctypes.c_void_p(int(d_right)),
                                        ctypes.c_void_p(int(d_steps)) if d_steps else None,
                                        ctypes.c_void_p(int(stream)) if stream else None))


def set_option(name: str, value: int) -> None:
    """vr_set_option: a process-wide library option (include/vrhip.h)."""
    check(lib().vr_set_option(name.encode(), int(value)))


def enable_test_switches(on: bool = True) -> None:
    """Let the library read the kernel-variant / schedule switches of the environment (VR_NO_LDS,
    VR_DEPTH_LANES, VR_SCHED, ...; INTEGRATION.md "Runtime switches") -- the GPU tests and the
    measurement tools; the MATLAB MEX never does, so a MATLAB session's environment cannot.  (An A/B
    build of an earlier tree, VR_LIB_PATH, may predate the option: a DIAG=1 build reads them anyway.)"""
    if not hasattr(lib(), "vr_set_option"):
        return
    set_option("test_switches", 1 if on else 0)


def last_march_kernel() -> str:
    """The demangled name of the march kernel instantiation the last render launched."""
    buf = ctypes.create_string_buffer(256)
    check(lib().vr_last_march_kernel(buf, len(buf)))
    return buf.value.decode()


def assemble_partitions(d_parts: int, width: int, height: int, block_cols: int, num_parts: int, max_cols: int,
                        d_out: int, stream: int = 0) -> None:
    check(lib().vr_assemble_partitions(ctypes.c_void_p(int(d_parts)), int(width), int(height), int(block_cols),
                                       int(num_parts), int(max_cols), ctypes.c_void_p(int(d_out)),
                                       ctypes.c_void_p(int(stream)) if stream else None))


def synth_shell_device(d_out: int, n: int, stream: int = 0) -> None:
    check(lib().vr_synth_shell_device(ctypes.c_void_p(int(d_out)), int(n),
                                      ctypes.c_void_p(int(stream)) if stream else None))


def synth_shell_planes_device(d_out: int, n: int, z_first: int, count: int, stream: int = 0) -> None:
    check(lib().vr_synth_shell_planes_device(ctypes.c_void_p(int(d_out)), int(n), int(z_first), int(count),
                                             ctypes.c_void_p(int(stream))))


def gradient_device(d_data: int, dims, d_gx: int, d_gy: int, d_gz: int, stream: int = 0) -> None:
    """Volume.grad on the device (vr_gradient_device): MATLAB gradient() of the column-major single
    array at d_data with dims (d0, d1, d2) into d_gx (dim 2), d_gy (dim 1), d_gz (dim 3)."""
    dd = (ctypes.c_uint64 * 3)(*[int(x) for x in dims])
    _lib.check(_lib.lib().vr_gradient_device(d_data, dd, d_gx, d_gy, d_gz, stream))


def henyey_greenstein_device(n: int, g: float, d_out: int, stream: int = 0) -> None:
    """vr_henyey_greenstein_device: HenyeyGreenstein(n, g) into device memory (n^3 floats)."""
    check(lib().vr_henyey_greenstein_device(ctypes.c_uint32(int(n)), ctypes.c_float(g), ctypes.c_void_p(int(d_out)),
                                            ctypes.c_void_p(int(stream)) if stream else None))


def normalize_device(d_in: int, n: int, new_min: float, new_max: float, d_out: int, stream: int = 0) -> None:
    """vr_normalize_device: Volume.normalize of n single values in device memory (d_out may be d_in)."""
    check(lib().vr_normalize_device(ctypes.c_void_p(int(d_in)), int(n), float(new_min), float(new_max),
                                    ctypes.c_void_p(int(d_out)), ctypes.c_void_p(int(stream)) if stream else None))


def resize_device(d_in: int, in_dims, out_dims, d_out: int, stream: int = 0) -> None:
    """vr_resize_device: Volume.resize (imresize3 cubic) of a column-major device volume."""
    a = (ctypes.c_uint64 * 3)(*(list(int(x) for x in in_dims) + [1] * (3 - len(in_dims))))
    b = (ctypes.c_uint64 * 3)(*(list(int(x) for x in out_dims) + [1] * (3 - len(out_dims))))
    check(lib().vr_resize_device(ctypes.c_void_p(int(d_in)), a, b, ctypes.c_void_p(int(d_out)),
                                 ctypes.c_void_p(int(stream)) if stream else None))


def resize_contributions(in_len: int, out_len: int):
    """(weights [out_len, P] float64, 0-based indices [out_len, P] int32) of one resize axis."""
    P = ctypes.c_int32(0)
    check(lib().vr_resize_contributions(int(in_len), int(out_len), ctypes.byref(P), None, None))
    w = np.zeros((int(out_len), P.value), np.float64)
    i = np.zeros((int(out_len), P.value), np.int32)
    check(lib().vr_resize_contributions(int(in_len), int(out_len), ctypes.byref(P), w.ctypes.data_as(ctypes.c_void_p),
                                        i.ctypes.data_as(ctypes.c_void_p)))
    return w, i


def channel(handle, t_sync, volumes, render_argv):
    """One vr_channel: handle, the 'sync_volumes' arguments after the handle (t_sync, Emission,
    Reflection, Absorption[, dx, dy, dz]) and the positional 'render' arguments after the handle.
    Returns (VrChannel, keep-alive list)."""
    c = _lib.VrChannel()
    c.handle = _handle(handle)
    c.time_last_mem_sync = int(np.asarray(t_sync).reshape(-1)[0])
    vols = [_vr_volume(v) for v in volumes]
    if len(vols) not in (3, 6):
        raise _lib.VrError(5, "channel: expected 3 or 6 volumes")
    c.emission, c.reflection, c.absorption = (ctypes.pointer(v) for v in vols[:3])
    if len(vols) == 6:
        c.dx, c.dy, c.dz = (ctypes.pointer(v) for v in vols[3:])
    ra, keep = render_args(*render_argv)
    c.args = ctypes.pointer(ra)
    return c, [vols, ra, keep, [getattr(v, "Data", None) for v in volumes]]


def render_channels(channels, stereo: bool = False, base: float = 0.0):
    """Multi-channel frame (vr_render_channels): `channels` = [(handle, t_sync, volumes,
    render_argv), ...]; returns one image (H, W, 3) per channel, or per channel a (left, right)
    pair when stereo."""
    built = [channel(*c) for c in channels]
    arr = (_lib.VrChannel * len(built))(*[b[0] for b in built])
    res = np.asarray(channels[0][3][4]).reshape(-1)
    H, W = int(res[0]), int(res[1])
    nv = 2 if stereo else 1
    out = np.zeros((len(built) * nv, H * W * 3), dtype=np.float32)
    check(lib().vr_render_channels(arr, len(built), 1 if stereo else 0, float(base),
                                   out.ctypes.data_as(ctypes.c_void_p) if out.size else None))
    del built
    imgs = [out[k].reshape((H, W, 3), order="F") for k in range(out.shape[0])]
    return [(imgs[2 * i], imgs[2 * i + 1]) for i in range(len(channels))] if stereo else imgs


def render_channels_device(channels, d_out: int, stereo: bool = False, base: float = 0.0, stream: int = 0) -> None:
    """vr_render_channels_device: channel i's view e into d_out + (i * eyes + e) * H*W*3 floats."""
    built = [channel(*c) for c in channels]
    arr = (_lib.VrChannel * len(built))(*[b[0] for b in built])
    check(lib().vr_render_channels_device(arr, len(built), 1 if stereo else 0, float(base),
                                          ctypes.c_void_p(int(d_out)), ctypes.c_void_p(int(stream)) if stream else None))
    del built


def sum_channels_device(d_in: int, n: int, views: int, image_floats: int, d_out: int, stream: int = 0) -> None:
    """vr_sum_channels_device: d_out[e] = d_in[0][e] + d_in[1][e] + ... (fp32, channel order)."""
    check(lib().vr_sum_channels_device(ctypes.c_void_p(int(d_in)), int(n), int(views), int(image_floats),
                                       ctypes.c_void_p(int(d_out)), ctypes.c_void_p(int(stream)) if stream else None))


def _group_devices():
    """VR_DEVICES (comma-separated device indices, primary first) selects multi-device handles."""
    import os
    ev = os.environ.get("VR_DEVICES", "").strip()
    return [int(x) for x in ev.split(",") if x.strip()] if ev else []


def volumeRender(cmd, *args):
    """The `volumeRender` mex: commands 'new', 'delete', 'mem_info', 'sync_volumes', 'render'."""
    nrhs = 1 + len(args)
    if not isinstance(cmd, str) or len(cmd) >= 64:
        raise _lib.VrError(1, "First input should be a command string less than 64 characters long.")
    L = lib()
    if cmd == "new":
        p = ctypes.c_void_p()
        devs = _group_devices()
        if devs:  # VR_DEVICES="0,1,...": a multi-device group (vr_new_multi), as the MEX adaptor does
            arr = (ctypes.c_int32 * len(devs))(*devs)
            check(L.vr_new_multi(arr, len(devs), ctypes.byref(p)))
        else:
            check(L.vr_new(ctypes.byref(p)))
        return np.uint64(p.value)
    if cmd == "render_channels":  # vr_render_channels: ('render_channels', channels[, stereo, base])
        return render_channels(*args)
    if nrhs < 2:
        raise _lib.VrError(1, "Second input should be a class instance handle.")
    h = _handle(args[0])
    if cmd == "delete":
        check(L.vr_delete(h))
        if nrhs != 2:
            warnings.warn("Delete: Unexpected arguments ignored.")
        return None
    if cmd == "mem_info":
        buf = ctypes.create_string_buffer(1 << 14)
        check(L.vr_mem_info(h, buf, len(buf)))
        print(buf.value.decode(), end="")
        return None
    if cmd == "sync_volumes":
        if nrhs < 6:
            raise _lib.VrError(1, "insufficient parameter!")
        t_sync = int(np.asarray(args[1]).reshape(-1)[0])
        em, re, ab = (_vr_volume(v) for v in args[2:5])  # order: Emission, Reflection, Absorption
        if nrhs == 9:
            gx, gy, gz = (_vr_volume(v) for v in args[5:8])
            check(L.vr_sync_volumes(h, t_sync, ctypes.byref(em), ctypes.byref(re), ctypes.byref(ab),
                                    ctypes.byref(gx), ctypes.byref(gy), ctypes.byref(gz)))
        elif nrhs == 6:
            check(L.vr_sync_volumes(h, t_sync, ctypes.byref(em), ctypes.byref(re), ctypes.byref(ab),
                                    None, None, None))
        else:  # 7, 8 or > 9 arguments: the previous gradient volumes are kept (render.cpp:105-113)
            flag = VrVolume()  # not read: only its presence selects the form
            check(L.vr_sync_volumes(h, t_sync, ctypes.byref(em), ctypes.byref(re), ctypes.byref(ab),
                                    ctypes.byref(flag), ctypes.byref(flag) if nrhs != 7 else None, None))
        if nrhs > 9:
            warnings.warn("SyncVolumes: Unexpected arguments ignored.")
        return None
    if cmd == "render_stereo":  # fused stereo pair (vr_render_stereo): args as 'render' + base
        ra, keep = render_args(*args[1:10])
        res = np.asarray(args[5]).reshape(-1)
        H, W = int(res[0]), int(res[1])
        left = np.zeros((H, W, 3), dtype=np.float32, order="F")
        right = np.zeros((H, W, 3), dtype=np.float32, order="F")
        check(L.vr_render_stereo(h, ctypes.byref(ra), float(args[10]),
                                 left.ctypes.data_as(ctypes.c_void_p) if left.size else None,
                                 right.ctypes.data_as(ctypes.c_void_p) if right.size else None))
        del keep
        return left, right
    if cmd == "render":
        if nrhs < 11:
            raise _lib.VrError(1, "insufficient parameter!")
        ra, keep = render_args(*args[1:10])
        res = np.asarray(args[5]).reshape(-1)
        H, W = int(res[0]), int(res[1])
        out = np.zeros((H, W, 3), dtype=np.float32, order="F")
        check(L.vr_render(h, ctypes.byref(ra), out.ctypes.data_as(ctypes.c_void_p) if out.size else None))
        del keep
        return out
    return None
