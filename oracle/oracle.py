"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (the checker, never the product).

Python side of the CPU oracle: an independent restatement of the reference's mex-level state and
host arithmetic, driving the C restatement of the ray march in oracle/vr_oracle.c.

Restated here (cite: /root/reference/...):
  - mxMake_volume dims / memory_size       src/C/vr/volumeRender.cpp:64-74, 307-342
  - Volume operator==                       src/C/vr/volumeRender.cpp:24-26
  - MManager sync / resetGradients          src/C/vr/mm/mmanager.hxx:178-213
  - syncWithDevice / referenceTexture /     src/C/vr/volumeRender_kernel.cu:631-672, 703-722, 739-867
    syncVolume / setGradientTextures        (module-global slot indices + texture bindings)
  - render marshalling                      src/C/mex/render.cpp:134-259
  - initRender, gradient step               src/C/vr/volumeRender.cpp:112-156, 273-275 (in C: vr_oracle_host.c)
  - cudaDeviceReset on delete               src/C/vr/mm/mmanager.hxx:103-105

PARITY STATUS: parity unpinned for the ray march (no reference outputs exist -- SURVEY.md 8c);
the HG LUT is pinned by the reference generator's known answers (tests/test_oracle.py).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_int32, c_int64, c_uint, c_uint64, c_void_p, POINTER

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")


class OrTex(ctypes.Structure):
    _fields_ = [("data", c_void_p), ("nx", c_int64), ("ny", c_int64), ("nz", c_int64)]


class OrParams(ctypes.Structure):
    _fields_ = [("width", c_int64), ("height", c_int64),
                ("factor_emission", c_float), ("factor_absorption", c_float), ("factor_reflection", c_float),
                ("boxmin", c_float * 3), ("boxmax", c_float * 3), ("rot", (c_float * 3) * 4),
                ("opacity_threshold", c_float), ("tstep", c_float), ("color", c_float * 3),
                ("grad_step", c_float * 3), ("grad_method", c_int32), ("num_lights", c_int32),
                ("lights", c_void_p), ("max_steps", c_int64),
                ("em", OrTex), ("ab", OrTex), ("re", OrTex), ("grad_em", OrTex),
                ("gx", OrTex), ("gy", OrTex), ("gz", OrTex), ("lut", OrTex)]


_libs = {}


def lib(path: str = LIB_PATH):
    """The oracle's shared object (default liboracle.so).  bench.py's cpu_baseline leg passes the
    -O3 build of the same sources (libcpubase.so, or a -march=native build made on the box)."""
    if path not in _libs:
        if not os.path.exists(path):
            raise ImportError(f"oracle not built: make -C {_HERE}")
        L = ctypes.CDLL(path)
        for sfx in ("f32", "f64"):
            if not hasattr(L, f"or_render_{sfx}"):  # libcpubase.so: f32 only
                continue
            f = getattr(L, f"or_render_{sfx}")
            f.restype = c_uint64
            f.argtypes = [POINTER(OrParams), c_void_p, c_void_p, c_int64, c_int]
            f = getattr(L, f"or_render_pixels_{sfx}")
            f.restype = c_uint64
            f.argtypes = [POINTER(OrParams), c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int]
            f = getattr(L, f"or_tex3d_{sfx}")
            f.restype = c_float
            f.argtypes = [c_void_p, c_int64, c_int64, c_int64, c_float, c_float, c_float]
        L.or_init_render.restype = None
        L.or_init_render.argtypes = [c_uint64, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]
        L.or_grad_step.restype = None
        L.or_grad_step.argtypes = [c_uint64, c_uint64, c_uint64, c_void_p]
        L.or_hg_lut.restype = c_int
        L.or_hg_lut.argtypes = [c_uint, c_float, c_void_p]
        _libs[path] = L
    return _libs[path]


def hg_lut(n: int, g: float = 0.8) -> np.ndarray:
    """Restated HenyeyGreenstein(n, g) as a MATLAB-shaped (n,n,n) column-major array."""
    out = np.empty(n ** 3, dtype=np.float32)
    rc = lib().or_hg_lut(n, c_float(g), out.ctypes.data)
    if rc:
        raise ValueError("g must be in interval [-1,1]")
    return out.reshape((n, n, n), order="F")


def tex3d(vol: np.ndarray, x: float, y: float, z: float, double: bool = False) -> float:
    """One tex3D fetch (normalized coords, linear filter, clamp) on a MATLAB-shaped volume."""
    v = np.asfortranarray(vol, dtype=np.float32)
    d = v.shape + (1,) * (3 - v.ndim)
    f = lib().or_tex3d_f64 if double else lib().or_tex3d_f32
    return float(f(v.ctypes.data, d[0], d[1], d[2], c_float(x), c_float(y), c_float(z)))


# ---------------------------------------------------------------------------------------------
# host-side model of the mex / MManager / module globals

EM, AB, RE, DX, DY, DZ, LIGHT = range(7)


class OVolume:
    """mxMake_volume: identity (data pointer), dims, memory_size, last_update."""

    def __init__(self, data: np.ndarray, last_update: int):
        a = np.asarray(data)
        self.array = a
        self.ptr = a.ctypes.data if a.size else 0
        if a.ndim == 3:
            self.dims = tuple(int(s) for s in a.shape)
        elif a.ndim == 2:
            self.dims = (a.shape[0], a.shape[1], 1)
        elif a.ndim == 1:
            self.dims = (a.shape[0], 1, 1)
        else:
            self.dims = (1, 1, 1)
        self.memory_size = self.dims[0] * self.dims[1] * self.dims[2] * 4
        self.last_update = int(last_update)

    def __eq__(self, o):  # volumeRender.cpp:24-26
        return self.ptr == o.ptr and self.last_update == o.last_update and self.memory_size == o.memory_size


EMPTY = None


def _empty():
    v = OVolume.__new__(OVolume)
    v.array, v.ptr, v.dims, v.memory_size, v.last_update = None, 0, (0, 0, 0), 0, 0
    return v


class DevArray:
    """A device copy ('cudaArray'): snapshot of the data at upload time.  copy=False keeps a view
    (full-size tests whose volumes are never edited after the sync: no second 4-32 GiB copy)."""

    def __init__(self, vol: OVolume, copy: bool = True):
        self.data = np.array(np.asarray(vol.array, dtype=np.float32).reshape(-1, order="F"), copy=True if copy else None)
        self.dims = vol.dims


class Handle:
    def __init__(self):
        self.time_last_mem_sync = 0
        self.vol = [_empty() for _ in range(7)]
        self.arr = [None] * 7


class OracleSession:
    """The state the reference keeps across mex calls, and `render` on top of the C oracle."""

    def __init__(self, copy: bool = True):
        self.handles = {}
        self._next = 1
        self.copy = copy  # snapshot volumes at sync (False: views of the caller's arrays)
        self._reset_globals()

    def _reset_globals(self):
        self.bind = [None] * 7                     # texture -> DevArray
        self.idx = {EM: EM, AB: EM, RE: RE}        # d_idxEmmission, d_idxAbsorption, d_idxReflection
        self.grad_method = 0                       # dc_activeGradientMethod
        self.lights = np.zeros((0, 6), np.float32) # d_lightSources / c_numLightSources

    # 'new' / 'delete'
    def new(self) -> int:
        h = self._next
        self._next += 1
        self.handles[h] = Handle()
        return h

    def delete(self, h: int) -> None:
        del self.handles[h]
        self._reset_globals()             # cudaDeviceReset
        for o in self.handles.values():
            o.arr = [None] * 7

    # 'sync_volumes'
    def sync_volumes(self, h: int, t_sync: int, em, re, ab, gx=None, gy=None, gz=None, nrhs=None) -> None:
        """render.cpp:93-129.  nrhs (the mex argument count, default 9 with gradients, else 6):
        9 takes the gradient volumes, 6 resets them, any other count keeps the previous ones
        (render.cpp:105-113); setGradientMethod(lookup if 9 else compute) precedes the sync."""
        m = self.handles[h]
        m.time_last_mem_sync = int(t_sync)
        m.vol[EM], m.vol[RE], m.vol[AB] = em, re, ab
        if nrhs is None:
            nrhs = 9 if gx is not None else 6
        if nrhs == 9:
            m.vol[DX], m.vol[DY], m.vol[DZ] = gx, gy, gz
        elif nrhs == 6:
            self._reset_gradients(m)
        self.grad_method = 1 if nrhs == 9 else 0
        self._mm_sync(m)

    def _reset_gradients(self, m):
        for s in (DX, DY, DZ):
            m.vol[s] = _empty()

    def _sync_volume(self, m, tex, slot):
        self.bind[tex] = None
        m.arr[slot] = DevArray(m.vol[slot], copy=self.copy)
        self.bind[tex] = m.arr[slot]

    def _reference(self, m, tex, bufslot, idxslot, target):
        if m.arr[bufslot] is not None:
            self.bind[tex] = None
            m.arr[bufslot] = None
        self.idx[idxslot] = target

    def _mm_sync(self, m):
        if any(m.vol[s].last_update == 0 and m.arr[s] is not None for s in (DX, DY, DZ)):
            self._reset_gradients(m)
        em, ab, re, T = m.vol[EM], m.vol[AB], m.vol[RE], m.time_last_mem_sync
        simEmAb, simEmRe, simAbRe = em == ab, em == re, ab == re
        reqEm = em.last_update > T or T == 0
        reqAb = ab.last_update > T or T == 0
        reqRe = re.last_update > T or T == 0
        updEm = updAb = updRe = False
        if reqEm:
            self._sync_volume(m, EM, EM)
            updEm = True
            if simEmRe and not updRe:
                self._reference(m, RE, RE, RE, EM)
                updRe = True
            if simEmAb and not updAb:
                self._reference(m, AB, AB, AB, EM)
                updAb = True
        if reqAb:
            if not updAb:
                self._sync_volume(m, AB, AB)
                updAb = True
            if simAbRe and not updRe:
                self._reference(m, RE, RE, RE, AB)
                updRe = True
            if simEmAb and not updEm:
                self._reference(m, EM, AB, EM, AB)
                updEm = True
        if reqRe:
            if not updRe:
                self._sync_volume(m, RE, RE)
                updRe = True
            if simAbRe and not updAb:
                self._reference(m, AB, AB, AB, RE)
                updAb = True
            if simEmAb and not updEm:
                self._reference(m, EM, EM, EM, RE)
                updEm = True
        if m.vol[DX].last_update and m.vol[DY].last_update and m.vol[DZ].last_update:
            for s in (DX, DY, DZ):
                self._sync_volume(m, s, s)
            self.grad_method = 1

    # 'render'
    def params(self, h: int, lights, illum, factors, element_size_um, resolution, rot_flipped, props, thr,
               color):
        """Marshal one 'render' call into OrParams (+ keep-alive list).  lights: None (logical
        false) or an (n, 6) array [Position(MATLAB order), Color]; illum: None or OVolume."""
        m = self.handles[h]
        if lights is not None and illum is not None:
            L = np.asarray(lights, dtype=np.float32).reshape(-1, 6)
            kernel_lights = np.concatenate([L[:, 2::-1], L[:, 3:6]], axis=1)  # position reversed
            self.lights = np.ascontiguousarray(kernel_lights, dtype=np.float32)
            m.vol[LIGHT] = illum
            self._sync_volume(m, LIGHT, LIGHT)
        fac = np.asarray(factors, np.float32).reshape(-1)
        es = np.asarray(element_size_um, np.float32).reshape(-1)[::-1].copy()  # make_float3Inv
        H, W = (int(v) for v in np.asarray(resolution).reshape(-1)[:2])
        r = np.asarray(rot_flipped, np.float32).reshape(-1, order="F")
        pr = np.asarray(props, np.float32).reshape(-1)
        P = OrParams()
        P.width, P.height = W, H
        P.factor_emission, P.factor_reflection, P.factor_absorption = fac[0], fac[1], fac[2]
        bmin, bmax, tstep, gstep = (c_float * 3)(), (c_float * 3)(), c_float(), (c_float * 3)()
        esa = (c_float * 3)(*es)
        w, hh, d = m.vol[EM].dims
        lib().or_init_render(w, hh, d, esa, bmin, bmax, ctypes.byref(tstep))
        lib().or_grad_step(w, hh, d, gstep)
        for i in range(3):
            P.boxmin[i], P.boxmax[i], P.grad_step[i], P.color[i] = bmin[i], bmax[i], gstep[i], float(
                np.float32(np.asarray(color, np.float32).reshape(-1)[i]))
        cols = [(r[2], r[1], r[0]), (r[5], r[4], r[3]), (r[8], r[7], r[6]), (pr[0], pr[1], pr[2])]
        for j in range(4):
            for i in range(3):
                P.rot[j][i] = cols[j][i]
        P.opacity_threshold = np.float32(thr)
        P.tstep = tstep.value
        P.grad_method = self.grad_method
        P.num_lights = len(self.lights)
        P.lights = self.lights.ctypes.data if len(self.lights) else None
        # safety cap on samples per ray (same rule as the product; never reached by a terminating ray)
        b = np.array([bmax[0], bmax[1], bmax[2]], dtype=np.float64)
        diag = float(np.sqrt(4.0 * (b * b).sum()))
        finite = np.isfinite(tstep.value) and tstep.value > 0 and np.all(np.isfinite(b))
        cap = 2.0 * diag / float(tstep.value) + 64.0 if finite else np.inf
        P.max_steps = int(cap) if cap < 2.0e9 else 2000000000
        keep = [self.lights]

        def tex(arr):
            t = OrTex()
            if arr is not None and arr.data.size:
                t.data = arr.data.ctypes.data
                t.nx, t.ny, t.nz = arr.dims
                keep.append(arr)
            return t

        P.em = tex(self.bind[self.idx[EM]])
        P.ab = tex(self.bind[self.idx[AB]])
        P.re = tex(self.bind[self.idx[RE]])
        P.grad_em = tex(self.bind[EM])
        P.gx, P.gy, P.gz = tex(self.bind[DX]), tex(self.bind[DY]), tex(self.bind[DZ])
        P.lut = tex(self.bind[LIGHT])
        degenerate = not finite
        return P, keep, degenerate

    def render(self, h: int, *args, double: bool = False, threads: int = 0, cols=None, pixels=None,
               lib_path: str = LIB_PATH, **kw):
        """Returns (image [H,W,3] float32 column-major, total samples).  With `pixels=(xs, ys)`
        returns (values [n,3], per-pixel samples) instead."""
        P, keep, degenerate = self.params(h, *args, **kw)
        threads = threads or os.cpu_count() or 1
        L = lib(lib_path)
        f = L.or_render_f64 if double else L.or_render_f32
        fp = L.or_render_pixels_f64 if double else L.or_render_pixels_f32
        if pixels is not None:
            xs = np.ascontiguousarray(pixels[0], dtype=np.int64)
            ys = np.ascontiguousarray(pixels[1], dtype=np.int64)
            out = np.zeros((len(xs), 3), np.float32)
            steps = np.zeros(len(xs), np.uint64)
            if not degenerate:
                fp(ctypes.byref(P), xs.ctypes.data, ys.ctypes.data, len(xs), out.ctypes.data, steps.ctypes.data,
                   threads)
            return out, steps
        W, H = P.width, P.height
        img = np.zeros((H, W, 3), dtype=np.float32, order="F")
        if degenerate or W * H == 0:
            return img, 0
        if cols is not None:
            c = np.ascontiguousarray(cols, dtype=np.int64)
            total = f(ctypes.byref(P), img.ctypes.data, c.ctypes.data, len(c), threads)
        else:
            total = f(ctypes.byref(P), img.ctypes.data, None, 0, threads)
        del keep
        return img, int(total)


# ---------------------------------------------------------------------------------------------
# synthetic inputs of SURVEY.md 8d

def shell_volume(n: int) -> np.ndarray:
    """V_shell(n) (closed form, float64 arithmetic rounded to float32), MATLAB-shaped (n,n,n)."""
    c = (np.arange(n, dtype=np.float64) + 0.5) / n
    x = c[:, None, None]
    y = c[None, :, None]
    z = c[None, None, :]
    r = np.sqrt((x - 0.5) ** 2 + (y - 0.5) ** 2 + (z - 0.5) ** 2)
    v = np.clip(1.0 - np.abs(r - 0.32) / 0.14, 0.0, 1.0)
    tp = 6.0 * np.pi
    shaded = v * (0.6 + 0.4 * np.sin(tp * x) * np.sin(tp * y) * np.sin(tp * z)) + 0.05 * (x + 2 * y + 3 * z) / 6.0
    v = np.where(v > 0, shaded, 0.0)
    return np.asfortranarray(v.astype(np.float32))


def rand_volume(n: int = 32, seed: int = 20241218) -> np.ndarray:
    """V_rand(n) of SURVEY.md 8d (sampler known-answer inputs)."""
    return np.asfortranarray(np.random.default_rng(seed).random((n, n, n), dtype=np.float32))


def matlab_gradient(data: np.ndarray):
    """MATLAB [gx, gy, gz] = gradient(Data) in single: gx along dim 2, gy along dim 1, gz dim 3."""
    d = np.asarray(data, dtype=np.float32)
    out = []
    for axis in (1, 0, 2):
        g = np.empty_like(d)
        sl = [slice(None)] * 3

        def s(a, b):
            q = list(sl)
            q[axis] = slice(a, b)
            return tuple(q)

        n = d.shape[axis]
        if n > 1:
            g[s(1, n - 1)] = (d[s(2, n)] - d[s(0, n - 2)]) / np.float32(2)
            g[s(0, 1)] = d[s(1, 2)] - d[s(0, 1)]
            g[s(n - 1, n)] = d[s(n - 1, n)] - d[s(n - 2, n - 1)]
        else:
            g[...] = 0
        out.append(np.asfortranarray(g))
    return tuple(out)


def rotation(alpha=0.0, beta=0.0, gamma=0.0, R=None) -> np.ndarray:
    """VolumeRender.rotate (VolumeRender.m:239-262) in float64 with MATLAB's exact cosd/sind."""
    def sd(a):
        r = np.fmod(a, 360.0)
        if r == int(r) and int(r) % 90 == 0:
            return [0.0, 1.0, 0.0, -1.0][(int(r) // 90) % 4]
        return float(np.sin(np.deg2rad(a)))

    def cd(a):
        r = np.fmod(a, 360.0)
        if r == int(r) and int(r) % 90 == 0:
            return [1.0, 0.0, -1.0, 0.0][(int(r) // 90) % 4]
        return float(np.cos(np.deg2rad(a)))

    R = np.eye(3) if R is None else np.asarray(R, dtype=np.float64)
    Rx = np.array([[1, 0, 0], [0, cd(alpha), -sd(alpha)], [0, sd(alpha), cd(alpha)]])
    Ry = np.array([[cd(beta), 0, sd(beta)], [0, 1, 0], [-sd(beta), 0, cd(beta)]])
    Rz = np.array([[cd(gamma), -sd(gamma), 0], [sd(gamma), cd(gamma), 0], [0, 0, 1]])
    return R @ Rx @ Ry @ Rz


# ---------------------------------------------------------------------------------------------
# MATLAB-side volume preprocessing, restated for the device versions' tests.
# Parity unpinned: no MATLAB here; these follow the published imresize / imresize3 algorithm
# (contributions(): cubic kernel, antialiasing when shrinking, mirrored ends) and Volume.m.

def _cubic(x):
    """imresize's cubic kernel (a = -0.5), double."""
    ax = np.abs(x)
    ax2 = ax * ax
    ax3 = ax * ax * ax
    return ((1.5 * ax3 - 2.5 * ax2 + 1.0) * (ax <= 1.0) +
            (-0.5 * ax3 + 2.5 * ax2 - 4.0 * ax + 2.0) * ((1.0 < ax) & (ax <= 2.0)))


def resize_contributions(in_len: int, out_len: int):
    """imresize contributions() for one axis (Volume.m:93-106 -> imresize3): weights [out, P]
    (double, row-normalised) and 0-based source indices [out, P] (mirrored at the ends), columns
    zero for every output dropped."""
    scale = out_len / in_len
    aa = scale < 1.0
    width = 4.0 / scale if aa else 4.0
    x = np.arange(1, out_len + 1, dtype=np.float64)[:, None]
    u = x / scale + 0.5 * (1.0 - 1.0 / scale)
    left = np.floor(u - width / 2.0)
    P = int(np.ceil(width)) + 2
    ind = left + np.arange(P, dtype=np.float64)[None, :]
    d = u - ind
    w = scale * _cubic(scale * d) if aa else _cubic(d)
    s = np.zeros((out_len, 1))
    for p in range(P):  # row sums in tap order
        s[:, 0] = s[:, 0] + w[:, p]
    w = w / s
    n = in_len
    k = np.mod(ind.astype(np.int64) - 1, 2 * n)
    idx = np.where(k < n, k, 2 * n - 1 - k)
    keep = np.any(w != 0.0, axis=0)
    return w[:, keep], idx[:, keep].astype(np.int32)


def resize(data: np.ndarray, newsize) -> np.ndarray:
    """Volume.resize: separable passes along the axes in order of increasing scale (stable), each
    out = sum_p w * in[idx] accumulated in double in tap order and rounded to single; axes whose
    length does not change are skipped."""
    a = np.asarray(data, np.float32)
    new = tuple(int(v) for v in np.asarray(newsize).reshape(-1))
    shp = a.shape + (1,) * (3 - a.ndim)
    out_shape = new + (1,) * (3 - len(new))
    a = a.reshape(shp, order="F")
    scales = [out_shape[i] / shp[i] for i in range(3)]
    order = sorted(range(3), key=lambda i: scales[i])
    for dim in order:
        if out_shape[dim] == a.shape[dim]:
            continue
        w, idx = resize_contributions(a.shape[dim], out_shape[dim])
        src = np.moveaxis(a, dim, 0).astype(np.float64)
        acc = np.zeros((out_shape[dim],) + src.shape[1:], np.float64)
        for p in range(w.shape[1]):
            acc = acc + w[:, p].reshape((-1,) + (1,) * (src.ndim - 1)) * src[idx[:, p]]
        a = np.moveaxis(acc.astype(np.float32), 0, dim)
    return np.asfortranarray(a.reshape(new if len(new) == np.asarray(data).ndim else out_shape, order="F"))


def normalize(data: np.ndarray, new_min: float, new_max: float) -> np.ndarray:
    """Volume.normalize (Volume.m:208-220) in single: max / min omit NaN; each operation rounded."""
    d = np.asarray(data, np.float32)
    valid = d[d == d]
    mx = valid.max() if valid.size else np.float32(np.nan)
    mn = valid.min() if valid.size else np.float32(np.nan)
    with np.errstate(all="ignore"):
        t1 = d - mn
        t2 = t1 * np.float32(float(new_max) - float(new_min))
        t3 = t2 / np.float32(mx - mn)
        return t3 + np.float32(new_min)
