"""Python mirror of the reference's MATLAB classes ``Volume`` and ``LightSource``.

``Volume``      /root/reference/src/matlab/VolumeRender/Volume.m
``LightSource`` /root/reference/src/matlab/VolumeRender/LightSource.m

Data is kept exactly as MATLAB holds it: a single-precision, column-major (Fortran-order) array
``Data(d0, d1, d2)``.  Assigning ``Data`` stamps ``TimeLastUpdate`` (Volume.m:225-238), which is
what the renderer's upload deduplication keys on.  In-place edits of the numpy array bypass the
stamp (MATLAB cannot do that); call ``touch()`` after such an edit.
"""
from __future__ import annotations

import numpy as np

from .mex import timestamp


def _single(data) -> np.ndarray:
    a = np.asarray(data, dtype=np.float32)
    return np.asfortranarray(a)


class Volume:
    """Volume data container with change timestamp (Volume.m:1-222)."""

    def __init__(self, data):
        self.TimeLastUpdate = np.uint64(0)
        self.Data = data

    @property
    def Data(self) -> np.ndarray:
        return self._data

    @Data.setter
    def Data(self, data) -> None:  # set.Data + PostSet listener (Volume.m:82-90, 225-238)
        self._data = _single(data)
        self.TimeLastUpdate = timestamp()

    def touch(self) -> None:
        """Stamp TimeLastUpdate after an in-place edit of Data."""
        self.TimeLastUpdate = timestamp()

    def size(self):
        return self._data.shape

    def mean(self):
        return self._data.mean(dtype=np.float64)

    def max(self):
        return self._data.max()

    def min(self):
        return self._data.min()

    def mip(self) -> np.ndarray:
        """Maximum intensity projection: max(permute(Data,[2 1 3]), [], 3) (Volume.m:138-146)."""
        d = self._data if self._data.ndim == 3 else self._data.reshape(self._data.shape + (1,) * (3 - self._data.ndim))
        return np.max(np.transpose(d, (1, 0, 2)), axis=2)

    def grad(self):
        """[gx, gy, gz] = gradient(Data) with MATLAB's axis convention (Volume.m:181-205):
        gx = d/d(dim 2), gy = d/d(dim 1), gz = d/d(dim 3); central differences inside,
        one-sided at the edges, computed in single precision."""
        d = self._data
        if d.ndim != 3:
            raise ValueError("grad expects 3-D data")
        gy, gx, gz = (np.asfortranarray(g.astype(np.float32)) for g in np.gradient(d, axis=(0, 1, 2)))
        return Volume(gx), Volume(gy), Volume(gz)

    def normalize(self, new_min, new_max) -> None:
        """Linear normalisation to [new_min, new_max] (Volume.m:208-220) in MATLAB's single
        arithmetic: (Data - min) * single(newMax - newMin) / (max - min) + single(newMin), each step
        rounded to single (vr_normalize_device does the same on device data)."""
        d = self._data
        ok = d[~np.isnan(d)]
        mx = ok.max() if ok.size else np.float32(np.nan)
        mn = ok.min() if ok.size else np.float32(np.nan)
        with np.errstate(all="ignore"):
            t = (d - mn) * np.float32(float(new_max) - float(new_min))
            t = t / np.float32(mx - mn)
            self.Data = t + np.float32(new_min)

    def resize(self, newsize) -> None:
        """Volume.resize (Volume.m:93-106: imresize3 for 3-D data, imresize for 2-D) on the GPU
        (vr_resize_device: cubic, antialiasing when shrinking).  newsize: 3 (or, for 2-D data, 2)
        sizes."""
        import torch
        from .mex import resize_device
        d = self._data
        dims = tuple(d.shape) + (1,) * (3 - d.ndim)
        new = tuple(int(x) for x in np.asarray(newsize).reshape(-1))
        out_dims = new + (1,) * (3 - len(new))
        src = torch.from_numpy(np.ascontiguousarray(d.reshape(-1, order="F"))).cuda()
        dst = torch.empty(int(np.prod(out_dims)), dtype=torch.float32, device="cuda")
        resize_device(src.data_ptr(), dims, out_dims, dst.data_ptr(), torch.cuda.current_stream().cuda_stream)
        out = dst.cpu().numpy().reshape(out_dims, order="F")
        self.Data = out if d.ndim == 3 else out.reshape(new, order="F")

    def pad(self, padding: int, value=0) -> None:
        """Pad all three dimensions by `padding` on both sides with `value` (Volume.m:119-135)."""
        if self._data.ndim == 3:
            self.Data = np.pad(self._data, int(padding), mode="constant", constant_values=value)


class LightSource:
    """A light: Position and Color, both 1x3 single (LightSource.m:32-104)."""

    def __init__(self, pos, col):
        pos = np.asarray(pos)
        col = np.asarray(col)
        if pos.size != 3:
            raise ValueError("dimensions of position must be [1,3]")
        if col.size != 3:
            raise ValueError("dimensions of color must be [1,3]")
        self.Position = np.asarray(pos, dtype=np.float32).reshape(3)
        self.Color = np.asarray(col, dtype=np.float32).reshape(3)

    def __repr__(self) -> str:
        return f"LightSource(Position={self.Position.tolist()}, Color={self.Color.tolist()})"
