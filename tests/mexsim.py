"""TEST-ONLY: call a MEX adaptor of mex/ (built against tests/mexstub/ into libmex_<name>.so) the way
MATLAB does: Python values become mxArrays of the stand-in model, mexFunction(nlhs, plhs, nrhs,
prhs) runs, mexErrMsgTxt comes back as MexError, plhs come back as numpy arrays.

Value mapping (what VolumeRender.m hands the mex): str -> char row; bool -> logical scalar;
numpy arrays / scalars keep their dtype (float32 -> single, uint64 -> uint64, float64 -> double),
column-major; a Volume -> a 'Volume' object with properties Data and TimeLastUpdate; a LightSource
or a list of them -> a 1 x N 'LightSource' object array with Position and Color; a list / tuple
-> a cell row."""
from __future__ import annotations

import ctypes
import os
from ctypes import c_char_p, c_int, c_size_t, c_void_p, POINTER

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
STUB_DIR = os.path.join(HERE, "mexstub")

CLS = {np.dtype(np.float64): 6, np.dtype(np.float32): 7, np.dtype(np.int8): 8, np.dtype(np.uint8): 9,
       np.dtype(np.int16): 10, np.dtype(np.uint16): 11, np.dtype(np.int32): 12, np.dtype(np.uint32): 13,
       np.dtype(np.int64): 14, np.dtype(np.uint64): 15}
DTYPE = {v: k for k, v in CLS.items()}
LOGICAL, CHAR = 3, 4


class MexError(RuntimeError):
    pass


_libs = {}


def lib(name: str):
    if name not in _libs:
        path = os.path.join(STUB_DIR, f"libmex_{name}.so")
        if not os.path.exists(path):
            raise ImportError(f"{path} not built: make -C {STUB_DIR}")
        L = ctypes.CDLL(path)
        L.stub_numeric.restype = c_void_p
        L.stub_numeric.argtypes = [c_int, c_int, POINTER(c_size_t), c_void_p]
        L.stub_string.restype = c_void_p
        L.stub_string.argtypes = [c_char_p]
        L.stub_object.restype = c_void_p
        L.stub_object.argtypes = [c_char_p, c_size_t]
        L.stub_set_prop.restype = None
        L.stub_set_prop.argtypes = [c_void_p, c_size_t, c_char_p, c_void_p]
        L.stub_cell.restype = c_void_p
        L.stub_cell.argtypes = [c_size_t]
        L.stub_set_cell.restype = None
        L.stub_set_cell.argtypes = [c_void_p, c_size_t, c_void_p]
        L.stub_class.restype = c_int
        L.stub_class.argtypes = [c_void_p]
        L.stub_ndim.restype = c_size_t
        L.stub_ndim.argtypes = [c_void_p]
        L.stub_dims.restype = POINTER(c_size_t)
        L.stub_dims.argtypes = [c_void_p]
        L.stub_data.restype = c_void_p
        L.stub_data.argtypes = [c_void_p]
        L.stub_bytes.restype = c_size_t
        L.stub_bytes.argtypes = [c_void_p]
        L.stub_free.restype = None
        L.stub_free.argtypes = [c_void_p]
        for f in ("stub_last_error", "stub_warnings", "stub_printed"):
            getattr(L, f).restype = c_char_p
            getattr(L, f).argtypes = []
        L.stub_lock_count.restype = c_int
        L.stub_clear_log.restype = None
        L.stub_call.restype = c_int
        L.stub_call.argtypes = [c_int, POINTER(c_void_p), c_int, POINTER(c_void_p)]
        _libs[name] = L
    return _libs[name]


def _numeric(L, a: np.ndarray):
    a = np.asarray(a)
    if a.dtype == np.bool_:
        a = a.astype(np.uint8)
        cls = LOGICAL
    else:
        cls = CLS[a.dtype]
    shape = a.shape if a.ndim >= 2 else ((1, a.size) if a.ndim == 1 else (1, 1))
    buf = np.asfortranarray(a.reshape(shape, order="F"))
    dims = (c_size_t * len(shape))(*shape)
    return L.stub_numeric(cls, len(shape), dims, buf.ctypes.data if buf.size else None)


def to_mx(L, x):
    """A Python value as a new mxArray of the stand-in model (see the module docstring)."""
    from volume_renderer_amd.volume import LightSource, Volume
    if isinstance(x, str):
        return L.stub_string(x.encode())
    if isinstance(x, (bool, np.bool_)):
        return _numeric(L, np.array(bool(x)))
    if isinstance(x, Volume):
        o = L.stub_object(b"Volume", 1)
        L.stub_set_prop(o, 0, b"Data", _numeric(L, x.Data))
        L.stub_set_prop(o, 0, b"TimeLastUpdate", _numeric(L, np.uint64(x.TimeLastUpdate)))
        return o
    if isinstance(x, LightSource) or (isinstance(x, list) and x and all(isinstance(l, LightSource) for l in x)):
        ls = x if isinstance(x, list) else [x]
        o = L.stub_object(b"LightSource", len(ls))
        for i, l in enumerate(ls):
            L.stub_set_prop(o, i, b"Position", _numeric(L, np.float32(l.Position)))
            L.stub_set_prop(o, i, b"Color", _numeric(L, np.float32(l.Color)))
        return o
    if isinstance(x, (list, tuple)):
        c = L.stub_cell(len(x))
        for i, e in enumerate(x):
            L.stub_set_cell(c, i, to_mx(L, e))
        return c
    return _numeric(L, np.asarray(x))


def from_mx(L, p):
    """plhs entry -> numpy array (MATLAB dims, column-major); None if unset."""
    if not p:
        return None
    cls = L.stub_class(p)
    nd = L.stub_ndim(p)
    dims = tuple(L.stub_dims(p)[i] for i in range(nd))
    dt = np.dtype(np.uint8) if cls == LOGICAL else DTYPE[cls]
    n = L.stub_bytes(p)
    raw = np.ctypeslib.as_array(ctypes.cast(L.stub_data(p), POINTER(ctypes.c_ubyte)), shape=(n,)).copy() if n \
        else np.zeros(0, np.uint8)
    a = raw.view(dt).reshape(dims, order="F")
    return a.astype(bool) if cls == LOGICAL else a


def call(name: str, nlhs: int, *args):
    """[plhs...] = name(args...): returns a list of nlhs outputs; raises MexError on mexErrMsgTxt."""
    L = lib(name)
    L.stub_clear_log()
    prhs = (c_void_p * max(len(args), 1))(*[to_mx(L, a) for a in args])
    plhs = (c_void_p * max(nlhs, 1))()
    try:
        rc = L.stub_call(nlhs, plhs, len(args), prhs)
        if rc:
            raise MexError(L.stub_last_error().decode())
        return [from_mx(L, plhs[i]) for i in range(nlhs)]
    finally:
        for i in range(len(args)):
            L.stub_free(prhs[i])
        for i in range(max(nlhs, 1)):
            if plhs[i]:
                L.stub_free(plhs[i])


def warnings(name: str) -> str:
    return lib(name).stub_warnings().decode()


def printed(name: str) -> str:
    return lib(name).stub_printed().decode()


def lock_count(name: str) -> int:
    return lib(name).stub_lock_count()
