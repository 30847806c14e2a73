"""ctypes mirrors of the plain-C types in include/orbfe.h (shared by the product binding and the
test-only oracle binding).  No torch, no device code here."""
from __future__ import annotations

import ctypes as C

import numpy as np

ORBFE_OK = 0
ORBFE_ERR_ARG = -1
ORBFE_ERR_CAPACITY = -2
ORBFE_ERR_HIP = -3
ORBFE_ERR_UNSUPPORTED = -4
ORBFE_ERR_NOMEM = -5

STATUS_NAMES = {
    ORBFE_OK: "ok", ORBFE_ERR_ARG: "bad argument", ORBFE_ERR_CAPACITY: "capacity",
    ORBFE_ERR_HIP: "HIP error", ORBFE_ERR_UNSUPPORTED: "unsupported input",
    ORBFE_ERR_NOMEM: "device out of memory",
}


class OrbfeError(RuntimeError):
    def __init__(self, fn: str, status: int):
        super().__init__(f"{fn} failed: {status} ({STATUS_NAMES.get(status, 'unknown')})")
        self.status = status


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class Keypoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


# numpy view of orbfe_keypoint / cv::KeyPoint (28 bytes)
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == C.sizeof(Keypoint) == 28


class FrameView(C.Structure):
    _fields_ = [("n", C.c_int32), ("keys_un", C.c_void_p), ("desc", C.c_void_p),
                ("u_right", C.c_void_p), ("min_x", C.c_float), ("max_x", C.c_float),
                ("min_y", C.c_float), ("max_y", C.c_float), ("grid_w_inv", C.c_float),
                ("grid_h_inv", C.c_float), ("scale_factors", C.c_void_p),
                ("nlevels", C.c_int32)]


class MapPointView(C.Structure):
    _fields_ = [("m", C.c_int32), ("track_in_view", C.c_void_p), ("is_bad", C.c_void_p),
                ("proj_x", C.c_void_p), ("proj_y", C.c_void_p), ("proj_xr", C.c_void_p),
                ("pred_level", C.c_void_p), ("view_cos", C.c_void_p), ("desc", C.c_void_p),
                ("n_obs", C.c_void_p)]


class Camera(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("bf", C.c_float), ("b", C.c_float)]


def ptr(a: np.ndarray | None) -> C.c_void_p | None:
    """Raw pointer of a C-contiguous numpy array (None passes NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays handed to the C ABI must be C-contiguous"
    return C.c_void_p(a.ctypes.data)


class Frame:
    """Host-side stand-in for the Frame members the matchers read (Frame.h): undistorted
    keypoints, descriptors, mvuRight, image bounds and the 64x48 grid constants
    (Frame.cc:212-213, 554-582).  Keeps the numpy arrays alive for the FrameView."""

    GRID_COLS, GRID_ROWS = 64, 48  # Frame.h:37-38

    def __init__(self, keys: np.ndarray, desc: np.ndarray, width: int, height: int,
                 scale_factors: np.ndarray, u_right: np.ndarray | None = None):
        self.keys = np.ascontiguousarray(keys, dtype=KEYPOINT_DTYPE)
        self.desc = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
        assert len(self.desc) == len(self.keys)
        self.u_right = None if u_right is None else np.ascontiguousarray(u_right, np.float32)
        self.scale_factors = np.ascontiguousarray(scale_factors, np.float32)
        self.min_x, self.max_x, self.min_y, self.max_y = 0.0, float(width), 0.0, float(height)
        self.grid_w_inv = np.float32(self.GRID_COLS) / np.float32(self.max_x - self.min_x)
        self.grid_h_inv = np.float32(self.GRID_ROWS) / np.float32(self.max_y - self.min_y)

    @property
    def n(self) -> int:
        return len(self.keys)

    def view(self) -> FrameView:
        return FrameView(self.n, ptr(self.keys), ptr(self.desc), ptr(self.u_right),
                         self.min_x, self.max_x, self.min_y, self.max_y,
                         float(self.grid_w_inv), float(self.grid_h_inv),
                         ptr(self.scale_factors), len(self.scale_factors))


class MapPoints:
    """SoA of MapPoint tracking scratch (MapPoint.h:106-111) for SearchByProjection."""

    def __init__(self, proj_x, proj_y, pred_level, view_cos, desc, n_obs=None,
                 track_in_view=None, is_bad=None, proj_xr=None):
        m = len(proj_x)
        self.proj_x = np.ascontiguousarray(proj_x, np.float32)
        self.proj_y = np.ascontiguousarray(proj_y, np.float32)
        self.proj_xr = (np.full(m, -1, np.float32) if proj_xr is None
                        else np.ascontiguousarray(proj_xr, np.float32))
        self.pred_level = np.ascontiguousarray(pred_level, np.int32)
        self.view_cos = np.ascontiguousarray(view_cos, np.float32)
        self.desc = np.ascontiguousarray(desc, np.uint8).reshape(m, 32)
        self.n_obs = (np.ones(m, np.int32) if n_obs is None
                      else np.ascontiguousarray(n_obs, np.int32))
        self.track_in_view = (np.ones(m, np.uint8) if track_in_view is None
                              else np.ascontiguousarray(track_in_view, np.uint8))
        self.is_bad = (np.zeros(m, np.uint8) if is_bad is None
                       else np.ascontiguousarray(is_bad, np.uint8))

    @property
    def m(self) -> int:
        return len(self.proj_x)

    def view(self) -> MapPointView:
        return MapPointView(self.m, ptr(self.track_in_view), ptr(self.is_bad), ptr(self.proj_x),
                            ptr(self.proj_y), ptr(self.proj_xr), ptr(self.pred_level),
                            ptr(self.view_cos), ptr(self.desc), ptr(self.n_obs))
