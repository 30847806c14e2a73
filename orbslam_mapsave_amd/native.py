"""ctypes binding of liborbfe.so (the HIP product library) and the host-side mirror of the
reference interface for the hot path:

* :class:`ORBextractor` mirrors ``ORB_SLAM2::ORBextractor`` (include/ORBextractor.h:50-119):
  same ctor arguments, ``__call__(image, mask)`` for ``operator()`` and the six getters;
* :class:`ORBmatcher` mirrors the hot subset of ``ORB_SLAM2::ORBmatcher``
  (include/ORBmatcher.h:38-110): ``DescriptorDistance``, ``SearchForInitialization`` and the two
  tracking ``SearchByProjection`` overloads, plus the brute-force match of config 3.

There is no CPU fallback: importing works anywhere, but constructing an extractor or matcher
needs the built library and a gfx950 device, and raises otherwise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .abi import (KEYPOINT_DTYPE, ORBFE_ERR_CAPACITY, ORBFE_OK, Camera, Frame, FrameView,
                  MapPoints, MapPointView, OrbfeError, Params, ptr)

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORBFE_LIB selects another build of the same library (A/B runs of build variants)
LIB_PATH = os.environ.get("ORBFE_LIB") or os.path.join(_HERE, "lib", "liborbfe.so")
_lib: C.CDLL | None = None

# every symbol include/orbfe.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "orbfe_create", "orbfe_destroy", "orbfe_get_levels", "orbfe_get_scale_factor",
    "orbfe_get_scale_tables", "orbfe_get_features_per_level", "orbfe_keypoint_capacity",
    "orbfe_keypoint_capacity_for", "orbfe_keypoint_capacity_params", "orbfe_set_arithmetic", "orbfe_get_arithmetic",
    "orbfe_get_reference_constants",
    "orbfe_extract", "orbfe_input_buffer", "orbfe_extract_staged", "orbfe_staged_outputs",
    "orbfe_extract_color", "orbfe_human_mask_rect", "orbfe_extract_batch",
    "orbfe_extract_batch_device", "orbfe_extract_color_batch_device", "orbfe_set_stream",
    "orbfe_synchronize", "orbfe_compute_stereo_matches", "orbfe_compute_stereo_matches_device",
    "orbfe_stereo_status", "orbfe_profile", "orbfe_profile_read", "orbfe_pyramid_path", "orbfe_debug_replay", "orbfe_set_stage_mask", "orbfe_get_level", "orbfe_get_blurred_level", "orbfe_get_fast_keys",
    "orbfe_matcher_create", "orbfe_matcher_destroy", "orbfe_matcher_set_stream",
    "orbfe_matcher_profile", "orbfe_matcher_profile_read", "orbfe_matcher_profile_read_stages", "orbfe_hamming",
    "orbfe_bf_match", "orbfe_bf_match_batch_device", "orbfe_search_for_initialization",
    "orbfe_search_by_projection_local", "orbfe_search_by_projection_last",
    "orbfe_search_by_projection_keyframe", "orbfe_distinctive_descriptors",
    "orbfe_distinctive_descriptors_device", "orbfe_search_local_points_device",
    "orbfe_search_by_projection_local_device",
    "orbfe_matcher_last_rounds", "orbfe_matcher_capacity_retries", "orbfe_features_in_area", "orbfe_is_in_frustum", "orbfe_vocabulary_load_text",
    "orbfe_vocabulary_create", "orbfe_vocabulary_destroy", "orbfe_vocabulary_info",
    "orbfe_vocabulary_set_stream", "orbfe_bow_transform", "orbfe_bow_transform_batch_device",
    "orbfe_search_by_bow", "orbfe_search_by_bow_batch_device", "orbfe_archive_mat_bytes",
    "orbfe_archive_write_keypoints_device", "orbfe_archive_read_keypoints_device",
    "orbfe_archive_write_descriptors_device", "orbfe_archive_read_descriptors_device",
]


def lib() -> C.CDLL:
    """Load liborbfe.so; raise loudly if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with "
                               "`python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        L.orbfe_create.restype = C.c_void_p
        L.orbfe_create.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.orbfe_destroy.argtypes = [C.c_void_p]
        L.orbfe_get_scale_factor.restype = C.c_float
        for fn in ("orbfe_get_levels", "orbfe_get_scale_factor", "orbfe_keypoint_capacity",
                   "orbfe_synchronize"):
            getattr(L, fn).argtypes = [C.c_void_p]
        L.orbfe_pyramid_path.argtypes = [C.c_void_p, C.c_int]
        if hasattr(L, "orbfe_matcher_create"):
            L.orbfe_matcher_create.restype = C.c_void_p
            L.orbfe_matcher_create.argtypes = [C.c_int, C.c_void_p]
            L.orbfe_matcher_destroy.argtypes = [C.c_void_p]
        if hasattr(L, "orbfe_vocabulary_load_text"):
            L.orbfe_vocabulary_load_text.restype = C.c_void_p
            L.orbfe_vocabulary_load_text.argtypes = [C.c_char_p, C.c_int, C.c_void_p]
            L.orbfe_vocabulary_create.restype = C.c_void_p
            L.orbfe_vocabulary_destroy.argtypes = [C.c_void_p]
        if hasattr(L, "orbfe_archive_mat_bytes"):
            L.orbfe_archive_mat_bytes.restype = C.c_int64
            sz, vp, i = C.c_size_t, C.c_void_p, C.c_int
            L.orbfe_archive_write_keypoints_device.argtypes = [i, vp, sz, vp, i, vp, sz, vp]
            L.orbfe_archive_read_keypoints_device.argtypes = [i, vp, sz, vp, i, vp, sz, vp]
            L.orbfe_archive_write_descriptors_device.argtypes = [i, vp, sz, vp, i, i, vp, sz, vp, vp]
            L.orbfe_archive_read_descriptors_device.argtypes = [i, vp, sz, i, vp, sz, vp, vp, vp]
        _lib = L
    return _lib


# hipStreamLegacy (hip_runtime_api.h): the device's legacy default stream as an explicit handle
HIP_STREAM_LEGACY = 1


def _stream_arg(stream_handle: int | None):
    """set_stream's argument: None = the handle's own stream; 0 (torch's default stream, the
    legacy null stream) = hipStreamLegacy, since a NULL hip_stream selects the handle's own
    stream in the C ABI; anything else is a hipStream_t as is."""
    if stream_handle is None:
        return None
    return C.c_void_p(HIP_STREAM_LEGACY if stream_handle == 0 else stream_handle)


def _check(fn: str, st: int) -> None:
    if st != ORBFE_OK:
        raise OrbfeError(fn, st)


def reference_constants() -> dict:
    """The reference's compile-time constants as the HIP library uses them
    (orbfe_get_reference_constants: ORBextractor.cc:71-73, ORBmatcher.cc:37-39); no device."""
    out = (C.c_int32 * 6)()
    _check("orbfe_get_reference_constants", lib().orbfe_get_reference_constants(out))
    return dict(zip(("PATCH_SIZE", "HALF_PATCH_SIZE", "EDGE_THRESHOLD", "TH_HIGH", "TH_LOW",
                     "HISTO_LENGTH"), list(out)))


def keypoint_capacity(nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int,
                      minThFAST: int, w: int, h: int) -> int:
    """Per-frame keypoint capacity at w x h for these extractor parameters, without a handle or
    a device (orbfe_keypoint_capacity_params): the slab rows an extraction can fill."""
    p = Params(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
    c = lib().orbfe_keypoint_capacity_params(C.byref(p), int(w), int(h))
    _check("orbfe_keypoint_capacity_params", min(c, 0))
    return c


# ORBFE_PIX_* (include/orbfe.h): the cvtColor codes of Tracking::GrabImage*
PIX_GRAY, PIX_RGB, PIX_BGR, PIX_RGBA, PIX_BGRA = range(5)
PIX_CHANNELS = {PIX_GRAY: 1, PIX_RGB: 3, PIX_BGR: 3, PIX_RGBA: 4, PIX_BGRA: 4}


def human_mask_rect(joints: np.ndarray, w: int, h: int) -> tuple[int, int, int, int]:
    """OpDetector::SkeletonSquareMask's zeroed rectangle from (n, 3) joints
    (DetectHumanPose.cpp:453-489), via orbfe_human_mask_rect."""
    j = np.ascontiguousarray(joints, np.float32).reshape(-1, 3)
    out = (C.c_int32 * 4)()
    _check("orbfe_human_mask_rect", lib().orbfe_human_mask_rect(ptr(j), len(j), w, h, out))
    return tuple(out)


class ORBextractor:
    """``ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)`` on a gfx950 GPU
    (ORBextractor.cc:409-469).  One instance is not reentrant; use one per thread."""

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int,
                 minThFAST: int, device: int = 0, max_width: int = 0, max_height: int = 0,
                 max_batch: int = 1):
        self._p = Params(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        st = C.c_int(0)
        h = lib().orbfe_create(C.byref(self._p), device, max_width, max_height, max_batch,
                               C.byref(st))
        if not h:
            raise OrbfeError("orbfe_create", st.value)
        self._h = C.c_void_p(h)
        self.nlevels = nlevels

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().orbfe_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- getters (ORBextractor.h:68-88)
    def GetLevels(self) -> int:
        return lib().orbfe_get_levels(self._h)

    def GetScaleFactor(self) -> float:
        return lib().orbfe_get_scale_factor(self._h)

    def _tables(self):
        t = [np.zeros(self.nlevels, np.float32) for _ in range(4)]
        _check("orbfe_get_scale_tables", lib().orbfe_get_scale_tables(self._h, *map(ptr, t)))
        return t

    def GetScaleFactors(self) -> np.ndarray:
        return self._tables()[0]

    def GetInverseScaleFactors(self) -> np.ndarray:
        return self._tables()[1]

    def GetScaleSigmaSquares(self) -> np.ndarray:
        return self._tables()[2]

    def GetInverseScaleSigmaSquares(self) -> np.ndarray:
        return self._tables()[3]

    def features_per_level(self) -> np.ndarray:
        out = np.zeros(self.nlevels, np.int32)
        _check("orbfe_get_features_per_level", lib().orbfe_get_features_per_level(self._h, ptr(out)))
        return out

    ARITH_SCALAR, ARITH_X86_SIMD = 0, 1

    def set_arithmetic(self, mode: int) -> None:
        """orbfe_set_arithmetic: ARITH_X86_SIMD (the default: the SSE2 resize / blur bodies and
        FMA-contracted rotation of the reference's x86-64 build) or ARITH_SCALAR (OpenCV's
        portable scalar paths)."""
        _check("orbfe_set_arithmetic", lib().orbfe_set_arithmetic(self._h, int(mode)))

    def capacity(self, w: int | None = None, h: int | None = None) -> int:
        """Keypoints per frame that can never overflow: for a w x h input when given
        (orbfe_keypoint_capacity_for), else for every supported size."""
        if w is None or h is None:
            return lib().orbfe_keypoint_capacity(self._h)
        c = lib().orbfe_keypoint_capacity_for(self._h, int(w), int(h))
        _check("orbfe_keypoint_capacity_for", min(c, 0))
        return c

    # ---- operator() (ORBextractor.cc:1042-1108)
    def __call__(self, image: np.ndarray, mask: np.ndarray | None = None):
        """Returns (keypoints[KEYPOINT_DTYPE], descriptors uint8 (n, 32)); an empty image
        returns (None, None) like the reference, which leaves its outputs untouched."""
        image = np.asarray(image)
        if image.size == 0:
            return None, None
        # a row-strided u8 view (a cv::Mat ROI: step > cols) is passed as is, with its stride
        if not (image.dtype == np.uint8 and image.ndim == 2 and image.strides[1] == 1 and
                image.strides[0] >= image.shape[1]):
            image = np.ascontiguousarray(image, np.uint8)
        h, w = image.shape
        stride = image.strides[0]
        m = None if mask is None or np.size(mask) == 0 else np.ascontiguousarray(mask, np.uint8)
        cap = self.capacity(w, h)
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        _check("orbfe_extract", lib().orbfe_extract(
            self._h, C.c_void_p(image.ctypes.data), w, h, C.c_size_t(stride), ptr(m),
            C.c_size_t(w), ptr(kps), cap, ptr(desc), C.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def input_buffer(self, w: int, h: int) -> np.ndarray:
        """The handle's pinned staging buffer as a writable (h, w) uint8 view
        (orbfe_input_buffer): write the gray frame into it (as GrabImageMonocular's cvtColor
        would), then call :meth:`extract_staged`."""
        buf = C.POINTER(C.c_uint8)()
        stride = C.c_size_t(0)
        _check("orbfe_input_buffer", lib().orbfe_input_buffer(self._h, w, h, C.byref(buf),
                                                              C.byref(stride)))
        flat = np.ctypeslib.as_array(buf, shape=(h * stride.value,))
        return np.lib.stride_tricks.as_strided(flat, (h, w), (stride.value, 1))

    def extract_staged(self, w: int, h: int, copy_out: bool = True):
        """operator() on the staged frame (orbfe_extract_staged).  copy_out=False leaves the
        outputs in the handle's pinned buffers (kps_cap 0) and returns views of them
        (orbfe_staged_outputs), valid until the next call."""
        n = C.c_int(0)
        if copy_out:
            cap = self.capacity(w, h)
            kps = np.zeros(cap, KEYPOINT_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            _check("orbfe_extract_staged", lib().orbfe_extract_staged(
                self._h, w, h, ptr(kps), cap, ptr(desc), C.byref(n)))
            return kps[:n.value].copy(), desc[:n.value].copy()
        _check("orbfe_extract_staged", lib().orbfe_extract_staged(self._h, w, h, None, 0, None,
                                                                  C.byref(n)))
        return self.staged_outputs()

    def staged_outputs(self):
        """Views of the last single-frame call's outputs in handle-owned memory."""
        k = C.c_void_p()
        d = C.c_void_p()
        n = C.c_int(0)
        _check("orbfe_staged_outputs", lib().orbfe_staged_outputs(self._h, C.byref(k), C.byref(d),
                                                                  C.byref(n)))
        if not k.value or n.value == 0:
            return np.zeros(0, KEYPOINT_DTYPE), np.zeros((0, 32), np.uint8)
        kb = (C.c_uint8 * (n.value * KEYPOINT_DTYPE.itemsize)).from_address(k.value)
        db = (C.c_uint8 * (n.value * 32)).from_address(d.value)
        return (np.frombuffer(kb, KEYPOINT_DTYPE, n.value),
                np.frombuffer(db, np.uint8).reshape(n.value, 32))

    def extract_color(self, image: np.ndarray, pix: int, mask: np.ndarray | None = None,
                      rect: tuple[int, int, int, int] | None = None):
        """``cvtColor(image, gray, CV_*2GRAY)`` (Tracking.cc:409-422) fused with
        ``operator()(gray, mask)``; `pix` is one of PIX_*; `rect` = (x0, y0, x1, y1) zeroed
        rectangle of the human mask (DetectHumanPose.cpp:484-489)."""
        image = np.ascontiguousarray(image, np.uint8)
        if image.size == 0:
            return None, None
        h, w = image.shape[:2]
        cn = 1 if image.ndim == 2 else image.shape[2]
        if cn != PIX_CHANNELS[pix]:
            raise ValueError(f"pix {pix} needs {PIX_CHANNELS[pix]} channels, image has {cn}")
        m = None if mask is None or np.size(mask) == 0 else np.ascontiguousarray(mask, np.uint8)
        r = None if rect is None else (C.c_int32 * 4)(*rect)
        cap = self.capacity(w, h)
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        _check("orbfe_extract_color", lib().orbfe_extract_color(
            self._h, ptr(image), pix, w, h, C.c_size_t(w * cn), ptr(m), C.c_size_t(w),
            r, ptr(kps), cap, ptr(desc), C.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def extract_color_batch_device(self, d_imgs: int, pix: int, n: int, w: int, h: int,
                                   stride: int, frame_pitch: int, d_kps: int, kps_cap: int,
                                   d_desc: int, d_n_out: int, d_masks: int | None = None,
                                   mask_stride: int = 0, mask_frame_pitch: int = 0,
                                   d_rects: int | None = None) -> None:
        """Device-resident colour batch (orbfe_extract_color_batch_device); async."""
        _check("orbfe_extract_color_batch_device", lib().orbfe_extract_color_batch_device(
            self._h, C.c_void_p(d_imgs), pix, n, w, h, C.c_size_t(stride),
            C.c_size_t(frame_pitch), C.c_void_p(d_masks) if d_masks else None,
            C.c_size_t(mask_stride), C.c_size_t(mask_frame_pitch),
            C.c_void_p(d_rects) if d_rects else None, C.c_void_p(d_kps), kps_cap,
            C.c_void_p(d_desc), C.c_void_p(d_n_out)))

    def ComputeStereoMatches(self, right: "ORBextractor", kl: np.ndarray, dl: np.ndarray,
                             kr: np.ndarray, dr: np.ndarray, bf: float, b: float,
                             frame: int = 0):
        """Frame::ComputeStereoMatches (Frame.cc:584-756) with this handle as
        mpORBextractorLeft and `right` as mpORBextractorRight (their last extractions' pyramids).
        Returns (mvuRight, mvDepth) float32 arrays of len(kl)."""
        kl = np.ascontiguousarray(kl, KEYPOINT_DTYPE)
        kr = np.ascontiguousarray(kr, KEYPOINT_DTYPE)
        dl = np.ascontiguousarray(dl, np.uint8)
        dr = np.ascontiguousarray(dr, np.uint8)
        ur = np.full(len(kl), -1, np.float32)
        dp = np.full(len(kl), -1, np.float32)
        _check("orbfe_compute_stereo_matches", lib().orbfe_compute_stereo_matches(
            self._h, right._h, frame, ptr(kl), ptr(dl), len(kl), ptr(kr), ptr(dr), len(kr),
            C.c_float(bf), C.c_float(b), ptr(ur), ptr(dp)))
        return ur, dp

    def compute_stereo_matches_device(self, right: "ORBextractor", n: int, d_kl: int, d_dl: int,
                                      d_nl: int, d_kr: int, d_dr: int, d_nr: int, kps_cap: int,
                                      bf: float, b: float, d_ur: int, d_dp: int) -> None:
        """Batched device form (orbfe_compute_stereo_matches_device); async."""
        _check("orbfe_compute_stereo_matches_device", lib().orbfe_compute_stereo_matches_device(
            self._h, right._h, n, C.c_void_p(d_kl), C.c_void_p(d_dl), C.c_void_p(d_nl),
            C.c_void_p(d_kr), C.c_void_p(d_dr), C.c_void_p(d_nr), kps_cap, C.c_float(bf),
            C.c_float(b), C.c_void_p(d_ur), C.c_void_p(d_dp)))

    def stereo_status(self) -> None:
        _check("orbfe_stereo_status", lib().orbfe_stereo_status(self._h))

    def extract_batch(self, images: np.ndarray, masks: np.ndarray | None = None):
        """Host batch: (n, h, w) uint8 -> (kps (n, cap), desc (n, cap, 32), counts (n,))."""
        images = np.ascontiguousarray(images, np.uint8)
        n, h, w = images.shape
        cap = self.capacity(w, h)
        kps = np.zeros((n, cap), KEYPOINT_DTYPE)
        desc = np.zeros((n, cap, 32), np.uint8)
        cnt = np.zeros(n, np.int32)
        arr = (C.c_void_p * n)(*[images[i].ctypes.data for i in range(n)])
        marr = None
        if masks is not None:
            masks = np.ascontiguousarray(masks, np.uint8)
            marr = (C.c_void_p * n)(*[masks[i].ctypes.data for i in range(n)])
        _check("orbfe_extract_batch", lib().orbfe_extract_batch(
            self._h, arr, n, w, h, C.c_size_t(w), marr, C.c_size_t(w), ptr(kps), cap, ptr(desc),
            ptr(cnt)))
        return kps, desc, cnt

    def extract_batch_device(self, d_imgs: int, n: int, w: int, h: int, stride: int,
                             frame_pitch: int, d_kps: int, kps_cap: int, d_desc: int,
                             d_n_out: int, d_masks: int | None = None) -> None:
        """Device-resident batch (raw device pointers, e.g. torch ``data_ptr()``); async."""
        _check("orbfe_extract_batch_device", lib().orbfe_extract_batch_device(
            self._h, C.c_void_p(d_imgs), n, w, h, C.c_size_t(stride), C.c_size_t(frame_pitch),
            C.c_void_p(d_masks) if d_masks else None, C.c_void_p(d_kps), kps_cap,
            C.c_void_p(d_desc), C.c_void_p(d_n_out)))

    def set_stream(self, stream_handle: int | None) -> None:
        _check("orbfe_set_stream", lib().orbfe_set_stream(
            self._h, _stream_arg(stream_handle)))

    def synchronize(self) -> None:
        _check("orbfe_synchronize", lib().orbfe_synchronize(self._h))

    STAGES = ("mask", "resize", "fast", "octree", "blur", "describe")

    def profile(self, enable: bool, stages=None) -> None:
        """Record a HIP event pair around every kernel launch (orbfe_profile), or only around
        the launches of the named stages (e.g. ("fast",))."""
        mode = int(bool(enable))
        if enable and stages is not None:
            mode = 0
            for st in stages:
                mode |= 2 << self.STAGES.index(st)
        _check("orbfe_profile", lib().orbfe_profile(self._h, mode))

    def set_stages(self, stages=None) -> None:
        """orbfe_set_stage_mask: later extraction calls run only the named stages (None: all)."""
        mask = 0
        for st in stages or ():
            mask |= 1 << self.STAGES.index(st)
        _check("orbfe_set_stage_mask", lib().orbfe_set_stage_mask(self._h, C.c_uint(mask)))

    def replay(self, stages, reps: int = 1) -> None:
        """orbfe_debug_replay: relaunch the named stages of the last extraction reps times."""
        mask = 0
        for st in stages:
            mask |= 1 << self.STAGES.index(st)
        _check("orbfe_debug_replay", lib().orbfe_debug_replay(self._h, C.c_uint(mask), int(reps)))

    def profile_read(self) -> dict:
        """{stage: (total_ms, launches)} since the previous read (orbfe_profile_read)."""
        ms = np.zeros(len(self.STAGES), np.float64)
        n = np.zeros(len(self.STAGES), np.int32)
        _check("orbfe_profile_read", lib().orbfe_profile_read(self._h, ptr(ms), ptr(n)))
        return {s: (float(ms[i]), int(n[i])) for i, s in enumerate(self.STAGES)}

    PYR_PATHS = ("per_level", "bands")

    def pyramid_path(self, nframes: int) -> str:
        """The pyramid kernel an extraction of `nframes` frames at the last extracted size takes
        (orbfe_pyramid_path): "per_level" or "bands"."""
        r = lib().orbfe_pyramid_path(self._h, int(nframes))
        _check("orbfe_pyramid_path", r if r < 0 else 0)
        return self.PYR_PATHS[r]

    # ---- probes of the last extraction
    def _level(self, fn, frame: int, level: int) -> np.ndarray:
        w, h = C.c_int(0), C.c_int(0)
        _check(fn.__name__, fn(self._h, frame, level, None, C.byref(w), C.byref(h)))
        out = np.zeros((h.value, w.value), np.uint8)
        _check(fn.__name__, fn(self._h, frame, level, ptr(out), C.byref(w), C.byref(h)))
        return out

    def get_level(self, level: int, frame: int = 0) -> np.ndarray:
        """mvImagePyramid[level] of the last extraction (ORBextractor.h:90)."""
        return self._level(lib().orbfe_get_level, frame, level)

    @property
    def mvImagePyramid(self) -> list[np.ndarray]:
        return [self.get_level(l) for l in range(self.nlevels)]

    def get_blurred_level(self, level: int, frame: int = 0) -> np.ndarray:
        return self._level(lib().orbfe_get_blurred_level, frame, level)

    def get_fast_keys(self, level: int, frame: int = 0) -> np.ndarray:
        cap = 65536
        while True:
            out = np.zeros(cap, KEYPOINT_DTYPE)
            n = C.c_int(0)
            st = lib().orbfe_get_fast_keys(self._h, frame, level, ptr(out), cap, C.byref(n))
            if st == ORBFE_ERR_CAPACITY:
                cap = n.value
                continue
            _check("orbfe_get_fast_keys", st)
            return out[:n.value].copy()


def archive_mat_bytes(rows: int, cols: int = 32, elem_size: int = 1) -> int:
    """Bytes of one cv::Mat archive record (MapPoint.h:215-247)."""
    return int(lib().orbfe_archive_mat_bytes(rows, cols, elem_size))


def archive_write_keypoints_device(n_frames: int, d_keys: int, keys_pitch: int, d_n: int,
                                   cap: int, d_out: int, out_pitch: int, stream=None) -> None:
    """Keypoint records (serialize(Archive&, cv::KeyPoint&), MapPoint.h:196-209) from HBM."""
    _check("orbfe_archive_write_keypoints_device", lib().orbfe_archive_write_keypoints_device(
        n_frames, d_keys, keys_pitch, d_n, cap, d_out, out_pitch, stream))


def archive_read_keypoints_device(n_frames: int, d_in: int, in_pitch: int, d_n: int, cap: int,
                                  d_keys: int, keys_pitch: int, stream=None) -> None:
    _check("orbfe_archive_read_keypoints_device", lib().orbfe_archive_read_keypoints_device(
        n_frames, d_in, in_pitch, d_n, cap, d_keys, keys_pitch, stream))


def archive_write_descriptors_device(n_mats: int, d_desc: int, desc_pitch: int, d_rows,
                                     rows_fixed: int, cap: int, d_out: int, out_pitch: int,
                                     d_len=None, stream=None) -> None:
    """rows x 32 CV_8UC1 cv::Mat records (MapPoint.h:215-229) from HBM descriptors."""
    _check("orbfe_archive_write_descriptors_device", lib().orbfe_archive_write_descriptors_device(
        n_mats, d_desc, desc_pitch, d_rows, rows_fixed, cap, d_out, out_pitch, d_len, stream))


def archive_read_descriptors_device(n_mats: int, d_in: int, in_pitch: int, cap: int,
                                    d_desc: int, desc_pitch: int, d_rows, d_status: int,
                                    stream=None) -> None:
    _check("orbfe_archive_read_descriptors_device", lib().orbfe_archive_read_descriptors_device(
        n_mats, d_in, in_pitch, cap, d_desc, desc_pitch, d_rows, d_status, stream))


class Vocabulary:
    """ORBVocabulary (DBoW2 TemplatedVocabulary<FORB>) held in HBM: loadFromTextFile and
    transform (Frame::ComputeBoW)."""

    def __init__(self, path: str, device: int = 0):
        st = C.c_int(0)
        h = lib().orbfe_vocabulary_load_text(path.encode(), device, C.byref(st))
        if not h:
            raise OrbfeError("orbfe_vocabulary_load_text", st.value)
        self._h = C.c_void_p(h)
        info = np.zeros(6, np.int32)
        _check("orbfe_vocabulary_info", lib().orbfe_vocabulary_info(self._h, ptr(info)))
        self.k, self.L, self.scoring, self.weighting, self.nodes, self.words = map(int, info)

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().orbfe_vocabulary_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def transform(self, desc: np.ndarray, levelsup: int = 4):
        """-> (word_ids, values, node_ids, node_off, feat) = BowVector + FeatureVector."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        cap = max(n, 1)
        wid = np.zeros(cap, np.int32)
        val = np.zeros(cap, np.float64)
        nid = np.zeros(cap, np.int32)
        off = np.zeros(cap + 1, np.int32)
        feat = np.zeros(cap, np.int32)
        nw, nn = C.c_int32(0), C.c_int32(0)
        _check("orbfe_bow_transform", lib().orbfe_bow_transform(
            self._h, ptr(d), n, levelsup, ptr(wid), ptr(val), C.byref(nw), ptr(nid), ptr(off),
            ptr(feat), C.byref(nn)))
        return (wid[:nw.value].copy(), val[:nw.value].copy(), nid[:nn.value].copy(),
                off[:nn.value + 1].copy(), feat[:off[nn.value]].copy())

    def transform_batch_device(self, nframes: int, d_desc: int, d_n: int, cap: int,
                               levelsup: int, d_wid: int, d_val: int, d_nw: int, d_nid: int,
                               d_noff: int, d_feat: int, d_nn: int) -> None:
        _check("orbfe_bow_transform_batch_device", lib().orbfe_bow_transform_batch_device(
            self._h, nframes, C.c_void_p(d_desc), C.c_void_p(d_n), cap, levelsup,
            C.c_void_p(d_wid), C.c_void_p(d_val), C.c_void_p(d_nw), C.c_void_p(d_nid),
            C.c_void_p(d_noff), C.c_void_p(d_feat), C.c_void_p(d_nn)))

    def set_stream(self, stream_handle: int | None) -> None:
        _check("orbfe_vocabulary_set_stream", lib().orbfe_vocabulary_set_stream(
            self._h, _stream_arg(stream_handle)))


class ORBmatcher:
    """``ORBmatcher(nnratio=0.6, checkOri=true)`` (ORBmatcher.cc:41-43), GPU-backed."""

    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30  # ORBmatcher.cc:37-39

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        st = C.c_int(0)
        h = lib().orbfe_matcher_create(device, C.byref(st))
        if not h:
            raise OrbfeError("orbfe_matcher_create", st.value)
        self._h = C.c_void_p(h)

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().orbfe_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def DescriptorDistance(self, a: np.ndarray, b: np.ndarray) -> np.ndarray | int:
        """Row-wise Hamming distance (ORBmatcher.cc:1650-1666)."""
        a2 = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
        b2 = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
        out = np.zeros(len(a2), np.int32)
        _check("orbfe_hamming", lib().orbfe_hamming(self._h, ptr(a2), ptr(b2), len(a2), ptr(out)))
        return int(out[0]) if np.ndim(a) == 1 else out

    def bf_match(self, q: np.ndarray, r: np.ndarray):
        q = np.ascontiguousarray(q, np.uint8).reshape(-1, 32)
        r = np.ascontiguousarray(r, np.uint8).reshape(-1, 32)
        bi, bd, sd = (np.zeros(len(q), np.int32) for _ in range(3))
        _check("orbfe_bf_match", lib().orbfe_bf_match(self._h, ptr(q), len(q), ptr(r), len(r),
                                                      ptr(bi), ptr(bd), ptr(sd)))
        return bi, bd, sd

    def bf_match_batch_device(self, d_q: int, q_pitch: int, d_nq: int, nq_cap: int, d_r: int,
                              r_pitch: int, d_nr: int, nb: int, d_out: int) -> None:
        _check("orbfe_bf_match_batch_device", lib().orbfe_bf_match_batch_device(
            self._h, C.c_void_p(d_q), C.c_size_t(q_pitch), C.c_void_p(d_nq), nq_cap,
            C.c_void_p(d_r), C.c_size_t(r_pitch), C.c_void_p(d_nr), nb, C.c_void_p(d_out)))

    def profile(self, enable: bool) -> None:
        _check("orbfe_matcher_profile", lib().orbfe_matcher_profile(self._h, int(enable)))

    def profile_read(self) -> tuple[float, int]:
        """(total ms, launches) of the brute-force match kernels since the previous read."""
        ms = np.zeros(1, np.float64)
        n = np.zeros(1, np.int32)
        _check("orbfe_matcher_profile_read", lib().orbfe_matcher_profile_read(self._h, ptr(ms), ptr(n)))
        return float(ms[0]), int(n[0])

    def profile_read_stages(self) -> dict:
        """{"bf_match": (ms, launches), "bf_expand": (ms, launches)} since the previous read:
        the match kernels and the shared-reference expansion (orbfe_matcher_profile_read_stages)."""
        ms = np.zeros(2, np.float64)
        n = np.zeros(2, np.int32)
        _check("orbfe_matcher_profile_read_stages",
               lib().orbfe_matcher_profile_read_stages(self._h, ptr(ms), ptr(n)))
        return {"bf_match": (float(ms[0]), int(n[0])), "bf_expand": (float(ms[1]), int(n[1]))}

    def set_stream(self, stream_handle: int | None) -> None:
        _check("orbfe_matcher_set_stream", lib().orbfe_matcher_set_stream(
            self._h, _stream_arg(stream_handle)))

    def SearchForInitialization(self, F1: Frame, F2: Frame, vbPrevMatched: np.ndarray,
                                windowSize: int = 10):
        """Returns (vnMatches12, nmatches, updated vbPrevMatched) (ORBmatcher.cc:408-523)."""
        prev = np.ascontiguousarray(vbPrevMatched, np.float32).reshape(-1, 2).copy()
        m12 = np.zeros(F1.n, np.int32)
        nm = C.c_int32(0)
        v1, v2 = F1.view(), F2.view()
        _check("orbfe_search_for_initialization", lib().orbfe_search_for_initialization(
            self._h, C.c_float(self.mfNNratio), int(self.mbCheckOrientation), C.byref(v1),
            C.byref(v2), ptr(prev), windowSize, ptr(m12), C.byref(nm)))
        return m12, nm.value, prev

    def SearchByProjection(self, F: Frame, mps: MapPoints, th: float = 3.0, frame_mp=None,
                           frame_mp_obs=None, mp_ids=None):
        """Local-map overload (ORBmatcher.cc:45-129).  Returns (frame_mp, frame_mp_obs,
        nmatches): the MapPoint id held by each keypoint (-1 = none)."""
        fmp = (np.full(F.n, -1, np.int32) if frame_mp is None
               else np.ascontiguousarray(frame_mp, np.int32).copy())
        fobs = (np.zeros(F.n, np.int32) if frame_mp_obs is None
                else np.ascontiguousarray(frame_mp_obs, np.int32).copy())
        ids = None if mp_ids is None else np.ascontiguousarray(mp_ids, np.int32)
        nm = C.c_int32(0)
        fv, mv = F.view(), mps.view()
        _check("orbfe_search_by_projection_local", lib().orbfe_search_by_projection_local(
            self._h, C.c_float(self.mfNNratio), C.byref(fv), ptr(fmp), ptr(fobs), C.byref(mv),
            ptr(ids), C.c_float(th), C.byref(nm)))
        return fmp, fobs, nm.value

    def SearchByProjectionLast(self, cur: Frame, tcw_cur, cam: Camera, last_keys, last_valid,
                               last_outlier, last_xyz, last_desc, last_nobs, tcw_last,
                               th: float, bMono: bool, frame_mp=None, frame_mp_obs=None,
                               last_ids=None):
        """Last-frame overload (ORBmatcher.cc:1331-1473)."""
        fmp = (np.full(cur.n, -1, np.int32) if frame_mp is None
               else np.ascontiguousarray(frame_mp, np.int32).copy())
        fobs = (np.zeros(cur.n, np.int32) if frame_mp_obs is None
                else np.ascontiguousarray(frame_mp_obs, np.int32).copy())
        a = [np.ascontiguousarray(tcw_cur, np.float32).reshape(12),
             np.ascontiguousarray(last_keys, KEYPOINT_DTYPE),
             np.ascontiguousarray(last_valid, np.uint8),
             np.ascontiguousarray(last_outlier, np.uint8),
             np.ascontiguousarray(last_xyz, np.float32).reshape(-1, 3),
             np.ascontiguousarray(last_desc, np.uint8).reshape(-1, 32),
             np.ascontiguousarray(last_nobs, np.int32),
             np.ascontiguousarray(tcw_last, np.float32).reshape(12)]
        ids = None if last_ids is None else np.ascontiguousarray(last_ids, np.int32)
        nm = C.c_int32(0)
        cv = cur.view()
        _check("orbfe_search_by_projection_last", lib().orbfe_search_by_projection_last(
            self._h, int(self.mbCheckOrientation), C.byref(cv), ptr(a[0]), C.byref(cam),
            ptr(fmp), ptr(fobs), len(a[1]), ptr(a[1]), ptr(a[2]), ptr(a[3]), ptr(a[4]),
            ptr(a[5]), ptr(a[6]), ptr(ids), ptr(a[7]), C.c_float(th), int(bMono),
            C.byref(nm)))
        return fmp, fobs, nm.value

    def SearchByProjectionKeyFrame(self, cur: Frame, tcw_cur, cam: Camera, log_scale: float,
                                   kf_angle, kf_valid, kf_bad, already_found, kf_xyz, kf_desc,
                                   kf_min_dist, kf_max_dist, th: float, ORBdist: int,
                                   frame_mp=None, kf_ids=None):
        """Relocalisation overload SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th,
        ORBdist) (ORBmatcher.cc:1475-1602).  Returns (frame_mp, nmatches)."""
        fmp = (np.full(cur.n, -1, np.int32) if frame_mp is None
               else np.ascontiguousarray(frame_mp, np.int32).copy())
        a = [np.ascontiguousarray(tcw_cur, np.float32).reshape(12),
             np.ascontiguousarray(kf_angle, np.float32),
             np.ascontiguousarray(kf_valid, np.uint8),
             np.ascontiguousarray(kf_bad, np.uint8),
             np.ascontiguousarray(already_found, np.uint8),
             np.ascontiguousarray(kf_xyz, np.float32).reshape(-1, 3),
             np.ascontiguousarray(kf_desc, np.uint8).reshape(-1, 32),
             np.ascontiguousarray(kf_min_dist, np.float32),
             np.ascontiguousarray(kf_max_dist, np.float32)]
        ids = None if kf_ids is None else np.ascontiguousarray(kf_ids, np.int32)
        nm = C.c_int32(0)
        cv = cur.view()
        _check("orbfe_search_by_projection_keyframe", lib().orbfe_search_by_projection_keyframe(
            self._h, int(self.mbCheckOrientation), C.byref(cv), ptr(a[0]), C.byref(cam),
            C.c_float(log_scale), ptr(fmp), len(a[1]), *(ptr(x) for x in a[1:]), ptr(ids),
            C.c_float(th), int(ORBdist), C.byref(nm)))
        return fmp, nm.value

    def ComputeDistinctiveDescriptors(self, obs_off: np.ndarray, obs_desc: np.ndarray):
        """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:483-548) over a CSR of the
        points' observation descriptors -> (best row per point or -1, mDescriptor (n, 32))."""
        off = np.ascontiguousarray(obs_off, np.int32)
        d = np.ascontiguousarray(obs_desc, np.uint8).reshape(-1, 32)
        n = len(off) - 1
        best = np.zeros(n, np.int32)
        out = np.zeros((n, 32), np.uint8)
        _check("orbfe_distinctive_descriptors", lib().orbfe_distinctive_descriptors(
            self._h, n, ptr(off), ptr(d), ptr(best), ptr(out)))
        return best, out

    def search_local_points_device(self, n_kp: int, d_keys: int, d_desc: int,
                                   d_u_right: int | None, width: int, height: int,
                                   scale_factors: np.ndarray, tcw, cam: Camera,
                                   log_scale: float, cos_limit: float, n_mp: int, d_xyz: int,
                                   d_normal: int, d_min: int, d_max: int, d_mdesc: int,
                                   d_nobs: int, d_bad: int, d_skip: int | None,
                                   d_ids: int | None, nnratio: float, th: float, d_fmp: int,
                                   d_fobs: int, d_in_view: int) -> tuple[int, int]:
        """Tracking::SearchLocalPoints on device-resident frame + local map
        (orbfe_search_local_points_device) -> (nmatches, nToMatch)."""
        sf = np.ascontiguousarray(scale_factors, np.float32)
        gw = np.float32(64) / np.float32(width)
        gh = np.float32(48) / np.float32(height)
        fv = FrameView(n_kp, C.c_void_p(d_keys), C.c_void_p(d_desc),
                       C.c_void_p(d_u_right) if d_u_right else None, 0.0, float(width), 0.0,
                       float(height), float(gw), float(gh), ptr(sf), len(sf))
        t = np.ascontiguousarray(tcw, np.float32).reshape(12)
        counts = np.zeros(2, np.int32)
        vp = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        _check("orbfe_search_local_points_device", lib().orbfe_search_local_points_device(
            self._h, C.byref(fv), ptr(t), C.byref(cam), C.c_float(log_scale),
            C.c_float(cos_limit), n_mp, vp(d_xyz), vp(d_normal), vp(d_min), vp(d_max),
            vp(d_mdesc), vp(d_nobs), vp(d_bad), vp(d_skip), vp(d_ids), C.c_float(nnratio),
            C.c_float(th), vp(d_fmp), vp(d_fobs), vp(d_in_view), ptr(counts)))
        return int(counts[0]), int(counts[1])

    def search_by_projection_local_device(self, n_kp: int, d_keys: int, d_desc: int,
                                          d_u_right: int | None, width: int, height: int,
                                          scale_factors: np.ndarray, n_mp: int,
                                          d_in_view: int, d_bad: int, d_px: int, d_py: int,
                                          d_pxr: int, d_lvl: int, d_vcos: int, d_mdesc: int,
                                          d_nobs: int, d_ids: int | None, nnratio: float,
                                          th: float, d_fmp: int, d_fobs: int) -> int:
        """SearchByProjection(F, vpLocalMapPoints, th) alone on device-resident isInFrustum
        outputs (orbfe_search_by_projection_local_device) -> nmatches."""
        sf = np.ascontiguousarray(scale_factors, np.float32)
        gw = np.float32(64) / np.float32(width)
        gh = np.float32(48) / np.float32(height)
        fv = FrameView(n_kp, C.c_void_p(d_keys), C.c_void_p(d_desc),
                       C.c_void_p(d_u_right) if d_u_right else None, 0.0, float(width), 0.0,
                       float(height), float(gw), float(gh), ptr(sf), len(sf))
        vp = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        mv = MapPointView(n_mp, vp(d_in_view), vp(d_bad), vp(d_px), vp(d_py), vp(d_pxr),
                          vp(d_lvl), vp(d_vcos), vp(d_mdesc), vp(d_nobs))
        nm = C.c_int32(0)
        _check("orbfe_search_by_projection_local_device",
               lib().orbfe_search_by_projection_local_device(
                   self._h, C.c_float(nnratio), C.byref(fv), vp(d_fmp), vp(d_fobs), C.byref(mv),
                   vp(d_ids), C.c_float(th), C.byref(nm)))
        return nm.value

    def last_rounds(self) -> int:
        return lib().orbfe_matcher_last_rounds(self._h)

    def GetFeaturesInArea(self, F: Frame, x, y, r, min_level=-1, max_level=-1, wave=False):
        """Frame::GetFeaturesInArea (Frame.cc:445-498) for arrays of queries on F's grid
        (orbfe_features_in_area).  Returns one int32 array of keypoint indices per query, in
        the reference's candidate order."""
        x = np.ascontiguousarray(np.atleast_1d(x), np.float32)
        nq = len(x)
        y = np.ascontiguousarray(np.broadcast_to(np.asarray(y, np.float32), (nq,)))
        r = np.ascontiguousarray(np.broadcast_to(np.asarray(r, np.float32), (nq,)))
        lo = np.ascontiguousarray(np.broadcast_to(np.asarray(min_level, np.int32), (nq,)))
        hi = np.ascontiguousarray(np.broadcast_to(np.asarray(max_level, np.int32), (nq,)))
        off = np.zeros(nq + 1, np.int32)
        fv = F.view()
        st = lib().orbfe_features_in_area(self._h, C.byref(fv), nq, ptr(x), ptr(y), ptr(r),
                                          ptr(lo), ptr(hi), int(bool(wave)), ptr(off), None, 0)
        items = np.zeros(max(int(off[nq]), 1), np.int32)
        if st == ORBFE_ERR_CAPACITY:
            st = lib().orbfe_features_in_area(self._h, C.byref(fv), nq, ptr(x), ptr(y), ptr(r),
                                              ptr(lo), ptr(hi), int(bool(wave)), ptr(off),
                                              ptr(items), len(items))
        _check("orbfe_features_in_area", st)
        return [items[off[q]:off[q + 1]].copy() for q in range(nq)]

    def capacity_retries(self) -> int:
        """Calls rerun because their candidates outgrew the device buffer (diagnostics)."""
        return lib().orbfe_matcher_capacity_retries(self._h)

    def SearchByBoW(self, kf_desc, kf_angle, kf_mp_ok, kf_fv, f_desc, f_angle, f_fv):
        """SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches) (ORBmatcher.cc:159-291); *_fv are
        (node_ids, node_off, feat) FeatureVectors.  Returns (matches per frame feature, n)."""
        kd = np.ascontiguousarray(kf_desc, np.uint8).reshape(-1, 32)
        fd = np.ascontiguousarray(f_desc, np.uint8).reshape(-1, 32)
        ka = np.ascontiguousarray(kf_angle, np.float32)
        fa = np.ascontiguousarray(f_angle, np.float32)
        ok = np.ascontiguousarray(kf_mp_ok, np.uint8)
        kn, ko, kfe = (np.ascontiguousarray(x, np.int32) for x in kf_fv)
        fn, fo, ffe = (np.ascontiguousarray(x, np.int32) for x in f_fv)
        out = np.zeros(len(fd), np.int32)
        nm = C.c_int32(0)
        _check("orbfe_search_by_bow", lib().orbfe_search_by_bow(
            self._h, C.c_float(self.mfNNratio), int(self.mbCheckOrientation), len(kd), ptr(kd),
            ptr(ka), ptr(ok), len(kn), ptr(kn), ptr(ko), ptr(kfe), len(fd), ptr(fd), ptr(fa),
            len(fn), ptr(fn), ptr(fo), ptr(ffe), ptr(out), C.byref(nm)))
        return out, nm.value

    def search_by_bow_batch_device(self, n_pairs: int, d_pair_kf: int, d_pair_f: int,
                                   kf_cap: int, d_kf_desc: int, d_kf_angle: int, d_kf_mp_ok: int,
                                   d_kf_nn: int, d_kf_node_ids: int, d_kf_node_off: int,
                                   d_kf_feat: int, f_cap: int, d_f_desc: int, d_f_angle: int,
                                   d_f_nn: int, d_f_node_ids: int, d_f_node_off: int,
                                   d_f_feat: int, d_matches: int, d_nmatches: int,
                                   d_status: int) -> None:
        """SearchByBoW over n_pairs (keyframe slot, frame slot) pairs (Tracking::Relocalization's
        candidate loop, Tracking.cc:1636-1656); device pointers in the layout of
        Vocabulary.transform_batch_device.  Asynchronous on the matcher's stream."""
        v = C.c_void_p
        _check("orbfe_search_by_bow_batch_device", lib().orbfe_search_by_bow_batch_device(
            self._h, C.c_float(self.mfNNratio), int(self.mbCheckOrientation), n_pairs,
            v(d_pair_kf), v(d_pair_f), kf_cap, v(d_kf_desc), v(d_kf_angle), v(d_kf_mp_ok),
            v(d_kf_nn), v(d_kf_node_ids), v(d_kf_node_off), v(d_kf_feat), f_cap, v(d_f_desc),
            v(d_f_angle), v(d_f_nn), v(d_f_node_ids), v(d_f_node_off), v(d_f_feat),
            v(d_matches), v(d_nmatches), v(d_status)))

    def is_in_frustum(self, xyz, normal, min_dist, max_dist, tcw, cam: Camera, bounds,
                      log_scale: float, cos_limit: float = 0.5):
        """Frame::isInFrustum + MapPoint::PredictScale over all map points (Frame.cc:387)."""
        xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
        n = len(xyz)
        normal = np.ascontiguousarray(normal, np.float32).reshape(-1, 3)
        mn = np.ascontiguousarray(min_dist, np.float32)
        mx = np.ascontiguousarray(max_dist, np.float32)
        t = np.ascontiguousarray(tcw, np.float32).reshape(12)
        inv = np.zeros(n, np.uint8)
        px, py, pxr, vc = (np.zeros(n, np.float32) for _ in range(4))
        pl = np.zeros(n, np.int32)
        _check("orbfe_is_in_frustum", lib().orbfe_is_in_frustum(
            self._h, n, ptr(xyz), ptr(normal), ptr(mn), ptr(mx), ptr(t), C.byref(cam),
            *(C.c_float(b) for b in bounds), C.c_float(log_scale), C.c_float(cos_limit),
            ptr(inv), ptr(px), ptr(py), ptr(pxr), ptr(pl), ptr(vc)))
        return inv, px, py, pxr, pl, vc
