"""Host-side mirror of the reference's ORBextractor (include/ORBextractor.h:22-79) on the HIP path.

    ex = ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
    mono_index, keypoints, descriptors = ex(image, mask, vLappingArea)   # operator()

mirrors `int operator()(InputArray image, InputArray mask, vector<KeyPoint>& kps,
OutputArray desc, vector<int>& vLappingArea)` (src/ORBextractor.cc:987-1071): the mask is
ignored, an empty image returns -1, keypoints come back in the reference's order (mono block at
the front, lapping block reversed at the back).  `extract_batch` is the batched device entry point
used by the multi-camera frame and the benchmark (inputs already in HBM, outputs left in HBM).
"""
import ctypes

import numpy as np

from . import _lib


class ORBextractor:
    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, width=None, height=None,
                 max_images=1):
        self.nfeatures = int(nfeatures)
        self.scaleFactor = float(scaleFactor)
        self.nlevels = int(nlevels)
        self.iniThFAST = int(iniThFAST)
        self.minThFAST = int(minThFAST)
        self._lib = _lib.load()
        self._h = None
        self._wh = None
        self._max_images = int(max_images)
        if width is not None:
            self._create(int(width), int(height), self._max_images)

    # -- lifetime ---------------------------------------------------------------------------------
    def _create(self, w, h, max_images):
        self.close()
        p = _lib.OrbParams(self.nfeatures, self.scaleFactor, self.nlevels, self.iniThFAST, self.minThFAST)
        h_ = ctypes.c_void_p()
        _lib.check(self._lib.omv_orb_create(ctypes.byref(p), w, h, max_images, ctypes.byref(h_)), "omv_orb_create")
        self._h = h_
        self._wh = (w, h)
        self._max_images = max_images

    def close(self):
        if self._h is not None:
            self._lib.omv_orb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ensure(self, w, h, n=1):
        if self._h is None or self._wh != (w, h) or n > self._max_images:
            self._create(w, h, max(n, self._max_images))

    # -- getters (include/ORBextractor.h:40-50) --------------------------------------------------
    def _tables(self):
        if self._h is None:
            self._ensure(640, 480)
        t = [np.zeros(self.nlevels, np.float32) for _ in range(4)]
        _lib.check(self._lib.omv_orb_scale_tables(self._h, *[_lib.ptr(a) for a in t]), "omv_orb_scale_tables")
        return t

    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return self.scaleFactor

    def GetScaleFactors(self):
        return self._tables()[0]

    def GetInverseScaleFactors(self):
        return self._tables()[1]

    def GetScaleSigmaSquares(self):
        return self._tables()[2]

    def GetInverseScaleSigmaSquares(self):
        return self._tables()[3]

    def max_keypoints(self):
        return self._lib.omv_orb_max_keypoints(self._h)

    # -- operator() -------------------------------------------------------------------------------
    def __call__(self, image, mask=None, vLappingArea=(0, 0)):
        """Returns (monoIndex, keypoints[structured KP_DTYPE], descriptors (N,32) u8)."""
        img = np.ascontiguousarray(image)
        if img.size == 0:
            return -1, np.zeros(0, _lib.KP_DTYPE), np.zeros((0, 32), np.uint8)
        assert img.dtype == np.uint8 and img.ndim == 2, "CV_8UC1 expected (src/ORBextractor.cc:998)"
        h, w = img.shape
        self._ensure(w, h)
        cap = self.max_keypoints()
        kps = np.zeros(cap, _lib.KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int()
        mono = ctypes.c_int()
        _lib.check(self._lib.omv_orb_extract_host(self._h, _lib.ptr(img), w, int(vLappingArea[0]),
                                                  int(vLappingArea[1]), _lib.ptr(kps), _lib.ptr(desc),
                                                  ctypes.byref(n), ctypes.byref(mono)), "omv_orb_extract_host")
        return mono.value, kps[:n.value].copy(), desc[:n.value].copy()

    # -- batched device path ------------------------------------------------------------------------
    def extract_batch(self, images, lapping, kps, desc, n_out, mono, stream=None, harris=None):
        """images: torch uint8 cuda tensor [n, H, W] (contiguous rows); lapping: host int array [n, 2];
        kps: torch [n, N_max, 6] 32-bit (omv_kp rows); desc: torch uint8 [n, N_max, 32];
        n_out / mono: torch int32 [n]; harris: optional torch float32 [n, N_max], OpenCV ORB's Harris response
        per row (an extra: the reference's response is FAST's).  Asynchronous on `stream` (torch stream or None)."""
        n, h, w = images.shape
        self._ensure(w, h, n)
        _lib.check(self._lib.omv_orb_set_harris(self._h, _lib.ptr(harris) if harris is not None else None),
                   "omv_orb_set_harris")
        lap = np.ascontiguousarray(np.asarray(lapping, dtype=np.int32).reshape(n, 2))
        s = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
        pitch = images.stride(1)
        _lib.check(self._lib.omv_orb_extract_batch(self._h, n, _lib.ptr(images), images.stride(0), pitch,
                                                   _lib.ptr(lap), _lib.ptr(kps), _lib.ptr(desc), _lib.ptr(n_out),
                                                   _lib.ptr(mono), s), "omv_orb_extract_batch")

    def last_error(self):
        return self._lib.omv_orb_last_error(self._h)

    def debug_level(self, img, level):
        w, h = ctypes.c_int(), ctypes.c_int()
        _lib.check(self._lib.omv_orb_debug_level(self._h, img, level, None, ctypes.byref(w), ctypes.byref(h)))
        out = np.zeros((h.value, w.value), np.uint8)
        _lib.check(self._lib.omv_orb_debug_level(self._h, img, level, _lib.ptr(out), ctypes.byref(w),
                                                 ctypes.byref(h)))
        return out

    # -- measurement ------------------------------------------------------------------------------
    def last_counts(self):
        """(FAST candidates, distributed keypoints) of the last batch, summed over its images."""
        c, k = ctypes.c_longlong(), ctypes.c_longlong()
        _lib.check(self._lib.omv_orb_last_counts(self._h, ctypes.byref(c), ctypes.byref(k)), "omv_orb_last_counts")
        return c.value, k.value

    STAGES = ("pyr_resize", "fast_cells", "octree", "describe")

    def enable_timing(self, on=True):
        _lib.check(self._lib.omv_orb_enable_timing(self._h, int(bool(on))))

    def stage_ms(self, reset=True):
        ms = np.zeros(len(self.STAGES), np.float64)
        calls = ctypes.c_longlong()
        _lib.check(self._lib.omv_orb_stage_ms(self._h, _lib.ptr(ms), ctypes.byref(calls), int(bool(reset))))
        return dict(zip(self.STAGES, ms.tolist())), calls.value
