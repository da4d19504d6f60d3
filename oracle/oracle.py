"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/liboracle.so, the CPU restatement of the
reference (see orb_oracle.cpp / match_oracle.cpp headers).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker / baseline, never as
the thing measured or shipped.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4")])

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", HERE])
        _lib = ctypes.CDLL(LIB)
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def orb_tables(nfeatures=1200, scale=1.2, nlevels=8):
    sc, isc, s2, is2 = (np.zeros(nlevels, np.float32) for _ in range(4))
    q = np.zeros(nlevels, np.int32)
    um = np.zeros(16, np.int32)
    lib().oracle_orb_tables(nfeatures, ctypes.c_float(scale), nlevels, _p(sc), _p(isc), _p(s2), _p(is2), _p(q), _p(um))
    return dict(scale=sc, inv_scale=isc, sigma2=s2, inv_sigma2=is2, quota=q, umax=um)


def pyramid_level(img, level, nfeatures=1200, scale=1.2, nlevels=8):
    img = np.ascontiguousarray(img)
    h, w = img.shape
    ow, oh = ctypes.c_int(), ctypes.c_int()
    lib().oracle_orb_pyramid_level(_p(img), w, h, w, nfeatures, ctypes.c_float(scale), nlevels, level, None,
                                   ctypes.byref(ow), ctypes.byref(oh))
    out = np.zeros((oh.value, ow.value), np.uint8)
    lib().oracle_orb_pyramid_level(_p(img), w, h, w, nfeatures, ctypes.c_float(scale), nlevels, level, _p(out),
                                   ctypes.byref(ow), ctypes.byref(oh))
    return out


def level_candidates(level_img, ini_th, min_th):
    L = np.ascontiguousarray(level_img)
    h, w = L.shape
    cap = 200000
    xs, ys, rs = (np.zeros(cap, np.float32) for _ in range(3))
    n = lib().oracle_orb_level_candidates(_p(L), w, h, ini_th, min_th, _p(xs), _p(ys), _p(rs), cap)
    return xs[:n].copy(), ys[:n].copy(), rs[:n].copy()


def distribute(xs, ys, resp, minX, maxX, minY, maxY, N):
    xs, ys, resp = (np.ascontiguousarray(a, dtype=np.float32) for a in (xs, ys, resp))
    cap = len(xs) + 8
    sel = np.zeros(cap, np.int32)
    n = lib().oracle_orb_distribute(_p(xs), _p(ys), _p(resp), len(xs), minX, maxX, minY, maxY, N, _p(sel), cap)
    return sel[:n].copy()


def orb_extract(img, nfeatures=1200, scale=1.2, nlevels=8, ini_th=15, min_th=7, lapping=(0, 0)):
    """ORBextractor::operator() restated: returns (monoIndex, kps[KP_DTYPE], desc (n,32) u8)."""
    img = np.ascontiguousarray(img)
    h, w = img.shape
    cap = nfeatures + 64 * nlevels
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    mono = ctypes.c_int()
    n = lib().oracle_orb_extract(_p(img), w, h, w, nfeatures, ctypes.c_float(scale), nlevels, ini_th, min_th,
                                 int(lapping[0]), int(lapping[1]), _p(kps), _p(desc), cap, ctypes.byref(mono))
    return mono.value, kps[:n].copy(), desc[:n].copy()


def orb_extract_frame(imgs, nfeatures, lapping, scale=1.2, nlevels=8, ini_th=15, min_th=7, threaded=True):
    """Multi-camera frame, one std::thread per camera like src/Frame.cc:1841-1862."""
    imgs = np.ascontiguousarray(imgs)
    nc, h, w = imgs.shape
    cap = nfeatures + 64 * nlevels
    kps = np.zeros((nc, cap), KP_DTYPE)
    desc = np.zeros((nc, cap, 32), np.uint8)
    n_out = np.zeros(nc, np.int32)
    mono = np.zeros(nc, np.int32)
    ptrs = (ctypes.c_void_p * nc)(*[imgs[c].ctypes.data for c in range(nc)])
    lap = np.ascontiguousarray(np.asarray(lapping, np.int32).reshape(nc, 2))
    lib().oracle_orb_extract_frame(nc, ptrs, w, h, w, nfeatures, ctypes.c_float(scale), nlevels, ini_th, min_th,
                                   _p(lap), _p(kps), _p(desc), cap, _p(n_out), _p(mono), int(threaded))
    return n_out, mono, kps, desc


def fast_atan2(y, x):
    f = lib().oracle_fast_atan2
    f.restype = ctypes.c_float
    return f(ctypes.c_float(y), ctypes.c_float(x))
