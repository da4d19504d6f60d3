"""CPU checks of native pieces that do not need a GPU: the introsort replica against libstdc++'s
std::sort, the glibc sincosf restatement against the host libm, and the C ABI export table."""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HARNESS = r'''
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
#include "omv_introsort.h"
struct P { int k1, k2, id; };
static bool less_(const P &a, const P &b) { return a.k1 < b.k1 || (a.k1 == b.k1 && a.k2 < b.k2); }
int main() {
    std::mt19937 rng(1234);
    int stack[192];
    for (int trial = 0; trial < 3000; ++trial) {
        int n = trial < 100 ? trial : (int)(rng() % 2000);
        int kmax = 1 + (int)(rng() % 6), xmax = 1 + (int)(rng() % 4);
        std::vector<P> a(n);
        for (int i = 0; i < n; ++i) a[i] = P{(int)(rng() % kmax), (int)(rng() % xmax), i};
        if (trial % 7 == 0) std::sort(a.begin(), a.end(), [](const P &x, const P &y) { return x.id > y.id; });
        if (trial % 11 == 0)   // median-of-3 killer-ish pattern to reach the heapsort fallback
            for (int i = 0; i < n; ++i) a[i].k1 = (i % 2) ? i : n - i, a[i].k2 = 0;
        std::vector<omv::SortItem> b(n);
        for (int i = 0; i < n; ++i) b[i] = omv::SortItem{a[i].k1, a[i].k2, a[i].id};
        std::sort(a.begin(), a.end(), less_);
        omv::libstdcxx_sort(b.data(), n, stack);
        for (int i = 0; i < n; ++i)
            if (a[i].id != b[i].payload) { std::printf("MISMATCH trial %d n %d at %d\n", trial, n, i); return 1; }
    }
    std::printf("OK\n");
    return 0;
}
'''


def test_introsort_replica_matches_std_sort():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "h.cpp")
        open(src, "w").write(HARNESS)
        exe = os.path.join(d, "h")
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "openmavis_amd", "csrc"),
                               src, "-o", exe])
        out = subprocess.run([exe], capture_output=True, text=True)
        assert out.returncode == 0 and "OK" in out.stdout, out.stdout


def test_sincosf_restatement_matches_libm():
    """tools/check_sincosf.c carries the same constants/ops as omv_device.h::glibc_sincosf; here a
    strided sweep of [0, 2*pi] (the full sweep is bit-exact too: 1,086,918,620 floats)."""
    src = os.path.join(ROOT, "tools", "check_sincosf.c")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "cs")
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-DUSEFMA", "-DSTRIDE=97", src, "-o", exe, "-lm"])
        out = subprocess.run([exe], capture_output=True, text=True, timeout=120).stdout
        m = re.search(r"cos_bad (\d+) sin_bad (\d+)", out)
        assert m and m.group(1) == "0" and m.group(2) == "0", out


def test_atan2f_restatement_matches_libm():
    """tools/check_atan2f.c carries the same constants/ops as omv_device.h::glibc_atan2f (KB8 projection)."""
    src = os.path.join(ROOT, "tools", "check_atan2f.c")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "at")
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-DN=3000000L", src, "-o", exe, "-lm"])
        out = subprocess.run([exe], capture_output=True, text=True, timeout=120).stdout
        m = re.search(r"n (\d+) bad (\d+)", out)
        assert m and int(m.group(1)) > 2000000 and m.group(2) == "0", out


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "omv.h")).read()
    return sorted(set(re.findall(r"^\s*(?:omv_status|int|void)\s+(omv_\w+)\s*\(", hdr, re.M)))


def test_library_exports_every_declared_symbol():
    from openmavis_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from openmavis_amd import build
        build.build_hip()
    lib = _lib.load()
    declared = _declared_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in include/omv.h but not exported"
        assert name in _lib.SIGNATURES, f"{name} has no ctypes binding"
    assert _lib.missing == []


def test_no_device_means_loud_failure():
    """No CPU fallback: without a GPU the product entry points raise."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from openmavis_amd import _lib
    from openmavis_amd.orb import ORBextractor
    with pytest.raises(_lib.OmvError):
        ORBextractor(500, 1.2, 8, 20, 7, width=640, height=480)


def test_unknown_camera_model_is_rejected():
    """Every projecting entry point rejects a camera type other than KB8 / Pinhole before touching the device
    (a stray cam_model used to mean KB8 silently): omv_frustum through omv_rig.model."""
    import ctypes
    from openmavis_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from openmavis_amd import build
        build.build_hip()
    lib = _lib.load()
    rig = _lib.Rig()
    rig.n_cams, rig.n_levels, rig.log_scale_factor = 2, 8, 0.18232156
    rig.min_x, rig.max_x, rig.min_y, rig.max_y = 0.0, 720.0, 0.0, 540.0
    dummy = (ctypes.c_byte * 4096)()
    poses, world, track = ctypes.cast(dummy, ctypes.c_void_p), _lib.MpWorld(), _lib.MpTrack()
    for bad in (2, -1, 7):
        rig.model[1] = bad
        st = lib.omv_frustum(1, poses, ctypes.byref(rig), ctypes.byref(world), 0, ctypes.c_float(0.5),
                             ctypes.byref(track), None, None)
        assert st == _lib.OMV_ERR_ARG, (bad, st)
    rig.model[1] = 1   # Pinhole: accepted (M = 0 returns before any launch)
    st = lib.omv_frustum(1, poses, ctypes.byref(rig), ctypes.byref(world), 0, ctypes.c_float(0.5),
                         ctypes.byref(track), None, None)
    assert st == 0
