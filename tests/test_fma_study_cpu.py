"""Contraction sensitivity of the ORB restatement (full study: tools/fma_study.py ->
profiles/fma_study.json).  The parity mode rounds every float operation; the reference is built with
-O3 -march=native, where GCC fuses a*b+c.  Pinned here on the golden EuRoC-size image:
- fusing the reference's own steering products (ORBextractor.cc:56-57, GCC's pattern) changes nothing;
- fusing the whole restatement (OpenCV's fastAtan2 included) changes only IC angles, by at most 2 ulp, and
  no descriptor, position, response, octave, count or order."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


@pytest.fixture(scope="module")
def golden_image():
    from openmavis_amd import synth
    g = np.load(os.path.join(ROOT, "tests", "golden", "orb_euroc_752x480.npz"))
    img = synth.synth_image(int(g["seed"]), int(g["w"]), int(g["h"]))
    kw = dict(nfeatures=int(g["nfeatures"]), ini_th=int(g["ini"]), min_th=int(g["mn"]),
              lapping=tuple(int(v) for v in g["lapping"]))
    return img, kw


def test_contraction_modes(golden_image):
    import oracle
    img, kw = golden_image
    base = os.path.join(ROOT, "oracle", "liboracle.so")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle_fma.so"])
    try:
        oracle.use_library(base)
        oracle.set_contract(0)
        m0, k0, d0 = oracle.orb_extract(img, **kw)
        oracle.set_contract(1)
        m1, k1, d1 = oracle.orb_extract(img, **kw)
        oracle.set_contract(0)
        assert m0 == m1 and np.array_equal(k0.view(np.uint32), k1.view(np.uint32)) and np.array_equal(d0, d1)
        oracle.use_library(os.path.join(ROOT, "oracle", "liboracle_fma.so"))
        m2, k2, d2 = oracle.orb_extract(img, **kw)
    finally:
        oracle.use_library(base)
        oracle.set_contract(0)
    assert m0 == m2 and len(k0) == len(k2) and np.array_equal(d0, d2)
    for f in ("x", "y", "size", "response", "octave"):
        assert np.array_equal(k0[f].view(np.uint32), k2[f].view(np.uint32)), f
    ulp = np.abs(k0["angle"].view(np.int32).astype(np.int64) - k2["angle"].view(np.int32).astype(np.int64))
    assert ulp.max() <= 2
    assert 0 < np.count_nonzero(ulp) < 0.1 * len(ulp)   # the fused fastAtan2 polynomial moves a few percent
