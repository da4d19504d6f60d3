"""One batch of each BoW / initialisation search (for rocprofv3 kernel traces): python tools/bow_once.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("OMV_LIB"):   # an instrumented variant of the library (e.g. -DOMV_BOW_PROFILE)
    from openmavis_amd import _lib  # noqa: E402
    _lib.load(os.environ["OMV_LIB"])
import bench  # noqa: E402

out = bench.aux_legs(torch.device("cuda", 0), False)
for k in ("search_by_bow", "search_by_bow_kf_kf", "search_for_initialization"):
    print(k, out[k]["ms_per_batch"])
