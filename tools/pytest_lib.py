"""Run pytest against another build of the library (an instrumented variant from
`python -m openmavis_amd.build variant NAME DEFINE...`), for debugging only:
    OMV_LIB=openmavis_amd/variants/libomv_NAME.so python tools/pytest_lib.py <pytest args>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from openmavis_amd import _lib  # noqa: E402

_lib.load(os.environ["OMV_LIB"])
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[1:]))
