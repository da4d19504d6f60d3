"""Run bench.py against another build of the library (A/B of an instrumented or older variant):
    OMV_LIB=openmavis_amd/variants/libomv_NAME.so python tools/bench_lib.py <bench.py args>"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("OMV_LIB"):
    from openmavis_amd import _lib  # noqa: E402
    _lib.load(os.environ["OMV_LIB"])
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
