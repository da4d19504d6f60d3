"""Time LocalInertialBA optimize() on the config-5 window (for rocprofv3 runs): python tools/lba_time.py [runs]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("OMV_LIB"):   # e.g. a -DOMV_LDLT_PROFILE build of the library
    from openmavis_amd import _lib  # noqa: E402
    _lib.load(os.environ["OMV_LIB"])
from openmavis_amd import synth_ba  # noqa: E402
from openmavis_amd.optimizer import LocalInertialBA  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
prob = synth_ba.make_lba_problem()
ba = LocalInertialBA(max_kf=50, max_cams=5, max_pts=20000, max_mono=len(prob["mono_pt"]), max_imu=25)
ba.set_problem(prob)
for i in range(runs):
    ba.reset()
    t = time.time()
    r, s = ba.optimize(opt_it=4, lambda_init=1e-2, large=True, chi2=False)
    dt = time.time() - t
    print(json.dumps(dict(wall_ms=round(dt * 1e3, 3), err=r["err"], err_end=r["err_end"],
                          **{k: round(float(v), 4) for k, v in ba.stage_ms().items()})))
