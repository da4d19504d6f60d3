import time, json, numpy as np
from openmavis_amd import synth_ba
from openmavis_amd.optimizer import LocalInertialBA
prob = synth_ba.make_lba_problem()
ba = LocalInertialBA(max_kf=50, max_cams=5, max_pts=20000, max_mono=len(prob["mono_pt"]), max_imu=25)
ba.set_problem(prob)
for i in range(3):
    t = time.time(); r, s = ba.optimize(opt_it=4, lambda_init=1e-2, large=True); dt = time.time() - t
    print(json.dumps(dict(wall_ms=dt * 1e3, trials=r["trials"], err=r["err"], err_end=r["err_end"], **ba.stage_ms())))
