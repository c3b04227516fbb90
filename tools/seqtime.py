import sys, time, os
sys.path.insert(0, os.getcwd())
import numpy as np
import aicp_mapping_amd._lib as L
from aicp_mapping_amd import synthetic as sy
st = sy.make_stream(n_readings=64, n_points=120000, seed=1)
ctx = L.Context(0)
tn = os.environ.get('SEQ_TIMENN', '0') == '1'
prm = L.default_sequence_params(flags=L.AICP_RUN_OVERLAP | (L.AICP_RUN_TIME_NN if tn else 0))
for k in range(6):
    t = time.perf_counter()
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    dt = time.perf_counter() - t
    tm = ctx.last_sequence_timing(); nn = ctx.last_nn_timing()
    print(f"run {k}: {dt*1e3:.1f} ms wall, {64/dt:.0f} clouds/s; timing {tm}; nn {nn['launches']} launches {nn['total_ms']:.2f} ms, mean iters {np.mean([o['icp']['iterations'] for o in out]):.2f}", flush=True)
