"""Host-output table pass on cfg5 (the drop-in's first-query shape, experiments only):
wall time of Engine.compute into fresh host arrays with and without registering
them for the D2H (SHDR_HOST_REGISTER), against the pass's own kernel time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shadow_amd.routes import SHDR_TIMING, Engine  # noqa: E402

g, hosts, _, _ = bench.make_workload(sys.argv[1] if len(sys.argv) > 1 else "cfg5")
eng = Engine(g)
eng.compute(hosts[:64], hosts)  # warm: landmarks, arena
for reg in ("1", "0", "1"):
    os.environ["SHDR_HOST_REGISTER"] = reg
    t0 = time.perf_counter()
    t = eng.compute(hosts, hosts, flags=SHDR_TIMING)
    wall = time.perf_counter() - t0
    print(f"register={reg}: wall {wall:.2f} s, pass {eng.timing()['routes_pass'] / 1e3:.2f} s", flush=True)
    del t
