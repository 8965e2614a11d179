"""Does a process that ran a ksim engine (libksim_hip -> /opt/rocm's HIP runtime) and then imported
torch (which carries its own HIP runtime) exit cleanly?  Prints the order and exits 0 if it gets to
the end; a crash in interpreter teardown shows as the exit status."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
order = sys.argv[1] if len(sys.argv) > 1 else "ksim-first"
if order == "torch-first":
    import torch  # noqa: F401
import ksim  # noqa: E402

t = ksim.Trace.openb("default")
rp = t.replay(seed=42)
arr, n = t.typical()
e = ksim.Engine(t.num_nodes, 1)
e.set_nodes(0, rp.nodes)
e.set_typical(0, arr, n)
e.set_policy(0, "BestFit")
e.load_events(0, rp.events, 200)
e.run()
if order == "ksim-first":
    import torch  # noqa: F401,E402
if len(sys.argv) > 2 and sys.argv[2] == "close":
    e.close()
print("reached the end:", order, flush=True)
