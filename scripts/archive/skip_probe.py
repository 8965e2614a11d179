"""Dead-class skip probe: k_memo (lean) on C2 seed 42 -- the whole stream against its prefix before the
first failure; with the skip, the tail's repeated failures cost little."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-scheduler-simulator_amd")]
import ksim
t = ksim.Trace.openb("default")
rp = t.replay(seed=42, tune_ratio=1.3, shuffle=True)
arr, n = t.typical()
for n_ev in (7885, 9000, 10000, rp.n):
    eng = ksim.Engine(t.num_nodes, 1, run_mode=3)
    eng.set_nodes(0, rp.nodes)
    eng.set_typical(0, arr, n)
    eng.set_policy(0, "FGD")
    eng.load_events(0, rp.events, n_ev)
    best = min(eng.run() for _ in range(3))
    res = eng.results(0)
    print("events %5d  ms %.3f  us/event %.3f  failed %d  path %s" % (n_ev, best, best * 1000 / n_ev,
          sum(1 for r in res if r[0] < 0), eng.last_run_path()), flush=True)
    eng.close()
