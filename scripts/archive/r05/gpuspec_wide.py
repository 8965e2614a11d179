"""One long FGD replay (gpuspec33, seed 42: the N-GPU C4 floor) on k_hmemo at 1, 2, 4 and 8 workgroups per
replica (run_mode 5; K > 1 is the wide form): ms per replay, and every K's decisions equal to K = 1's."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd")]
import ksim  # noqa: E402


def main(name="gpuspec33", seed=42, reps=3):
    t = ksim.Trace.openb(name)
    rp = t.replay(seed=seed)
    arr, n = t.typical()
    base = None
    for wgs in (1, 2, 4, 8):
        eng = ksim.Engine(t.num_nodes, 1, run_mode=5, wgs_per_replica=wgs)
        eng.set_nodes(0, rp.nodes)
        eng.set_typical(0, arr, n)
        eng.set_policy(0, "FGD")
        eng.load_events(0, rp.events, rp.n)
        eng.run()
        res = eng.results(0)
        ts = []
        for _ in range(reps):
            eng.set_nodes(0, rp.nodes)
            t0 = time.perf_counter()
            eng.run()
            ts.append((time.perf_counter() - t0) * 1e3)
        same = base is None or res == base
        base = base or res
        print("%s seed %d wgs %d (ran %d, path %s): %.2f ms (min of %d), decisions %s" % (
            name, seed, wgs, eng.last_run_wgs(), eng.last_run_path(), min(ts), reps,
            "= K 1" if same else "DIFFER"), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
