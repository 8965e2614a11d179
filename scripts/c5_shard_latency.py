"""Per-pod latency of the node-sharded C5 cluster as an in-process shard group:
the 100k-node C5 cluster, the first N events, world = 1 (unsharded k_replay), 2 and 8 shards on one
device.  Checks the merged decisions equal the unsharded run's and prints one JSON object.
Usage (GPU box): python3 scripts/c5_shard_latency.py [--events 5000] [--worlds 2 8]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))

import ksim  # noqa: E402
import ksim.shard as SH  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=5000)
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 8])
    a = ap.parse_args()
    t = ksim.Trace.openb("default").synthetic(100_000, 1_000_000, seed=0)
    rp = t.replay(seed=1, tune_ratio=0.0, shuffle=False)
    arr, n = t.typical()
    e = ksim.Engine(t.num_nodes, 1, run_mode=2)
    e.set_nodes(0, rp.nodes)
    e.set_typical(0, arr, n)
    e.set_policy(0, "FGD")
    e.load_events(0, rp.events, a.events)
    e.run()
    ms1 = e.run()
    want = e.results(0)
    out = {"events": a.events, "nodes": t.num_nodes, "unsharded": {"kernel": e.last_run_path(),
           "wgs": e.last_run_wgs(), "device_ms": ms1, "us_per_pod": ms1 * 1e3 / a.events}, "groups": []}
    e.close()
    for w in a.worlds:
        for mode in ("hmemo", "step"):
            # hmemo: one k_hmemo launch over every shard's slices, one granule exchange per pod (the default);
            # step: KSIM_VARIANT=shard_hmemo=0, the per-pod k_step + gather + commit launches (round 2's path)
            os.environ["KSIM_VARIANT"] = "shard_hmemo=%d" % (mode == "hmemo")
            g = SH.ShardGroup(rp.nodes, (arr, n), w)
            g.load_events(rp.events, a.events)
            g.run()
            t0 = time.perf_counter()
            ms = g.run()
            wall = time.perf_counter() - t0
            same = g.results() == want
            wgs = g.engines[0].last_run_wgs()
            g.close()
            out["groups"].append({"world": w, "mode": mode, "wgs_per_shard": wgs, "device_ms": ms,
                                  "us_per_pod": ms * 1e3 / a.events, "wall_us_per_pod": wall * 1e6 / a.events,
                                  "results_equal_unsharded": same})
            print("world %d %s: %.2f us/pod, equal %s" % (w, mode, ms * 1e3 / a.events, same), file=sys.stderr,
                  flush=True)
    os.environ.pop("KSIM_VARIANT", None)
    out["note"] = ("in-process shard group on one device. hmemo: every shard's k_hmemo slices in one launch, the "
                   "pod step's slice maxima exchanged as world x K granules (no host, no collective per pod); "
                   "step: per pod every shard's Filter+Score (k_step mode 2), a gather kernel and the commit. The "
                   "cross-process exchange (one process per GPU) stays unmeasured on a 1-GPU lease")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
