import os, sys
sys.path[:0] = ["kubernetes-scheduler-simulator_amd", "oracle", "tests"]
import ksim, ksim.shard as SH, pyoracle as O
from fuzz_cases import make_case
case = make_case(3, 250, 1200, 0.1)
want, _, _ = O.run_events(case["onodes"], case["otypical"], case["oevents"], policy=O.POL_FGD, gpu_sel=O.SEL_FGD, seed=5, threads=16)
for world in (2,):
    g = SH.ShardGroup(case["nodes"], (case["typical"], case["typical_n"]), world, policy="FGD", seed=5)
    g.load_events(case["events"], case["n_events"])
    g.run()
    per = [e.results(0) for e in g.engines]
    got = SH.merge_results(per, g.parts)
    print("K", g.engines[0].last_run_wgs(), "parts", [(p[0], len(p[2])) for p in g.parts])
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    print("bad", bad[:10], len(bad))
    ev = case["events"]
    for i in bad[:3]:
        ref = ev[i].ref
        print("event", i, "delete", ev[i].is_delete, "ref", ref, "want", want[i], "got", got[i])
        for k in range(world):
            print("  shard", k, "rec", per[k][i], "creation rec", per[k][ref])
        print("  want creation", want[ref], "got creation", got[ref])
    g.close()
