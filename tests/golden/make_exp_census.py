"""Generates tests/golden/exp_census.json: the math.Exp census of the FGD path.

The reference's FGD score is int64(sigmoid((cur-new)/1000)*100) (fgd_score.go:123,144,
plugin_utils.go:76-78), and sigmoid calls Go's math.Exp.  The product (and the oracle) restate Go's
portable exp algorithm; the reference binary may have used Go's amd64 assembly routine, which is not
in the container.  For every FGD experiment of the paper sweep (17 traces x seeds 42-51, tune 1.3,
the reference's own event streams) this script replays the oracle and records:
  - every score delta the path evaluates (Score of every node + Reserve's selector), its closest
    approach to a step of the score function, how many come within 1e-10 of a step;
  - of those, how many get a different score from a correctly rounded exp (x87 expl rounded to double):
    `crdiff`, and how many would change score if exp's result moved by one ulp: `sensitive` (with the
    largest |delta| among them);
  - whether the whole decision stream (node, GPUs, score, feasible count, status per event) is the
    same when the oracle's exp is replaced by the correctly rounded one: `same_decisions_cr`.
For two default-trace seeds it also replays with every exp result moved by +1 / -1 ulp (a worst case
no accurate exp implementation exhibits: exp(0) = 1 exactly) and records how many decisions change.
Run: python tests/golden/make_exp_census.py [--threads N] (about 30 min on 8 cores).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import helpers  # noqa: E402
import ksim  # noqa: E402
import ksim.sweep as SW  # noqa: E402
import pyoracle as O  # noqa: E402

PREFIX = 1500  # the bounded sample tests/test_exp_census.py re-runs (default trace, seed 42)


def one(trace, seed, threads, limit=None, nudges=()):
    rp = trace.replay(seed=seed, tune_ratio=1.3, shuffle=True)
    args = (helpers.oracle_nodes(trace, rp), helpers.oracle_typical(trace), helpers.oracle_events(trace, rp, limit))
    O.census_begin()
    base, _, _ = O.run_events(*args, threads=threads)
    c = O.census_end()
    O.set_exp_mode(1)
    cr, _, _ = O.run_events(*args, threads=threads)
    O.set_exp_mode(0)
    c["events"] = len(base)
    c["same_decisions_cr"] = cr == base
    for j in nudges:
        O.set_exp_nudge(j)
        nj, _, _ = O.run_events(*args, threads=threads)
        O.set_exp_nudge(0)
        c["decisions_changed_nudge%+d" % j] = sum(1 for a, b in zip(nj, base) if a != b)
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--out", default=os.path.join(HERE, "exp_census.json"))
    args = ap.parse_args()
    th = O.score_thresholds()
    out = {"thresholds": th[1:101], "near": 1e-10, "experiments": {}}
    t0 = time.time()
    default = ksim.Trace.openb("default")
    out["prefix"] = one(default, 42, args.threads, limit=PREFIX)
    for tname in SW.TRACES:
        t = ksim.Trace.openb(tname[len("openb_pod_list_"):])
        for seed in SW.SEEDS:
            nud = (1, -1) if tname == "openb_pod_list_default" and seed in (42, 43) else ()
            c = one(t, seed, args.threads, nudges=nud)
            out["experiments"]["%s/06-FGD/%d" % (tname, seed)] = c
            print("%-30s %d: %d deltas, min dist %.3g, near %d, crdiff %d, sensitive %d (max |delta| %.3g), "
                  "same decisions %s %s [%.0f s]" % (tname, seed, c["deltas"], c["min_dist"], c["near"], c["crdiff"],
                                                   c["sensitive"], c["sensitive_max_abs_delta"], c["same_decisions_cr"],
                                                   {k: v for k, v in c.items() if k.startswith("decisions_changed")},
                                                   time.time() - t0), flush=True)
    ex = out["experiments"].values()
    out["summary"] = {
        "experiments": len(out["experiments"]),
        "deltas": sum(c["deltas"] for c in ex),
        "near": sum(c["near"] for c in ex),
        "crdiff": sum(c["crdiff"] for c in ex),
        "sensitive": sum(c["sensitive"] for c in ex),
        "sensitive_max_abs_delta": max(c["sensitive_max_abs_delta"] for c in ex),
        "all_same_decisions_cr": all(c["same_decisions_cr"] for c in ex),
        "min_dist_nonsensitive_note": "deltas farther than 1e-10 from every step keep their score under any "
                                      "exp within 400 ulps",
    }
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["summary"], indent=1))


if __name__ == "__main__":
    main()
