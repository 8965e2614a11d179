"""How often does a PWR + FGD cycle's raw PWR min / max repeat?  (CPU, the oracle's diagnostics hook.)

Runs the oracle on the openb default trace under "PWR 500 FGD 500" and records every scored cycle's raw PWR
(lo, hi).  Prints the hit rate of three predictors a speculative NormalizeScore range could use: the previous
scored cycle's range, the previous range of the same pod class, and the same class's range with hi alone.
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import helpers  # noqa: E402
import ksim  # noqa: E402
import pyoracle as O  # noqa: E402


def main(seed=0, n_ev=None):
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=seed)
    n = n_ev or rp.n
    buf = (C.c_int64 * (2 * n))(*([1, 0] * n))
    L = O.lib()
    L.orc_pwr_lohi_trace.argtypes = [C.c_void_p, C.c_int]
    L.orc_pwr_lohi_trace(C.cast(buf, C.c_void_p), n)
    os.environ["KSIM_ORACLE_CACHE"] = "0"
    evs = helpers.oracle_events(t, rp, n)
    O.run_events(helpers.oracle_nodes(t, rp), helpers.oracle_typical(t), evs, policy=O.POL_PWR_FGD,
                 gpu_sel=O.SEL_FGD, threads=8, w_pwr=500, w_fgd=500)
    L.orc_pwr_lohi_trace(None, 0)
    last, by_cls = None, {}
    tot = h_last = h_cls = h_cls_hi = 0
    for s in range(n):
        lo, hi = buf[2 * s], buf[2 * s + 1]
        if lo > hi:
            continue  # no normalisation this cycle (0 or 1 feasible node)
        e = evs[s]
        cls = (e["cpu"], e["mem"], e["milli"], e["num"], e["type"])
        tot += 1
        h_last += last == (lo, hi)
        h_cls += by_cls.get(cls) == (lo, hi)
        h_cls_hi += by_cls.get(cls, (None, None))[1] == hi
        last = (lo, hi)
        by_cls[cls] = (lo, hi)
    print("seed %d: %d scored cycles, %d classes; hit rate: previous cycle %.3f, previous of the class %.3f "
          "(hi alone %.3f)" % (seed, tot, len(by_cls), h_last / tot, h_cls / tot, h_cls_hi / tot))
    # the M most recent distinct ranges of the class (k_replay<PWR+FGD> keys two), or of any class
    for M in (1, 2, 3, 4):
        hist, glob, hit, hit_any = {}, [], 0, 0
        for s in range(n):
            lo, hi = buf[2 * s], buf[2 * s + 1]
            if lo > hi:
                continue
            e = evs[s]
            h = hist.setdefault((e["cpu"], e["mem"], e["milli"], e["num"], e["type"]), [])
            hit += (lo, hi) in h
            hit_any += (lo, hi) in glob
            for lst in (h, glob):
                if (lo, hi) in lst:
                    lst.remove((lo, hi))
                lst.insert(0, (lo, hi))
                del lst[M:]
        print("M %d class-recent hit %.4f global-recent hit %.4f" % (M, hit / tot, hit_any / tot))


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
