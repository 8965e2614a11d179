"""bench.py's counter-backed rooflines: every bench configuration's profile is
committed under profiles/<round>/prof/<profile_key> (the newest round first), and bench.py picks it up
only for the kernel the run launched.  CPU only (reads the committed summaries)."""
import argparse
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _args(**kw):
    a = dict(config="c2", policy="FGD", run_mode=0, report=False, sharded=False)
    a.update(kw)
    return argparse.Namespace(**a)


def test_profile_keys():
    import bench
    assert bench.profile_key(_args()) == "c2"
    assert bench.profile_key(_args(run_mode=5)) == "c2-rm5"
    assert bench.profile_key(_args(policy="BestFit")) == "c2-BestFit"
    assert bench.profile_key(_args(policy="PWR 500 FGD 500")) == "c2-PWR_500_FGD_500"
    assert bench.profile_key(_args(config="c4", report=True)) == "c4"
    assert bench.profile_key(_args(config="c5", sharded=True)) == "c5-sharded"


def test_rank_share_lines_do_not_borrow_the_whole_sweep_profile():
    # a --rank-share line times one share's launches: the whole C4 profile's traffic is not its traffic
    import bench
    ns = _args(config="c4", report=True, rank_share="3/8")
    assert bench.profile_key(ns) == "c4-share3of8"
    assert bench.profile_rooflines(ns, ["k_hmemo", "k_scan1_mix"]) == (None, None, None)


@pytest.mark.parametrize("key,path", [("c2", ["k_memo"]), ("c4", ["k_hmemo", "k_scan1_mix"]), ("c5", ["k_hmemo_wide"]),
                                      ("c2-rm5", ["k_hmemo"]), ("c2-BestFit", ["k_replay"]), ("c2-DotProd", ["k_replay"]),
                                      ("c2-PWR", ["k_replay"]), ("c2-PWR_500_FGD_500", ["k_replay"])])
def test_committed_profiles_feed_the_bench_line(key, path):
    import bench
    pf = bench.profile_file(key)
    with open(pf) as f:
        dom = json.load(f)["dominant"]
    assert dom["hbm_bytes_per_dispatch"] > 0 and dom["mean_duration_ns"] > 0
    # the fp64 split of the VALU issue: both parts present and within the whole
    assert 0 <= dom["f64_share"] < 1 and 0 < dom["valu_frac"] < 1
    assert dom["f64_frac"] / 2 + dom["nonf64_frac"] >= dom["valu_frac"] * 0.999
    ns = _args()
    ns.config, rest = key.split("-")[0], key.split("-")[1:]
    for r in rest:
        if r.startswith("rm"):
            ns.run_mode = int(r[2:])
        else:
            ns.policy = r.replace("_", " ")
    assert bench.profile_key(ns) == key
    traffic, src, valu = bench.profile_rooflines(ns, path)
    assert traffic == dom["hbm_bytes_per_dispatch"] and src.endswith(key + "/pmc.json")
    assert valu["frac"] == dom["valu_frac"] and valu["f64_frac"] == dom["f64_frac"]
    # a run that launched another kernel does not borrow this profile
    assert bench.profile_rooflines(ns, ["k_step"]) == (None, None, None)
