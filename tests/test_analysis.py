"""ksim.analysis (cluster-report log lines -> curves) against the reference's own Python harness.

tests/golden/curve_golden.json holds what scripts/analysis.py + experiments/analysis/
merge_*_discrete.py produced on synthetic report logs (tests/golden/make_curve_golden.py);
here the same synthetic reports go through ksim.analysis and must give the same curves.
"""
import math
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "kubernetes-scheduler-simulator_amd"))

import json  # noqa: E402

import ksim.analysis as A  # noqa: E402
from make_curve_golden import synth_reports  # noqa: E402

with open(os.path.join(HERE, "golden", "curve_golden.json")) as f:
    GOLD = json.load(f)


@pytest.mark.parametrize("seed", GOLD["seeds"])
def test_curves_match_reference_harness(seed):
    reps = synth_reports(seed, GOLD["total_gpus"])
    want = GOLD["curves"][str(seed)]
    assert len(reps) == want["n_events"]
    got = A.curves(reps)
    assert {str(k): v for k, v in got["alloc"].items()} == want["alloc"]
    assert {str(k): v for k, v in got["frag"].items()} == want["frag"]
    fr = {str(k): v for k, v in got["frag_ratio"].items()}
    assert fr.keys() == want["frag_ratio"].keys()
    for k, v in want["frag_ratio"].items():  # unrounded mean, through the reference's CSV round trip
        assert math.isclose(fr[k], v, rel_tol=1e-12, abs_tol=1e-12), (k, fr[k], v)


def test_log_lines_parse_back(tmp_path):
    reps = synth_reports(GOLD["seeds"][0])[:50]
    p = tmp_path / "x.log"
    A.write_log(p, reps)
    frag, allo = A.parse_log(p)
    assert allo["arrived_gpu_milli"] == [r["arrived_gpu_milli"] for r in reps]
    assert allo["used_gpu_milli"] == [r["used_gpu_milli"] for r in reps]
    assert frag["origin_milli"] == [float("%.2f" % A.report_values(r)["frag_milli"]) for r in reps]


def test_report_messages_format():
    rep = dict(frag_bins=[1.0, 2.005, 1000.0, 3.0, 4.0, 5.0, 0.5], used_nodes=3, used_gpus=12, used_gpu_milli=4500,
               total_gpus=6212, arrived_gpu_milli=5000, used_cpu_milli=7000, arrived_cpu_milli=9000)
    m = A.report_messages(rep)
    v = A.report_values(rep)
    idle = 0.0
    for x in rep["frag_bins"]:
        idle += x
    assert v["idle_milli"] == idle
    assert m[0] == "[Report]; Frag amount: %.2f; Frag ratio: %.2f%%; Q124 ratio: %.2f%%; (origin)\n" % (
        v["frag_milli"], 100 * v["frag_milli"] / idle, 100 * (1.0 + 2.005 + 3.0) / idle)
    assert m[1] == "[Alloc]; Used nodes: 3; Used GPUs: 12; Used GPU Milli: 4500; Total GPUs: 6212; Arrived GPU Milli: 5000\n"
    assert m[2] == "[AllocCPU]; Used CPU Milli: 7000; Arrived CPU Milli: 9000\n"
    line = A.logrus_line(m[1])
    assert line.endswith('Arrived GPU Milli: 5000\\n"\n')
    empty = dict(rep, frag_bins=[0.0] * 7)
    assert "Frag ratio: NaN%" in A.report_messages(empty)[0]


def test_curves_arrays_fast_path_matches():
    # the vectorised sweep path equals the merge_*_discrete.py path up to a 0.01 rounding tie
    import numpy as np
    for seed in GOLD["seeds"]:
        reps = synth_reports(seed, GOLD["total_gpus"])
        arrs = {k: np.array([r[k] for r in reps]) for k in reps[0] if k != "frag_bins"}
        arrs["frag_bins"] = np.array([r["frag_bins"] for r in reps])
        fast = A.curves_arrays(arrs)
        want = GOLD["curves"][str(seed)]
        assert {str(k) for k in fast["alloc"]} == set(want["alloc"])
        for kind in ("alloc", "frag"):
            for k, v in fast[kind].items():
                assert abs(v - want[kind][str(k)]) <= 0.0100001, (kind, k, v, want[kind][str(k)])
        for k, v in fast["frag_ratio"].items():
            assert math.isclose(v, want["frag_ratio"][str(k)], rel_tol=1e-9)
