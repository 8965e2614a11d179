"""The paper's experiments against the reference's own end-to-end results.

experiments/analysis/expected_results/analysis_{allo,frag}_discrete.csv hold the reference's
curves for 17 traces x 6 policies x seeds 42-51 (tune 1.3).  A seed's event stream and node
names come from the restated Go math/rand (csrc/go_rand.hpp), so every experiment is compared
ROW FOR ROW: our 131-point allocation and fragmentation curves against the reference's row for
the same (trace, policy, seed).  Random is the exception (the reference draws it over a
goroutine-timing-dependent order): it is compared on its 10-seed mean.
Every test needs a gfx950 device.
"""
import os

import pytest

import ksim.sweep as SW

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ALLO = os.path.join(HERE, "golden", "expected_results", "analysis_allo_discrete.csv")
FRAG = os.path.join(HERE, "golden", "expected_results", "analysis_frag_discrete.csv")
# full precision (merge_frag_ratio_discrete.py:77-88): per arrived-GPU %, the mean of every event's
# 2-decimal "Frag ratio"; compared at north_star's 1e-9 relative curve tolerance
FRAG_RATIO = os.path.join(HERE, "golden", "expected_results", "analysis_frag_ratio_discrete.csv")
RATIO_TOL = 1e-9
POINTS = [20, 40, 60, 80, 90, 100, 110, 120, 130]


@pytest.fixture(scope="module")
def default_sweep():
    # the cheap-policy groups with their node records in LDS (KSIM_VARIANT=scan1=1); the full sweep below runs
    # the default placement (records in VGPRs), so both k_scan1 placements meet the reference's rows
    os.environ["KSIM_VARIANT"] = "scan1=1"
    try:
        sw = SW.Sweep(SW.plan(traces=["openb_pod_list_default"]))
    finally:
        del os.environ["KSIM_VARIANT"]
    dev_ms, wall = sw.run()
    curves = sw.curves()
    sw.close()
    return curves, dev_ms


def table(curves, trace):
    rows = []
    for p in SW.POLICY_DIRS:
        ours = SW.mean_curve(curves, trace, p, "alloc")
        ref = SW.expected_mean_curve(ALLO, trace, p)
        fo = SW.mean_curve(curves, trace, p, "frag")
        fr = SW.expected_mean_curve(FRAG, trace, p)
        rows.append((p, ours, ref, fo, fr))
    return rows


def test_default_trace_all_policies_vs_expected_results(default_sweep):
    curves, dev_ms = default_sweep
    rows = table(curves, "openb_pod_list_default")
    for p, ours, ref, fo, fr in rows:
        print("%-17s alloc ours/ref " % p + " ".join("%d:%.2f/%.2f" % (k, ours[k], ref[k]) for k in POINTS))
        print("%-17s frag  ours/ref " % p + " ".join("%d:%.2f/%.2f" % (k, fo[k], fr[k]) for k in POINTS))
    print("60 experiments replayed in %.1f ms of device time" % dev_ms)
    for p, ours, ref, fo, fr in rows:
        for k in POINTS:
            # seed-to-seed spread of the reference at 100-130% is 0.3-1.2 points; means of 10 seeds
            # (measured: within 0.1 point of the reference at every point, for every policy)
            assert abs(ours[k] - ref[k]) <= 0.3, (p, k, ours[k], ref[k])
            assert abs(fo[k] - fr[k]) <= 0.3, (p, "frag", k, fo[k], fr[k])
    at130 = {p: ours[130] for p, ours, _, _, _ in rows}
    assert max(at130, key=at130.get) == "06-FGD" and min(at130, key=at130.get) == "01-Random"


def test_default_trace_rows_identical_to_expected_results(default_sweep):
    curves, _ = default_sweep
    for kind, csv in (("alloc", ALLO), ("frag", FRAG)):
        mm = SW.row_mismatches(curves, kind, SW.expected_rows(csv))
        assert len(mm) == 60
        bad = {k: v for k, v in mm.items() if v and k[1] != "01-Random"}
        assert not bad, (kind, sorted(bad.items())[:5])
    ratio_rows = ratio_deviations(curves)
    assert len(ratio_rows) == 50
    assert max(ratio_rows.values()) <= RATIO_TOL, sorted(ratio_rows.items(), key=lambda kv: -kv[1])[:3]


def ratio_deviations(curves):
    """Per deterministic experiment, the largest relative deviation of our fragmentation-ratio curve
    from the reference's full-precision row (inf when the arrived-% points differ)."""
    exp = SW.expected_rows(FRAG_RATIO)
    return {k: SW.max_rel_dev(c["frag_ratio"], exp[k]) for k, c in curves.items()
            if k[1] != "01-Random" and k in exp}


def test_full_paper_sweep_vs_expected_results():
    # C4: all 1020 experiments (17 traces x 6 policies x 10 seeds) as replicas of one engine;
    # every (trace, policy) 10-seed mean curve near the reference's, at every arrived-GPU %.
    # The cheap-policy groups run on k_scan1 (one workgroup per replica, node records in VGPRs: the
    # default; the LDS placement is covered by the default-trace sweep above).
    sw = SW.Sweep(SW.plan())
    dev_ms, wall = sw.run()
    curves = sw.curves()
    # the cheap group (850 replicas, more than the CUs beside the FGD group hold at once) reports replica by replica
    # through k_report_overlap's queue, each of its workgroups taking several replicas
    n_ovl = sw.eng.last_run_report_overlap()
    sw.close()
    assert n_ovl == 850, n_ovl
    worst = {}
    for t in SW.TRACES:
        for p in SW.POLICY_DIRS:
            for kind, csv in (("alloc", ALLO), ("frag", FRAG)):
                ours, ref = SW.mean_curve(curves, t, p, kind), SW.expected_mean_curve(csv, t, p)
                keys = [k for k in ours if k in ref]
                assert len(keys) >= 125, (t, p, kind)
                worst[(t, p, kind)] = max(abs(ours[k] - ref[k]) for k in keys)
    print("1020 experiments: %.0f ms device time; worst deviations:" % dev_ms,
          sorted(worst.items(), key=lambda kv: -kv[1])[:5])
    det = {}
    for kind, csv in (("alloc", ALLO), ("frag", FRAG)):
        mm = SW.row_mismatches(curves, kind, SW.expected_rows(csv))
        det[kind] = {k: v for k, v in mm.items() if k[1] != "01-Random"}
        same = sum(1 for v in det[kind].values() if not v)
        print("%s: %d of %d deterministic rows identical to expected_results" % (kind, same, len(det[kind])))
        print("  differing:", sorted((k, v[:4]) for k, v in det[kind].items() if v)[:10])
    # measured (profiles/r01/sweep_compare.json): worst 0.85 (Random, itself not reproducible in the
    # reference), <= 0.62 for every other policy; the reference's own seed spread is up to ~1.2
    for (t, p, kind), dev in worst.items():
        assert dev <= (1.5 if p == "01-Random" else 1.0), (t, p, kind, dev)
    for kind in det:
        assert len(det[kind]) == 850
        assert all(not v for v in det[kind].values()), kind
    # every deterministic row's 131 full-precision fragmentation-ratio points (measured: <= 2.2e-16,
    # i.e. the reference's and our means of the same 2-decimal values differ by at most an ulp of
    # summation order)
    ratio_rows = ratio_deviations(curves)
    assert len(ratio_rows) == 850
    worst_ratio = max(ratio_rows.values())
    print("frag_ratio: 850 rows x 131 points, worst relative deviation %.3g" % worst_ratio)
    assert worst_ratio <= RATIO_TOL, sorted(ratio_rows.items(), key=lambda kv: -kv[1])[:3]


def test_sweep_with_pwr_runs():
    # the fork's PWR experiments (generate_run_scripts.py:31-42) next to FGD in one sweep: two
    # engines (persistent kernels / per-pod PWR path); FGD stays row-identical to the reference
    pols = ("06-FGD",) + tuple(SW.PWR_POLICY_DIRS)
    sw = SW.Sweep(SW.plan(traces=["openb_pod_list_default"], policies=pols, seeds=[42, 43]))
    assert len(sw.groups) == 2
    dev_ms, _ = sw.run()
    curves = sw.curves()
    sw.close()
    assert len(curves) == 10
    for (t, p, s), c in curves.items():
        assert len(c["alloc"]) == 131 and len(c["frag"]) == 131, (p, s)
        assert c["alloc"][130] > 85.0, (p, s, c["alloc"][130])
    for kind, csv in (("alloc", ALLO), ("frag", FRAG)):
        mm = SW.row_mismatches({k: v for k, v in curves.items() if k[1] == "06-FGD"}, kind, SW.expected_rows(csv))
        assert len(mm) == 2 and not any(mm.values())
    print("PWR sweep: %.0f ms device time; alloc at 130%%:" % dev_ms,
          {(p, s): c["alloc"][130] for (t, p, s), c in sorted(curves.items())})


def test_sweep_fgd_batches_rows_identical():
    # --fgd-batch: the FGD experiments as separate engines of `fgd_batch` replicas (k_memo where they fit);
    # rows identical to expected_results, one engine per batch
    sw = SW.Sweep(SW.plan(traces=["openb_pod_list_default"], policies=("06-FGD", "05-BestFit")), fgd_batch=3)
    assert len(sw.groups) == 1 + 4  # BestFit; FGD seeds in batches of 3, 3, 3, 1
    sw.run()
    curves = sw.curves()
    sw.close()
    for kind, csv in (("alloc", ALLO), ("frag", FRAG)):
        mm = SW.row_mismatches(curves, kind, SW.expected_rows(csv))
        assert len(mm) == 20 and not any(mm.values()), kind


def test_default_sweep_fgd_group_is_memoised():
    # the FGD group of a sweep (10 replicas here, next to 50 others) replays memoised, not k_replay
    sw = SW.Sweep(SW.plan(traces=["openb_pod_list_default"]))
    sw.run()
    path = sw.eng.last_run_path()
    sw.close()
    assert path == "memo+k_replay", path


@pytest.mark.parametrize("widths", [(16, 16), (12, 12), (24, 32), (32, 12)], ids=lambda w: "%d-%d" % w)
def test_share_with_widened_fgd_rows_identical(widths):
    # round-5 verdict item 1: an N-GPU share's longest FGD replays on k_memo, each at its own width (SW.WIDE_KS; the
    # gpuspec traces' keys in HBM, the untyped ones' in LDS) beside the one-workgroup FGD replicas (k_hmemo) and the
    # cheap policies' k_scan1_mix, all concurrently: three launches, each gated before the next, every row still
    # identical to expected_results
    assert set(widths) <= set(SW.WIDE_KS)
    items = SW.plan(traces=["openb_pod_list_gpuspec33", "openb_pod_list_gpushare100", "openb_pod_list_default"],
                    seeds=[42, 43, 48])
    pick = {("openb_pod_list_gpuspec33", 42): widths[0], ("openb_pod_list_gpushare100", 48): widths[1]}
    wide = {i: pick[(e[0], e[2])] for i, e in enumerate(items) if e[1] == "06-FGD" and (e[0], e[2]) in pick}
    assert len(wide) == 2
    sw = SW.Sweep(items, wgs=1, wide=wide)
    sw.run()
    kernels, gate = sw.eng.last_run_kernels(), sw.eng.last_run_gate()
    launches, streams = sw.eng.last_run_launches()
    curves = sw.curves()
    sw.close()
    assert kernels == ["k_memo_hkeys", "k_hmemo", "k_scan1_mix"], kernels  # gpuspec33's classes: keys in HBM
    assert launches == 3 and streams == 2 and gate == (1, 0)  # k_memo on the engine stream, two side streams
    for kind, csv in (("alloc", ALLO), ("frag", FRAG)):
        mm = SW.row_mismatches({k: v for k, v in curves.items() if k[1] != "01-Random"}, kind, SW.expected_rows(csv))
        assert len(mm) == 45 and not any(mm.values()), kind
    ratio_rows = ratio_deviations({k: v for k, v in curves.items() if k[1] != "01-Random"})
    assert len(ratio_rows) == 45 and max(ratio_rows.values()) <= RATIO_TOL


@pytest.mark.parametrize("overlap", ["1", "0"], ids=["overlapped", "after"])
def test_overlapped_report_rows_identical(overlap, monkeypatch):
    # the cheap group's cluster report replica by replica as each replay ends (k_report_overlap, behind the FGD
    # group on its stream; forced here, on the full sweep it runs when the cheap group outnumbers the free CUs) and
    # after the whole group (KSIM_VARIANT report_overlap=0): every row identical to expected_results either way
    if overlap == "1":
        monkeypatch.setenv("KSIM_TEST", "report_overlap=1")
    else:
        monkeypatch.setenv("KSIM_VARIANT", "report_overlap=0")
    sw = SW.Sweep(SW.plan(traces=["openb_pod_list_default", "openb_pod_list_gpushare40"], seeds=[42, 44, 47]), wgs=1)
    for _ in range(2):  # the second run reuses the queue (its entries carry the run's epoch)
        sw.run()
        n_ovl = sw.eng.last_run_report_overlap()
        curves = sw.curves()
        assert n_ovl == (30 if overlap == "1" else 0), n_ovl
        for kind, csv in (("alloc", ALLO), ("frag", FRAG)):
            mm = SW.row_mismatches({k: v for k, v in curves.items() if k[1] != "01-Random"}, kind,
                                   SW.expected_rows(csv))
            assert len(mm) == 30 and not any(mm.values()), kind
        ratio_rows = ratio_deviations({k: v for k, v in curves.items() if k[1] != "01-Random"})
        assert len(ratio_rows) == 30 and max(ratio_rows.values()) <= RATIO_TOL
    sw.close()
