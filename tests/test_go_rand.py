"""Go math/rand restatement (csrc/go_rand.hpp) and the event streams it produces.

Pins, weakest to strongest:
  1. Go's published outputs after rand.Seed(1) (the default source of every Go program before
     1.20): Int63, Intn(100), Float64.  Each value depends on rngCooked, so these also pin the
     recomputed table (tools/gen_go_rng_cooked.c).
  2. The recomputed table equals the committed csrc/go_rng_cooked.inc.
  3. The event stream of every (trace, seed) of the paper sweep: while every pod fits, the
     reference's allocation curve depends only on the order and sizes of arriving pods, so the
     first 30 arrived-GPU % of each expected_results row (13 traces x 10 seeds x 5 deterministic
     policies) pin the rand.Int / Shuffle / tuning draws.  On the gpuspec traces a pod restricted
     to a scarce GPU model fails under every policy from the first 1-2 %, so their streams are
     pinned by a whole experiment (5) instead.
  4. One whole experiment through the oracle: the 131-point allocation and fragmentation rows
     of openb default / BestFit / seed 42, which also pin rand.Perm (node names decide every
     score tie, generic_scheduler.go:187-212) and the informer draws before it.
  5. The same for gpuspec10 / GpuPacking / seed 50 (model-constrained pods, early failures).
The GPU side of 4 is tests/test_gpu_sweep.py: all 850 deterministic experiments row for row.
"""
import os
import subprocess

import numpy as np
import pytest

import helpers
import ksim
import ksim.analysis as A
import ksim.sweep as SW

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "kubernetes-scheduler-simulator_amd")
ALLO = os.path.join(HERE, "golden", "expected_results", "analysis_allo_discrete.csv")
FRAG = os.path.join(HERE, "golden", "expected_results", "analysis_frag_discrete.csv")
FRAG_RATIO = os.path.join(HERE, "golden", "expected_results", "analysis_frag_ratio_discrete.csv")

# Go's documented outputs for the default seed 1 (math/rand before Go 1.20)
SEED1_INT63 = [5577006791947779410, 8674665223082153551, 6129484611666145821, 4037200794235010051,
               3916589616287113937, 6334824724549167320, 605394647632969758, 1443635317331776148,
               894385949183117216, 2775422040480279449]
SEED1_INTN100 = [81, 87, 47, 59, 81, 18, 25, 40, 56, 0]
SEED1_FLOAT64 = [0.6046602879796196, 0.9405090880450124, 0.6645600532184904]


def test_seed1_published_outputs():
    assert ksim.go_rand(1, ksim.GO_INT63, 10) == SEED1_INT63
    assert ksim.go_rand(1, ksim.GO_INTN, 10, 100) == SEED1_INTN100
    assert ksim.go_rand(1, ksim.GO_FLOAT64, 3) == SEED1_FLOAT64


def test_seed_normalisation():
    # rng.go Seed: seed %= 2^31-1, negative -> +2^31-1, 0 -> 89482311
    m = 2 ** 31 - 1
    assert ksim.go_rand(1 + m, ksim.GO_INT63, 5) == SEED1_INT63[:5]
    assert ksim.go_rand(0, ksim.GO_INT63, 5) == ksim.go_rand(89482311, ksim.GO_INT63, 5)
    assert ksim.go_rand(-5, ksim.GO_INT63, 5) == ksim.go_rand(m - 5, ksim.GO_INT63, 5)


def test_perm_shuffle_intn_properties():
    for seed in (42, 51, 233):
        p = ksim.go_rand(seed, ksim.GO_PERM, 1213, 1213)
        assert sorted(p) == list(range(1213))
        s = ksim.go_rand(seed, ksim.GO_SHUFFLE, 8152)
        assert sorted(s) == list(range(8152)) and s != list(range(8152))
        for n in (1, 2, 3, 64, 1000, 8152, 2 ** 31 - 1, 2 ** 31, 2 ** 40):
            v = ksim.go_rand(seed, ksim.GO_INTN, 50, n)
            assert all(0 <= x < n for x in v)
    # Intn(power of two) masks Int31 (rand.go Int31n), Intn(n > 2^31-1) goes through Int63n
    assert ksim.go_rand(1, ksim.GO_INTN, 10, 1 << 20) == [(x >> 32) & ((1 << 20) - 1) for x in SEED1_INT63]
    assert ksim.go_rand(1, ksim.GO_INTN, 10, 1 << 40) == [x & ((1 << 40) - 1) for x in SEED1_INT63]
    with pytest.raises(ksim.KsimError):
        ksim.go_rand(1, ksim.GO_INTN, 1, 0)


def test_cooked_table_regenerates(tmp_path):
    exe = str(tmp_path / "gen")
    subprocess.run(["gcc", "-O3", "-o", exe, os.path.join(PKG, "tools", "gen_go_rng_cooked.c")], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    with open(os.path.join(PKG, "csrc", "go_rng_cooked.inc")) as f:
        assert out == f.read()


@pytest.fixture(scope="module")
def expected_alloc():
    return SW.expected_rows(ALLO)


@pytest.mark.parametrize("trace", [t[len("openb_pod_list_"):] for t in SW.TRACES if "gpuspec" not in t])
def test_event_streams_match_expected_results(trace, expected_alloc):
    t = ksim.Trace.openb(trace)
    pods = t.pods()
    total = sum(n["gpu"] for n in t.nodes())
    for seed in SW.SEEDS:
        rp = t.replay(seed=seed, tune_ratio=1.3, shuffle=True)
        gpu = np.array([pods[rp.pod_index[k]]["milli"] * pods[rp.pod_index[k]]["num"] for k in range(rp.n)])
        arrived = np.cumsum(gpu)
        # every pod placed: used GPU milli == arrived GPU milli (merge_alloc_discrete.py:96-121)
        arrs = {"frag_bins": np.zeros((rp.n, 7)), "total_gpus": np.full(rp.n, total, dtype=np.int64),
                "arrived_gpu_milli": arrived, "used_gpu_milli": arrived}
        ours = A.curves_arrays(arrs)["alloc"]
        refs = [expected_alloc[("openb_pod_list_" + trace, p, seed)] for p in SW.POLICY_DIRS if p != "01-Random"]
        # points before any policy failed a pod: there all five reference rows agree
        pts = [a for a in range(31) if len({r.get(a) for r in refs}) == 1]
        assert len(pts) >= 20, (trace, seed, pts)
        bad = [a for a in pts if ours.get(a) != refs[0].get(a)]
        assert not bad, (trace, seed, bad[:5])


@pytest.mark.parametrize("trace,policy,seed", [("default", "05-BestFit", 42), ("gpuspec10", "04-GpuPacking", 50)])
def test_whole_experiment_row_identical_via_oracle(trace, policy, seed):
    import pyoracle as O
    pol = {"05-BestFit": O.POL_BESTFIT, "04-GpuPacking": O.POL_PACKING}[policy]
    t = ksim.Trace.openb(trace)
    rp = t.replay(seed=seed, tune_ratio=1.3, shuffle=True)
    _, _, reps = O.run_events(helpers.oracle_nodes(t, rp), helpers.oracle_typical(t), helpers.oracle_events(t, rp),
                              policy=pol, gpu_sel=O.SEL_BEST, threads=min(8, os.cpu_count() or 1),
                              with_report=True)
    cv = A.curves(reps)
    key = ("openb_pod_list_" + trace, policy, seed)
    for kind, csv in (("alloc", ALLO), ("frag", FRAG)):
        ref = SW.expected_rows(csv)[key]
        assert len(ref) == 131
        assert cv[kind] == ref, (kind, [a for a in ref if cv[kind].get(a) != ref[a]][:5])
    # the full-precision fragmentation-ratio row (merge_frag_ratio_discrete.py:77-88: the mean of every
    # event's 2-decimal "Frag ratio" in an arrived-% bin): north_star's 1e-9 relative curve contract
    ref = SW.expected_rows(FRAG_RATIO)[key]
    assert len(ref) == 131 and set(cv["frag_ratio"]) == set(ref)
    assert SW.max_rel_dev(cv["frag_ratio"], ref) <= 1e-9


def test_informer_draws_are_what_pins_the_node_names():
    # node names (rand.Perm) move with the number of draws before it; the event stream does not
    t = ksim.Trace.openb("default")
    a, b = t.replay(seed=42), t.replay(seed=42, informer_draws=0)
    assert a.n == b.n and list(a.pod_index[:a.n]) == list(b.pod_index[:b.n])
    assert list(a.prefix) != list(b.prefix)
    assert list(t.replay(seed=42, informer_draws=10).prefix) == list(a.prefix)


def test_oracle_go_source_published_outputs():
    # the oracle's own restatement of the source (fgd_oracle.c orc_go_*), which checks the Random
    # draw structure on the device: Go's seed-1 outputs, Int63 and Intn(100) (= Int31n)
    import pyoracle as O
    g = O.go_seed(1)
    assert [v & ((1 << 63) - 1) for v in O.go_uint64(g, 10)] == SEED1_INT63
    g = O.go_seed(1)
    assert [O.go_int31n(g, 100) for _ in range(10)] == SEED1_INTN100
    g = O.go_seed(1)
    assert [O.go_int31n(g, 1 << 20) for _ in range(10)] == [(x >> 32) & ((1 << 20) - 1) for x in SEED1_INT63]


@pytest.mark.parametrize("trace,seed,tune", [("default", 42, 1.3), ("multigpu50", 51, 1.3), ("default", 7, 0.0)])
def test_replay_go_state_is_seed_plus_the_replays_draws(trace, seed, tune):
    # ksim_trace_replay_go_state (the stream the first scheduling cycle finds) == rand.Seed(seed)
    # advanced by exactly the replay's draw count, by the oracle's restatement
    import pyoracle as O
    t = ksim.Trace.openb(trace)
    vec, tap, feed, draws = t.go_state(seed=seed, tune_ratio=tune)
    assert draws > 1000  # rand.Int, the shuffle, the tuning draws, the informers' and rand.Perm
    g = O.go_seed(seed)
    O.go_uint64(g, draws)
    assert (list(g.vec), g.tap, g.feed) == (vec, tap, feed)
