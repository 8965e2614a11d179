"""Host-side replay driver (C++): trace loading, GetTypicalPods, event order, tuning, node naming."""
import csv
import os
from collections import Counter

import pytest

import helpers
import ksim

TRACES = ["default", "cpu050", "cpu100", "cpu200", "cpu250", "gpushare40", "gpushare60", "gpushare80",
          "gpushare100", "gpuspec10", "gpuspec20", "gpuspec25", "gpuspec33", "multigpu20", "multigpu30",
          "multigpu40", "multigpu50"]


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


def test_openb_node_stats(default_trace):
    # SURVEY §8 (derived from data/csv): 1213 nodes, GPUs per node {8:617, 2:518, 4:54, 1:24}, 6212 GPUs
    nodes = default_trace.nodes()
    assert len(nodes) == 1213
    assert Counter(n["gpu"] for n in nodes) == {8: 617, 2: 518, 4: 54, 1: 24}
    assert sum(n["gpu"] for n in nodes) == 6212
    assert sum(n["cpu"] for n in nodes) == 107018000
    types = default_trace.type_names()
    by = Counter(types[n["type"]] for n in nodes)
    assert by == {"G2": 549, "T4": 404, "P100": 134, "V100M16": 55, "G3": 39, "V100M32": 30, "A10": 2}
    assert [n["name"] for n in nodes] == sorted(n["name"] for n in nodes)


def test_openb_pod_stats(default_trace):
    # 8152 pods: 1088 CPU-only, 3078 GPU-share, 3911 whole 1-GPU, 16 2-GPU, 15 4-GPU, 44 8-GPU
    pods = default_trace.pods()
    assert len(pods) == 8152
    kinds = Counter("cpu" if p["num"] == 0 else ("share" if p["milli"] < 1000 else "%d" % p["num"]) for p in pods)
    assert kinds == {"cpu": 1088, "share": 3078, "1": 3911, "2": 16, "4": 15, "8": 44}
    assert all(p["mask"] == ksim.KSIM_TYPE_ANY for p in pods)


def test_loader_matches_plain_csv_parse(default_trace):
    rows = list(csv.DictReader(open(os.path.join(ksim.DATA_DIR, "openb_pod_list_default.csv"))))
    by_name = {r["name"]: r for r in rows}
    for p in default_trace.pods()[:500]:
        r = by_name[p["name"]]
        assert p["cpu"] == int(r["cpu_milli"]) and p["mem"] == int(r["memory_mib"])
        assert p["num"] == int(r["num_gpu"])
        assert p["milli"] == (int(r["gpu_milli"]) if int(r["num_gpu"]) else 0)


def test_gpuspec_masks():
    t = ksim.Trace.openb("gpuspec33")
    types = t.type_names()
    n_spec = 0
    for p in t.pods():
        if p["spec"]:
            n_spec += 1
            want = 0
            for m in p["spec"].split("|"):
                want |= 1 << types.index(m)
            assert p["mask"] == want
    assert n_spec > 1000


@pytest.mark.parametrize("name", TRACES)
def test_typical_pods_product_equals_oracle(name):
    # frag.go:285-380 restated twice (C++ product, C oracle) -> identical table, bit-exact freqs
    t = ksim.Trace.openb(name)
    arr, n = t.typical()
    mine = [(arr[i].cpu_milli, arr[i].gpu_milli, arr[i].gpu_count, arr[i].freq) for i in range(n)]
    ref = helpers.oracle_typical(t)
    assert [(c, m, k, f) for (c, m, k, _, f) in ref] == mine
    types = t.type_names()
    for i, (_, _, _, spec, _) in enumerate(ref):
        want = 0
        for x in filter(None, spec.split("|")):
            want |= 1 << types.index(x)
        want = want or ksim.KSIM_TYPE_ANY
        assert arr[i].type_mask == want
    assert abs(sum(x[3] for x in mine) - 1) < 1e-9
    if name == "default":
        assert n == 35  # T = 35 at C2


def test_replay_event_stream(default_trace):
    rp = default_trace.replay(seed=42, tune_ratio=1.3, shuffle=True)
    pods = default_trace.pods()
    # originals first (a permutation), then "-tuned-i" clones
    first = rp.pod_index[:8152]
    assert sorted(first.tolist()) == list(range(8152))
    assert first.tolist() != list(range(8152))
    # tuneUpPods stops before exceeding ratio * capacity (MilliGpu check, simulator.go:1273)
    total = sum(pods[i]["milli"] * pods[i]["num"] for i in rp.pod_index)
    assert total <= 1.3 * 6212000
    assert 10500 < rp.n < 11200
    # node prefixes are a permutation; ranks follow byte-wise order of "%04d-name"
    assert sorted(rp.prefix.tolist()) == list(range(1213))
    names = rp.node_names(default_trace.nodes())
    order = sorted(range(1213), key=lambda i: names[i])
    assert [rp.nodes[i].name_rank for i in order] == list(range(1213))
    # events carry the pod rows
    for k in (0, 100, 9000):
        p = pods[rp.pod_index[k]]
        e = rp.events[k]
        assert (e.cpu_milli, e.mem_mib, e.gpu_milli, e.gpu_count) == (p["cpu"], p["mem"], p["milli"], p["num"])


def test_replay_deterministic_and_seeded(default_trace):
    a = default_trace.replay(seed=7)
    b = default_trace.replay(seed=7)
    c = default_trace.replay(seed=8)
    assert a.n == b.n and (a.pod_index == b.pod_index).all() and (a.prefix == b.prefix).all()
    assert (a.pod_index[: c.n] != c.pod_index[: a.n]).any()


def test_replay_no_shuffle_no_tune(default_trace):
    rp = default_trace.replay(seed=1, tune_ratio=0, shuffle=False)
    assert rp.n == 8152 and rp.pod_index.tolist() == list(range(8152))


def test_replay_tune_down():
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=3, tune_ratio=0.5)
    pods = t.pods()
    total = sum(pods[i]["milli"] * pods[i]["num"] for i in rp.pod_index)
    assert total <= 0.5 * 6212000 and rp.n < 8152


def test_synthetic_cluster(default_trace):
    s = default_trace.synthetic(20000, 5000, seed=0)
    assert s.num_nodes == 20000 and s.num_pods == 5000
    rp = s.replay(seed=1, tune_ratio=0, shuffle=False)
    # >= 10000 nodes: "%04d-" prefixes grow to 5 digits, ranks still follow string order
    names = rp.node_names(s.nodes())
    order = sorted(range(20000), key=lambda i: names[i])
    assert [rp.nodes[i].name_rank for i in order] == list(range(20000))


def _write(path, rows):
    with open(path, "w", newline="") as f:
        csv.writer(f).writerows(rows)


NODE_HDR = ["sn", "cpu_milli", "memory_mib", "gpu", "model"]
POD_HDR = ["name", "cpu_milli", "memory_mib", "num_gpu", "gpu_milli", "gpu_spec"]


def test_loader_rejects_short_rows(tmp_path):
    # a row without the required columns is KSIM_EIO, not an out-of-range read
    nodes, pods = tmp_path / "n.csv", tmp_path / "p.csv"
    _write(pods, [POD_HDR, ["p0", "1000", "1024", "1", "500", "V100M16"]])
    _write(nodes, [NODE_HDR, ["n0", "96000", "786432", "8", "V100M16"], ["n1", "96000"]])
    with pytest.raises(ksim.KsimError) as ei:
        ksim.Trace.openb(str(pods), node_csv=str(nodes))
    assert ei.value.code == ksim.KSIM_EIO
    _write(nodes, [NODE_HDR, ["n0", "96000", "786432", "8", "V100M16"]])
    _write(pods, [POD_HDR, ["p0", "1000", "1024", "1", "500", "V100M16"], ["p1", "1000"]])
    with pytest.raises(ksim.KsimError) as ei:
        ksim.Trace.openb(str(pods), node_csv=str(nodes))
    assert ei.value.code == ksim.KSIM_EIO


def test_tuning_needs_gpu_demand_and_capacity(tmp_path):
    # simulator.go:1203-1211: with a tune ratio the reference panics on a workload or cluster without
    # CPU or GPU (tuneUpPods would never end); the replay driver returns KSIM_EINVAL instead
    nodes, pods = tmp_path / "n.csv", tmp_path / "p.csv"
    _write(nodes, [NODE_HDR, ["n0", "96000", "786432", "8", "V100M16"]])
    _write(pods, [POD_HDR, ["p0", "1000", "1024", "0", "0", ""], ["p1", "2000", "1024", "0", "0", ""]])
    t = ksim.Trace.openb(str(pods), node_csv=str(nodes))
    with pytest.raises(ksim.KsimError) as ei:
        t.replay(seed=1, tune_ratio=1.3)
    assert ei.value.code == ksim.KSIM_EINVAL
    assert t.replay(seed=1, tune_ratio=0.0).n == 2  # no tuning: fine
