"""C1: the reference's own example, example/original/test-cluster-config.yaml (BASELINE.json configs[0]).

Two nodes (pai-node-00: 64 CPU, 2 x V100; pai-node-01: 64 CPU, 4 x V100; 110 pods each) and three pods
(gpu-pod-00: 4 CPU, 0.5 GPU; gpu-pod-01: 8 CPU, no GPU; gpu-pod-02: 12 CPU, 2 whole GPUs), FGD with
the FGD GPU selector (test-scheduler-config.yaml), shufflePod false, workload tuning ratio 0.9 with
seed 233.  The YAML files are restated here as the two CSV tables the replay driver reads (the
values are the YAMLs' own; no reference file is copied).

CPU: the event stream -- the three pods in name order (no creation-time annotation: SortClusterPods
falls back to names), then the tuneUpPods clones drawn with Go's rand.Intn(3) after the debug
rand.Int(), recomputed here from the restated source's raw Int63 stream.
GPU: the engine's decisions equal the oracle's, event by event.
"""
import os

import pytest

import helpers
import ksim
import pyoracle as O

NODES = "sn,cpu_milli,memory_mib,gpu,model\npai-node-00,64000,256000,2,V100\npai-node-01,64000,256000,4,V100\n"
PODS = ("name,cpu_milli,memory_mib,num_gpu,gpu_milli,gpu_spec\n"
        "gpu-pod-00,4000,9216,1,500,\n"
        "gpu-pod-01,8000,17408,0,0,\n"
        "gpu-pod-02,12000,18432,2,1000,\n")
PODS_ALLOC = 110  # node YAMLs: allocatable pods


@pytest.fixture(scope="module")
def c1(tmp_path_factory):
    d = tmp_path_factory.mktemp("c1")
    with open(os.path.join(d, "nodes.csv"), "w") as f:
        f.write(NODES)
    with open(os.path.join(d, "pods.csv"), "w") as f:
        f.write(PODS)
    t = ksim.Trace.openb(str(os.path.join(d, "pods.csv")), node_csv=str(os.path.join(d, "nodes.csv")))
    rp = t.replay(seed=233, tune_ratio=0.9, shuffle=False)
    for i in range(t.num_nodes):
        rp.nodes[i].pods_alloc = PODS_ALLOC
    return t, rp


def go_intn_stream(seed, n, skip):
    """Go's Rand.Intn(n) (Int31n: rejection above the largest multiple of n) on the Int63 stream."""
    raw = ksim.go_rand(seed, ksim.GO_INT63, 400)[skip:]
    mx = (1 << 31) - 1 - (1 << 31) % n
    out = []
    for v in raw:
        v31 = v >> 32
        if v31 <= mx:
            out.append(v31 % n)
    return out


def test_c1_event_stream(c1):
    t, rp = c1
    pods = t.pods()
    assert [p["name"] for p in pods] == ["gpu-pod-00", "gpu-pod-01", "gpu-pod-02"]
    order = [int(i) for i in rp.pod_index[:rp.n]]
    assert order[:3] == [0, 1, 2]  # shufflePod false: name order
    # tuneUpPods (simulator.go:1263-1282): draw until podTotalMilliGpuReq + MilliGpu > 0.9 * 6000
    total, target, want = 500 + 2000, 0.9 * 6000, []
    for idx in go_intn_stream(233, 3, 1):  # after core.go:116's rand.Int()
        p = pods[idx]
        if total + p["milli"] > target:
            break
        total += p["milli"] * p["num"]
        want.append(idx)
    assert order[3:] == want and len(want) > 0
    assert rp.n == 3 + len(want)


@pytest.mark.gpu
def test_c1_fgd_matches_oracle(c1):
    t, rp = c1
    arr, n = t.typical()
    eng = ksim.Engine(t.num_nodes, 1)
    eng.set_nodes(0, rp.nodes)
    eng.set_typical(0, arr, n)
    eng.set_policy(0, "FGD")
    eng.load_events(0, rp.events, rp.n)
    eng.run()
    got = eng.results(0)
    eng.close()
    onodes = helpers.oracle_nodes(t, rp)
    for d in onodes:
        d["pods"] = PODS_ALLOC
    want, _, _ = O.run_events(onodes, helpers.oracle_typical(t), helpers.oracle_events(t, rp), policy=O.POL_FGD,
                              gpu_sel=O.SEL_FGD)
    assert got == want
    assert sum(1 for r in got if r[0] >= 0) >= 3
