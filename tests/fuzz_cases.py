"""Adversarial synthetic clusters for the parity fuzz (tests/test_gpu_fuzz.py, tests/test_fuzz_cases.py).

One seed gives matching engine inputs (ksim.Node / ksim.Pod / ksim.Typical: model ids, type
bitmasks, name ranks) and oracle inputs (model strings, pipe-list GPU specs, "%04d-" node names),
built side by side from the same random draws.  The draws reach the corners the openb traces do
not: GPU-less nodes, 3/5/6/7-GPU nodes, tight pod limits (the pods+1 <= allowed Filter), tiny
memory, zero-CPU pods (Score's non-zero 100m, utils.go:1008-1029), 8-GPU pods, GPU specs naming a
model no node has (IsNodeAccessibleToPodByType, utils.go:957-1006), pipe lists of two models, and
deletions of earlier creations (open_gpu_share.go:58-70).
"""
import ctypes as C

import numpy as np

import ksim

MODELS = ["G2", "T4", "P100", "V100M16", "A10"]
UNKNOWN = "H100"  # a model no node has: its bit never matches
VOCAB = MODELS + [UNKNOWN]


def _mask(spec, vocab=VOCAB):
    if not spec:
        return ksim.KSIM_TYPE_ANY
    m = 0
    for s in spec.split("|"):
        m |= 1 << vocab.index(s)
    return m


def make_case(seed, n_nodes, n_create, p_delete=0.0, models=None):
    """-> dict(nodes, events, n_events, typical, typical_n, onodes, oevents, otypical)
    models: the GPU model vocabulary (model id = index; default MODELS), e.g. a trace's type_names()
    so that its PWR power model applies."""
    import pyoracle as O

    MODELS_ = list(models) if models is not None else MODELS
    VOCAB_ = MODELS_ + [UNKNOWN]

    rnd = np.random.default_rng(seed)
    # node names: "%04d-" + name from a permutation (simulator.go:584-588); rank = byte order
    perm = rnd.permutation(n_nodes)
    names = ["%04d-node-%d" % (perm[i], i) for i in range(n_nodes)]
    order = sorted(range(n_nodes), key=lambda i: names[i].encode())
    rank = [0] * n_nodes
    for r, i in enumerate(order):
        rank[i] = r
    nodes = (ksim.Node * n_nodes)()
    onodes = []
    for i in range(n_nodes):
        gpu = int(rnd.choice([0, 1, 2, 3, 4, 5, 6, 7, 8], p=[.12, .1, .15, .05, .15, .03, .05, .05, .3]))
        model = int(rnd.integers(len(MODELS_))) if gpu > 0 else 0
        cpu = int(rnd.choice([2000, 8000, 32000, 64000, 96000, 128000]))
        mem = int(rnd.choice([4096, 16384, 65536, 262144, 786432]))
        pods = int(rnd.choice([1, 2, 3, 8, 110], p=[.05, .1, .1, .25, .5]))
        n = nodes[i]
        n.cpu_alloc_milli, n.mem_alloc_mib, n.pods_alloc = cpu, mem, pods
        n.gpu_count, n.gpu_type, n.name_rank = gpu, model, rank[i]
        onodes.append(dict(name=names[i], cpu=cpu, mem=mem, pods=pods, gpu=gpu, model=MODELS_[model] if gpu else ""))
    creates = []
    for _ in range(n_create):
        kind = rnd.choice(["cpu", "share", "whole"], p=[.2, .45, .35])
        # (few CPU sizes for GPU pods: the target-workload table stays within the engine's 256
        # entries; the real traces have at most 127)
        cpu = int(rnd.choice([0, 100, 500, 1000, 4000, 8000, 16000, 48000] if kind == "cpu" else [0, 4000, 16000]))
        mem = int(rnd.choice([0, 512, 2048, 8192, 30000, 120000]))
        if kind == "cpu":
            milli, num = 0, 0
        elif kind == "share":
            milli, num = int(rnd.choice([1, 100, 250, 333, 500, 700, 999])), 1
        else:
            milli, num = 1000, int(rnd.choice([1, 1, 1, 2, 3, 4, 8]))
        spec = ""
        if num > 0 and rnd.random() < 0.2:
            k = int(rnd.integers(1, 3))
            spec = "|".join(rnd.choice(VOCAB_, size=k, replace=False))
        creates.append((cpu, mem, milli, num, spec))
    # event stream: creations, each followed with probability p_delete by the deletion of a random
    # live earlier creation
    evs, oev, live = [], [], []
    for cpu, mem, milli, num, spec in creates:
        e = ksim.make_pod(cpu, milli, num, mem, _mask(spec, VOCAB_), cpu_nz=cpu if cpu > 0 else 100)
        evs.append(e)
        oev.append(dict(cpu=cpu, cpu_nz=cpu if cpu > 0 else 100, mem=mem, milli=milli, num=num, type=spec))
        live.append(len(evs) - 1)
        if p_delete > 0 and rnd.random() < p_delete and live:
            ref = live.pop(int(rnd.integers(len(live))))
            d = ksim.Pod()
            C.memmove(C.byref(d), C.byref(evs[ref]), C.sizeof(ksim.Pod))
            d.is_delete, d.ref = 1, ref
            evs.append(d)
            od = dict(oev[ref])
            od.update(delete=1, ref=ref)
            oev.append(od)
    # target workload: the created pods (GetTypicalPods, frag.go:285-380) by the oracle; the
    # engine gets the same list with model bitmasks
    otyp = O.get_typical_pods([(c, m, n, s) for c, _, m, n, s in creates])
    typ = (ksim.Typical * max(1, len(otyp)))()
    for i, (cpu, milli, num, spec, freq) in enumerate(otyp):
        typ[i].cpu_milli, typ[i].gpu_milli, typ[i].gpu_count = cpu, milli, num
        typ[i].type_mask, typ[i].freq = _mask(spec, VOCAB_), freq
    return dict(nodes=nodes, events=(ksim.Pod * max(1, len(evs)))(*evs), n_events=len(evs), typical=typ,
                typical_n=len(otyp), onodes=onodes, oevents=oev, otypical=otyp)
