"""Shared test helpers: build matching engine and oracle inputs from one trace.

The engine gets the product's encodings (type bitmasks, name ranks, typical
table from the C++ host driver); the oracle gets strings (GPU model names,
"%04d-<name>" node names) and computes its own typical table, so the encodings
are checked rather than shared.
"""
import ksim
import pyoracle as O


def oracle_typical(trace, threshold=95, step=1):
    wl = [(p["cpu"], p["milli"], p["num"], p["spec"] if p["num"] > 0 else "") for p in trace.pods()]
    return O.get_typical_pods(wl, threshold=threshold, step=step)


def product_typical_list(trace, threshold=95, step=1):
    arr, n = trace.typical(threshold=threshold, step=step)
    return arr, n


def oracle_nodes(trace, replay):
    tn = trace.nodes()
    names = replay.node_names(tn)
    types = trace.type_names()
    return [dict(name=names[i], cpu=tn[i]["cpu"], mem=tn[i]["mem"], pods=1001, gpu=tn[i]["gpu"],
                 model=types[tn[i]["type"]] if tn[i]["gpu"] > 0 else "") for i in range(len(tn))]


def oracle_subset(trace, replay, keep):
    """oracle_nodes restricted to the node indices `keep` (built once, not once per index)."""
    full = oracle_nodes(trace, replay)
    return [full[i] for i in keep]


def oracle_events(trace, replay, limit=None):
    pods = trace.pods()
    n = replay.n if limit is None else min(limit, replay.n)
    out = []
    for k in range(n):
        p = pods[replay.pod_index[k]]
        out.append(dict(cpu=p["cpu"], cpu_nz=p["cpu"], mem=p["mem"], milli=p["milli"], num=p["num"],
                        type=p["spec"] if p["num"] > 0 else ""))
    return out


def subset_nodes(replay, keep):
    """Engine nodes for a subset of node indices, re-ranked by their relative order."""
    import ctypes as C
    sub = (ksim.Node * len(keep))()
    ranks = sorted(range(len(keep)), key=lambda j: replay.nodes[keep[j]].name_rank)
    rank_of = {j: r for r, j in enumerate(ranks)}
    for j, i in enumerate(keep):
        C.memmove(C.byref(sub[j]), C.byref(replay.nodes[i]), C.sizeof(ksim.Node))
        sub[j].name_rank = rank_of[j]
    return sub


def delete_stream(trace, replay, n_create, p_delete=0.3, seed=0):
    """A create/delete event stream (simulator.go:416-422): after each creation, with probability
    p_delete, a deletion of a random live earlier creation.  Returns (engine events, oracle events)."""
    import ctypes as C
    import random
    rnd = random.Random(seed)
    evs, oev, live = [], [], []
    base = oracle_events(trace, replay, n_create)
    for k in range(n_create):
        e = ksim.Pod()
        C.memmove(C.byref(e), C.byref(replay.events[k]), C.sizeof(ksim.Pod))
        evs.append(e)
        oev.append(dict(base[k]))
        live.append(len(evs) - 1)
        if rnd.random() < p_delete and live:
            ref = live.pop(rnd.randrange(len(live)))
            d = ksim.Pod()
            C.memmove(C.byref(d), C.byref(evs[ref]), C.sizeof(ksim.Pod))
            d.is_delete, d.ref = 1, ref
            evs.append(d)
            od = dict(oev[ref])
            od.update(delete=1, ref=ref)
            oev.append(od)
    return (ksim.Pod * len(evs))(*evs), oev
