"""The paper sweep's split over ranks: ksim.sweep.shard with the cost model.

Every split tiles the 1020 experiments (each on exactly one rank), is deterministic, spreads the long FGD
replays over the ranks and balances the estimated totals; without costs it is the round robin.
"""
import pytest

import ksim.sweep as SW


@pytest.fixture(scope="module")
def plan():
    items = SW.plan()
    return items, SW.plan_costs(items)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_split_tiles_the_sweep(plan, world):
    items, costs = plan
    assert len(items) == 1020 and len(costs) == 1020
    shares = [SW.shard(items, k, world, costs) for k in range(world)]
    flat = [e for sh in shares for e in sh]
    assert sorted(flat) == sorted(items) and len(set(flat)) == len(items)
    assert shares == [SW.shard(items, k, world, costs) for k in range(world)]  # deterministic
    for sh in shares:  # each rank keeps plan order
        pos = [items.index(e) for e in sh]
        assert pos == sorted(pos)
    idx = {e: i for i, e in enumerate(items)}
    tot = [sum(costs[idx[e]] for e in sh) for sh in shares]
    assert max(tot) <= 1.01 * (sum(costs) / world) + max(costs)  # LPT: within one item of the mean
    if world > 1:
        # the 40 longest experiments (gpuspec FGD) spread: no rank holds more than its share plus one
        longest = sorted(range(len(items)), key=lambda i: -costs[i])[:40]
        per = [sum(1 for i in longest if items[i] in set(sh)) for sh in shares]
        assert max(per) <= 40 // world + 1


def test_round_robin_without_costs(plan):
    items, _ = plan
    assert SW.shard(items, 1, 4) == items[1::4]


def test_cost_model_orders_policies(plan):
    items, costs = plan
    by = {}
    for e, c in zip(items, costs):
        by.setdefault((e[0], e[1]), []).append(c)
    # gpuspec33's FGD replays (127 typical pods) are the longest; a cheap policy costs less than FGD on a trace
    # the measured table (profiles/r06/c4_costs.jsonl): the longest chains are FGD on the typed gpuspec traces (127
    # typical pods) and the long gpushare streams (16 805 events)
    top = sorted(by, key=lambda k: -max(by[k]))[:6]
    assert all(p == "06-FGD" and ("gpuspec" in t or "gpushare" in t) for t, p in top), top
    assert ("openb_pod_list_gpuspec33", "06-FGD") in top
    assert max(by[("openb_pod_list_default", "05-BestFit")]) < min(by[("openb_pod_list_default", "06-FGD")])


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_widths_fit_the_cus_and_take_the_longest_fgd_chains(plan, world):
    # round-5 verdict item 1: after the LPT split, each share's FGD replays whose one-workgroup chain is longer than
    # every chain widening cannot shorten take k_memo at one of WIDTHS' widths, longest first, within the 256 CUs
    items, costs = plan
    wide_costs = SW.plan_wide_costs(items)
    widths = {k: (pc, slow) for k, pc, slow in SW.WIDTHS}
    chosen = []
    for k in range(world):
        sh = SW.shard(items, k, world, costs)
        idx = [items.index(e) for e in sh]
        c = [costs[i] for i in idx]
        wc = {kw: [v[i] for i in idx] for kw, v in wide_costs.items()}
        wide = SW.plan_widths(sh, c, wc)
        assert wide == SW.plan_widths(sh, c, wc)  # deterministic
        assert len(set(wide.values())) <= 1 and all(sh[i][1] == "06-FGD" for i in wide)  # one width per share
        if not wide:
            continue
        kw = next(iter(wide.values()))
        chosen.append(kw)
        per_cu, slow = widths[kw]
        n_fgd = sum(1 for e in sh if e[1] == "06-FGD")
        n_cheap = len(sh) - n_fgd
        assert n_fgd + len(wide) * (kw - 1) + -(-n_cheap // per_cu) <= 256
        # the widened ones are the longest FGD chains, each longer than every (slowed) cheap chain
        narrow = [c[i] for i in range(len(sh)) if sh[i][1] == "06-FGD" and i not in wide]
        assert min(c[i] for i in wide) >= max(narrow, default=0.0)
        assert min(c[i] for i in wide) > slow * max((c[i] for i in range(len(sh)) if sh[i][1] != "06-FGD"), default=0.0)
        # the chosen width predicts no longer a share than any other candidate's plan
        t = SW._widen(sh, c, wc[kw], 256, kw, per_cu, slow)[0]
        assert all(t <= SW._widen(sh, c, wc[k2], 256, k2, pc2, s2)[0] for k2, pc2, s2 in SW.WIDTHS)
    if world == 1:  # the whole sweep leaves no CU for a wide replica
        assert SW.plan_widths(items, costs, wide_costs) == {}
    if world == 8:  # every long chain fits at 16 workgroups (profiles/r06/c4_shares/widths_r06.txt)
        assert set(chosen) == {16}
    if world == 4:  # more long chains than 16-wide slots: 12 workgroups, the cheap replicas 6 to a CU
        assert set(chosen) == {12}


def test_widths_stop_where_a_wide_chain_would_not_be_shorter():
    items = [("t", "06-FGD", s, 1.3) for s in range(4)] + [("t", "05-BestFit", 0, 1.3)]
    costs = [100.0, 90.0, 50.0, 40.0, 60.0]
    wide = {16: [70.0, 95.0, 30.0, 30.0, 60.0]}
    one = ((16, 3, 1.0),)
    # item 1 would be no shorter wide: the widening stops there, and item 2 is under the cheap chain anyway
    assert SW.plan_widths(items, costs, wide, widths=one) == {0: 16}
    assert SW.plan_widths(items, costs, wide, cus=16, widths=one) == {}  # no CUs to spare
    assert SW.plan_widths(items, costs, wide, widths=((16, 6, 1.0),)) == {0: 16}


def test_widths_choose_the_shorter_predicted_share():
    # two long FGD chains and one cheap chain: at 16 workgroups only one fits the CUs, at 12 both do
    items = [("t", "06-FGD", s, 1.3) for s in range(2)] + [("t", "05-BestFit", 0, 1.3)]
    costs = [100.0, 95.0, 40.0]
    wide = {16: [60.0, 58.0, 40.0], 12: [62.0, 60.0, 40.0]}
    widths = ((16, 3, 1.0), (12, 6, 1.4))
    assert SW.plan_widths(items, costs, wide, cus=30, widths=widths) == {0: 12, 1: 12}  # 62 against 95
    assert SW.plan_widths(items, costs, wide, cus=40, widths=widths) == {0: 16, 1: 16}  # 60 against 62
    # equal predictions: the width that widens more, then the first
    assert SW.plan_widths(items, costs, {16: [60.0, 58.0, 40.0], 12: [60.0, 58.0, 40.0]}, cus=40, widths=widths) == \
        {0: 16, 1: 16}


def test_costs_come_from_the_measured_table(plan):
    # each table row is one experiment measured alone (its seed with the most events): the model prices that
    # experiment at the measured device time
    import json
    items, costs = plan
    with open(SW.COST_TABLE) as f:
        rows = [json.loads(ln) for ln in f]
    assert {(r["trace"], r["policy"], r["form"]) for r in rows} >= {(t, p, "one") for t in SW.TRACES for p in SW.POLICY_DIRS}
    for r in rows:
        if r["form"] != "one":
            continue
        i = items.index((r["trace"], r["policy"], r["seed"], 1.3))
        assert costs[i] == pytest.approx(r["device_ms"] * 1000, rel=1e-3)
