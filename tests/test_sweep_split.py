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
    # round-5 verdict item 1: after the LPT split, each share's longest FGD replays take k_memo, each at the fewest
    # workgroups (of WIDE_KS) that bring it under the share's predicted time, within the 256 CUs
    items, costs = plan
    wide_costs = SW.plan_wide_costs(items)
    seen = set()
    for k in range(world):
        sh = SW.shard(items, k, world, costs)
        idx = [items.index(e) for e in sh]
        c = [costs[i] for i in idx]
        wc = {kw: [v[i] for i in idx] for kw, v in wide_costs.items()}
        wide = SW.plan_widths(sh, c, wc)
        assert wide == SW.plan_widths(sh, c, wc)  # deterministic
        assert all(sh[i][1] == "06-FGD" and kw in SW.WIDE_KS for i, kw in wide.items())
        seen |= set(wide.values())
        if not wide:
            continue
        n_fgd = sum(1 for e in sh if e[1] == "06-FGD")
        n_cheap = len(sh) - n_fgd
        loosest = max(p for p, _ in SW.CHEAP_PACKS)
        assert n_fgd + sum(kw - 1 for kw in wide.values()) + -(-n_cheap // loosest) <= 256 - SW.CU_SLACK
        # the widened ones are the longest FGD chains, and each is shorter widened
        narrow = [c[i] for i in range(len(sh)) if sh[i][1] == "06-FGD" and i not in wide]
        assert min(c[i] for i in wide) >= max(narrow, default=0.0)
        assert all(wc[kw][i] < c[i] for i, kw in wide.items())
        # the predicted share time is shorter than the longest chain was
        t = max([wc[kw][i] for i, kw in wide.items()] + narrow)
        assert t < max(c[i] for i in wide)
    if world == 1:  # the whole sweep leaves no CU for a wide replica
        assert SW.plan_widths(items, costs, wide_costs) == {}
    if world == 8:  # room for the longest chains (gpushare100) at 24 or 32 workgroups
        assert seen & {24, 32}, seen
    if world == 4:  # more long chains than CUs at 16: 12 and narrower
        assert 12 in seen and max(seen) <= 12, seen


def test_widths_take_the_fewest_workgroups_under_the_predicted_time():
    items = [("t", "06-FGD", s, 1.3) for s in range(3)] + [("t", "05-BestFit", 0, 1.3)]
    costs = [100.0, 90.0, 50.0, 60.0]
    wide = {12: [80.0, 70.0, 40.0, 60.0], 16: [70.0, 60.0, 38.0, 60.0], 32: [62.0, 59.0, 35.0, 60.0]}
    one = ((3, 1.0),)
    # T = 62: item 0 needs 32 workgroups, item 1 16 (the fewest under 62), item 2 is under the cheap chain (60)
    assert SW.plan_widths(items, costs, wide, packs=one, margin=1.0, slack=0) == {0: 32, 1: 16}
    # fewer CUs: 3 FGD + 1 cheap + 31 + 15 = 50 > 44, so T = 70 (item 0 at 16, item 1 at 12)
    assert SW.plan_widths(items, costs, wide, cus=44, packs=one, margin=1.0, slack=0) == {0: 16, 1: 12}
    assert SW.plan_widths(items, costs, wide, cus=3, packs=one, slack=0) == {}  # no CUs to spare
    # the margin widens item 2 too (50 > 0.75 x 62) at the fewest workgroups that shorten it
    assert SW.plan_widths(items, costs, wide, packs=one, margin=0.75, slack=0) == {0: 32, 1: 16, 2: 12}


def test_widths_choose_the_shorter_packing():
    # two long FGD chains beside six cheap ones (40 alone, 56 packed 6 to a CU)
    items = [("t", "06-FGD", s, 1.3) for s in range(2)] + [("t", "05-BestFit", s, 1.3) for s in range(6)]
    costs = [100.0, 95.0] + [40.0] * 6
    wide = {12: [62.0, 60.0] + [40.0] * 6, 32: [50.0, 48.0] + [40.0] * 6}
    packs = ((3, 1.0), (6, 1.4))
    # T = 60 needs item 0 at 32 and item 1 at 12 (42 CUs beyond one each), T = 62 both at 12 (22)
    assert SW.plan_widths(items, costs, wide, cus=30, packs=packs, margin=1.0, slack=0) == {0: 12, 1: 12}
    # 45 CUs: packed 3 to a CU the cheap replicas leave 41 (T 62), 6 to a CU 42 (T 60, over their 56): the tighter wins
    assert SW.plan_widths(items, costs, wide, cus=45, packs=packs, margin=1.0, slack=0) == {0: 32, 1: 12}
    assert SW.plan_widths(items, costs, wide, cus=45, packs=packs[:1], margin=1.0, slack=0) == {0: 12, 1: 12}


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
