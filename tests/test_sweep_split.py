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
    top = max(by, key=lambda k: max(by[k]))
    assert top == ("openb_pod_list_gpuspec33", "06-FGD")
    assert max(by[("openb_pod_list_default", "05-BestFit")]) < min(by[("openb_pod_list_default", "06-FGD")])
