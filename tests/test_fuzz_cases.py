"""CPU checks of the fuzz-case generator (tests/fuzz_cases.py) and the oracle on it: the oracle
replays every case for every policy, the cases reach the corners they are meant to reach, and the
engine-side encodings (name ranks, model bitmasks) agree with the oracle-side strings."""
import pytest

import ksim
import pyoracle as O
from fuzz_cases import MODELS, VOCAB, make_case
from test_gpu_fuzz import CASES, POLICIES


@pytest.mark.parametrize("seed,n,e,pdel", CASES)
def test_oracle_replays_every_case(seed, n, e, pdel):
    c = make_case(seed, n, e, pdel)
    statuses = set()
    for name, pol, sel in POLICIES:
        res, state, _ = O.run_events(c["onodes"], c["otypical"], c["oevents"], policy=pol, gpu_sel=sel, seed=5)
        assert len(res) == c["n_events"]
        statuses |= {r[4] for r in res}
        for cpu_left, mem_left, pods, gl in state:
            assert cpu_left >= 0 and mem_left >= 0 and all(0 <= g <= 1000 for g in gl)
    assert 0 in statuses  # something binds
    if n > 1:
        assert 1 in statuses  # and something fails (the cluster fills or the filter rejects)


def test_cases_reach_the_corners():
    c = make_case(2, 97, 900, 0.25)
    gpus = {d["gpu"] for d in c["onodes"]}
    assert 0 in gpus and 8 in gpus and gpus & {3, 5, 6, 7}
    ev = c["oevents"]
    assert any(e.get("delete") for e in ev)
    assert any(e["cpu"] == 0 and e["cpu_nz"] == 100 for e in ev)
    assert any(e["num"] == 8 for e in ev)
    assert any("H100" in e["type"] for e in ev) and any("|" in e["type"] for e in ev)
    assert any(d["pods"] <= 2 for d in c["onodes"])


def test_engine_encodings_match_oracle_strings():
    c = make_case(3, 250, 300, 0.1)
    names = [d["name"].encode() for d in c["onodes"]]
    for i, d in enumerate(c["onodes"]):
        n = c["nodes"][i]
        assert n.name_rank == sorted(names).index(names[i])
        assert n.gpu_count == d["gpu"]
        if d["gpu"]:
            assert MODELS[n.gpu_type] == d["model"]
    for k, e in enumerate(c["oevents"]):
        p = c["events"][k]
        if e["type"]:
            assert p.type_mask == sum(1 << VOCAB.index(s) for s in e["type"].split("|"))
        else:
            assert p.type_mask == ksim.KSIM_TYPE_ANY
        assert (p.cpu_milli, p.cpu_nz_milli, p.mem_mib, p.gpu_milli, p.gpu_count) == \
            (e["cpu"], e["cpu_nz"], e["mem"], e["milli"], e["num"])
