"""The device's reports written as `simon apply`'s log: byte-identical to the oracle's log, which the
reference's own scripts/analysis.py read into tests/golden/log_golden.json (tests/test_log_contract.py).
Covers the per-event [Power] report (analysis.go:24-56) and the end-of-run ClusterAnalysis block from
the device's final state.  Needs a gfx950 device.
"""
import hashlib
import json
import os

import pytest

import ksim.analysis as A
import log_case

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "log_golden.json")) as f:
    GOLD = json.load(f)


@pytest.mark.parametrize("policy", sorted(log_case.POLICIES))
def test_gpu_log_equals_golden(policy, tmp_path):
    log = tmp_path / "gpu.log"
    res, path = log_case.engine_log(log, policy)
    want = GOLD["policies"][policy]
    with open(log) as f:
        got = A.parse_log_full(f.readlines())
    assert {k: float(v) for k, v in got["row"].items()} == want["row"], path
    assert got["power"] == want["power"], path
    assert hashlib.sha256(log.read_bytes()).hexdigest() == want["log_sha256"], path
