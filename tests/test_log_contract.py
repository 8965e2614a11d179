"""The log contract: our `simon apply` log, read by the reference's own harness.

tests/golden/log_golden.json holds what the reference's scripts/analysis.py (log_to_csv) produced
from the oracle's log of one openb run (tests/log_case.py; tests/golden/make_log_golden.py): the
per-experiment analysis.csv row -- unscheduled and original pods, the InitSchedule allocation ratios,
amounts and totals, the quadrant shares -- and the per-event [Power] columns (analysis_pwr.csv).
Here the log is rebuilt from the oracle (byte-identical: same sha256) and read back by ksim.analysis'
restatement of that parser, which must give the reference script's row and columns.  The GPU side
(tests/test_gpu_log_contract.py) writes the same bytes from the device's reports.
"""
import hashlib
import json
import os

import pytest

import ksim.analysis as A
import log_case

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "log_golden.json")) as f:
    GOLD = json.load(f)


@pytest.mark.parametrize("policy", sorted(log_case.POLICIES))
def test_oracle_log_read_like_the_reference_harness(policy, tmp_path):
    log = tmp_path / "run.log"
    log_case.oracle_log(log, policy)
    want = GOLD["policies"][policy]
    assert hashlib.sha256(log.read_bytes()).hexdigest() == want["log_sha256"]
    with open(log) as f:
        got = A.parse_log_full(f.readlines())
    assert {k: float(v) for k, v in got["row"].items()} == want["row"]
    assert got["power"] == want["power"]
    assert len(got["allo"]["arrived_gpu_milli"]) == log_case.N_EVENTS
    # every line kind is there: failures, the ClusterAnalysis block, the unscheduled count
    assert want["row"]["unscheduled"] > 0 and want["row"]["origin_pods"] == 8152
    assert 0 < want["row"]["milli_gpu_init_schedule"] <= 100 and want["row"]["gpu_total"] > 0


def test_logrus_formatting_rules():
    # text_formatter.go:151-153 (no msg key when empty), :298-337 (bare when every char is safe)
    assert A.logrus_line("", ts="T") == 'time="T" level=info\n'
    assert A.logrus_line("--------------------", ts="T") == 'time="T" level=info msg=--------------------\n'
    assert A.logrus_line("a: b\n", ts="T") == 'time="T" level=info msg="a: b\\n"\n'


def test_pod_repr_and_power_line():
    # resource.go:104-127; analysis.go:54
    assert A.pod_repr(6000, 460, 1, "") == "<CPU:   6.00, GPU: 1 x {460 }m (CPUREQ: ANY) (GPUREQ: ANY)>"
    assert A.pod_repr(88000, 0, 0, "") == "<CPU:  88.00, GPU: 0 x {0   }m (CPUREQ: ANY) (GPUREQ: NONE)>"
    assert A.pod_repr(12000, 1000, 8, "V100M16|V100M32") == \
        "<CPU:  12.00, GPU: 8 x {1000}m (CPUREQ: ANY) (GPUREQ: V100M16|V100M32)>"
    assert A.power_message(dict(cpu_w=11190.0, gpu_w=35875.0)) == \
        "[Power]; cluster: 47065.0; ClusterCPU: 11190.0; ClusterGPU: 35875.0\n"


def test_cluster_analysis_block_shape():
    nodes = [dict(cpu_alloc=64000, cpu_used=8000, mem_alloc_mib=1024, mem_used_mib=512, gpu_count=2,
                  gpu_used=[1000, 300, 0, 0, 0, 0, 0, 0]),
             dict(cpu_alloc=32000, cpu_used=0, mem_alloc_mib=1024, mem_used_mib=0, gpu_count=0, gpu_used=[0] * 8)]
    msgs = A.cluster_analysis_messages(nodes, [1000.0, 200.0, 500.0, 0.0, 0.0, 0.0, 0.0])
    # the header, then the 15 lines scripts/analysis.py reads (its NUM_CLUSTER_ANALYSIS_LINE = 16)
    assert msgs[1] == "========== Cluster Analysis Results (InitSchedule) =========="
    assert msgs[3] == "    MilliCpuLeft:  8.3% (8000/96000)\n"
    assert msgs[4] == "    Memory  : 25.0%% (%d/%d)\n" % (512 * A.MIB, 2048 * A.MIB)
    assert msgs[5] == "    Gpu     : 100.0% (2/2)\n"
    assert msgs[6] == "    MilliGpu: 65.0% (1300/2000)\n"
    assert msgs[7] == "q1_lack_both :   1.00 x 10^3 (58.82%)\n"
    assert msgs[-2] == "=============================================="
    assert msgs[-3] == "frag_gpu_milli:   1.20 x 10^3 (70.59%)\n"
    lines = [A.logrus_line(m) for m in msgs]
    row = A.parse_log_full(lines)["row"]
    assert row["gpu_init_schedule"] == 100.0 and row["milli_gpu_amount_init_schedule"] == 1300.0
    assert row["q2_lack_gpu_init_schedule"] == 11.76 and row["frag_gpu_milli_init_schedule"] == 70.59
    assert "milli_cpu_init_schedule" not in row  # analysis.py:7 ALLO_KEYS has MilliCpu, the log MilliCpuLeft
