"""Writes tests/golden/go_known_answers.json: the known-answer vectors held by the
reference's own Go unit tests for the Filter+Score path, transcribed as data.

Sources (reference tree Fr4nz83/kubernetes-scheduler-simulator @ 2024_08_07):
  pkg/utils/frag_test.go:13-51    TestingGenerateGetTypicalPods (35 typical pods)
  pkg/utils/frag_test.go:53-87    TestingGenerateGetTypicalPodsWithNonGpu (31 typical pods)
  pkg/utils/frag_test.go:100-121  TestNodeGpuShareFragAmountScore
  pkg/utils/frag_test.go:123-140  TestNodeGpuShareFragAmountWithNonGpu
  pkg/utils/frag_test.go:142-163  TestNodeGpuShareFragAmount
  pkg/utils/frag_test.go:165-185  TestGetGpuFragMilliByNodeResAndPodRes
  pkg/simulator/plugin/gpu_packing_score_test.go:9-35  TestGpuPackingScorePlugin_Score
  pkg/type/resource_test.go:9-41  Flatten / Add / Sub / Copy
  pkg/utils/utils_test.go:25-55   TestCalculateVectorDotProduct (NormalizeVector + CalculateVectorDotProduct
                                  of nodeRes.ToResourceVec / podRes.ToResourceVec; InDelta 1e-3)

Percentages are Go untyped-constant expressions such as `9.33 / 100`; Go evaluates
them exactly and rounds once, so they are stored as [numerator, denominator]
integer pairs and converted with fractions.Fraction (one correct rounding).
Run:  python tests/golden/make_go_known_answers.py
"""
import json
import os

# (MilliCpu, MilliGpu, GpuNumber, GpuType, Percentage numerator (x100), 100)
TYPICAL_35 = [
    (6000, 465, 1, "", 933), (8000, 440, 1, "2080", 915), (8000, 475, 1, "T4", 876),
    (8000, 440, 1, "P100", 872), (2000, 465, 1, "", 868), (12000, 900, 1, "", 865),
    (4000, 900, 1, "", 843), (16000, 678, 1, "T4", 836), (8000, 500, 1, "", 829),
    (6000, 511, 1, "", 811), (14000, 1000, 2, "2080", 54), (4000, 1000, 1, "2080", 43),
    (32000, 1000, 2, "T4", 43), (16000, 1000, 1, "V100M16", 40), (64000, 1000, 2, "", 40),
    (10000, 1000, 2, "", 40), (11400, 1000, 1, "T4", 36), (16000, 1000, 1, "T4", 36),
    (4000, 1000, 2, "", 36), (14000, 1000, 2, "V100M16", 36), (8000, 1000, 4, "", 36),
    (16000, 1000, 2, "", 32), (2000, 1000, 1, "T4", 32), (6000, 1000, 1, "", 32),
    (4000, 1000, 1, "", 32), (5000, 1000, 1, "", 32), (32000, 1000, 4, "V100M16", 32),
    (32000, 1000, 2, "", 32), (24000, 1000, 8, "2080", 32), (40000, 1000, 4, "", 29),
    (32000, 1000, 8, "", 29), (32000, 1000, 1, "T4", 29), (16000, 1000, 1, "", 25),
    (7000, 1000, 1, "V100M16", 25), (24000, 1000, 1, "T4", 25),
]
TYPICAL_NONGPU_31 = [
    (15700, 1000, 1, "", 2869), (11900, 1000, 1, "", 1893), (11400, 1000, 1, "", 1227),
    (1000, 0, 0, "", 736), (18710, 1000, 1, "", 485), (8200, 1000, 1, "", 379),
    (16400, 1000, 1, "", 331), (9810, 1000, 1, "", 197), (15200, 1000, 1, "", 187),
    (11200, 1000, 1, "", 181), (14200, 1000, 1, "", 176), (12000, 0, 0, "", 165),
    (14900, 1000, 1, "", 139), (60200, 1000, 4, "", 123), (64200, 1000, 8, "", 107),
    (32200, 1000, 4, "", 101), (17400, 1000, 2, "", 91), (30200, 1000, 2, "", 69),
    (16000, 1000, 1, "", 64), (15000, 1000, 1, "", 59), (64000, 1000, 8, "", 53),
    (15000, 0, 0, "", 53), (11910, 1000, 1, "", 53), (120200, 1000, 8, "", 48),
    (11300, 1000, 1, "", 37), (30000, 1000, 2, "", 32), (9800, 1000, 1, "", 32),
    (8000, 1000, 1, "", 32), (2000, 1000, 1, "", 27), (2000, 80, 1, "", 27),
    (1000, 1000, 1, "", 27),
]


def tp(rows):
    # percentage = (x / 100) / 100 as an exact rational: x / 10000
    return [dict(cpu=c, milli=m, num=n, type=t, pct=[x, 10000]) for (c, m, n, t, x) in rows]


def node(name, cpu_left, gpu_left, gpu_number, gpu_type, cpu_cap=64000):
    return dict(name=name, cpu_left=cpu_left, cpu_cap=cpu_cap, gpu_left=gpu_left, gpu_number=gpu_number,
                type=gpu_type)


DATA = {
    "typical_35": tp(TYPICAL_35),
    "typical_nongpu_31": tp(TYPICAL_NONGPU_31),
    "typical_single": tp([(6000, 465, 1, "", 933)]),
    # frag_test.go:100-121 and :142-163 (same inputs, InDelta 0.01)
    "frag_score_cases": [
        dict(src="frag_test.go:103-105", typical="typical_35",
             node=node("4x1080_used", 1000, [200, 1000, 1000, 500], 4, "1080"), want=2566.62),
        dict(src="frag_test.go:107-109", typical="typical_35",
             node=node("4x1080_full", 1000, [1000] * 4, 4, "1080"), want=3802.40),
        dict(src="frag_test.go:111-113", typical="typical_35",
             node=node("8x1080_full", 1000, [1000] * 8, 8, "1080"), want=7604.80),
        dict(src="frag_test.go:115-120", typical="typical_single",
             node=node("4x1080_used_lack_CPU", 1000, [200, 1000, 1000, 500], 4, "1080"), want=251.91,
             want_class="q4_lack_cpu", want_left_total=2700),
        # frag_test.go:123-140
        dict(src="frag_test.go:126-128", typical="typical_nongpu_31",
             node=node("8xP100_empty", 64000, [1000] * 8, 8, "P100"), want=887.20),
        dict(src="frag_test.go:131-133", typical="typical_nongpu_31",
             node=node("8xP100_halved", 32000, [1000] * 4 + [0] * 4, 8, "P100"), want=554.4),
        dict(src="frag_test.go:136-139", typical="typical_nongpu_31",
             node=node("8xP100_nocpu", 0, [1000] * 4 + [0] * 4, 8, "P100"), want=4000),
    ],
    # frag_test.go:165-185 GetGpuFragMilliByNodeResAndPodRes (exact)
    "frag_milli_cases": [
        dict(node=node("4x1080_used", 1000, [200, 1000, 1000, 500], 4, "1080"),
             pod=dict(cpu=100, milli=1000, num=2, type="1080"), want=700),
        dict(node=node("4x1080_full", 1000, [1000] * 4, 4, "1080"),
             pod=dict(cpu=100, milli=1000, num=2, type="1080"), want=0),
        dict(node=node("8x1080_full", 1000, [1000] * 8, 8, "1080"),
             pod=dict(cpu=100, milli=1000, num=2, type="1080"), want=0),
        dict(node=node("4x1080_used", 1000, [200, 1000, 1000, 500], 4, "1080"),
             pod=dict(cpu=100, milli=200, num=2, type="1080"), want=0),
    ],
    # gpu_packing_score_test.go:9-35 (exact)
    "packing_cases": [
        dict(node=node("Hello", 1000, [200, 1000, 1000, 500], 4, "1080", 96000),
             pod=dict(cpu=100, milli=1000, num=2, type="1080"), want=48),
        dict(node=node("Hello", 1000, [1000] * 4, 4, "1080", 96000),
             pod=dict(cpu=100, milli=1000, num=2, type="1080"), want=29),
        dict(node=node("Hello", 1000, [1000] * 8, 8, "1080", 96000),
             pod=dict(cpu=100, milli=1000, num=2, type="1080"), want=25),
        dict(node=node("Hello", 1000, [200, 1000, 1000, 500], 4, "1080", 96000),
             pod=dict(cpu=100, milli=200, num=2, type="1080"), want=93),
    ],
    # resource_test.go:9-17 Flatten("bellman").MilliGpu
    "flatten_cases": [
        dict(node=node("Hello", 1000, [200, 600, 350, 0], 4, "1080", 96000), want="600,350,200,0,0,0,0,0,"),
        dict(node=node("Hello", 300, [0, 0, 0, 0], 1, "", 96000), want="0,0,0,0,0,0,0,0,"),
        dict(node=node("Hello", 65535, [1000, 2000, 3000, 4000, 5000, 6000, 7000, 8000, 9000], 9, "", 96000),
             want="9000,8000,7000,6000,5000,4000,3000,2000,"),
    ],
    # resource_test.go:19-27 Add, :29-35 Sub (exact)
    "add_cases": [
        dict(node=node("Hello", 1000, [200, 0, 0, 500], 4, "1080", 96000),
             pod=dict(cpu=100, milli=1000, num=2, type="1080"), idl=[1, 2],
             want_cpu_left=1100, want_gpu_left=[200, 1000, 1000, 500]),
    ],
    # utils_test.go:25-55: node [MilliCpuLeft, total GPU milli left], pod [MilliCpu, MilliGpu * GpuNumber],
    # both normalized by cap, dot product within 1e-3 of want (the Go test's assert.InDelta)
    "dot_product_cases": [
        dict(node_vec=[1000, 200 + 600 + 350 + 0], pod_vec=[500, 500], cap=[2000, 4000], want=0.1609375),
        dict(node_vec=[1000, 1000 + 150], pod_vec=[500, 500], cap=[2000, 4000], want=0.1609375),
        dict(node_vec=[500, 500 + 75], pod_vec=[500, 500], cap=[2000, 4000], want=0.08046875),
        dict(node_vec=[0, 2000], pod_vec=[1000, 20], cap=[2000, 2000], want=0.01),
        dict(node_vec=[8000, 1000], pod_vec=[4000, 1000], cap=[8000, 1000], want=1.5),
    ],
    "sub_cases": [
        dict(node=node("Hello", 1000, [200, 1000, 1000, 500], 4, "1080", 96000),
             pod=dict(cpu=100, milli=1000, num=2, type="1080"),
             want_cpu_left=900, want_gpu_left=[200, 0, 0, 500]),
    ],
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "go_known_answers.json")
    with open(out, "w") as f:
        json.dump(DATA, f, indent=1)
    print("wrote", out)
