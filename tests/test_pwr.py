"""PWRScore (pkg/simulator/plugin/pwr_score.go) and its energy model, on the CPU.

The reference has no test for PWR (parity against reference outputs: unpinned).  The oracle
restates pwr_score.go + GetEnergyConsumptionNode (resource.go:536-563) + the const.go tables;
these tests pin it with hand-computed known answers from those formulas, then check the engine's
__host__ __device__ PWR math (ksim_device.hpp, compiled for the host) against the oracle on fuzzed
nodes.  tests/test_gpu_pwr.py covers the device runs.
"""
import ctypes as C
import os
import random
import subprocess

import pytest

import ksim
import pyoracle as O

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
CPU_MODELS = ["", "Intel-Xeon-8269CY", "Intel-Xeon-8163", "Intel-Xeon-ES-2682-V4", "Intel-Xeon-6326",
              "Intel-Xeon-8369B"]


def pwr(cpu_left, gl, gpu_type="T4", cap=64000, cpu_type="", cpu=4000, milli=500, num=1):
    n = O.node_res(cpu_left, gl, len(gl), gpu_type, cap, cpu_type)
    return O.pwr_score(n, O.pod_res(cpu, milli, num))


def test_energy_known_answers():
    # T4 x2 idle, 64 cores of the "" CPU profile (15 W idle / 120 W full, 16 cores per CPU):
    # 32 physical cores, 2 CPUs idle -> 30 W; 2 idle T4 -> 20 W
    assert O.energy_node(O.node_res(64000, [1000, 1000], 2, "T4", 64000)) == (0, 30.0, 20.0)
    # 4000 milli used -> 2 working cores -> one active CPU: 15 + 120; one T4 busy: 10 + 70
    assert O.energy_node(O.node_res(60000, [500, 1000], 2, "T4", 64000)) == (0, 135.0, 80.0)
    # odd capacity: ceil(31.5) = 32 real cores, floor(31.5) = 31 idle
    assert O.energy_node(O.node_res(63000, [1000], 1, "P100", 63000)) == (0, 135.0, 25.0)
    # Intel-Xeon-8163 (20 / 165 W, 24 cores): 48 real cores = 2 idle CPUs
    assert O.energy_node(O.node_res(96000, [1000] * 8, 8, "G2", 96000, "Intel-Xeon-8163")) == (0, 40.0, 240.0)
    # G3 uses the A100 profile (50 / 400 W)
    assert O.energy_node(O.node_res(96000, [0, 1000], 2, "G3", 96000))[2] == 450.0
    # no gpu-card-model label: no GPU term; unknown GPU / CPU models fail
    assert O.energy_node(O.node_res(64000, [], 0, "", 64000)) == (0, 30.0, 0.0)
    assert O.energy_node(O.node_res(64000, [1000], 1, "H100", 64000))[0] == -1
    assert O.energy_node(O.node_res(64000, [1000], 1, "T4", 64000, "EPYC"))[0] == -2


def test_pwr_score_known_answers():
    # share pod on a fresh T4 x2 node: both GPUs cost 50 -> 215 W; the first GPU is kept on ties
    assert pwr(64000, [1000, 1000]) == (-165, 0b01, 0)
    # GPU 0 already busy (300 left): packing onto it costs nothing, GPU 1 costs 60 W
    assert pwr(60000, [300, 1000], cpu=2000, milli=200) == (0, 0b01, 0)
    assert pwr(60000, [1000, 300], cpu=2000, milli=200) == (0, 0b10, 0)
    # whole-GPU pod: NodeResource.Sub takes GPU 0, AllocateExclusiveGpuId reports it
    assert pwr(64000, [1000, 1000], cpu=8000, milli=1000, num=1) == (-165, 0b01, 0)
    # CPU-only pod: only the CPU term moves
    assert pwr(64000, [1000, 1000], cpu=8000, milli=0, num=0) == (-105, 0, 0)
    # unknown GPU model: the Score fails
    assert pwr(64000, [1000], gpu_type="H100")[2] == 1


def test_normalize_known_answers():
    assert O.normalize_pwr([-165, 0, -60]) == [0, 100, 63]
    assert O.normalize_pwr([-7, -7, -7]) == [100, 100, 100]   # pwr_score.go:121-131: all equal -> 100
    assert O.normalize_pwr([-400, -1]) == [0, 100]


def test_policy_strings():
    assert ksim.parse_policy("PWR 500 FGD 500") == ("PWR+FGD", (500, 500))
    assert ksim.parse_policy("PWR 50 FGD 950") == ("PWR+FGD", (50, 950))
    assert ksim.parse_policy("PWR") == ("PWR", None)
    assert ksim.parse_policy("FGD") == ("FGD", None)


def test_trace_power_model():
    t = ksim.Trace.openb("default")
    pm = t.power_model()
    names = t.type_names()
    watts = {"T4": (10, 70), "A10": (30, 150), "P100": (25, 250), "V100M16": (30, 300), "V100M32": (30, 300),
             "G2": (30, 150), "G3": (50, 400)}
    for i, nm in enumerate(names):
        if nm == "":
            assert (pm.gpu_unlabelled >> i) & 1
            continue
        assert (pm.gpu_valid >> i) & 1, nm
        assert (pm.gpu_idle_w[i], pm.gpu_full_w[i]) == watts[nm]
    assert pm.cpu_valid == 0b111111
    assert [(pm.cpu_idle_w[c], pm.cpu_full_w[c], pm.cpu_cores[c]) for c in range(6)] == [
        (15, 120, 16), (20, 205, 26), (20, 165, 24), (15, 120, 16), (20, 185, 16), (20, 270, 32)]


@pytest.fixture(scope="module")
def dm():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    L = C.CDLL(os.path.join(HERE, "libdevmath.so"))
    I8 = C.c_int * 8
    L.dm_pwr_score.argtypes = [C.c_int, C.c_int, C.c_int, I8, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                               C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.dm_pwr_normalize.argtypes = [C.c_int, C.c_int, C.c_int]
    return L


def test_device_pwr_math_equals_oracle(dm):
    # vocabulary of the fuzz: the openb models, one model without an energy model, the empty label
    types = ["T4", "A10", "P100", "V100M16", "V100M32", "G2", "G3", "H100", ""]
    pm = ksim.PowerModel()
    ref = ksim.Trace.openb("default")
    rpm, rnames = ref.power_model(), ref.type_names()
    for i, nm in enumerate(types):
        if nm == "":
            pm.gpu_unlabelled |= 1 << i
        elif nm in rnames:
            j = rnames.index(nm)
            pm.gpu_idle_w[i], pm.gpu_full_w[i] = rpm.gpu_idle_w[j], rpm.gpu_full_w[j]
            pm.gpu_valid |= 1 << i
    for c in range(6):
        pm.cpu_idle_w[c], pm.cpu_full_w[c], pm.cpu_cores[c] = rpm.cpu_idle_w[c], rpm.cpu_full_w[c], rpm.cpu_cores[c]
    pm.cpu_valid = rpm.cpu_valid
    rnd = random.Random(7)
    checked = 0
    for _ in range(6000):
        ty = rnd.randrange(len(types))
        cnt = 0 if types[ty] == "" else rnd.choice([1, 2, 4, 8])
        gl = [rnd.choice([0, 1000, 1000, rnd.randint(0, 1000)]) for _ in range(cnt)] + [0] * (8 - cnt)
        cap = rnd.choice([32000, 63000, 64000, 96000, 128000, 88000])
        cpu_left = rnd.randint(0, cap)
        cm = rnd.randrange(6)
        k = rnd.random()
        if k < 0.2:
            cpu, milli, num = rnd.choice([1000, 4000, 12000]), 0, 0
        elif k < 0.6:
            cpu, milli, num = rnd.choice([2000, 4000, 8000]), rnd.choice([100, 250, 500, 999]), 1
        else:
            cpu, milli, num = rnd.choice([4000, 16000]), 1000, rnd.choice([1, 2, 4, 8])
        node = O.node_res(cpu_left, gl[:cnt], cnt, types[ty], cap, CPU_MODELS[cm])
        s_o, m_o, e_o = O.pwr_score(node, O.pod_res(cpu, milli, num))
        g, e = C.c_int(-1), C.c_int(0)
        s_d = dm.dm_pwr_score(cpu_left, cap, cm, (C.c_int * 8)(*gl), cnt, ty, cpu, milli, num,
                              C.addressof(pm), C.byref(g), C.byref(e))
        assert e.value == e_o, (types[ty], cnt)
        if e_o:
            continue
        # share pods: the chosen GPU is the score's; others report no GPU (Reserve takes
        # AllocateExclusiveGpuId, checked in test_device_math_cpu.py)
        fits = num == 1 and milli < 1000 and any(gl[i] >= milli for i in range(cnt))
        if num == 1 and milli < 1000 and not fits:
            continue  # Filter removes the node before Score
        assert s_d == s_o, (types[ty], cpu_left, cap, cm, gl, cpu, milli, num)
        if num == 1 and milli < 1000:
            assert (1 << g.value) == m_o
        checked += 1
    assert checked > 3000
    for _ in range(2000):
        xs = [rnd.randint(-600, 0) for _ in range(rnd.randint(1, 9))]
        lo, hi = min(xs), max(xs)
        assert [dm.dm_pwr_normalize(x, lo, hi) for x in xs] == O.normalize_pwr(xs)
