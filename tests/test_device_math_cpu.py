"""The engine's __host__ __device__ math (ksim_device.hpp), compiled for the host, against the oracle.

Fuzzed node states x pods x typical tables: F, FGD score + GPU choice, Filter, BestFit, DotProduct,
GpuPacking, GpuClustering and AllocateExclusiveGpuId must agree bit for bit.  This is the same source
the gfx950 kernels inline; tests/test_gpu_parity.py covers the device execution itself.
"""
import ctypes as C
import os
import random
import subprocess

import pytest

import helpers
import ksim
import pyoracle as O

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


@pytest.fixture(scope="module")
def dm():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    L = C.CDLL(os.path.join(HERE, "libdevmath.so"))
    I8 = C.c_int * 8
    L.dm_go_exp.argtypes = [C.c_double]
    L.dm_go_exp.restype = C.c_double
    L.dm_frag_F.argtypes = [C.c_int, I8, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_double)]
    L.dm_frag_F.restype = C.c_double
    L.dm_fgd_score.argtypes = [C.c_int, I8, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                               C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_int)]
    L.dm_filter.argtypes = [C.c_int, C.c_int, I8, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                            C.c_uint]
    L.dm_filter_scan.argtypes = L.dm_filter.argtypes
    L.dm_bestfit.argtypes = [C.c_int, I8, C.c_int, C.c_int, C.c_int, C.c_int]
    L.dm_dotprod.argtypes = [C.c_int, I8, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
    L.dm_dotprod_mm.argtypes = [C.c_int, I8, C.c_int, C.c_int, C.c_int, C.c_int]
    L.dm_go_tanh.argtypes = [C.c_double]
    L.dm_go_tanh.restype = C.c_double
    L.dm_packing.argtypes = [I8, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
    L.dm_clustering.argtypes = [C.c_int * 9, I8, C.c_int, C.c_int, C.c_int]
    L.dm_clustering_mask.argtypes = [C.c_int * 9, I8, C.c_int, C.c_int, C.c_int]
    L.dm_exclusive.argtypes = [I8, C.c_int, C.c_int, C.c_int]
    L.dm_frag_bins7.argtypes = [C.c_int, I8, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_double),
                                C.c_double * 7]
    L.dm_fix80.argtypes = [C.c_double, C.POINTER(C.c_uint64), C.POINTER(C.c_int64)]
    return L


TYPES = ["A10", "G2", "G3", "P100", "T4", "V100M16", "V100M32"]


def rand_gl(rnd, cnt):
    gl = [rnd.choice([0, 1000, 1000, 1000, rnd.randint(0, 1000), rnd.randint(0, 1000)]) for _ in range(cnt)]
    return gl + [0] * (8 - cnt)


def rand_pod(rnd):
    k = rnd.random()
    if k < 0.15:
        return rnd.choice([1000, 4000, 12000, 32000]), 0, 0
    if k < 0.55:
        return rnd.choice([2000, 4000, 6000, 8000, 11908]), rnd.choice([100, 250, 300, 460, 500, 810, 999]), 1
    return rnd.choice([4000, 8000, 16000, 64000]), 1000, rnd.choice([1, 1, 1, 2, 4, 8])


def table(tlist):
    tpi = (C.c_int * (4 * len(tlist)))()
    tpf = (C.c_double * len(tlist))()
    for i, (cpu, milli, num, spec, f) in enumerate(tlist):
        mask = 0
        for x in filter(None, spec.split("|")):
            mask |= 1 << TYPES.index(x)
        tpi[4 * i:4 * i + 4] = [cpu, milli, max(num, 1), C.c_int(mask or -1).value]
        tpf[i] = f
    return tpi, tpf


@pytest.fixture(scope="module")
def tables():
    t = ksim.Trace.openb("gpuspec33")
    d = ksim.Trace.openb("default")
    return [helpers.oracle_typical(d), helpers.oracle_typical(t)]


def test_go_exp_host_equals_oracle(dm):
    rnd = random.Random(1)
    for _ in range(20000):
        x = rnd.uniform(-30, 30) if rnd.random() < 0.9 else rnd.uniform(-1e-6, 1e-6)
        assert dm.dm_go_exp(x) == O.lib().orc_go_exp(x)


def test_frag_F_and_fgd_score_fuzz(dm, tables):
    rnd = random.Random(2)
    for tlist in tables:
        tpi, tpf = table(tlist)
        otp = O.typical(tlist)
        for _ in range(1500):
            cnt = rnd.choice([1, 2, 4, 8])
            gl = rand_gl(rnd, cnt)
            cpu_left = rnd.choice([0, 500, 2000, 8000, 32000, 64000, 96000])
            ty = rnd.randrange(len(TYPES))
            node = O.node_res(cpu_left, gl[:cnt], cnt, TYPES[ty], 96000)
            f = dm.dm_frag_F(cpu_left, (C.c_int * 8)(*gl), ty, len(tlist), tpi, tpf)
            assert f == O.frag_score(node, otp)
            cpu, milli, num = rand_pod(rnd)
            pr = O.pod_res(cpu, milli, num, "")
            # only states that pass Filter are scored by the reference
            if not dm.dm_filter(cpu_left, 10 ** 6, (C.c_int * 8)(*gl), cnt, ty, 10, cpu, 0, milli, num, 0xFFFFFFFF):
                continue
            g = C.c_int(0)
            s = dm.dm_fgd_score(cpu_left, (C.c_int * 8)(*gl), cnt, ty, cpu, milli, num, len(tlist), tpi, tpf,
                                C.byref(g))
            ws, wm = O.fgd_score(node, pr, otp)
            assert s == ws
            if num == 1 and milli < 1000:
                assert wm == (1 << g.value)


def test_cheap_scores_and_exclusive_fuzz(dm):
    rnd = random.Random(3)
    L = O.lib()
    for _ in range(20000):
        cnt = rnd.choice([1, 2, 4, 8])
        gl = rand_gl(rnd, cnt)
        cpu_left = rnd.choice([0, 100, 2000, 8000, 32000, 64000, 128000])
        cpu, milli, num = rand_pod(rnd)
        node = O.node_res(cpu_left, gl[:cnt], cnt, "G2", 128000)
        pr = O.pod_res(cpu, milli, num, "")
        g8 = (C.c_int * 8)(*gl)
        assert dm.dm_bestfit(cpu_left, g8, cnt, cpu, milli, num) == L.orc_best_fit_score(C.byref(node), C.byref(pr))
        g = C.c_int(0)
        want = L.orc_dot_product_score(C.byref(node), C.byref(pr))
        assert dm.dm_dotprod(cpu_left, g8, cnt, cpu, milli, num, 128000, 0, C.byref(g)) == want
        assert dm.dm_dotprod_mm(cpu_left, g8, cnt, cpu, milli, num) == want
        if milli > 0:
            e1, e2 = C.c_int(0), C.c_int(0)
            a = dm.dm_packing(g8, cnt, cpu, milli, num, C.byref(e1))
            b = L.orc_packing_score(C.byref(node), C.byref(pr), C.byref(e2))
            assert e1.value == e2.value and (e1.value or a == b)
            assert dm.dm_exclusive(g8, cnt, milli, num) == L.orc_allocate_exclusive_gpu_id(C.byref(node),
                                                                                            C.byref(pr))
        if milli > 0:  # GpuPacking's closed forms (whole GPUs, one share) against its general loop's shapes too
            for m2, n2 in ((milli, num), (1000, 0), (1000, rnd.choice([1, 2, 3])), (rnd.choice([1, 300, 999, 1000]), 1)):
                pr2 = O.pod_res(cpu, m2, n2, "")
                e1, e2 = C.c_int(0), C.c_int(0)
                a = dm.dm_packing(g8, cnt, cpu, m2, n2, C.byref(e1))
                b = L.orc_packing_score(C.byref(node), C.byref(pr2), C.byref(e2))
                assert e1.value == e2.value and (e1.value or a == b), (gl, cnt, m2, n2, a, b)
        tags = [rnd.choice([0, 0, 0, 1, 2]) for _ in range(9)]
        tag = -1 if num == 0 else (0 if (num == 1 and milli < 1000) else num)
        want = L.orc_clustering_score(C.byref(node), C.byref(pr), tag, (C.c_int32 * 9)(*tags))
        assert dm.dm_clustering((C.c_int * 9)(*tags), g8, cnt, milli, num) == want
        assert dm.dm_clustering_mask((C.c_int * 9)(*tags), g8, cnt, milli, num) == want  # k_scan1's presence bits


def test_frag_bins7_fuzz(dm, tables):
    # the report's per-node term: every NodeGpuShareFragAmount bin bit-identical to the oracle
    rnd = random.Random(4)
    for tlist in tables:
        tpi, tpf = table(tlist)
        otp = O.typical(tlist)
        for _ in range(1500):
            cnt = rnd.choice([1, 2, 4, 8])
            gl = rand_gl(rnd, cnt)
            cpu_left = rnd.choice([0, 500, 2000, 8000, 32000, 64000, 96000])
            ty = rnd.randrange(len(TYPES))
            out = (C.c_double * 7)()
            dm.dm_frag_bins7(cpu_left, (C.c_int * 8)(*gl), ty, len(tlist), tpi, tpf, out)
            assert list(out) == O.frag_bins(O.node_res(cpu_left, gl[:cnt], cnt, TYPES[ty], 96000), otp)


def test_fix80_exact_scaling(dm):
    # x * 2^80 as an integer, exactly, for report-sized values (and truncation below 2^-80)
    from fractions import Fraction
    rnd = random.Random(5)
    vals = [0.0, 1.0, 0.5, 2.0 ** -80, 2.0 ** -81, 1e-30, 123456.789, 8e8, 2.0 ** 45]
    vals += [rnd.uniform(0, 1e6) for _ in range(2000)] + [rnd.random() * 10 ** rnd.randint(-20, 8) for _ in range(2000)]
    for x in vals:
        lo, hi = C.c_uint64(0), C.c_int64(0)
        dm.dm_fix80(x, C.byref(lo), C.byref(hi))
        got = (hi.value << 64) | lo.value
        assert got == int(Fraction(x) * 2 ** 80), x


def test_fgd_score_threshold_table(dm):
    # k_memo scores through a table of the 100 score steps of int64(sigmoid(delta/1000)*100)
    # (ksim_device.hpp build_score_thresholds / fgd_score_lookup): equal to the direct
    # expression (and so to the oracle's) on random deltas and on every step +-3 ulps
    import struct
    th = (C.c_double * 102)()
    dm.dm_score_thresholds.argtypes = [C.c_double * 102]
    dm.dm_score_lookup.argtypes = [C.c_double, C.c_double * 102]
    dm.dm_score_of_delta.argtypes = [C.c_double]
    assert dm.dm_score_thresholds(th) == 1
    L = O.lib()

    def direct(x):
        return dm.dm_score_of_delta(x)

    def nxt(x, k):
        b = struct.unpack("<q", struct.pack("<d", x))[0]
        key = b if b >= 0 else -(b & 0x7FFFFFFFFFFFFFFF)
        key += k
        b = key if key >= 0 else (-key) | (1 << 63)
        return struct.unpack("<d", struct.pack("<Q", b))[0]

    rnd = random.Random(6)
    xs = [rnd.uniform(-1e4, 1e4) for _ in range(40000)] + [rnd.uniform(-50, 50) for _ in range(20000)]
    xs += [0.0, -0.0, 1e9, -1e9, 1e300, -1e300]
    for k in range(1, 101):
        xs += [nxt(th[k], j) for j in range(-3, 4)]
    for x in xs:
        s = direct(x)
        assert dm.dm_score_lookup(x, th) == s, x
        # the oracle computes the same expression from (cur, new) = (x, 0)
        sig = 1.0 / (1.0 + L.orc_go_exp(-(x / 1000)))
        assert s == int(sig * 100)
    assert [direct(th[k]) for k in range(1, 101)] == list(range(1, 101))


@pytest.mark.parametrize("dim", [O.DIM_MERGE, O.DIM_SHARE, O.DIM_DIVIDE, O.DIM_EXTEND])
@pytest.mark.parametrize("norm", [O.NORM_MAX, O.NORM_NODE, O.NORM_POD])
def test_dotprod_variants_fuzz(dm, dim, norm):
    # every dimExtMethod x normMethod: the device's single-loop restatement against the oracle's
    # literal GenerateSchedulingMatchGroups lists -- the score and the best group's GPU id
    rnd = random.Random(100 + 4 * norm + dim)
    for _ in range(6000):
        cnt = rnd.choice([0, 1, 2, 4, 6, 8])
        gl = rand_gl(rnd, cnt) if cnt else [0] * 8
        cpu_left = rnd.choice([0, 100, 2000, 8000, 32000, 64000, 96000])
        cap = rnd.choice([cpu_left, 96000, 128000])
        cpu, milli, num = rand_pod(rnd)
        cpu = max(cpu, 100)  # PodResource.MilliCpu carries the non-zero default
        node = O.node_res(cpu_left, gl[:cnt], cnt, "G2", cap)
        pr = O.pod_res(cpu, milli, num, "")
        g = C.c_int(0)
        s = dm.dm_dotprod(cpu_left, (C.c_int * 8)(*gl), cnt, cpu, milli, num, cap, dim | norm << 4, C.byref(g))
        ws, wg = O.dot_product_score(node, pr, dim, norm)
        assert (s, g.value) == (ws, wg), (cpu_left, gl[:cnt], cap, cpu, milli, num)


def test_go_tanh_host_equals_oracle(dm):
    rnd = random.Random(5)
    xs = [0.0, -0.0, 1e-300, 0.1, 0.5, 0.6249999, 0.625, 0.7, 1.0, 2.0, 10.0, 44.0, 44.02, 45.0, 300.0]
    xs += [rnd.uniform(-3, 3) for _ in range(4000)] + [rnd.uniform(0, 0.3) for _ in range(2000)]
    for x in xs + [-x for x in xs]:
        a, b = dm.dm_go_tanh(x), O.go_tanh(x)
        assert a == b or (a != a and b != b), x
    # Go's tanh: exact at 0 and saturated beyond 0.5 * log(2**127)
    assert O.go_tanh(50.0) == 1.0 and O.go_tanh(-50.0) == -1.0


def test_filter_scan_equals_filter_node(dm):
    # k_scan1's branch-free Filter (filter_scan) against filter_node, which every other path and the GPU parity
    # tests check against the oracle: every corner -- no pod slot left, zero requests, CPU / memory at and past
    # the boundary, GPU-less nodes, a model the pod does not accept, share / whole / partial multi-GPU requests
    rnd = random.Random(11)
    n = 0
    for _ in range(40000):
        cnt = rnd.choice([0, 1, 2, 4, 8])
        gl = rand_gl(rnd, cnt) if cnt else [0] * 8
        cpu_left = rnd.choice([0, 50, 100, 1000, 4000, 32000, 96000, -5])
        mem_left = rnd.choice([0, 100, 1024, 10 ** 6])
        pods_left = rnd.choice([0, 1, 5])
        ty = rnd.randrange(len(TYPES))
        cpu = rnd.choice([0, 100, 1000, 4000, 32000, 96000])
        mem = rnd.choice([0, 100, 1024])
        k = rnd.random()
        if k < 0.2:
            milli, num = 0, 0
        elif k < 0.6:
            milli, num = rnd.choice([100, 250, 500, 999, 1000]), 1
        elif k < 0.85:
            milli, num = 1000, rnd.choice([2, 4, 8])
        else:
            milli, num = rnd.choice([300, 500]), rnd.choice([0, 2, 3])
        mask = rnd.choice([0xFFFFFFFF, 1 << ty, 1 << ((ty + 1) % len(TYPES)), 0])
        args = (cpu_left, mem_left, (C.c_int * 8)(*gl), cnt, ty, pods_left, cpu, mem, milli, num, mask)
        a, b = dm.dm_filter(*args), dm.dm_filter_scan(*args)
        assert a == b, args
        n += a
    assert 1000 < n < 39000  # both outcomes well represented
