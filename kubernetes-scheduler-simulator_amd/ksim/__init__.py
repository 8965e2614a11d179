"""ksim -- Python binding of libksim_hip.so (the MI355X scoring engine).

A thin ctypes layer over the C ABI in include/ksim_engine.h and
include/ksim_trace.h.  It mirrors the reference's plugin vocabulary
(Filter / Score / Reserve / Unreserve / schedule cycle; FGDScore, BestFitScore,
DotProductScore, GpuPackingScore, GpuClusteringScore, RandomScore, PWRScore and the weighted
PWRScore + FGDScore combinations) so tests and
bench.py read like the reference's own tests.

There is no CPU fallback: compute calls raise KsimError(KSIM_ENODEV) when no
gfx950 device is present, and importing the extension fails loudly when
lib/libksim_hip.so has not been built.
"""
import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
# KSIM_LIB_PATH: another build of the library (A/B runs of two builds on one box); default the in-tree one
LIB_PATH = os.environ.get("KSIM_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libksim_hip.so")
DATA_DIR = os.path.join(REPO_DIR, "data", "openb")

KSIM_OK, KSIM_EINVAL, KSIM_ENOMEM, KSIM_EHIP, KSIM_ERANGE, KSIM_ESTATE, KSIM_ENOTSUP, KSIM_ENODEV, KSIM_EIO, KSIM_EPEER = \
    0, -1, -2, -3, -4, -5, -6, -7, -8, -9
KSIM_TYPE_ANY = 0xFFFFFFFF
MAX_GPU = 8
NUM_TAGS = 9

POLICY = {"FGD": 0, "BestFit": 1, "DotProd": 2, "GpuPacking": 3, "GpuClustering": 4, "Random": 5,
          "PWR": 6, "PWR+FGD": 7}
GPUSEL = {"best": 0, "worst": 1, "random": 2, "FGD": 3, "PWR": 4, "DotProd": 5}
# DotProduct's GpuPluginCfg (pkg/type/config.go:3-55)
DIM_EXT = {"merge": 0, "share": 1, "divide": 2, "extend": 3}
NORM = {"max": 0, "node": 1, "pod": 2}
# experiments/run_scripts/expected_run_scripts_0511.sh and generate_run_scripts.py:31-42:
# policy -> gpuSelMethod
DEFAULT_GPUSEL = {"FGD": "FGD", "BestFit": "best", "DotProd": "best", "GpuPacking": "best",
                  "GpuClustering": "best", "Random": "random", "PWR": "PWR", "PWR+FGD": "FGD"}


def parse_policy(name):
    """generate_run_scripts.py policy strings: "FGD", "PWR", "PWR 500 FGD 500", ... ->
    (POLICY key, weights or None)."""
    parts = name.replace("_", " ").split()  # the directory form "PWR_500_FGD_500" too (get_dir_name_from_method)
    if len(parts) == 4 and parts[0] == "PWR" and parts[2] == "FGD":
        return "PWR+FGD", (int(parts[1]), int(parts[3]))
    return name, None
SCHEDULED, UNSCHEDULABLE, ERROR, DELETED = 0, 1, 2, 3


class KsimError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = lib().ksim_strerror(code).decode() if _LIB is not None else str(code)
        super().__init__("%s: %s (%d)" % (what, msg, code))


class Node(C.Structure):
    _fields_ = [("cpu_alloc_milli", C.c_int64), ("mem_alloc_mib", C.c_int64), ("pods_alloc", C.c_int32),
                ("gpu_count", C.c_int32), ("gpu_type", C.c_int32), ("name_rank", C.c_uint32),
                ("cpu_used_milli", C.c_int64), ("mem_used_mib", C.c_int64), ("pods_used", C.c_int32),
                ("gpu_used_milli", C.c_int32 * MAX_GPU), ("tag_count", C.c_int32 * NUM_TAGS),
                ("cpu_model", C.c_int32)]


MAX_CPU_MODELS = 8


class PowerModel(C.Structure):
    _fields_ = [("gpu_idle_w", C.c_double * 32), ("gpu_full_w", C.c_double * 32),
                ("cpu_idle_w", C.c_double * MAX_CPU_MODELS), ("cpu_full_w", C.c_double * MAX_CPU_MODELS),
                ("cpu_cores", C.c_double * MAX_CPU_MODELS), ("gpu_valid", C.c_uint32),
                ("gpu_unlabelled", C.c_uint32), ("cpu_valid", C.c_uint32), ("reserved", C.c_uint32)]


class Pod(C.Structure):
    _fields_ = [("cpu_milli", C.c_int64), ("cpu_nz_milli", C.c_int64), ("mem_mib", C.c_int64),
                ("gpu_milli", C.c_int32), ("gpu_count", C.c_int32), ("type_mask", C.c_uint32),
                ("is_delete", C.c_int32), ("ref", C.c_int32), ("reserved", C.c_int32)]


class Typical(C.Structure):
    _fields_ = [("cpu_milli", C.c_int64), ("gpu_milli", C.c_int32), ("gpu_count", C.c_int32),
                ("type_mask", C.c_uint32), ("reserved", C.c_int32), ("freq", C.c_double)]


class Result(C.Structure):
    _fields_ = [("node", C.c_int32), ("gpu_mask", C.c_int32), ("score", C.c_int64), ("n_feasible", C.c_int32),
                ("status", C.c_int32)]


class Report(C.Structure):
    _fields_ = [("frag_bins", C.c_double * 7), ("used_nodes", C.c_int64), ("used_gpus", C.c_int64),
                ("used_gpu_milli", C.c_int64), ("total_gpus", C.c_int64), ("arrived_gpu_milli", C.c_int64),
                ("used_cpu_milli", C.c_int64), ("arrived_cpu_milli", C.c_int64)]


class PowerReport(C.Structure):
    _fields_ = [("cluster_w", C.c_double), ("cpu_w", C.c_double), ("gpu_w", C.c_double),
                ("invalid_nodes", C.c_int64)]


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("nodes_per_block", C.c_int32), ("steps_per_graph", C.c_int32),
                ("wgs_per_replica", C.c_int32), ("run_mode", C.c_int32), ("reserved", C.c_int32 * 3)]


class TraceNode(C.Structure):
    _fields_ = [("name", C.c_char * 64), ("cpu_milli", C.c_int64), ("mem_mib", C.c_int64),
                ("gpu_count", C.c_int32), ("gpu_type", C.c_int32)]


class TracePod(C.Structure):
    _fields_ = [("name", C.c_char * 64), ("cpu_milli", C.c_int64), ("mem_mib", C.c_int64),
                ("gpu_milli", C.c_int32), ("gpu_count", C.c_int32), ("type_mask", C.c_uint32),
                ("gpu_spec", C.c_char * 64)]


class TypicalCfg(C.Structure):
    _fields_ = [("is_involved_cpu_pods", C.c_int32), ("pod_popularity_threshold", C.c_int32),
                ("pod_increase_step", C.c_int32), ("reserved", C.c_int32), ("gpu_res_weight", C.c_double)]


class ReplayCfg(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("tune_ratio", C.c_double), ("shuffle", C.c_int32), ("informer_draws", C.c_int32)]


assert C.sizeof(Node) == 128 and C.sizeof(Pod) == 48 and C.sizeof(Typical) == 32 and C.sizeof(Result) == 24
assert C.sizeof(Report) == 112 and C.sizeof(PowerReport) == 32

_LIB = None

# name -> (restype, argtypes); the set must equal the functions declared in include/*.h
_P = C.POINTER
_VP = C.c_void_p
SIGNATURES = {
    "ksim_strerror": (C.c_char_p, [C.c_int]),
    "ksim_abi_version": (C.c_int, []),
    "ksim_build_id": (C.c_char_p, []),
    "ksim_device_count": (C.c_int, []),
    "ksim_engine_create": (C.c_int, [_P(Config), C.c_int, C.c_int, _P(_VP)]),
    "ksim_engine_destroy": (None, [_VP]),
    "ksim_engine_set_nodes": (C.c_int, [_VP, C.c_int, _P(Node)]),
    "ksim_engine_set_typical": (C.c_int, [_VP, C.c_int, _P(Typical), C.c_int]),
    "ksim_engine_set_policy": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int, C.c_uint64]),
    "ksim_engine_set_power_model": (C.c_int, [_VP, C.c_int, _P(PowerModel)]),
    "ksim_engine_set_weights": (C.c_int, [_VP, C.c_int, C.c_int32, C.c_int32]),
    "ksim_engine_set_replica_wgs": (C.c_int, [_VP, C.c_int, C.c_int]),
    "ksim_trace_power_model": (C.c_int, [_VP, _P(PowerModel)]),
    "ksim_engine_filter_score": (C.c_int, [_VP, C.c_int, _P(Pod), C.c_int32, _P(C.c_uint8), _P(C.c_int32),
                                           _P(C.c_int32)]),
    "ksim_engine_reserve": (C.c_int, [_VP, C.c_int, _P(Pod), C.c_int, C.c_int32, _P(C.c_int32)]),
    "ksim_engine_unreserve": (C.c_int, [_VP, C.c_int, _P(Pod), C.c_int, C.c_int32]),
    "ksim_engine_bind": (C.c_int, [_VP, C.c_int, _P(Pod), C.c_int, C.c_int32]),
    "ksim_engine_schedule": (C.c_int, [_VP, C.c_int, _P(Pod), C.c_int32, _P(Result)]),
    "ksim_engine_load_events": (C.c_int, [_VP, C.c_int, _P(Pod), C.c_int]),
    "ksim_engine_run": (C.c_int, [_VP]),
    "ksim_engine_get_results": (C.c_int, [_VP, C.c_int, _P(Result), C.c_int]),
    "ksim_engine_get_nodes": (C.c_int, [_VP, C.c_int, _P(Node)]),
    "ksim_engine_time_steps": (C.c_int, [_VP, C.c_int, _P(C.c_double)]),
    "ksim_engine_last_run_ms": (C.c_int, [_VP, _P(C.c_double)]),
    "ksim_engine_last_run_steps": (C.c_int, [_VP, _P(C.c_int64)]),
    "ksim_engine_last_run_wgs": (C.c_int, [_VP, _P(C.c_int)]),
    "ksim_engine_last_run_launches": (C.c_int, [_VP, _P(C.c_int), _P(C.c_int)]),
    "ksim_engine_last_run_gate": (C.c_int, [_VP, _P(C.c_int), _P(C.c_longlong)]),
    "ksim_engine_last_run_report_overlap": (C.c_int, [_VP, _P(C.c_int)]),
    "ksim_engine_last_run_kernels": (C.c_int, [_VP, C.c_char_p, C.c_int]),
    "ksim_engine_last_run_path": (C.c_int, [_VP, _P(C.c_int)]),
    "ksim_engine_set_report": (C.c_int, [_VP, C.c_int]),
    "ksim_engine_get_reports": (C.c_int, [_VP, C.c_int, _P(Report), C.c_int]),
    "ksim_engine_get_power_reports": (C.c_int, [_VP, C.c_int, _P(PowerReport), C.c_int]),
    "ksim_engine_last_report_ms": (C.c_int, [_VP, _P(C.c_double)]),
    "ksim_shard_comm_id": (C.c_int, [_P(C.c_uint8)]),
    "ksim_engine_set_shard": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int, C.c_int, _P(C.c_uint8)]),
    "ksim_shard_group_run": (C.c_int, [_P(_VP), C.c_int]),
    "ksim_shard_peer_handle": (C.c_int, [_VP, _P(C.c_uint8)]),
    "ksim_engine_set_shard_peers": (C.c_int, [_VP, _P(C.c_uint8)]),
    "ksim_engine_set_shard_exchange": (C.c_int, [_VP, C.c_void_p, C.c_void_p]),
    "ksim_engine_set_plugin_cfg": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int]),
    "ksim_trace_load_openb": (C.c_int, [C.c_char_p, C.c_char_p, _P(_VP)]),
    "ksim_trace_synthetic": (C.c_int, [_VP, C.c_int, C.c_int, C.c_uint64, _P(_VP)]),
    "ksim_trace_free": (None, [_VP]),
    "ksim_trace_num_nodes": (C.c_int, [_VP]),
    "ksim_trace_num_pods": (C.c_int, [_VP]),
    "ksim_trace_num_types": (C.c_int, [_VP]),
    "ksim_trace_type_name": (C.c_int, [_VP, C.c_int, C.c_char_p, C.c_int]),
    "ksim_trace_node_at": (C.c_int, [_VP, C.c_int, _P(TraceNode)]),
    "ksim_trace_pod_at": (C.c_int, [_VP, C.c_int, _P(TracePod)]),
    "ksim_trace_typical": (C.c_int, [_VP, _P(TypicalCfg), _P(Typical), C.c_int, _P(C.c_int)]),
    "ksim_trace_replay": (C.c_int, [_VP, _P(ReplayCfg), _P(Pod), C.c_int, _P(C.c_int), _P(C.c_int32), _P(Node),
                                    _P(C.c_int32)]),
    "ksim_go_rand": (C.c_int, [C.c_int64, C.c_int, C.c_int64, C.c_int, _P(C.c_int64)]),
    "ksim_trace_replay_go_state": (C.c_int, [_VP, _P(ReplayCfg), _P(C.c_uint64), _P(C.c_int32), _P(C.c_int64)]),
    "ksim_engine_set_go_stream": (C.c_int, [_VP, C.c_int, _P(C.c_uint64), C.c_int, C.c_int]),
}


def build(quiet=True):
    """Compile libksim_hip.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    cmd = ["make", "-C", PKG_DIR] + (["-s"] if quiet else [])
    subprocess.run(cmd, check=True)


def hip_runtime_path():
    """The HIP runtime file this process binds libksim_hip.so to, or None for the one its RUNPATH finds
    (/opt/rocm).  One HIP / HSA runtime per process: torch ships its own libamdhip64
    (SONAME libamdhip64.so.7) and its libtorch_hip NEEDs it as "libamdhip64.so", a name the dynamic
    linker never matches with /opt/rocm's libamdhip64.so.7.2.x, so a process that loads ksim first and
    torch later maps two runtimes, each opening the device.  The other way round the linker does match:
    loaded first by path, torch's copy satisfies this library's NEEDED libamdhip64.so.7 (by SONAME) and
    torch's own later load (same file).  So where torch is installed its runtime is the process's --
    unless an HSA or HIP runtime is already mapped (a profiler's preload: rocprofv3 maps /opt/rocm's HSA
    before the program starts), whose directory's libamdhip64 then binds, so that HIP and HSA match.
    KSIM_HIP_RUNTIME: auto (default: as above), torch (required), system (/opt/rocm's: a process that
    never imports torch), or a path to a libamdhip64 file."""
    mode = os.environ.get("KSIM_HIP_RUNTIME", "auto")
    if mode == "system":
        return None
    if mode not in ("auto", "torch"):
        return mode
    if mode == "auto":
        mapped = hip_runtimes()
        for path in mapped["hip"] + mapped["hsa"]:
            d = os.path.dirname(path)
            for name in ("libamdhip64.so.7", "libamdhip64.so"):
                if os.path.exists(os.path.join(d, name)):
                    return os.path.join(d, name)
    import importlib.util
    spec = importlib.util.find_spec("torch")  # (locates torch without importing it)
    path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so") if spec and spec.origin else None
    if path and os.path.exists(path):
        return path
    if mode == "torch":
        raise ImportError("KSIM_HIP_RUNTIME=torch but torch's libamdhip64.so was not found")
    return None


def hip_runtimes():
    """The HIP and HSA runtime files mapped into this process (/proc/self/maps): one of each is the
    contract (tests/test_runtime.py)."""
    out = {"hip": set(), "hsa": set()}
    with open("/proc/self/maps") as f:
        for ln in f:
            parts = ln.split()
            if len(parts) < 6:
                continue
            base = os.path.basename(parts[5])
            if base.startswith("libamdhip64.so"):
                out["hip"].add(os.path.realpath(parts[5]))
            elif base.startswith("libhsa-runtime64.so"):
                out["hsa"].add(os.path.realpath(parts[5]))
    return {k: sorted(v) for k, v in out.items()}


def device_reset():
    """hipDeviceReset on the process's HIP runtime: every queue, stream and allocation of the device released
    now rather than by the runtime's exit handlers (bench.py before it exits, KSIM_DEVICE_RESET=1; DESIGN.md
    §3 on the profiler's exit-time fault).  Only for a process that holds no other device state (no torch)."""
    rt = hip_runtimes()["hip"]
    if rt:
        return C.CDLL(rt[0]).hipDeviceReset()
    return None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libksim_hip.so not built (%s); run `make -C %s` or __graft_entry__.build()"
                              % (LIB_PATH, PKG_DIR))
        rt = hip_runtime_path()
        if rt is not None:
            C.CDLL(rt, mode=C.RTLD_GLOBAL)  # the process's HIP runtime, before the library binds one
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("KSIM_LIB_PATH") and not hasattr(L, name):
                continue  # an older library loaded for an A/B run: its missing entry points fail when called
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def check(rc, what):
    if rc != KSIM_OK:
        raise KsimError(rc, what)
    return rc


def device_count():
    return lib().ksim_device_count()


def build_id():
    """sha256 prefix of the sources the loaded library was built from (Makefile HASH_SRCS)."""
    return lib().ksim_build_id().decode()


def source_hash():
    """The same prefix computed from the sources in this tree (equal to build_id() unless the library is stale)."""
    import hashlib
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mk = open(os.path.join(pkg, "Makefile")).read()
    var = {}
    for line in mk.splitlines():
        for name in ("DEV_HDRS", "HASH_SRCS"):
            if line.startswith(name + " :="):
                var[name] = line.split(":=", 1)[1].split()
    files = []
    for f in var["HASH_SRCS"]:
        files += var["DEV_HDRS"] if f == "$(DEV_HDRS)" else [f]
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(pkg, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


GO_INT63, GO_INTN, GO_FLOAT64, GO_PERM, GO_SHUFFLE = range(5)


def go_rand(seed, op, n, arg=0):
    """n draws of Go's math/rand after rand.Seed(seed) (include/ksim_trace.h ksim_go_rand)."""
    out = (C.c_int64 * max(1, n))()
    check(lib().ksim_go_rand(seed, op, arg, n, out), "ksim_go_rand")
    if op == GO_FLOAT64:
        import struct
        return [struct.unpack("<d", struct.pack("<q", v))[0] for v in out[:n]]
    return list(out[:n])


# ---------------------------------------------------------------------------
# trace / replay driver
# ---------------------------------------------------------------------------
class Trace:
    """An openb trace (nodes + original workload) loaded by the C++ host driver."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def openb(cls, pod_list="default", data_dir=DATA_DIR, node_csv=None):
        pod_csv = pod_list if pod_list.endswith(".csv") else os.path.join(data_dir, "openb_pod_list_%s.csv" % pod_list)
        node_csv = node_csv or os.path.join(data_dir, "openb_node_list_gpu_node.csv")
        h = _VP()
        check(lib().ksim_trace_load_openb(node_csv.encode(), pod_csv.encode(), C.byref(h)), "ksim_trace_load_openb")
        return cls(h)

    def synthetic(self, n_nodes, n_pods, seed=0):
        h = _VP()
        check(lib().ksim_trace_synthetic(self.h, n_nodes, n_pods, seed, C.byref(h)), "ksim_trace_synthetic")
        return Trace(h)

    def __del__(self):
        if getattr(self, "h", None) and _LIB is not None:
            _LIB.ksim_trace_free(self.h)
            self.h = None

    @property
    def num_nodes(self):
        return lib().ksim_trace_num_nodes(self.h)

    @property
    def num_pods(self):
        return lib().ksim_trace_num_pods(self.h)

    def type_names(self):
        out = []
        buf = C.create_string_buffer(64)
        for i in range(lib().ksim_trace_num_types(self.h)):
            check(lib().ksim_trace_type_name(self.h, i, buf, 64), "type_name")
            out.append(buf.value.decode())
        return out

    def nodes(self):
        out = []
        n = TraceNode()
        for i in range(self.num_nodes):
            check(lib().ksim_trace_node_at(self.h, i, C.byref(n)), "node_at")
            out.append(dict(name=n.name.decode(), cpu=n.cpu_milli, mem=n.mem_mib, gpu=n.gpu_count, type=n.gpu_type))
        return out

    def pods(self):
        out = []
        p = TracePod()
        for i in range(self.num_pods):
            check(lib().ksim_trace_pod_at(self.h, i, C.byref(p)), "pod_at")
            out.append(dict(name=p.name.decode(), cpu=p.cpu_milli, mem=p.mem_mib, milli=p.gpu_milli,
                            num=p.gpu_count, mask=p.type_mask, spec=p.gpu_spec.decode()))
        return out

    def power_model(self):
        """The reference's PWR energy model for this trace's GPU models (const.go:41-124)."""
        pm = PowerModel()
        check(lib().ksim_trace_power_model(self.h, C.byref(pm)), "ksim_trace_power_model")
        return pm

    def typical(self, threshold=95, step=1, involve_cpu=True, gpu_res_weight=0.0):
        """GetTypicalPods with the paper's TypicalPodsConfig (generate_config_and_run.py:59-62)."""
        cfg = TypicalCfg(1 if involve_cpu else 0, threshold, step, 0, gpu_res_weight)
        n = C.c_int(0)
        cap = 4096
        arr = (Typical * cap)()
        check(lib().ksim_trace_typical(self.h, C.byref(cfg), arr, cap, C.byref(n)), "ksim_trace_typical")
        return arr, n.value

    def replay(self, seed, tune_ratio=1.3, shuffle=True, informer_draws=-1):
        """Event stream + empty cluster for one replica (SortClusterPods + tuning + node naming)."""
        cfg = ReplayCfg(seed, tune_ratio, 1 if shuffle else 0, informer_draws)
        nn = self.num_nodes
        nodes = (Node * nn)()
        prefix = (C.c_int32 * nn)()
        n = C.c_int(0)
        rc = lib().ksim_trace_replay(self.h, C.byref(cfg), None, 0, C.byref(n), None, nodes, prefix)
        if rc not in (KSIM_OK, KSIM_ERANGE):
            check(rc, "ksim_trace_replay")
        cap = max(1, n.value)
        events = (Pod * cap)()
        pidx = (C.c_int32 * cap)()
        check(lib().ksim_trace_replay(self.h, C.byref(cfg), events, cap, C.byref(n), pidx, nodes, prefix),
              "ksim_trace_replay")
        return Replay(events, n.value, np.ctypeslib.as_array(pidx)[: n.value].copy(), nodes,
                      np.ctypeslib.as_array(prefix).copy())

    def go_state(self, seed, tune_ratio=1.3, shuffle=True, informer_draws=-1):
        """Go's math/rand source after that replay's draws (ksim_trace_replay_go_state):
        (vec[607] list, tap, feed, draws since rand.Seed)."""
        cfg = ReplayCfg(seed, tune_ratio, 1 if shuffle else 0, informer_draws)
        vec = (C.c_uint64 * 607)()
        tf = (C.c_int32 * 2)()
        draws = C.c_int64(0)
        check(lib().ksim_trace_replay_go_state(self.h, C.byref(cfg), vec, tf, C.byref(draws)),
              "ksim_trace_replay_go_state")
        return list(vec), tf[0], tf[1], draws.value


class Replay:
    def __init__(self, events, n, pod_index, nodes, prefix):
        self.events, self.n, self.pod_index, self.nodes, self.prefix = events, n, pod_index, nodes, prefix

    def node_names(self, trace_nodes):
        return ["%04d-%s" % (self.prefix[i], trace_nodes[i]["name"]) for i in range(len(trace_nodes))]


# ---------------------------------------------------------------------------
# engine
# ---------------------------------------------------------------------------
class Engine:
    """R independent simulated clusters of N nodes on one MI355X."""

    def __init__(self, n_nodes, n_replicas=1, device=0, nodes_per_block=0, steps_per_graph=0, wgs_per_replica=0,
                 run_mode=0):
        """run_mode (ksim_config.run_mode): 0 auto (FGD: k_memo, else k_hmemo, else k_replay), 1 k_step per
        pod (hipGraph), 2 k_replay only, 3 k_memo required, 4 k_memo decider mode, 5 k_hmemo required
        (anything else: KsimError KSIM_EINVAL)."""
        self.N, self.R = n_nodes, n_replicas
        cfg = Config(device, nodes_per_block, steps_per_graph, wgs_per_replica, run_mode)
        h = _VP()
        check(lib().ksim_engine_create(C.byref(cfg), n_nodes, n_replicas, C.byref(h)), "ksim_engine_create")
        self.h = h
        self.n_events = [0] * n_replicas

    def close(self):
        if getattr(self, "h", None):
            lib().ksim_engine_destroy(self.h)
            self.h = None

    __del__ = close

    def set_nodes(self, r, nodes):
        check(lib().ksim_engine_set_nodes(self.h, r, nodes), "set_nodes")

    def set_typical(self, r, tp, n):
        check(lib().ksim_engine_set_typical(self.h, r, tp, n), "set_typical")

    def set_policy(self, r, policy="FGD", gpusel=None, seed=0, dim_ext=None, norm=None):
        """policy: a POLICY key or a generate_run_scripts.py string such as "PWR 500 FGD 500".
        DotProd: dim_ext / norm as generate_config_and_run.py's -dimext / -norm.  The default here is
        merge / max, the paper sweep's configuration (expected_run_scripts_0511.sh passes -dimext merge);
        NOTE the reference CLI's own default is -dimext share (generate_config_and_run.py:80), which also
        switches gpuSelMethod to DotProductScore -- pass dim_ext="share" to get that.  Like that script, a
        dim_ext other than merge selects GPUs with the DotProduct selector ("DotProd") unless gpusel says
        otherwise."""
        policy, weights = parse_policy(policy)
        if policy == "DotProd" and dim_ext not in (None, "merge") and gpusel is None:
            gpusel = "DotProd"  # generate_config_and_run.py:271-275
        gs = gpusel or DEFAULT_GPUSEL[policy]
        check(lib().ksim_engine_set_policy(self.h, r, POLICY[policy], GPUSEL[gs], seed), "set_policy")
        if weights:
            self.set_weights(r, *weights)
        if policy == "DotProd" or dim_ext is not None or norm is not None:
            self.set_plugin_cfg(r, dim_ext or "merge", norm or "max")

    def set_plugin_cfg(self, r, dim_ext="merge", norm="max"):
        check(lib().ksim_engine_set_plugin_cfg(self.h, r, DIM_EXT[dim_ext], NORM[norm]), "set_plugin_cfg")

    def set_replica_wgs(self, r, wgs):
        """Workgroups for replica r (0: the engine's choice); an FGD replica hinted wide runs k_memo at that width
        beside one-workgroup replicas (ksim_engine_set_replica_wgs)."""
        check(lib().ksim_engine_set_replica_wgs(self.h, r, wgs), "set_replica_wgs")

    def set_weights(self, r, w_pwr, w_fgd):
        check(lib().ksim_engine_set_weights(self.h, r, w_pwr, w_fgd), "set_weights")

    def set_power_model(self, r, pm):
        check(lib().ksim_engine_set_power_model(self.h, r, C.byref(pm)), "set_power_model")

    # plugin-level entry points
    def filter_score(self, r, pod, step=0):
        feas = (C.c_uint8 * self.N)()
        score = (C.c_int32 * self.N)()
        gpu = (C.c_int32 * self.N)()
        check(lib().ksim_engine_filter_score(self.h, r, C.byref(pod), step, feas, score, gpu), "filter_score")
        return (np.ctypeslib.as_array(feas).copy(), np.ctypeslib.as_array(score).copy(),
                np.ctypeslib.as_array(gpu).copy())

    def reserve(self, r, pod, node, step=0):
        m = C.c_int32(0)
        rc = lib().ksim_engine_reserve(self.h, r, C.byref(pod), node, step, C.byref(m))
        check(rc, "reserve")
        return m.value

    def unreserve(self, r, pod, node, gpu_mask):
        check(lib().ksim_engine_unreserve(self.h, r, C.byref(pod), node, gpu_mask), "unreserve")

    def bind(self, r, pod, node, gpu_mask):
        """Reserve + Bind on the devices of a predefined gpu-index annotation (open_gpu_share.go:260-271)."""
        check(lib().ksim_engine_bind(self.h, r, C.byref(pod), node, gpu_mask), "bind")

    def schedule(self, r, pod, step=0):
        res = Result()
        check(lib().ksim_engine_schedule(self.h, r, C.byref(pod), step, C.byref(res)), "schedule")
        return res

    # whole-trace device loop
    def load_events(self, r, events, n):
        check(lib().ksim_engine_load_events(self.h, r, events, n), "load_events")
        self.n_events[r] = n
        if not hasattr(self, "events"):
            self.events = [None] * self.R
        self.events[r] = np.ctypeslib.as_array(events)[:n].copy() if n else None

    def work(self, memo_replicas=None):
        """Work the last run() did, from its results: feasible (pod, node) score evaluations (Score runs on
        every feasible node, framework.go:635-710; the single-feasible shortcut skips it,
        generic_scheduler.go:158-164), and for the memoised FGD replicas (memo_replicas; default all) the
        (class, node) keys the refreshes recomputed (every class, on the node the previous event changed)."""
        score_evals, refreshes = 0, 0
        memo = set(range(self.R) if memo_replicas is None else memo_replicas)
        for r in range(self.R):
            n = self.n_events[r]
            if not n:
                continue
            res = self.results_array(r)
            ev = self.events[r]
            create = ev["is_delete"] == 0
            nf = res["n_feasible"].astype(np.int64)
            score_evals += int(nf[create & (nf > 1)].sum())
            changed = ((res["status"] == SCHEDULED) & create) | ((res["status"] == DELETED) & ~create & (res["node"] >= 0))
            keys = np.stack([ev["cpu_milli"], ev["cpu_nz_milli"], ev["mem_mib"], ev["gpu_milli"], ev["gpu_count"],
                             ev["type_mask"].astype(np.int64)], axis=1)[create]
            classes = len(np.unique(keys, axis=0)) if len(keys) else 0
            if r in memo:
                refreshes += int(changed[:-1].sum()) * classes
        return score_evals, refreshes

    def run(self):
        check(lib().ksim_engine_run(self.h), "run")
        ms = C.c_double(0)
        check(lib().ksim_engine_last_run_ms(self.h, C.byref(ms)), "last_run_ms")
        return ms.value

    def set_shard(self, rank, world, node_offset, n_global, comm_id=None):
        """Make this engine shard `rank` of a node-sharded cluster (see ksim_engine.h); call before
        set_nodes.  comm_id: bytes from shard_comm_id() (RCCL, one process per GPU) or None."""
        cid = None if comm_id is None else (C.c_uint8 * SHARD_ID_BYTES).from_buffer_copy(bytes(comm_id))
        check(lib().ksim_engine_set_shard(self.h, rank, world, node_offset, n_global, cid), "set_shard")
        self._shard = (rank, world)

    def shard_peer_handle(self):
        """This shard's exchange buffer as an IPC handle (bytes; ksim_shard_peer_handle)."""
        buf = (C.c_uint8 * SHARD_HANDLE_BYTES)()
        check(lib().ksim_shard_peer_handle(self.h, buf), "shard_peer_handle")
        return bytes(buf)

    def set_shard_peers(self, handles):
        """Map every shard's exchange buffer (handles: the ranks' shard_peer_handle() in rank order)."""
        blob = b"".join(handles)
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        check(lib().ksim_engine_set_shard_peers(self.h, buf), "set_shard_peers")

    def set_go_stream(self, r, state):
        """Random on Go's math/rand stream (ksim_engine_set_go_stream) from state = (vec[607], tap,
        feed[, ...]) as Trace.go_state returns it; None restores the hash contract."""
        if state is None:
            check(lib().ksim_engine_set_go_stream(self.h, r, None, 0, 0), "set_go_stream")
            return
        vec = (C.c_uint64 * 607)(*state[0])
        check(lib().ksim_engine_set_go_stream(self.h, r, vec, state[1], state[2]), "set_go_stream")

    def set_shard_exchange(self, gather):
        """Host exchange of a sharded engine (ksim_engine_set_shard_exchange): per pod step run()
        calls gather(record) with this shard's 4-word record (a list of ints) and expects the
        `world` shards' records in rank order (a flat list of 4 * world ints).  None clears it."""
        if gather is None:
            self._xfn = None
            check(lib().ksim_engine_set_shard_exchange(self.h, None, None), "set_shard_exchange")
            return
        world = getattr(self, "_shard", (0, 0))[1]  # (set_shard first: the engine refuses otherwise)
        self._xfn = exchange_cfunc(gather, world)  # kept alive as long as the engine may call it
        check(lib().ksim_engine_set_shard_exchange(self.h, C.cast(self._xfn, C.c_void_p), None),
              "set_shard_exchange")

    def set_report(self, enable=True):
        """Per-event cluster report (analysis.go:59-119) computed on the device by run()."""
        check(lib().ksim_engine_set_report(self.h, 1 if enable else 0), "set_report")

    def reports(self, r):
        """The report after every event of replica r: list of dicts (ksim_report fields)."""
        n = self.n_events[r]
        out = (Report * max(1, n))()
        check(lib().ksim_engine_get_reports(self.h, r, out, n), "get_reports")
        return [dict(frag_bins=list(out[i].frag_bins), used_nodes=out[i].used_nodes, used_gpus=out[i].used_gpus,
                     used_gpu_milli=out[i].used_gpu_milli, total_gpus=out[i].total_gpus,
                     arrived_gpu_milli=out[i].arrived_gpu_milli, used_cpu_milli=out[i].used_cpu_milli,
                     arrived_cpu_milli=out[i].arrived_cpu_milli) for i in range(n)]

    def report_arrays(self, r):
        """The reports of replica r as numpy arrays (frag_bins [n,7] float64, counters [n] int64)."""
        n = self.n_events[r]
        out = (Report * max(1, n))()
        check(lib().ksim_engine_get_reports(self.h, r, out, n), "get_reports")
        a = np.ctypeslib.as_array(out)[:n]
        keys = ["used_nodes", "used_gpus", "used_gpu_milli", "total_gpus", "arrived_gpu_milli", "used_cpu_milli",
                "arrived_cpu_milli"]
        d = {k: np.array(a[k]) for k in keys}
        d["frag_bins"] = np.array(a["frag_bins"])
        return d

    def power_reports(self, r):
        """The [Power] report after every event of replica r (analysis.go:24-56; needs set_power_model):
        list of dicts cluster_w / cpu_w / gpu_w / invalid_nodes."""
        n = self.n_events[r]
        out = (PowerReport * max(1, n))()
        check(lib().ksim_engine_get_power_reports(self.h, r, out, n), "get_power_reports")
        return [dict(cluster_w=out[i].cluster_w, cpu_w=out[i].cpu_w, gpu_w=out[i].gpu_w,
                     invalid_nodes=out[i].invalid_nodes) for i in range(n)]

    def last_report_ms(self):
        ms = C.c_double(0)
        check(lib().ksim_engine_last_report_ms(self.h, C.byref(ms)), "last_report_ms")
        return ms.value

    def last_run_steps(self):
        s = C.c_int64(0)
        check(lib().ksim_engine_last_run_steps(self.h, C.byref(s)), "last_run_steps")
        return s.value

    def last_run_path(self):
        """'k_replay' | 'k_memo' | 'memo+k_replay' | 'k_step' | 'sharded' | 'k_hmemo' | 'k_random_go' | 'k_scan1': the kernels
        the last run()
        used ('memo+k_replay': a memoised kernel for the FGD replicas, k_replay / k_scan1 / k_random_go for the
        others)."""
        k = C.c_int(0)
        check(lib().ksim_engine_last_run_path(self.h, C.byref(k)), "last_run_path")
        return ["k_replay", "k_memo", "memo+k_replay", "k_step", "sharded", "k_hmemo", "k_random_go", "k_scan1"][k.value]

    def last_run_launches(self):
        """(replay launches, side streams they ran on concurrently; 0 = back to back) of the last run()."""
        n, s = C.c_int(0), C.c_int(0)
        check(lib().ksim_engine_last_run_launches(self.h, C.byref(n), C.byref(s)), "last_run_launches")
        return n.value, s.value

    def last_run_kernels(self):
        """The replay kernels the last run() launched, in launch order (e.g. ['k_hmemo', 'k_scan1_mix'])."""
        buf = C.create_string_buffer(256)
        check(lib().ksim_engine_last_run_kernels(self.h, buf, 256), "last_run_kernels")
        return [k for k in buf.value.decode().split("+") if k]

    def last_run_gate(self):
        """(gate, timeouts): the last run()'s residency gate (0 none, 1 opened, -1 given up at its bound) and the
        gates this engine gave up so far."""
        g, t = C.c_int(0), C.c_longlong(0)
        check(lib().ksim_engine_last_run_gate(self.h, C.byref(g), C.byref(t)), "last_run_gate")
        return g.value, t.value

    def last_run_report_overlap(self):
        """Replicas whose cluster report the last run() overlapped with the longer replays (0: none)."""
        n = C.c_int(0)
        check(lib().ksim_engine_last_run_report_overlap(self.h, C.byref(n)), "last_run_report_overlap")
        return n.value

    def last_run_wgs(self):
        k = C.c_int(0)
        check(lib().ksim_engine_last_run_wgs(self.h, C.byref(k)), "last_run_wgs")
        return k.value

    def time_steps(self, n_steps):
        us = C.c_double(0)
        check(lib().ksim_engine_time_steps(self.h, n_steps, C.byref(us)), "time_steps")
        return us.value

    def results(self, r):
        n = self.n_events[r]
        out = (Result * max(1, n))()
        check(lib().ksim_engine_get_results(self.h, r, out, n), "get_results")
        return [(out[i].node, out[i].gpu_mask, out[i].score, out[i].n_feasible, out[i].status) for i in range(n)]

    def results_array(self, r):
        """The results of replica r as a numpy structured array (node, gpu_mask, score, n_feasible, status)."""
        n = self.n_events[r]
        out = (Result * max(1, n))()
        check(lib().ksim_engine_get_results(self.h, r, out, n), "get_results")
        return np.ctypeslib.as_array(out)[:n].copy()

    def nodes(self, r):
        out = (Node * self.N)()
        check(lib().ksim_engine_get_nodes(self.h, r, out), "get_nodes")
        return out


SHARD_ID_BYTES = 128
SHARD_HANDLE_BYTES = 128
# ksim_shard_exchange_fn
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_void_p)


def exchange_cfunc(gather, world):
    """Wrap gather(record: 4 ints) -> 4 * world ints as a ksim_shard_exchange_fn; any exception or
    a wrong-sized gather returns 1 (the engine then ends the run with KSIM_ESTATE)."""
    def fn(send, recv, _user):
        try:
            out = gather([send[i] for i in range(4)])
            if len(out) != 4 * world:
                return 1
            for i, v in enumerate(out):
                recv[i] = int(v) & 0xFFFFFFFFFFFFFFFF
            return 0
        except Exception:  # noqa: BLE001 -- reported to the engine, which ends the run
            import traceback
            traceback.print_exc()
            return 1
    return EXCHANGE_FN(fn)


def shard_comm_id():
    """An RCCL unique id (ncclGetUniqueId) for ksim_engine_set_shard; make it on one rank."""
    buf = (C.c_uint8 * SHARD_ID_BYTES)()
    check(lib().ksim_shard_comm_id(buf), "shard_comm_id")
    return bytes(buf)


def shard_group_run(engines):
    """Run an in-process shard group (engines[k] = shard k, all on one device); returns device ms."""
    arr = (_VP * len(engines))(*[e.h for e in engines])
    check(lib().ksim_shard_group_run(arr, len(engines)), "shard_group_run")
    ms = C.c_double(0)
    check(lib().ksim_engine_last_run_ms(engines[0].h, C.byref(ms)), "last_run_ms")
    return ms.value


def make_pod(cpu, milli=0, num=0, mem=0, type_mask=KSIM_TYPE_ANY, cpu_nz=None):
    p = Pod()
    p.cpu_milli, p.cpu_nz_milli, p.mem_mib = cpu, cpu if cpu_nz is None else cpu_nz, mem
    p.gpu_milli, p.gpu_count, p.type_mask, p.ref = milli, num, type_mask, -1
    return p
