"""One HIP and one HSA runtime per process (DESIGN.md §1, round-3 verdict item 2).

torch ships its own libamdhip64 / libhsa-runtime64 and loads them under names the dynamic linker never
matches with /opt/rocm's, so a process that bound libksim_hip.so to /opt/rocm's runtime and then imported
torch held two of each, both opening the device at start and tearing it down at exit.  ksim.lib() now binds
the library to the runtime torch uses (ksim.hip_runtime_path).  These checks read /proc/self/maps of fresh
interpreters in the import orders the bench, the tests and the shard ranks use; no GPU is needed (mapping
a runtime does not initialise a device).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kubernetes-scheduler-simulator_amd")

PRELUDE = "import sys, json; sys.path[:0] = [%r, %r]\n" % (PKG, ROOT)


def maps_after(code, env=None):
    e = dict(os.environ)
    e.pop("KSIM_HIP_RUNTIME", None)
    e.update(env or {})
    out = subprocess.run([sys.executable, "-c", PRELUDE + code + "\nprint(json.dumps(ksim.hip_runtimes()))"],
                         capture_output=True, text=True, env=e, cwd=ROOT, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def torch_installed():
    import importlib.util
    return importlib.util.find_spec("torch") is not None


@pytest.mark.parametrize("order", ["ksim-then-torch", "torch-then-ksim", "torchrun-rank"])
def test_one_hip_and_hsa_runtime(order):
    if not torch_installed():
        pytest.skip("torch is not installed: only /opt/rocm's runtime exists")
    code = {
        "ksim-then-torch": "import ksim; ksim.lib(); import torch, torch.distributed",
        "torch-then-ksim": "import torch, torch.distributed; import ksim; ksim.lib()",
        # a bench.py rank under torchrun (world > 1): torch.distributed for the barrier, the engine, the shards
        "torchrun-rank": "import bench, ksim; import torch, torch.distributed; ksim.lib(); import ksim.shard, ksim.sweep",
    }[order]
    rt = maps_after(code)
    assert len(rt["hip"]) == 1 and len(rt["hsa"]) == 1, rt
    # and it is torch's: the runtime torch's own libraries and its RCCL are bound to
    assert os.path.dirname(rt["hip"][0]) == os.path.dirname(rt["hsa"][0])
    assert "torch" in rt["hip"][0]


def test_bench_world1_imports_no_torch():
    # bench.py at world 1 (the driver's default run) never imports torch: its one runtime is ksim's
    out = subprocess.run([sys.executable, "-c", PRELUDE + "import bench, ksim; ksim.lib(); import ksim.sweep\n"
                          "print('torch' in sys.modules)"], capture_output=True, text=True, cwd=ROOT, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == "False"
    src = open(os.path.join(ROOT, "bench.py")).read()
    main = src[src.index("def main():"):src.index("def _sharded_engine")]
    # torch appears in main() only under world > 1
    for i, ln in enumerate(main.splitlines()):
        if "import torch" in ln:
            assert "world > 1" in "\n".join(main.splitlines()[max(0, i - 8):i]), ln


def test_runtime_follows_a_preloaded_hsa():
    # under rocprofv3 /opt/rocm's HSA is mapped before the program runs: ksim then binds the HIP runtime
    # beside it, so HIP and HSA match (ksim.hip_runtime_path)
    hsa = "/opt/rocm/lib/libhsa-runtime64.so.1"
    if not os.path.exists(hsa):
        pytest.skip("no /opt/rocm HSA runtime")
    rt = maps_after("import ctypes; ctypes.CDLL(%r, mode=ctypes.RTLD_GLOBAL); import ksim; ksim.lib()" % hsa)
    assert len(rt["hip"]) == 1 and len(rt["hsa"]) == 1, rt
    assert os.path.dirname(rt["hip"][0]) == os.path.dirname(rt["hsa"][0]) and "torch" not in rt["hip"][0]


def test_system_runtime_without_torch():
    # a process that never imports torch may keep /opt/rocm's runtime (KSIM_HIP_RUNTIME=system)
    rt = maps_after("import ksim; ksim.lib()", env={"KSIM_HIP_RUNTIME": "system"})
    assert len(rt["hip"]) == 1 and len(rt["hsa"]) == 1, rt
    assert "torch" not in rt["hip"][0]


def test_hip_runtime_path_modes(monkeypatch):
    import ksim
    monkeypatch.setenv("KSIM_HIP_RUNTIME", "system")
    assert ksim.hip_runtime_path() is None
    monkeypatch.setenv("KSIM_HIP_RUNTIME", "/some/libamdhip64.so")
    assert ksim.hip_runtime_path() == "/some/libamdhip64.so"
    monkeypatch.setenv("KSIM_HIP_RUNTIME", "auto")
    p = ksim.hip_runtime_path()
    assert (p is None) == (not torch_installed())
