"""Writes tests/golden/curve_golden.json: outputs of the REFERENCE's own Python harness on a
synthetic cluster-report log, to pin ksim.analysis (log format, parsing, discretization).

Pipeline run here, in this container only (the reference tree never travels to the GPU box):
  1. synth_reports(seed)  -> per-event reports (numpy PCG64, deterministic; the test rebuilds them)
  2. ksim.analysis.write_log -> logrus text log, as `simon apply` writes it
  3. the reference's scripts/analysis.py log_to_csv (imported from /root/reference/scripts)
     -> analysis_allo.csv / analysis_frag.csv
  4. the reference's experiments/analysis/merge_{alloc,frag,frag_ratio}_discrete.py, run
     unmodified through symlinks in a scratch tree (they locate their data relative to
     their own path) -> analysis_*_discrete.csv
The JSON holds only data: the seed, the sizes and the discretized curves.
Run:  python tests/golden/make_curve_golden.py
"""
import importlib.util
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO / "kubernetes-scheduler-simulator_amd"))

REF = Path("/root/reference")
SEEDS = (7, 8)
TOTAL_GPUS = 6212


def synth_reports(seed, total_gpus=TOTAL_GPUS):
    """A synthetic report stream shaped like a 130%-inflated openb run: arrivals grow by pod-sized
    steps (small ones early, some large jumps later so that integer arrived-% buckets are skipped
    and the +-1 fallback is exercised), allocation saturates near 95%, the bins are positive."""
    rng = np.random.default_rng(seed)
    cap = total_gpus * 1000
    arrived = used = 0
    out = []
    while arrived < 1.3 * cap:
        big = arrived > 0.6 * cap and rng.random() < 0.08
        milli = int(rng.integers(1, 9)) * 1000 * (20 if big else 1) if rng.random() < 0.5 else int(rng.integers(0, 1001))
        arrived += milli
        if used + milli <= 0.95 * cap:
            used += milli
        idle = float(cap - used)
        w = rng.random(7)
        w /= w.sum()
        bins = [float(idle * x) + float(rng.integers(0, 4)) / 8 for x in w]
        nodes = min(1213, used // 3000 + 1)
        out.append(dict(frag_bins=bins, used_nodes=int(nodes), used_gpus=int(min(total_gpus, used // 900 + 1)),
                        used_gpu_milli=int(used), total_gpus=int(total_gpus), arrived_gpu_milli=int(arrived),
                        used_cpu_milli=int(used * 10), arrived_cpu_milli=int(arrived * 10)))
    return out


def _read_row(csv, seed):
    import pandas as pd
    df = pd.read_csv(csv)
    row = df[df["seed"] == seed].iloc[0]
    return {str(k): float(row[str(k)]) for k in range(131) if str(k) in row.index and row[str(k)] == row[str(k)]}


def main():
    import ksim.analysis as A
    spec = importlib.util.spec_from_file_location("ref_analysis", REF / "scripts" / "analysis.py")
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    out = {"seeds": list(SEEDS), "total_gpus": TOTAL_GPUS, "curves": {}}
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        (td / "analysis").mkdir()
        for name in ("merge_alloc_discrete.py", "merge_frag_discrete.py", "merge_frag_ratio_discrete.py"):
            os.symlink(REF / "experiments" / "analysis" / name, td / "analysis" / name)
        for seed in SEEDS:
            reps = synth_reports(seed)
            logdir = td / "logs" / str(seed)
            logdir.mkdir(parents=True)
            A.write_log(logdir / ("log-cc_tn1.3_ts%d.yaml-sc_fgd.yaml.log" % seed), reps)
            run = td / "data" / "openb_pod_list_default" / "06-FGD" / "1.3" / str(seed)
            run.mkdir(parents=True)
            ref.log_to_csv(logdir, run / "analysis.csv")
            out["curves"][str(seed)] = {"n_events": len(reps)}
        for name in ("merge_alloc_discrete.py", "merge_frag_discrete.py", "merge_frag_ratio_discrete.py"):
            subprocess.run([sys.executable, str(td / "analysis" / name)], check=True, cwd=td / "analysis",
                           stdout=subprocess.DEVNULL)
        res = td / "analysis" / "analysis_results"
        for seed in SEEDS:
            c = out["curves"][str(seed)]
            c["alloc"] = _read_row(res / "analysis_allo_discrete.csv", seed)
            c["frag"] = _read_row(res / "analysis_frag_discrete.csv", seed)
            c["frag_ratio"] = _read_row(res / "analysis_frag_ratio_discrete.csv", seed)
    with open(HERE / "curve_golden.json", "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", HERE / "curve_golden.json", {s: len(out["curves"][str(s)]["alloc"]) for s in SEEDS})


if __name__ == "__main__":
    main()
