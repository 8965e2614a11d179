"""Writes tests/golden/log_golden.json: what the REFERENCE's own log parser makes of our log.

Pipeline, run here in this container only (the reference tree never travels to the GPU box):
  1. tests/log_case.py oracle_log -> the `simon apply` log of one openb run (243 nodes, 3000 events),
     FGD and PWR, written by ksim.analysis.write_log from the oracle's reports, power reports and
     final cluster;
  2. the reference's scripts/analysis.py log_to_csv (imported from /root/reference/scripts) on a
     directory holding that log -> analysis.csv (the per-experiment summary row), analysis_frag.csv,
     analysis_allo.csv, analysis_pwr.csv.
The JSON holds only data: the log's sha256, the summary row and the per-event power columns the
reference's script produced (the frag / alloc columns are already pinned by curve_golden.json).
Run:  python tests/golden/make_log_golden.py
"""
import hashlib
import importlib.util
import json
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path[:0] = [str(REPO / "kubernetes-scheduler-simulator_amd"), str(REPO / "oracle"), str(REPO / "tests")]

REF = Path("/root/reference")


def main():
    import pandas as pd
    import log_case
    spec = importlib.util.spec_from_file_location("ref_analysis", REF / "scripts" / "analysis.py")
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    out = {"case": dict(trace=log_case.TRACE, seed=log_case.SEED, tune=log_case.TUNE, stride=log_case.STRIDE,
                        n_events=log_case.N_EVENTS), "policies": {}}
    for policy in log_case.POLICIES:
        with tempfile.TemporaryDirectory() as td:
            logdir = Path(td) / "logs"
            logdir.mkdir()
            log = logdir / ("log-cc_tn1.3_ts42.yaml-sc_%s.yaml.log" % policy.lower())
            log_case.oracle_log(log, policy)
            sha = hashlib.sha256(log.read_bytes()).hexdigest()
            ref.log_to_csv(logdir, Path(td) / "analysis.csv")
            row = pd.read_csv(Path(td) / "analysis.csv").iloc[0].to_dict()
            pwr = pd.read_csv(Path(td) / "analysis_pwr.csv")
            power = {c.split("-")[-1]: [float(x) for x in pwr[c].tolist()] for c in pwr.columns}
            out["policies"][policy] = {"log_sha256": sha, "log_lines": sum(1 for _ in open(log)),
                                       "row": {k: float(v) for k, v in row.items()}, "power": power}
            print(policy, sha[:16], {k: row[k] for k in list(row)[:6]}, len(power.get("power_cluster", [])))
    with open(HERE / "log_golden.json", "w") as f:
        json.dump(out, f, sort_keys=True)
    print("wrote", HERE / "log_golden.json")


if __name__ == "__main__":
    main()
