"""Copies the Alibaba openb trace inputs used by the replay driver out of the
reference tree (data/csv/, read-only at /root/reference), keeping only the
columns the hot path reads.  Provenance: Fr4nz83/kubernetes-scheduler-simulator
@ 2024_08_07 data/csv/*.csv (trace data, not source).  The GPU box has no
/root/reference, so the committed copies are what tests and bench.py read.

Run:  python data/make_openb_data.py [/root/reference]
"""
import csv
import os
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = os.path.join(REF, "data", "csv")
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "openb")
TRACES = ["default", "cpu050", "cpu100", "cpu200", "cpu250", "gpushare40", "gpushare60", "gpushare80",
          "gpushare100", "gpuspec10", "gpuspec20", "gpuspec25", "gpuspec33", "multigpu20", "multigpu30",
          "multigpu40", "multigpu50"]
POD_COLS = ["name", "cpu_milli", "memory_mib", "num_gpu", "gpu_milli", "gpu_spec"]


def copy(src, dst, cols):
    with open(src, newline="") as f, open(dst, "w", newline="") as g:
        r = csv.DictReader(f)
        keep = [c for c in cols if c in r.fieldnames]
        w = csv.writer(g, lineterminator="\n")
        w.writerow(keep)
        for row in r:
            w.writerow([row[c] for c in keep])


if __name__ == "__main__":
    os.makedirs(DST, exist_ok=True)
    copy(os.path.join(SRC, "openb_node_list_gpu_node.csv"), os.path.join(DST, "openb_node_list_gpu_node.csv"),
         ["sn", "cpu_milli", "memory_mib", "gpu", "model"])
    for t in TRACES:
        name = "openb_pod_list_%s.csv" % t
        copy(os.path.join(SRC, name), os.path.join(DST, name), POD_COLS)
    print("wrote", DST)
