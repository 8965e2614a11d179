"""Summarise a profile_config.sh (or profile_round.sh) run into pmc.json: per kernel the dispatches,
mean duration, HBM bytes (FETCH_SIZE x2 -- MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads -- + WRITE_SIZE, KiB), VALU instructions and the fp64 ones
(SQ_INSTS_VALU_{ADD,MUL,FMA}_F64), and the dominant kernel (largest total time) with its rooflines:
  hbm:  bytes per dispatch / duration vs 8 TB/s;
  valu: wave-level VALU instructions per dispatch / duration vs 256 CUs x 4 SIMDs x clock / 2 cycles
        (CDNA4 SIMDs are 32 lanes wide: a wave64 VALU instruction issues over 2 cycles, MI355X_MICROARCH.md;
        157.3 TF/s fp32 = 256 x 4 x 32 x 2 x 2.4 GHz; clock = GRBM_GUI_ACTIVE / 8 XCDs / duration, 2.4 GHz
        if that is implausible); the fp64 adds / muls / FMAs priced at their own rate, 4 cycles per wave64
        instruction (78.6 TF/s fp64 vector = 256 x 4 x 16 lanes x 2 flop x 2.4 GHz).
Usage: python3 scripts/pmc_summary.py DIR [bench args]"""
import csv
import glob
import json
import os
import re
import sys

HBM_PEAK = 8.0e12
CUS, SIMDS, XCDS = 256, 4, 8


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def kernel_of(name):
    """Kernel family from a (mangled or demangled) name: k_memo, k_hmemo, k_replay<policy>, ..."""
    for k in ("k_hinit_gk", "k_hinit_keys", "k_hmemo", "k_memo_finish", "k_pmemo", "k_memo", "k_random_go", "k_report_delta", "k_report_scan",
              "k_step_pwr", "k_step", "k_shard_commit", "k_shard_gather", "k_reserve", "k_advance"):
        if k in name:
            return k
    if "k_scan1_mix" in name:
        return "k_scan1_mix"
    if "k_scan1" in name:
        m = re.search(r"k_scan1<(\d+)", name) or re.search(r"k_scan1ILi(\d+)E", name)
        return "k_scan1<%s>" % (m.group(1) if m else "?")
    if "k_replay" in name:
        m = re.search(r"k_replay<(\d+)", name) or re.search(r"k_replayILi(\d+)E", name)
        return "k_replay<%s>" % (m.group(1) if m else "?")
    return name[:60]


def main(d, args=""):
    kt = rows(os.path.join(d, "kt", "**", "*kernel_trace.csv"))
    per = {}
    for r in kt:
        k = kernel_of(r.get("Kernel_Name", ""))
        e = per.setdefault(k, {"dispatches": 0, "total_ns": 0})
        e["dispatches"] += 1
        e["total_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])

    def counter(sub, name):
        acc = {}
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            if r.get("Counter_Name") != name:
                continue
            k = kernel_of(r.get("Kernel_Name", ""))
            a = acc.setdefault(k, {})
            a[r.get("Dispatch_Id", len(a))] = a.get(r.get("Dispatch_Id", len(a)), 0.0) + float(r["Counter_Value"])
        return {k: sum(v.values()) / len(v) for k, v in acc.items()}  # mean per dispatch (summed over SEs)

    fetch, write = counter("fetch", "FETCH_SIZE"), counter("write", "WRITE_SIZE")
    valu, waves, gui = counter("valu", "SQ_INSTS_VALU"), counter("valu", "SQ_WAVES"), counter("valu", "GRBM_GUI_ACTIVE")
    f64 = {n: counter("valu", "SQ_INSTS_VALU_%s_F64" % n) for n in ("ADD", "MUL", "FMA")}
    for k, e in per.items():
        e["mean_duration_ns"] = e["total_ns"] / e["dispatches"]
        t = e["mean_duration_ns"] * 1e-9
        if k in fetch and k in write:
            e["hbm_bytes_per_dispatch"] = (2 * fetch[k] + write[k]) * 1024
            e["hbm_frac"] = e["hbm_bytes_per_dispatch"] / t / HBM_PEAK
        if k in valu:
            e["valu_insts_per_dispatch"] = valu[k]
            e["waves_per_dispatch"] = waves.get(k)
            clock = gui[k] / XCDS / t if k in gui and t > 0 else 0.0
            if not 0.5e9 < clock < 3.0e9:
                clock = 2.4e9
            e["clock_hz"] = clock
            peak = CUS * SIMDS * clock / 2.0
            e["valu_peak_insts_per_s"] = peak
            e["valu_insts_per_s"] = valu[k] / t
            e["valu_frac"] = valu[k] / t / peak
            nf = sum(f64[n].get(k, 0.0) for n in f64)
            e["f64_insts_per_dispatch"] = nf
            e["f64_share"] = nf / valu[k] if valu[k] else 0.0
            e["f64_frac"] = nf / t / (CUS * SIMDS * clock / 4.0)
            e["nonf64_frac"] = (valu[k] - nf) / t / peak
    dom = max(per, key=lambda k: per[k]["total_ns"])
    out = {"args": args, "dominant": dict(kernel=dom, **per[dom]), "kernels": per,
           "note": "FETCH_SIZE x2 + WRITE_SIZE (KiB -> B), mean per dispatch; VALU fraction vs 2 cycles per wave64 "
                   "instruction (SIMD-32), fp64 at 4 cycles; clock from GRBM_GUI_ACTIVE / 8 XCDs"}
    # the fields bench.py reads (the dominant kernel)
    out.update(kernel=dom, hbm_bytes_per_dispatch=per[dom].get("hbm_bytes_per_dispatch"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
