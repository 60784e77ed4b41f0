"""Summarise PMC passes (scripts/pmc.sh output dirs) into profiles/: per config, the dominant
kernel's counters averaged over its dispatches, and the HBM bytes per launch computed as
MI355X_MICROARCH.md prescribes for gfx950: (2 x FETCH_SIZE + WRITE_SIZE) KiB.

    python scripts/pmc_json.py profiles/r03_pmc.json profiles/kernel1_pmc.json \\
        c2=gpurun_out/pmc_c2:k_pileup:pileup:1 c3=gpurun_out/pmc_c3:k_rc:rc:3 \\
        c5=gpurun_out/pmc_c5:k_sum_reads+k_sum_exact+k_sum_buffers:solo_sum:1:24

Each spec is dir:kernel-name-substring:bench-kernel-key:batch-copies[:launches-per-step[:mbq]]
(name c3_q20 for the C3 run at --mbq 20: bench.py looks entries up as <config>[_q<mbq>]).  The
second file is what bench.py reads as roofline.traffic: it carries the sha of the library the
counters were read from (bench.py reports traffic null for any other build).
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summarise(d, pat):
    """Per-dispatch averages of the kernels matching pat; "a+b+c" sums the averages of a, b and
    c (kernels that run once each per launch of the step's unit, e.g. C5's three summary kernels
    per contig)."""
    if "+" in pat:
        parts = [summarise(d, p) for p in pat.split("+")]
        out = {}
        for k in parts[0]:
            if k != "dispatches" and all(k in q for q in parts):
                out[k] = sum(q[k] for q in parts)
        out["dispatches"] = min(q["dispatches"] for q in parts)
        return out
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"] and (pat != "k_pileup" or "k_pileup_solo" not in r["Kernel_Name"]):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: sum(v) / len(v) for k, v in sorted(agg.items())}
    out["dispatches"] = max((len(v) for v in agg.values()), default=0)
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        out["hbm_bytes_per_launch"] = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024
    return out


def main():
    with open(os.path.join(REPO, "basecount_amd", "libbasecount_hip.so"), "rb") as fh:
        sha = hashlib.sha256(fh.read()).hexdigest()[:16]
    full = {"_doc": "rocprofv3 PMC passes (separate --pmc runs with --kernel-trace only, scripts/pmc.sh) of "
                    "`bench.py --lean --launch eager`, averaged per dispatch of the named kernel; FETCH_SIZE / "
                    "WRITE_SIZE in KiB; hbm_bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 "
                    "(gfx950 FETCH_SIZE counts half of 16 B/lane streaming reads, MI355X_MICROARCH.md).",
            "lib_sha16": sha}
    traffic = {"_doc": "HBM traffic per launch (per step for c5: 24 launches) of each config's dominant kernel "
                       "from the PMC passes in the companion r*_pmc.json; bench.py uses an entry only when "
                       "lib_sha16 matches the library it measures and copies matches its batch rotation.",
               }
    for arg in sys.argv[3:]:
        name, spec = arg.split("=", 1)
        parts = spec.split(":")
        d, pat, key, copies = parts[0], parts[1], parts[2], int(parts[3])
        per_step = int(parts[4]) if len(parts) > 4 else 1
        mbq = int(parts[5]) if len(parts) > 5 else 0
        s = summarise(d, pat)
        full[name] = dict(kernel=pat, **s)
        if "hbm_bytes_per_launch" in s:
            traffic[name] = {"mbq": mbq, "kernel": key, "copies": copies, "lib_sha16": sha,
                             "fetch_size_kib": s["FETCH_SIZE"], "write_size_kib": s["WRITE_SIZE"],
                             "hbm_bytes_per_launch": s["hbm_bytes_per_launch"] * per_step,
                             "dispatches": s["dispatches"], "launches_per_step": per_step}
    with open(sys.argv[1], "w") as fh:
        json.dump(full, fh, indent=1)
    with open(sys.argv[2], "w") as fh:
        json.dump(traffic, fh, indent=1)


if __name__ == "__main__":
    main()
