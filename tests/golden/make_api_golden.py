"""Golden fixtures for the library API (BaseCount rows / records / num_reads /
mean_coverage / mean_entropy / reference_lengths, main.py:208-359, and get_stats on caller lists,
main.py:14-79) produced by running the REFERENCE itself.

Run in the build container only (needs /root/reference, oracle/_ref and oracle/pysam_shim):

    python tests/golden/make_api_golden.py

Each case runs tests/golden/api_probe.py (our own probe: a fixed call sequence, results encoded as
type:repr strings) against the reference's ``basecount.main`` in a fresh process with
PYTHONHASHSEED=0 and PYTHONDONTWRITEBYTECODE=1, and writes api/<case>.json.gz plus api/cases.json.
tests/test_gpu_api.py runs the same probe against basecount_amd.main and compares.
"""
from __future__ import annotations

import gzip
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

CASES = {
    "edge_default": ("edge.bam", {}),
    "edge_shown": ("edge.bam", {"show_n_bases": True}),
    "edge_long": ("edge.bam", {"long_format": True}),
    "edge_long_shown": ("edge.bam", {"long_format": True, "show_n_bases": True}),
    "edge_q20_m30": ("edge.bam", {"min_base_quality": 20, "min_mapping_quality": 30}),
    # a strict subset raises KeyError in the reference when reads sit on other references
    "edge_refs_subset": ("edge.bam", {"references": ["chrA", "chrC"], "show_n_bases": True}),
    "edge_refs_all": ("edge.bam", {"references": ["chrD", "chrC", "chrB", "chrA"]}),
    "edge_chunk3": ("edge.bam", {"chunk_size": 3}),
    "c1_default": ("c1.bam", {}),
    "c1_long": ("c1.bam", {"long_format": True}),
    "mixed_shown_q20": ("mixed.bam", {"show_n_bases": True, "min_base_quality": 20}),
    "get_stats": ("-", {}),
}


def run_probe(bam: str, kw: dict) -> dict:
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", PYTHONHASHSEED="0",
               PYTHONPATH=os.pathsep.join([os.path.join(REPO, "oracle", "pysam_shim"),
                                           os.path.join(REPO, "oracle", "_ref"), REF, REPO]))
    p = subprocess.run([sys.executable, os.path.join(HERE, "api_probe.py"), "basecount.main", bam,
                        json.dumps(kw)], cwd=HERE, env=env, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(p.stderr[-3000:])
    return json.loads(p.stdout.strip().splitlines()[-1])


def main():
    os.makedirs(os.path.join(HERE, "api"), exist_ok=True)
    for name, (bam, kw) in CASES.items():
        res = run_probe(bam, kw)
        with open(os.path.join(HERE, "api", f"{name}.json.gz"), "wb") as fh:
            fh.write(gzip.compress(json.dumps(res, sort_keys=True).encode(), compresslevel=9, mtime=0))
        print(name, "ok")
    with open(os.path.join(HERE, "api", "cases.json"), "w") as fh:
        json.dump({k: {"bam": b, "kwargs": kw} for k, (b, kw) in CASES.items()}, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
