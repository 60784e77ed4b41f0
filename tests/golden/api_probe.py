"""The library-API probe (main.py:208-359): one fixed sequence of calls on a
``BaseCount`` module, with every result encoded as ``type:repr`` strings so ints, floats, numpy
scalars and NaN compare exactly.

The same function runs against the reference (make_api_golden.py, in the build container, through
oracle/pysam_shim) and against basecount_amd (tests/test_gpu_api.py, on the GPU), each in a
process with PYTHONHASHSEED=0 (the reference iterates a set of references, main.py:92).

    python tests/golden/api_probe.py MODULE BAM JSON_KWARGS      -> one JSON line on stdout
    python tests/golden/api_probe.py MODULE --cases CASES_JSON   -> {case: result}, one line
"""
from __future__ import annotations

import importlib
import json
import sys
import warnings


def enc(v):
    """Exact, type-carrying encoding of a result (lists / dicts recursively)."""
    if isinstance(v, dict):
        return {str(k): enc(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [enc(x) for x in v]
    return f"{type(v).__name__}:{v!r}"


def _err(fn):
    try:
        out = fn()
        return {"ok": enc(out)}
    except Exception as e:  # noqa: BLE001 - the exception text is part of the API
        return {"raise": f"{type(e).__name__}: {e}"}


def probe(M, bam: str, kw: dict, head: int = 400) -> dict:
    warnings.simplefilter("ignore")  # np.mean([]) warns in both implementations
    try:
        bc = M.BaseCount(bam, **kw)
    except Exception as e:  # noqa: BLE001 - e.g. the reference's KeyError for a strict subset
        return {"init_raise": f"{type(e).__name__}: {e}"}
    refs = list(bc.references)
    out = {
        "columns": enc(bc.columns),
        "references": enc(refs),
        "reference_lengths": enc(bc.reference_lengths),
        "num_reads": enc(bc.num_reads()),
        "mean_coverage": enc(bc.mean_coverage()),
        "mean_entropy": enc(bc.mean_entropy()),
    }
    rows = list(bc.rows())
    out["rows_n"] = len(rows)
    out["rows_head"] = enc(rows[:head])
    out["rows_tail"] = enc(rows[-head:])
    recs = list(bc.records())
    out["records_head"] = enc(recs[:head])
    per = {}
    for ref in sorted(refs):
        per[ref] = {
            "rows": enc(list(bc.rows(ref))[:head]),
            "records_tail": enc(list(bc.records(ref))[-head:]),
            "num_reads": enc(bc.num_reads(ref)),
            "mean_coverage": enc(bc.mean_coverage(ref)),
            "mean_entropy": {str(m): enc(bc.mean_entropy(ref, min_coverage=m)) for m in (0, 1, 3, 10**9)},
        }
    out["per_reference"] = per
    out["mean_entropy_min_cov"] = {str(m): enc(bc.mean_entropy(min_coverage=m)) for m in (0, 1, 3, 10**9)}
    out["errors"] = {
        "rows": _err(lambda: list(bc.rows("chrZ"))),
        "records": _err(lambda: list(bc.records("chrZ"))),
        "num_reads": _err(lambda: bc.num_reads("chrZ")),
        "mean_coverage": _err(lambda: bc.mean_coverage("chrZ")),
        "mean_entropy": _err(lambda: bc.mean_entropy("chrZ", min_coverage=2)),
    }
    return out


GET_STATS_CASES = [
    [[1, 2, 3, 4, 5, 6], [0, 0, 0, 0, 0, 7], [0, 0, 0, 0, 0, 0], [5, 5, 5, 5, 0, 0], [9, 0, 0, 0, 0, 0],
     [0, 3, 3, 0, 1, 0], [7, 7, 0, 0, 7, 2], [123456, 1, 0, 2, 3, 4]],
    [],
]


def probe_get_stats(M) -> dict:
    """get_stats on caller-owned lists (main.py:14-79), including the N-column pop it performs
    on the caller's own lists when show_n_bases is False (main.py:31)."""
    out = {}
    for ci, case in enumerate(GET_STATS_CASES):
        for show_n in (False, True):
            for long_format in (False, True):
                lists = [list(r) for r in case]
                rows = M.get_stats(lists, f"ref{ci}", show_n_bases=show_n, long_format=long_format)
                out[f"{ci}_{int(show_n)}_{int(long_format)}"] = {"rows": enc(rows), "inputs_after": enc(lists)}
    out["entropy"] = {str(i): enc(M.get_entropy(p)) for i, p in
                      enumerate([[0.5, 0.5], [1.0, 0.0], [0.25, 0.25, 0.5], [0.1, 0.2, 0.3, 0.4], []])}
    return out


def main():
    mod = sys.argv[1]
    M = importlib.import_module(mod)
    if sys.argv[2] == "--cases":  # every case of a cases.json in one process: {case: result}
        with open(sys.argv[3]) as fh:
            cases = json.load(fh)
        res = {name: (probe(M, c["bam"], c["kwargs"]) if c["bam"] != "-" else probe_get_stats(M))
               for name, c in cases.items()}
    else:
        bam, kw = sys.argv[2], json.loads(sys.argv[3])
        res = probe(M, bam, kw) if bam != "-" else probe_get_stats(M)
    sys.stdout.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
