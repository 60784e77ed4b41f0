"""Library-API parity: basecount_amd's BaseCount (rows, records,
num_reads, mean_coverage, mean_entropy with min_coverage, reference_lengths in wide and long
format, invalid-reference errors; main.py:208-359) and get_stats on caller-owned lists (the N
pop of main.py:31) against the reference's own outputs (tests/golden/api/, made by
make_api_golden.py running the reference).  Every value compares exactly, type included (int vs
float vs numpy float64): both sides run tests/golden/api_probe.py with PYTHONHASHSEED=0."""
import gzip
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")
API = os.path.join(GOLD, "api")


@pytest.fixture(scope="module")
def ours():
    env = dict(os.environ, PYTHONPATH=REPO, PYTHONHASHSEED="0")
    p = subprocess.run([sys.executable, os.path.join(GOLD, "api_probe.py"), "basecount_amd.main",
                        "--cases", os.path.join(API, "cases.json")], cwd=GOLD, env=env,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def _diff(a, b, path=""):
    if type(a) is not type(b):
        return f"{path}: {a!r:.200} != {b!r:.200}"
    if isinstance(a, dict):
        if set(a) != set(b):
            return f"{path}: keys {sorted(set(a) ^ set(b))}"
        for k in a:
            d = _diff(a[k], b[k], f"{path}.{k}")
            if d:
                return d
        return None
    if isinstance(a, list):
        if len(a) != len(b):
            return f"{path}: length {len(a)} != {len(b)}"
        for i, (x, y) in enumerate(zip(a, b)):
            d = _diff(x, y, f"{path}[{i}]")
            if d:
                return d
        return None
    return None if a == b else f"{path}: {a!r} != {b!r}"


with open(os.path.join(API, "cases.json")) as _fh:
    CASES = sorted(json.load(_fh))


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_api_matches_reference(ours, case):
    with gzip.open(os.path.join(API, f"{case}.json.gz")) as fh:
        gold = json.loads(fh.read())
    d = _diff(ours[case], gold)
    assert d is None, f"{case}: {d}"


@pytest.mark.gpu
def test_release_keeps_another_callers_scratch():
    """a get_basecounts call without _keep_scratch releases only scratch nobody asked
    to keep; release_device_memory() then gives back everything, the contexts' own kernel scratch
    (bc_ctx_release_scratch) included, and later calls still work."""
    sys.path.insert(0, REPO)
    from basecount_amd import main as M

    bam = os.path.join(GOLD, "mixed.bam")
    a = M.get_basecounts(bam, _mode="summary", _keep_scratch=True)
    kept = set(M._SCRATCHES)
    assert kept and kept <= M._KEPT
    b = M.get_basecounts(bam, _mode="summary")
    assert set(M._SCRATCHES) == kept  # the kept cache survived the plain call
    M.release_device_memory()
    assert not M._SCRATCHES and not M._KEPT
    c = M.get_basecounts(bam, _mode="summary")
    assert not M._SCRATCHES  # a plain call releases its own scratch
    for ref in a:
        assert a[ref]["summary"]["avg_cov"] == b[ref]["summary"]["avg_cov"] == c[ref]["summary"]["avg_cov"]
