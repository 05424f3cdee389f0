"""The bench line's contract, checked on the committed final-library line (profiles/r6af_bench.json,
a default `python bench.py` run on an MI355X): the driver's keys and types, the roofline and
cpu_baseline objects, and their internal arithmetic (frac = achieved / peak, achieved = algorithmic
bytes / kernel time). CPU only: it reads JSON."""

import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE = os.path.join(ROOT, "profiles", "r6af_bench.json")


@pytest.fixture(scope="module")
def line():
    with open(LINE) as f:
        rows = [r for r in f.read().splitlines() if r.strip().startswith("{")]
    assert rows, "no JSON line"
    return json.loads(rows[-1])


def test_driver_keys(line):
    for k, t in (("metric", str), ("value", float), ("unit", str), ("n_gpus", int),
                 ("steps", int), ("warmup", int), ("ms_per_step", float),
                 ("higher_is_better", bool), ("scaling", str), ("dtype", str), ("data", str),
                 ("config", dict)):
        assert isinstance(line[k], t), k
    assert line["n_gpus"] == 1 and line["higher_is_better"] is True
    assert line["vs_baseline"] is None  # BASELINE.md publishes no number for this metric
    assert "workload" in line["config"]
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert line["metric"] == json.load(f)["metric"]


def test_value_is_bytes_over_step_time(line):
    nbytes = line["config"]["bytes_per_step"]
    assert line["value"] == pytest.approx(nbytes / (line["ms_per_step"] * 1e-3) / 1e9, rel=2e-3)


def test_roofline_object(line):
    r = line["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=2e-4)
    assert r["achieved"] == pytest.approx(
        r["alg_bytes_per_step"] / (r["kernel_ms_per_step"] * 1e-3) / 1e9, rel=2e-3)
    # HBM bytes from the FETCH_SIZE pass of the same launches: within 1% of the algorithmic bytes
    assert r["traffic"] == pytest.approx(r["alg_bytes_per_step"], rel=1e-2)
    assert r["launches"] == 129


def test_cpu_baseline_object(line):
    c = line["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1
    assert c["value"] > 0 and c["unit"] == "GB/s" and c["sample"]
