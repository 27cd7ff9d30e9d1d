"""bench.py's one-line JSON contract on one GPU (a small, fast configuration)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


@pytest.mark.gpu
def test_bench_prints_the_contract_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2",
                        "--nsplit", "3", "--no-extra", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 2
    assert d["unit"] == "V-cycles/s" and d["higher_is_better"] is True and d["dtype"] == "f64"
    assert d["value"] > 0 and abs(d["ms_per_step"] - 1e3 / d["value"]) < 1e-3 * max(1.0, 1e3 / d["value"])
    assert "workload" in d["config"]
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    # the resident call (default) is fp64-issue-bound: its roofline is fp64 TFLOP/s against the 78.6
    # TFLOP/s peak; the other schedules' launches are HBM-bound
    if rf["bound"] == "fp64-valu":
        assert rf["unit"] == "TFLOP/s" and rf["peak"] == 78.6 and rf["cycles_per_launch"] == 4
    else:
        assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert 0 < rf["frac"] < 1.0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3


def test_pmc_traffic_is_reported_only_for_the_build_it_was_measured_on(tmp_path, monkeypatch):
    """bench.py reads roofline.traffic from the committed rocprofv3 PMC summary only when the
    summary's kernel-source digest (scripts/pmc_summary.py) matches the current sources"""
    sys.path.insert(0, ROOT)
    import bench
    import importlib.util
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "scripts", "pmc_summary.py"))
    ps = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ps)
    assert ps.source_digest() == bench.source_digest()
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    # the digest itself is computed over the real tree
    monkeypatch.setattr(bench, "source_digest", lambda: ps.source_digest())
    rec = {"n_split": 5, "levels": 3, "hbm_bytes_per_launch": 1.0e9, "commit": "abc1234",
           "source_digest": ps.source_digest()}
    (prof / "pmc_vcycle_res.json").write_text(json.dumps(rec))
    info = {}
    assert bench.pmc_traffic("vcycle_res", 5, 3, info) == 1.0e9
    assert info["source_matches_build"] is True and info["commit"] == "abc1234"
    assert bench.pmc_traffic("vcycle_res", 6, 3) is None   # another configuration
    rec["source_digest"] = "0" * 16                          # measured on other kernels: stale
    (prof / "pmc_vcycle_res.json").write_text(json.dumps(rec))
    info = {}
    assert bench.pmc_traffic("vcycle_res", 5, 3, info) is None
    assert info["source_matches_build"] is False
    assert bench.pmc_traffic("vcycle_pipe", 5, 3) is None    # no summary at all
