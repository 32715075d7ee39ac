"""bench.py output contract on the GPU: one JSON line with the driver's keys, the roofline and the
CPU-baseline objects, at a reduced window count (the C3 shape otherwise)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--windows", "2048", "--cpu-seconds", "1"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["unit"] == "windows/s" and rec["value"] > 0 and rec["higher_is_better"] is True
    assert "workload" in rec["config"]
    rf = rec["roofline"]
    assert rf["bound"] in ("hbm", "mfma") and rf["peak"] > 0 and rf["achieved"] > 0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    cb = rec["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["value"] > 0 and cb["cores"] >= 1
    # every window of the batch solved (the benchmark never times fallbacks)
    assert rec["solver"]["optimal_or_inaccurate"] == rec["solver"]["windows"]
