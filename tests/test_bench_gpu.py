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


@pytest.mark.gpu
def test_bench_sharded_path_with_real_kernels(tmp_path):
    """bench.py's N > 1 branch with the product kernels: two ranks under
    torch.distributed.run sharing cuda:0 (--share-device, --backend gloo: the W0 gather through host
    copies) over 16,384 windows of the global stream; the gathered W0 must equal the world-1 W0 of
    the same windows bit for bit (every window's rollout tiles and solve are the same at both batch
    sizes), and the line must carry the process group's own provenance."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    common = ["--global-windows", "16384", "--headline-only", "--cpu-seconds", "0", "--steps", "1", "--warmup", "1"]
    w1, w2 = str(tmp_path / "w0_world1.npy"), str(tmp_path / "w0_world2.npy")
    one = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *common, "--dump-w0", w1], cwd=ROOT,
                         capture_output=True, text=True, timeout=200, env=env)
    assert one.returncode == 0, one.stderr[-2000:]
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", "29541", os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--backend", "gloo", "--share-device", *common, "--dump-w0", w2],
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert two.returncode == 0, two.stderr[-3000:]
    lines = [l for l in two.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, two.stdout[-2000:]
    rec = json.loads(lines[0])
    d = rec["config"]["dist"]
    assert rec["n_gpus"] == 2 and d["backend"] == "gloo" and d["world_size"] == 2 and d["share_device"]
    assert d["windows_per_rank"] == [8192, 8192]
    import numpy as np
    a, b = np.load(w1), np.load(w2)
    assert a.shape == b.shape == (16384, 100)
    assert np.array_equal(a, b)
