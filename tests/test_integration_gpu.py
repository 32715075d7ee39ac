"""INTEGRATION.md §3's reference-side ctypes stub, executed as written (library path substituted):
it must agree with the package's drop-in `solve_mpc_log_utility` on a register-kernel window and
on a large-window one (N > 256, which needs the workspace the stub sizes)."""
import os
import re

import numpy as np
import pytest

from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, solve_mpc_log_utility, _lib

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = re.search(r"```python\n(# kmpc_ctypes\.py.*?)```", text, re.S).group(1)
    code = code.replace("/path/to/koopman_mpc_portfolio_rebalancing_amd/libkmpc.so", _lib.LIB_PATH)
    ns = {}
    exec(compile(code, "INTEGRATION.md:kmpc_ctypes.py", "exec"), ns)
    return ns["solve_mpc_log_utility"]


@pytest.mark.parametrize("N,H", [(20, 5), (300, 10)])
def test_ctypes_stub_matches_package(N, H):
    stub = _stub()
    rng = np.random.default_rng(N + H)
    wp = rng.dirichlet(np.ones(N))
    y = rng.normal(5e-4, 0.015, (H, N)).astype(np.float32)
    cfg = MPCConfig(horizon=H)
    Ws, infs = stub(wp, y, cfg)
    Wp, infp = solve_mpc_log_utility(wp, y, cfg)
    assert infs["status"] == infp["status"] == "optimal"
    assert np.array_equal(Ws, Wp)
    assert infs["value"] == infp["value"]
