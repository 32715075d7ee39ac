"""Build libkmpc.so in-tree: ``python -m koopman_mpc_portfolio_rebalancing_amd.build [--force]``.

hipcc cross-compiles for gfx950 without a GPU; the resulting .so lives next to this file (it is
git-ignored but travels with the repository snapshot to the GPU box).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libkmpc.so")


def sources():
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))
            if f.endswith((".hip", ".h", ".inc", "Makefile"))] + [os.path.join(os.path.dirname(HERE), "include", "kmpc.h")]


def is_stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in sources())


def build(force: bool = False, jobs: int = 7) -> str:
    if force:
        subprocess.run(["make", "-s", "-C", CSRC, "clean"], check=True)
    if force or is_stale():
        subprocess.run(["make", "-s", "-C", CSRC, f"-j{jobs}"], check=True)
    if not os.path.exists(LIB):
        raise RuntimeError("libkmpc.so was not produced")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
