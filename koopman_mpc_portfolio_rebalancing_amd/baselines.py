"""DMD (linear Koopman) baseline on the device window path.

Mirrors ``DMDStrategy`` of the reference (baselines.py:127-187): the operator A of x_{t+1} = A x_t
is fitted once on the host exactly as the reference does (``X' @ scipy.linalg.pinv(X)`` on the
float32 training embeddings, baselines.py:145-166 — a one-off fit, not on the path); the rollout
x <- A x over the horizon, the extraction of the first N entries, the de-standardisation and the
log-utility MPC solve run on the device. The rollout is the Koopman kernel chain with an identity
encoder / decoder and the latent operator A^T (row-vector convention, z <- z @ A^T), so DMD shares
``kmpc_window`` with the Koopman strategy.

The reference's Markowitz baseline (mean-variance QP, mpc.py:119-184) is SURVEY §8(f) row 3 and is
not provided on the device yet.
"""
from __future__ import annotations

from typing import Any, Sequence

import numpy as np
import torch

from .backtest import KoopmanMPCStrategy, Strategy
from .koopman import KoopmanModelSpec
from .mpc import MPCConfig


def fit_dmd(train_data) -> np.ndarray:
    """A = X' pinv(X) with X = data[:-1]^T, X' = data[1:]^T (baselines.py:145-166), float32 in,
    computed by scipy.linalg.pinv as in the reference."""
    from scipy.linalg import pinv
    data = train_data.cpu().numpy() if torch.is_tensor(train_data) else np.asarray(train_data)
    X = data[:-1].T
    X_prime = data[1:].T
    return X_prime @ pinv(X)


def dmd_model_spec(A: np.ndarray) -> KoopmanModelSpec:
    """The DMD rollout as a Koopman model: identity encoder, latent operator A^T, identity decoder."""
    n = A.shape[0]
    eye = torch.eye(n, dtype=torch.float32)
    return KoopmanModelSpec(kind="generic", encoder=[(eye, None)], kmat=torch.as_tensor(A, dtype=torch.float32).t().contiguous(),
                            decoder=[(eye, None)], enc_act="relu", enc_last_relu=False, norm_fn="id")


class DMDStrategy(KoopmanMPCStrategy):
    """Dynamic Mode Decomposition strategy (baselines.py:127-187) on the device window path.

    Args:
        train_data: [samples, obs_size] training embeddings (env.train_dataset.data).
        mpc_config: MPCConfig for the log-utility solve.
        device: as KoopmanMPCStrategy ('cpu' selects the current GPU; there is no CPU path).
    """

    def __init__(self, train_data: Any, mpc_config: MPCConfig, device: str = "cpu"):
        self.K = fit_dmd(train_data)
        self.n_assets = None
        super().__init__(dmd_model_spec(self.K), mpc_config, device)


__all__: Sequence[str] = ("DMDStrategy", "fit_dmd", "dmd_model_spec", "Strategy")
