"""Scorers — mirror ``evaluation/scorers.py:13-34`` (higher is better)."""

from __future__ import annotations

import numpy as np


class DummySklearWrapper:
    def __init__(self, model):
        self.model = model


def mle_log_likelihood_score(wrapped_model, x, y, **kwargs) -> float:
    """``scorers.py:30-34``: ``-nll(y, model(x)).mean()``; the sum is fused on the device."""
    return wrapped_model.model.score(np.asarray(x, np.float32), np.asarray(y, np.float32))


def bayesian_log_likelihood_score(wrapped_model, x, y, **kwargs) -> float:
    """``scorers.py:13-27``: ``logsumexp over posterior draws - log(draws)``, then the mean."""
    return wrapped_model.model.score(np.asarray(x, np.float32), np.asarray(y, np.float32))
