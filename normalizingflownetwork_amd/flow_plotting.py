"""Density heatmaps of a fitted model (``evaluation/visualization/flow_plotting.py:33-53``).

``model_density_heatmap`` computes exactly the array ``plot_model`` hands to
``plt.imshow`` — rows are the y grid from ``y_range[1]`` down to ``y_range[0]``,
columns the x batch, entries ``dist.prob((y - y_mean) / y_std) / sum(y_std)`` —
with one density-grid kernel (``nfn_chain_logprob_grid_f32``) instead of one
``dist.prob`` call per grid row.  ``plot_model`` draws it with matplotlib."""

from __future__ import annotations

import numpy as np


def model_density_heatmap(x, model, y_range, y_num: int = 100) -> np.ndarray:
    x = np.asarray(x, np.float32)
    assert len(x.shape) == 2 and x[0][0] < x[-1][0]  # flow_plotting.py:36
    assert len(y_range) == 2 and y_range[0] < y_range[1]  # flow_plotting.py:37
    dist = model(x)
    y_orig = np.linspace(y_range[1], y_range[0], num=y_num).reshape((y_num, 1))
    y = ((y_orig - model.y_mean) / model.y_std).astype(np.float32)
    heat = dist.prob_grid(y).cpu().numpy().astype(np.float64) / np.sum(model.y_std)
    assert heat.shape == (y_num, len(x))
    return heat


def plot_model(x, model, y_range, y_num: int = 100):
    """``flow_plotting.plot_model`` (matplotlib imshow of ``model_density_heatmap``)."""
    import matplotlib.pyplot as plt

    heat = model_density_heatmap(x, model, y_range, y_num)
    y_orig = np.linspace(y_range[1], y_range[0], num=y_num)
    plt.imshow(heat, aspect="equal")
    plt.xlabel("x")
    plt.ylabel("y")
    plt.xticks([0, x.shape[0] - 1], [x[0][0], x[-1][0]])
    plt.yticks([0, y_num - 1], [y_orig[0], y_orig[-1]])
    plt.colorbar()
    return heat
