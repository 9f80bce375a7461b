"""fit() wall time at the reference's training setting (Keras batch_size 32): the HIP-graph
replayed step vs the eager loop, same data and seeds (NormalizingFlowNetwork, 10 flows,
hidden (16, 16), 2048 samples, 20 epochs = 1280 steps)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflownetwork_amd import NormalizingFlowNetwork  # noqa: E402

rng = np.random.default_rng(0)
n = 2048
x = rng.uniform(-np.pi, np.pi, (n, 1)).astype(np.float32)
y = (np.sin(x) + 0.3 * rng.standard_normal((n, 1))).astype(np.float32)
for flows, bs, epochs in ((("planar", "radial") * 5, 32, 20), (("radial",) * 10, 256, 40)):
    res = {}
    for use_graph in (False, True, False, True):
        m = NormalizingFlowNetwork(1, flow_types=flows, hidden_sizes=(16, 16), trainable_base_dist=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h = m.fit(x, y, batch_size=bs, epochs=epochs, verbose=0, use_graph=use_graph)["loss"]
        torch.cuda.synchronize()
        res.setdefault(use_graph, []).append((time.perf_counter() - t0, h[-1]))
    steps = epochs * ((n + bs - 1) // bs)
    for g, v in res.items():
        t = min(a for a, _ in v)
        print(json.dumps({"flows": len(flows), "batch_size": bs, "epochs": epochs, "steps": steps, "graph": g,
                          "seconds": t, "ms_per_step": t / steps * 1e3, "final_loss": v[-1][1]}), flush=True)
