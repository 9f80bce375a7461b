"""Density grid A/B (diag build): per-row precomputed flow terms (NFN_GRID_PRE=1, the
release form) vs re-deriving them for every grid value (NFN_GRID_PRE=0), C2 chain,
G = 256 grid values x 2^16 rows, interleaved rounds in one process; and how the two
outputs compare."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflownetwork_amd import _lib, ops  # noqa: E402

_lib.use_diagnostic_build()
ft, d = ("planar", "radial") * 5, 1
P = ops.total_param_size(ft, d, True)
G, B = 256, 1 << 16
gen = torch.Generator(device="cuda").manual_seed(5)
t = torch.randn((B, P), generator=gen, device="cuda")
yg = torch.linspace(-4.0, 4.0, G, device="cuda").reshape(G, 1).contiguous()
lz = ops.GridLauncher(yg, t, ft, d, True)
outs, times = {}, {"1": [], "0": []}
for rnd in range(4):
    for v in ("1", "0"):
        os.environ["NFN_GRID_PRE"] = v
        for _ in range(3):
            lz.launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lz.launch()
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 20)
        outs[v] = lz.out.clone()
for v in ("1", "0"):
    print(f"NFN_GRID_PRE={v}: ms per launch {['%.4f' % x for x in times[v]]} "
          f"-> {G * B / (min(times[v]) * 1e-3):.3e} evals/s")
a, b = outs["1"], outs["0"]
fin = torch.isfinite(a) & torch.isfinite(b)
print(f"bitwise equal {(a == b).sum().item()} / {a.numel()}; finite-mismatch {(torch.isfinite(a) != torch.isfinite(b)).sum().item()}; "
      f"max |diff| / max(1,|b|) {((a - b).abs()[fin] / b.abs()[fin].clamp(min=1)).max().item():.3e}")
