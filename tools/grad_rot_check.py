"""Diag check: the backward with rotated tile slots (NFN_TILE_ROT_B) gives the plain walk's
gradients bitwise (the same per-sample math on the same rows)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflownetwork_amd import _lib  # noqa: E402

_lib.use_diagnostic_build()
from normalizingflownetwork_amd import ops  # noqa: E402

ft = ("planar", "radial") * 5
gen = torch.Generator(device="cuda").manual_seed(7)
for B in ((1 << 20) + 37, 1 << 22):
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((B, 32), generator=gen, device="cuda")
    g = torch.randn((B,), generator=gen, device="cuda")
    l0 = ops.GradLauncher(y, t, ft, 1, True, g_out=g)
    l0.launch()
    torch.cuda.synchronize()
    ref_t, ref_y = l0.grad_t.clone(), l0.grad_y.clone()
    os.environ["NFN_TILE_ROT_B"] = "4"
    l0.launch()
    torch.cuda.synchronize()
    os.environ.pop("NFN_TILE_ROT_B")
    assert torch.equal(l0.grad_t, ref_t) and torch.equal(l0.grad_y, ref_y), B
    print(f"B={B}: rotated backward bitwise the plain walk's")
