#!/usr/bin/env python3
"""Launch one config's forward kernel (or, with --grad, its fused backward) a few times
under a diagnostic-build knob (for rocprofv3 --pmc passes over a single variant: run it as
the program after `--`).

  python3 tools/run_variant.py C2 NFN_TILE_ROT=0 [--launches 5]
  python3 tools/run_variant.py C2 NFN_GRAD_WAVE1=1 --grad"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("cfg")
    ap.add_argument("knobs", nargs="*", help="NAME=VALUE diagnostic-build knobs")
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--grad", action="store_true", help="the fused backward (GradLauncher) instead")
    a = ap.parse_args()
    cfg, knobs, n = a.cfg, dict(k.split("=", 1) for k in a.knobs), a.launches
    os.environ.update(knobs)  # read by the diag library at each launch
    import torch

    from normalizingflownetwork_amd import _lib

    _lib.use_diagnostic_build()
    from normalizingflownetwork_amd import ops
    from tools.microbench import CFG

    ft, d, B, S = CFG[cfg]
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(1)
    y = torch.randn((B, d), generator=gen, device="cuda")
    t = torch.randn((B, P) if S is None else (S, B, P), generator=gen, device="cuda")
    if a.grad:
        g = torch.full((B,), -1.0 / B, device="cuda")
        L = ops.GradLauncher(y, t, ft, d, True, g_out=g)
        for _ in range(n):
            L.launch(int(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        print({"cfg": cfg, "knobs": knobs, "launches": n, "grad": True,
               "grad_t_abs_sum": float(L.grad_t.double().abs().sum().item())})
        return
    L = ops.ChainLauncher(y, t, ft, d, True, draws=S)
    for _ in range(n):
        L.launch()
    torch.cuda.synchronize()
    print({"cfg": cfg, "knobs": knobs, "launches": n, "mean_log_prob": float(L.out.double().mean().item())})


if __name__ == "__main__":
    main()
