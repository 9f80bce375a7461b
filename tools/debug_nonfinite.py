#!/usr/bin/env python3
"""Find non-finite kernel outputs on a config's synthetic data and compare those
rows with the oracle (fp64 / fp32).  Diagnostic only."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflownetwork_amd import ops  # noqa: E402
from oracle import nfn_oracle as O  # noqa: E402
from tools.microbench import CFG  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    ft, d, B, S = CFG[cfg]
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(1)
    y = torch.randn((B, d), generator=gen, device="cuda")
    t = torch.randn((B, P), generator=gen, device="cuda")
    for mode in ("auto", "tile"):
        if mode == "tile":
            os.environ["NFN_LOAD_MODE"] = "tile"
        for math in ("fast", "precise"):
            ops.set_math_mode(math)
            lp, _ = ops.chain_log_prob(y, t, ft, d, True)
            bad = torch.nonzero(~torch.isfinite(lp)).flatten()
            print(f"{cfg} mode={mode} math={math}: non-finite {bad.numel()} / {B}", flush=True)
            if bad.numel():
                idx = bad[:8]
                yn, tn = y[idx].cpu().numpy(), t[idx].cpu().numpy()
                with np.errstate(all="ignore"):
                    r64 = O.chain_log_prob(yn, tn, ft, d, True, np.float64)
                    r32 = O.chain_log_prob(yn, tn, ft, d, True, np.float32)
                for i, k in enumerate(idx.tolist()):
                    print(f"  row {k}: gpu {lp[k].item()!r} ref64 {r64[i]!r} ref32 {r32[i]!r}")
        os.environ.pop("NFN_LOAD_MODE", None)
    # check a random sample against the oracle too
    ops.set_math_mode("fast")
    lp, _ = ops.chain_log_prob(y, t, ft, d, True)
    idx = torch.randint(0, B, (2048,), generator=gen, device="cuda")
    yn, tn = y[idx].cpu().numpy(), t[idx].cpu().numpy()
    r64 = O.chain_log_prob(yn, tn, ft, d, True, np.float64)
    err = np.abs(lp[idx].cpu().numpy().astype(np.float64) - r64) / np.maximum(1, np.abs(r64))
    print(f"sample max rel err {np.nanmax(err):.3e}")


if __name__ == "__main__":
    main()
