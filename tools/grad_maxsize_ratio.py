"""max |gpu - ref64| / grad_tolerance of the fused backward at the widest shapes
(tests/test_gpu_parity.py::test_maximum_sizes' backward part), printed instead of asserted,
for the fp32 spread at 1 and at 3 input perturbations.  Run from a library tree's root.

  python tools/grad_maxsize_ratio.py"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from normalizingflownetwork_amd import ops
    from oracle import nfn_grad_oracle as G
    from oracle import nfn_oracle as O

    for d, K in ((32, 64), (16, 40), (5, 64), (1, 64)):
        rng = np.random.default_rng(d * 100 + K)
        ft = tuple(rng.choice(["planar", "radial", "affine"], size=K))
        P = O.total_param_size(ft, d, True)
        B = 37
        y = rng.standard_normal((B, d)).astype(np.float32)
        t = (0.3 * rng.standard_normal((B, P))).astype(np.float32)
        _, gt, gy = ops.chain_log_prob_grad(torch.from_numpy(y).cuda(), torch.from_numpy(t).cuda(), ft, d, True)
        out = {}
        for npert in (1, 3):
            gt64, gy64, dev_t, dev_y = G.fp32_spread(y, t, ft, d, True, n_perturbed=npert)
            for name, got, ref, dev in (("gt", gt.cpu().numpy(), gt64, dev_t), ("gy", gy.cpu().numpy(), gy64, dev_y)):
                ok = np.isfinite(ref)
                r = np.abs(got - ref)[ok] / G.grad_tolerance(ref, dev)[ok]
                out[f"{name}_n{npert}"] = round(float(r.max()), 3) if r.size else 0.0
        print({"d": d, "K": K, **out}, flush=True)


if __name__ == "__main__":
    main()
