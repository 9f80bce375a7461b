"""Diagnostic: how far inverse-then-forward lands from loc + scale * eps for the sampling
kernel (nfn_chain_sample_f32), against the fp32 conditioning of the forward chain at the
sample (d = 1: |J| = exp(fldj) amplifies the sample's own rounding)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflownetwork_amd import ops  # noqa: E402
from oracle import nfn_oracle as O  # noqa: E402

CASES = [(("planar", "radial") * 5, 1), (("radial", "radial"), 1), (("affine", "planar", "radial"), 3),
         (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8), (("planar",) * 6, 2)]
for ft, d in CASES:
    rng = np.random.default_rng(len(ft) * 10 + d)
    B = 1 << 16
    P = O.total_param_size(ft, d, True)
    t = (0.5 * rng.standard_normal((B, P))).astype(np.float32)
    eps = rng.standard_normal((B, d)).astype(np.float32)
    y, lp = ops.chain_sample(torch.from_numpy(eps).cuda(), torch.from_numpy(t).cuda(), ft, d, True)
    y = y.cpu().numpy().astype(np.float64)
    base, blocks = O.split_params(t.astype(np.float64), ft, d, True)
    z, ldj = y.copy(), np.zeros(B)
    zs, ls = [np.abs(y).max(1)], []
    for f, tk in zip(ft, blocks):
        z, l = O.flow_forward_fldj(f, z, tk, d)
        ldj += l
        zs.append(np.abs(z).max(1))
        ls.append(l)
    # every step of the inverse walk rounds its z_k once; the forward map from z_k to z_K
    # scales that by |J_{k->K}| (per coordinate: exp(sum_{j>=k} fldj_j / d))
    tail = np.zeros(B)
    partial_gain = np.maximum(1.0, zs[-1])
    for k in range(len(ls) - 1, -1, -1):
        tail = tail + ls[k]
        partial_gain = partial_gain + np.exp(tail / d) * np.maximum(1.0, zs[k])
    loc = t[:, :d].astype(np.float64)
    scale = 1e-3 + O.softplus(np.log(np.expm1(1.0)) + 0.1 * t[:, d:2 * d].astype(np.float64))
    target = loc + scale * eps
    err = np.abs(z - target).max(1) / np.maximum(1.0, np.abs(target).max(1))
    rec = {"flows": "+".join(ft), "d": d, "B": B, "max": float(err.max()), "q999": float(np.quantile(err, 0.999)),
           "q99": float(np.quantile(err, 0.99)), "median": float(np.median(err))}
    # conditioning: one ulp of every sample coordinate moved through the forward Jacobian
    # (|det J|^(1/d) as the per-coordinate gain) -> the error the sample's own rounding allows
    gain = np.exp(ldj / d) * np.maximum(1.0, np.abs(y).max(1)) * 2.0 ** -23 / np.maximum(1.0, np.abs(target).max(1))
    ratio = err / np.maximum(gain, 1e-30)
    pg = partial_gain * 2.0 ** -24 / np.maximum(1.0, np.abs(target).max(1))
    r2 = err / pg
    rec.update({"max_err_over_partial_gain": float(r2.max()), "q999_err_over_partial_gain": float(np.quantile(r2, 0.999))})
    rec.update({"max_err_over_rounding_gain": float(ratio.max()), "q999_err_over_gain": float(np.quantile(ratio, 0.999)),
                "worst": int(err.argmax()), "worst_gain": float(gain[err.argmax()]),
                "worst_ldj": float(ldj[err.argmax()])})
    print(json.dumps(rec), flush=True)
