"""Generate the committed golden fixtures in tests/golden/*.npz.

Run in the BUILD container (not on the GPU box):  ``python tests/golden/make_golden.py``

* Inputs are float32, seeded (``numpy.random.default_rng(22)``; seed 22 is the
  reference's convention, ``BaseEstimator.py:12``, ``dummy_data_gen.py:7``).
* Config C1's (x, y) come from the reference's own data generator
  ``simulation/dummy_data_gen.py:6-20`` (``gen_cosine_noise_data(4096)``),
  imported from /root/reference only while this script runs; the arrays are
  committed as data.
* Expected outputs come from the fp64 oracle (``oracle/nfn_oracle.py``); the
  fp32 op-by-op mirror is stored next to them (``ref32``) so tests can size the
  tolerance on ill-conditioned samples.  TF/TFP are not installed anywhere, so
  the reference's own TF path could not produce these values: numeric parity
  against TF itself is unpinned ("Oracle").
"""

from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import nfn_oracle as O  # noqa: E402

REFERENCE = "/root/reference"


def chain_case(name, flow_types, d, trainable, B, seed, t_scale=1.0, y_bcast=False, y=None, t=None, extra=None):
    rng = np.random.default_rng(seed)
    P = O.total_param_size(flow_types, d, trainable)
    if t is None:
        t = (rng.standard_normal((B, P)) * t_scale).astype(np.float32)
    if y is None:
        y = rng.standard_normal((1 if y_bcast else B, d)).astype(np.float32)
    ref64 = O.chain_log_prob(y, t, flow_types, d, trainable, np.float64)
    ref32 = O.chain_log_prob(y, t, flow_types, d, trainable, np.float32)
    arrs = dict(y=y, t=t, ref64=ref64, ref32=ref32, flow_types=np.array(flow_types, dtype="U8"),
                d=np.int32(d), trainable=np.int32(trainable))
    if extra:
        arrs.update(extra)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
    return arrs


def main():
    made = []
    # C1 plumbing: NFN d=1, ("radial","radial"), B=4096, data from the reference generator.
    sys.path.insert(0, REFERENCE)
    from simulation.dummy_data_gen import gen_cosine_noise_data  # reference code, build container only

    x, y = gen_cosine_noise_data(4096)
    assert hashlib.sha256(y.tobytes()).hexdigest().startswith("acca66247f03f832")
    y_mean = np.mean(y, axis=0, dtype=np.float32)  # BaseEstimator.py:49-53
    y_std = np.std(y, axis=0, dtype=np.float32)
    rng = np.random.default_rng(22)
    ft = ("radial", "radial")
    t = rng.standard_normal((4096, O.total_param_size(ft, 1, True))).astype(np.float32)
    logpdf64 = O.log_pdf(y, t, ft, 1, True, y_mean, y_std, np.float64)
    logpdf32 = O.log_pdf(y, t, ft, 1, True, y_mean, y_std, np.float32)
    y_circ = O.normalize_y(y, y_mean, y_std, np.float32)
    chain_case("c1_nfn_radial2_d1", ft, 1, True, 4096, 22, y=y_circ, t=t,
               extra=dict(x=x, y_raw=y, y_mean=y_mean, y_std=y_std, logpdf64=logpdf64, logpdf32=logpdf32))
    made.append("c1_nfn_radial2_d1")

    c2 = ("planar", "radial") * 5
    chain_case("c2_pr5_d1", c2, 1, True, 4096, 101)
    c3 = ("affine",) + ("planar",) * 4 + ("radial",) * 4
    chain_case("c3_apr_d8", c3, 8, True, 1024, 102)
    for d in (1, 3, 8):
        chain_case(f"asym_pra_d{d}", ("planar", "radial", "affine"), d, True, 1024, 110 + d)
    chain_case("asym_pra_d3_fixedbase", ("planar", "radial", "affine"), 3, False, 1024, 120)
    chain_case("noflows_d2", (), 2, True, 512, 121)
    chain_case("bcast_y1_pr_d2", ("planar", "radial"), 2, True, 256, 122, y_bcast=True)
    chain_case("stress_pr5_d1", c2, 1, True, 4096, 123, t_scale=3.0)
    chain_case("radial10_d5", ("radial",) * 10, 5, True, 512, 124)
    chain_case("planar_radial_d16", ("planar", "radial") * 2, 16, True, 256, 125)
    made += ["c2_pr5_d1", "c3_apr_d8", "asym_pra_d1", "asym_pra_d3", "asym_pra_d8", "asym_pra_d3_fixedbase",
             "noflows_d2", "bcast_y1_pr_d2", "stress_pr5_d1", "radial10_d5", "planar_radial_d16"]

    # Posterior (config C5 shape, reduced): S=8 draws, B=512, d=1, C2 flows, normalised y.
    rng = np.random.default_rng(130)
    S, B = 8, 512
    P = O.total_param_size(c2, 1, True)
    td = rng.standard_normal((S, B, P)).astype(np.float32)
    yp = rng.standard_normal((B, 1)).astype(np.float32)
    ym = np.array([0.25], np.float32)
    ys = np.array([1.5], np.float32)
    lse64 = O.posterior_lse(yp, td, c2, 1, True, ym, ys, np.float64)
    lse32 = O.posterior_lse(yp, td, c2, 1, True, ym, ys, np.float32)
    np.savez_compressed(os.path.join(HERE, "posterior_s8_pr5_d1.npz"), y=yp, t=td, y_mean=ym, y_std=ys,
                        ref64=lse64, ref32=lse32, flow_types=np.array(c2, dtype="U8"), d=np.int32(1),
                        trainable=np.int32(1))
    made.append("posterior_s8_pr5_d1")

    # Single bijectors (forward + fldj) at d in {1, 4}, plus the reference test inputs
    # of tests/test_flows.py:10-41 (t = ones, symmetric batch of ones/zeros).
    rng = np.random.default_rng(140)
    for ftype in ("planar", "radial", "affine"):
        for d in (1, 4):
            ps = O.param_size(ftype, d)
            tk = rng.standard_normal((256, ps)).astype(np.float32)
            z = rng.standard_normal((256, d)).astype(np.float32)
            f64, l64 = O.flow_forward_fldj(ftype, z.astype(np.float64), tk.astype(np.float64), d)
            f32, l32 = O.flow_forward_fldj(ftype, z, tk, d)
            ones = np.ones((10, ps), np.float32)
            sym = np.array([[1.0] * d] + [[0.0] * d] * 8 + [[1.0] * d], np.float32)
            sf64, sl64 = O.flow_forward_fldj(ftype, sym.astype(np.float64), ones.astype(np.float64), d)
            np.savez_compressed(os.path.join(HERE, f"flow_{ftype}_d{d}.npz"), z=z, t=tk, fwd64=f64, ldj64=l64,
                                fwd32=f32, ldj32=l32, sym_t=ones, sym_z=sym, sym_fwd64=sf64, sym_ldj64=sl64,
                                d=np.int32(d))
            made.append(f"flow_{ftype}_d{d}")
    with open(os.path.join(HERE, "MANIFEST.txt"), "w") as f:
        for m in made:
            h = hashlib.sha256(open(os.path.join(HERE, m + ".npz"), "rb").read()).hexdigest()[:16]
            f.write(f"{m}.npz {h}\n")
    print("wrote", len(made), "fixtures")


if __name__ == "__main__":
    main()
