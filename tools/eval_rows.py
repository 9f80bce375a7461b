"""Replay dumped samples (tests/test_gpu_fullbatch.py's gpurun_out/fullbatch_<cfg>_worst.npz)
through the library of a given tree, e.g. an older build under _ab/<name>, and compare
with the oracle values stored next to them.

    python tools/eval_rows.py <repo_dir> <npz> <C2|C3|C5> [fast|precise]
"""
import json
import sys

import numpy as np


def main():
    repo, path, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    mode = sys.argv[4] if len(sys.argv) > 4 else "fast"
    sys.path.insert(0, repo)
    import torch

    from normalizingflownetwork_amd import ops

    ops.set_math_mode(mode)
    z = np.load(path)
    ft, d = {"C2": (("planar", "radial") * 5, 1), "C5": (("planar", "radial") * 5, 1),
             "C3": (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8)}[cfg]
    y = torch.from_numpy(np.ascontiguousarray(z["y"])).cuda()
    t = torch.from_numpy(np.ascontiguousarray(z["t"])).cuda()
    if cfg == "C5":
        got = ops.posterior_lse(y, t, ft, d, True)[0].cpu().numpy()
    else:
        got = ops.chain_log_prob(y, t, ft, d, True)[0].cpu().numpy()
    r64 = z["ref64"]
    rel = np.abs(got - r64) / np.maximum(1.0, np.abs(r64))
    rel_dump = np.abs(z["got"] - r64) / np.maximum(1.0, np.abs(r64))
    print(json.dumps({"repo": repo, "cfg": cfg, "mode": mode, "n": int(len(got)),
                      "max_rel": float(rel.max()), "n_rel_gt_1e-5": int((rel > 1e-5).sum()),
                      "dump_max_rel": float(rel_dump.max()), "dump_n_rel_gt_1e-5": int((rel_dump > 1e-5).sum()),
                      "worst10_rel": [float(v) for v in np.sort(rel)[::-1][:10]]}))
    np.save(path.replace(".npz", f"_{mode}_{repo.strip('/').replace('/', '_')}.npy"), got)


if __name__ == "__main__":
    main()
