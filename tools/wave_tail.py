"""How much of a C2 forward launch is tail?  The diagnostic library's chain_wave1_kernel records
every wave's (start, end) wall clock (100 MHz; nfn_diag_wave_times, NFN_DIAG builds only); this
prints, over a few launches, the launch span (first start to last end), the spread of the wave
end times, and the share of the span during which fewer than all waves are still running —
the time a dynamic tile schedule could at most recover.

  python tools/wave_tail.py [config C2|R10] [launches]"""

import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflownetwork_amd import _lib  # noqa: E402

_lib.use_diagnostic_build()
from normalizingflownetwork_amd import ops  # noqa: E402

FLOWS = {"C2": ("planar", "radial") * 5, "R10": ("radial",) * 10}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    lib = _lib.load()
    fn = lib.nfn_diag_wave_times
    fn.restype = ctypes.c_int32
    fn.argtypes = [ctypes.c_void_p]
    gen = torch.Generator(device="cuda").manual_seed(22)
    B = 1 << 24
    ft = FLOWS[cfg]
    P = ops.total_param_size(ft, 1, True)
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((B, P), generator=gen, device="cuda")
    launcher = ops.ChainLauncher(y, t, ft, 1, True, write_values=True)
    sh = int(torch.cuda.current_stream().cuda_stream)
    for _ in range(800):  # clocks
        launcher.launch(sh)
    torch.cuda.synchronize()
    nw = 2 * torch.cuda.get_device_properties(0).multi_processor_count * 8  # >= the grid's waves
    buf = torch.zeros((2 * nw,), dtype=torch.int64, device="cuda")
    print(f"{cfg}: B = 2^24, wave start / end in 10 ns ticks, NFN_TILE_ROT={os.environ.get('NFN_TILE_ROT', '0')}")
    for rep in range(n):
        buf.zero_()
        fn(ctypes.c_void_p(buf.data_ptr()))
        launcher.launch(sh)
        fn(None)
        torch.cuda.synchronize()
        w = buf.view(-1, 2).cpu().numpy()
        w = w[w[:, 1] > 0].astype(np.float64) * 10e-3  # microseconds
        t0 = w[:, 0].min()
        s, e = w[:, 0] - t0, w[:, 1] - t0
        span = e.max()
        ends = np.sort(e)
        # time during which not all waves are still running: from the first wave end to the last
        tail = span - ends[0]
        q = np.percentile(e, [1, 10, 50, 90, 99])
        print(f"launch {rep}: {len(w)} waves; starts within {s.max():.1f} us; span {span:.1f} us; ends at "
              f"p1 {q[0]:.1f} p10 {q[1]:.1f} p50 {q[2]:.1f} p90 {q[3]:.1f} p99 {q[4]:.1f} max {span:.1f} us; "
              f"first end -> last end {tail:.1f} us ({100 * tail / span:.1f} % of the span); mean wave busy "
              f"{np.mean(e - s):.1f} us = {100 * np.mean(e - s) / span:.1f} % of the span", flush=True)
        if rep == n - 1:  # where the spread lives: by XCD (workgroups go round-robin over 8), by wave slot
            idx = np.nonzero(buf.view(-1, 2)[:, 1].cpu().numpy() > 0)[0]
            blk = idx // 4
            xcd = blk % 8
            print("  end time by XCD (mean / min / max us): " + "; ".join(
                f"{x}: {e[xcd == x].mean():.1f} / {e[xcd == x].min():.1f} / {e[xcd == x].max():.1f}" for x in range(8)))
            print("  end time by wave slot in the workgroup: " + "; ".join(
                f"{k}: {e[idx % 4 == k].mean():.1f}" for k in range(4)))
            cu = blk // 8 % 32  # the workgroup's slot within its XCD (2 per CU, so two slots per CU)
            per = np.array([e[(xcd == x) & (blk // 8 // 2 == c)].mean() for x in range(8) for c in range(16)])
            print(f"  end time by (XCD, CU guess) pair: min {per.min():.1f} max {per.max():.1f} sd {per.std():.1f} us; "
                  f"within-XCD sd of wave ends {np.mean([e[xcd == x].std() for x in range(8)]):.1f} us")
            order = np.argsort(e)
            print(f"  the earliest 5 % of waves finish by {e[order[len(e) // 20]]:.1f} us; their XCDs "
                  f"{np.bincount(xcd[order[:len(e) // 20]], minlength=8).tolist()}; latest 5 % XCDs "
                  f"{np.bincount(xcd[order[-len(e) // 20:]], minlength=8).tolist()}")


if __name__ == "__main__":
    main()
