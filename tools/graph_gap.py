"""Back-to-back C2 forward launches: stream launches vs one replayed HIP graph of the same
launches (torch.cuda.CUDAGraph over ChainLauncher.launch), wall clock per launch and the gap
it leaves beside the kernel's own duration (events recorded by the dispatch,
nfn_set_launch_events).  The question: does a graph shorten the ~6 us between consecutive
launches that bench.py's `value` carries?

  python tools/graph_gap.py [n_launches]"""

import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflownetwork_amd import _lib, ops  # noqa: E402

C2 = ("planar", "radial") * 5


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    lib = _lib.load()
    gen = torch.Generator(device="cuda").manual_seed(22)
    B = 1 << 24
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((B, 32), generator=gen, device="cuda")
    s = torch.cuda.Stream()
    launcher = ops.ChainLauncher(y, t, C2, 1, True, write_values=True)
    sh = int(s.cuda_stream)
    with torch.cuda.stream(s):
        for _ in range(800):  # clocks
            launcher.launch(sh)
    torch.cuda.synchronize()
    ref = launcher.out.clone()

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    e1.record(s)
    torch.cuda.synchronize()

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            launcher.launch(sh)
    torch.cuda.synchronize()

    rows = []
    for rep in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            launcher.launch(sh)
        torch.cuda.synchronize()
        w_stream = (time.perf_counter() - t0) / n * 1e3
        t0 = time.perf_counter()
        for _ in range(n):
            launcher.launch(0)  # the legacy default stream
        torch.cuda.synchronize()
        w_null = (time.perf_counter() - t0) / n * 1e3
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        w_graph = (time.perf_counter() - t0) / n * 1e3
        ks = []
        for _ in range(10):
            lib.nfn_set_launch_events(ctypes.c_void_p(e0.cuda_event), ctypes.c_void_p(e1.cuda_event))
            launcher.launch(sh)
            torch.cuda.synchronize()
            ks.append(e0.elapsed_time(e1))
        k = float(np.median(ks))
        rows.append((w_stream, w_graph, k))
        print(f"rep {rep}: kernel {k:.4f} ms | stream launches {w_stream:.4f} ms/launch (gap {1e3 * (w_stream - k):.1f} us)"
              f" | graph replay {w_graph:.4f} ms/launch (gap {1e3 * (w_graph - k):.1f} us)"
              f" | default stream {w_null:.4f} ms/launch (gap {1e3 * (w_null - k):.1f} us)", flush=True)
    assert torch.equal(launcher.out, ref)
    print("outputs bitwise equal after the graph replays")


if __name__ == "__main__":
    main()
