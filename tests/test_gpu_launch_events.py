"""The measurement hook nfn_set_launch_events (include/nfn.h, ABI 203): bench.py times the
dominant kernel with events that the launch itself records (hipExtLaunchKernel), instead of
hipEventRecord markers queued around every step.

* The armed launch records both events; the interval is the kernel's (positive, and within a
  few percent of a marker pair around the same launch on an idle stream).
* The hook clears after one launch: a second launch leaves the events where they were.
* Results are the plain launch's bitwise (the hook changes how a kernel is dispatched, not what
  it computes)."""

import ctypes

import pytest
import torch

from normalizingflownetwork_amd import ops

pytestmark = pytest.mark.gpu
C2 = ("planar", "radial") * 5


def _events():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream()
    e0.record(s)  # torch creates the HIP handle at the first record
    e1.record(s)
    torch.cuda.synchronize()
    return e0, e1


def test_dispatch_events_time_the_kernel(gpu):
    from normalizingflownetwork_amd import _lib

    lib = _lib.load()
    gen = torch.Generator(device="cuda").manual_seed(3)
    B = 1 << 22
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((B, 32), generator=gen, device="cuda")
    launcher = ops.ChainLauncher(y, t, C2, 1, True, write_values=True)
    sh = int(torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        launcher.launch(sh)
    torch.cuda.synchronize()
    ref = launcher.out.clone()

    m0, m1 = _events()
    d0, d1 = _events()
    marker, dispatch = [], []
    for _ in range(5):
        m0.record()
        launcher.launch(sh)
        m1.record()
        torch.cuda.synchronize()
        marker.append(m0.elapsed_time(m1))
        assert lib.nfn_set_launch_events(ctypes.c_void_p(d0.cuda_event), ctypes.c_void_p(d1.cuda_event)) == 0
        launcher.launch(sh)
        torch.cuda.synchronize()
        dispatch.append(d0.elapsed_time(d1))
        assert torch.equal(launcher.out, ref)
    km, kd = sorted(marker)[2], sorted(dispatch)[2]
    assert 0.0 < kd <= km * 1.05, (kd, km)
    assert kd >= 0.8 * km, (kd, km)

    # the hook cleared: an unarmed launch does not move the events
    before = d0.elapsed_time(d1)
    launcher.launch(sh)
    torch.cuda.synchronize()
    assert d0.elapsed_time(d1) == before
    assert torch.equal(launcher.out, ref)
