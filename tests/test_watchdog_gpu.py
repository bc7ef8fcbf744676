"""RCCL failure detection (csrc/runtime/rccl_comm.cpp CommWatchdog): a collective that completes is
retired silently; a stream that stays busy past the timeout (stand-in for a collective stuck on a
dead peer: a finite sleep kernel, so no RCCL kernel is in flight when the communicator is aborted)
aborts the communicator and latches an error that later calls raise."""
import time

import pytest
import torch

from pytorch_distributed_example_amd._ext import runtime

pytestmark = pytest.mark.gpu


def _comm():
    R = runtime()
    return R, R.RcclComm(R.RcclComm.make_unique_id(), 0, 1, torch.cuda.current_device())


def test_watchdog_retires_completed_collectives():
    R, comm = _comm()
    wd = R.CommWatchdog(comm, 10_000, 2)
    s = torch.cuda.Stream()
    t = torch.arange(4096, device="cuda", dtype=torch.float32)
    s.wait_stream(torch.cuda.current_stream())
    for _ in range(5):
        comm.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), 0, 0, s.cuda_stream)
        wd.watch(s.cuda_stream, "all_reduce")
    s.synchronize()
    deadline = time.time() + 5
    while wd.pending() and time.time() < deadline:
        time.sleep(0.005)
    assert wd.pending() == 0 and wd.error() == ""
    assert torch.equal(t.cpu(), torch.arange(4096, dtype=torch.float32))
    wd.stop()
    comm.destroy()


def test_watchdog_aborts_on_timeout():
    R, comm = _comm()
    wd = R.CommWatchdog(comm, 20, 2)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        torch.cuda._sleep(500_000_000)           # ~0.2 s of clock64() spinning: far past 20 ms
    wd.watch(s.cuda_stream, "stuck_all_reduce")
    deadline = time.time() + 30
    while not wd.error() and time.time() < deadline:
        time.sleep(0.005)
    err = wd.error()
    assert "stuck_all_reduce" in err and "aborted" in err, err
    s.synchronize()
    t = torch.ones(8, device="cuda")
    with pytest.raises(RuntimeError, match="destroyed or aborted"):
        comm.all_reduce(t.data_ptr(), t.data_ptr(), 8, 0, 0, s.cuda_stream)
    wd.stop()
