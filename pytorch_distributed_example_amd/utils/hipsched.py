"""Host-side wait policy of the HIP runtime.

By default a host thread blocked in ``hipDeviceSynchronize`` / ``hipStreamSynchronize`` may yield or
sleep.  After a long wait (e.g. the host ran far ahead of a deep queue of graph replays) the core it
wakes on is slow for the next ~ms, and the next ``hipGraphLaunch`` -- which writes one AQL packet per
node from the host -- then submits a 120-node LeNet graph at 5-9 us/node instead of ~0.5, slower
than the GPU retires the ~10 us nodes: the GPU starves at the start of the window
(profiles/r2_lenet_v3/host_launch_spin.txt: 180-1590 us vs 52-75 us to launch a 20-step graph).
``hipDeviceScheduleSpin`` keeps the waiting thread spinning, so the launch path stays hot.  It must
be set before the process creates its HIP context (before the first torch.cuda call that touches the
device); later calls are refused by the runtime and reported as False.
"""
from __future__ import annotations

import ctypes

HIP_DEVICE_SCHEDULE_AUTO = 0
HIP_DEVICE_SCHEDULE_SPIN = 1
HIP_DEVICE_SCHEDULE_YIELD = 2


def set_schedule(device: int = 0, flag: int = HIP_DEVICE_SCHEDULE_SPIN) -> bool:
    """``hipSetDevice(device)`` + ``hipSetDeviceFlags(flag)``; True on success.  No-op (False)
    without a HIP runtime library (CPU-only hosts)."""
    try:
        lib = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return False
    if lib.hipSetDevice(ctypes.c_int(device)) != 0:
        return False
    return lib.hipSetDeviceFlags(ctypes.c_uint(flag)) == 0
