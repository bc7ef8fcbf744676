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


def _cpu_list(spec: str):
    cpus = set()
    for part in spec.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def gpu_local_cpus(device: int = 0):
    """(PCI address, CPU set) of the host NUMA node nearest to visible GPU ``device``, read from the
    KFD topology and sysfs without initialising HIP; None when unavailable.  Visible GPUs are the KFD
    GPU nodes in node order, filtered by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES when set (the HIP
    runtime's own enumeration order)."""
    import glob
    import os
    try:
        nodes = []
        for path in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
            props = {}
            try:                      # a container may hide other GPUs' nodes (EPERM): not ours
                with open(path) as f:
                    for line in f:
                        k, _, v = line.partition(" ")
                        props[k] = v.strip()
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                nodes.append((int(path.split("/")[-2]), props))
        nodes.sort()
        for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
            sel = os.environ.get(var)
            if sel and all(s.strip().isdigit() for s in sel.split(",")):
                picked = [nodes[int(s)] for s in sel.split(",") if int(s) < len(nodes)]
                if len(picked) == len(sel.split(",")) and len(nodes) > len(picked):
                    nodes = picked
        props = nodes[device][1]
        loc, dom = int(props["location_id"]), int(props.get("domain", "0"))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"
        with open(f"/sys/bus/pci/devices/{bdf}/local_cpulist") as f:
            cpus = _cpu_list(f.read())
        return (bdf, cpus) if cpus else None
    except Exception:   # noqa: BLE001 - topology not readable: leave the affinity alone
        return None


def bind_local_numa(device: int = 0, node_devices=None, min_cpus_per_rank: int = 4):
    """Pin this process to the CPUs of the NUMA node nearest to GPU ``device`` (call before the first
    HIP call, so the runtime's own threads inherit it): the host side of every launch and of every
    synchronize (doorbell writes, completion-signal polling) then stays on the GPU's socket.
    ``node_devices``: the GPU of every rank on this host; the ranks whose GPU shares this NUMA node
    share its CPUs, and with fewer than ``min_cpus_per_rank`` each (a container granted few CPUs)
    nothing is pinned -- spinning host waits of several ranks on a handful of cores would cost more
    than the socket locality gains.  Returns the GPU's PCI address, or None if nothing was changed."""
    import os
    got = gpu_local_cpus(device)
    if got is None:
        return None
    bdf, cpus = got
    allowed = os.sched_getaffinity(0)
    use = cpus & allowed
    sharing = 1
    if node_devices is not None:
        sharing = max(1, sum(1 for d in node_devices
                             if d == device or ((g := gpu_local_cpus(d)) is not None and g[1] == cpus)))
    if not use or use == allowed or len(use) < min_cpus_per_rank * sharing:
        return None
    os.sched_setaffinity(0, use)
    _NUMA_PREV[0] = allowed
    return bdf


_NUMA_PREV = [None]   # the affinity bind_local_numa replaced


def verify_numa_binding(bdf, device: int = 0, props=None) -> bool:
    """After HIP is up: check that ``bdf`` (bind_local_numa's pick, from KFD node order) is the PCI
    address the runtime reports for ``device``.  On a mismatch (a runtime that orders GPUs otherwise)
    the previous affinity is restored and False returned; True when it matches or nothing was bound."""
    import os
    if bdf is None:
        return True
    if props is None:
        import torch
        props = torch.cuda.get_device_properties(device)
    want = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
    if bdf.lower().startswith(want):
        return True
    if _NUMA_PREV[0] is not None:
        os.sched_setaffinity(0, _NUMA_PREV[0])
        _NUMA_PREV[0] = None
    return False
