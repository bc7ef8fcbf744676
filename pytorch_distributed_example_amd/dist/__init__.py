"""torch.distributed-compatible process-group API over the framework's C++ runtime
(TCP rendezvous store, host TCP collectives, RCCL over xGMI).  See ``dist/api.py``."""
from .api import (  # noqa: F401
    Backend, DEFAULT_TIMEOUT, P2POp, batch_isend_irecv, EngineComm, GroupMember, ProcessGroup, ReduceOp, Work, all_gather,
    all_gather_into_tensor, all_reduce, all_to_all_single, barrier, broadcast, broadcast_coalesced, broadcast_parameters,
    destroy_process_group, engine_comm, gather, get_backend, gpu_launch, get_default_group, get_rank, get_world_size,
    init_process_group, irecv, is_available, is_initialized, isend, new_group, recv, reduce, reduce_op,
    reduce_scatter, reduce_scatter_tensor, scatter, send,
)
