"""Parallel execution: shard planner, one-process-per-GPU torch.distributed
(RCCL over xGMI) data parallelism, and host streaming / single-process
multi-GPU through the native engine."""
from . import shard
from .shard import Shard, chunks, ctr_add, equal_plan, plan

__all__ = ["shard", "Shard", "plan", "equal_plan", "ctr_add", "chunks"]
