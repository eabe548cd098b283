"""Distributed execution over RCCL (torch.distributed backend "nccl" on ROCm)."""
from .dp import GradReducer, init_distributed, world_info  # noqa: F401
