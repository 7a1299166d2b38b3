"""Pipeline-parallel planning (partitioner, piped-ring schedule model) and torchrun launch."""
from .pipeline import init_from_torchrun, plan_partition, simulate_piped_ring

__all__ = ["init_from_torchrun", "plan_partition", "simulate_piped_ring"]
