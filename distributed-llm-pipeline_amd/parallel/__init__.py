"""Pipeline-parallel planning (partitioner, piped-ring schedule model), torchrun launch and
rank restart (checkpointed elastic generation)."""
from .elastic import generate_elastic, latest_checkpoint
from .pipeline import init_from_torchrun, plan_partition, simulate_piped_ring

__all__ = ["generate_elastic", "init_from_torchrun", "latest_checkpoint", "plan_partition", "simulate_piped_ring"]
