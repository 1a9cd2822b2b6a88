"""Distribution: process groups (RCCL/gloo), FedAvg collectives, launcher, TCP compat transport."""
from .comm import DistInfo, barrier, init_distributed, shutdown  # noqa: F401
from .fedavg import aggregate_state_dicts, broadcast_model, fedavg_  # noqa: F401
