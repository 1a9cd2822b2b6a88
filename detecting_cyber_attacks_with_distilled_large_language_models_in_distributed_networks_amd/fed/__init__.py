"""Federated orchestration: per-GPU client rounds (collective FedAvg) and the TCP-compatible server."""
from .runner import FederatedClient, run_federated  # noqa: F401
