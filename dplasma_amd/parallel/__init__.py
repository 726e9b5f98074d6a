"""Inter-GPU communication: torch.distributed (RCCL over xGMI / gloo)."""
