"""Multi-GPU row sharding of GGUF weight matrices (one process per GPU, RCCL over xGMI)."""
from .row_shard import RowShardedMMQ, shard_rows, shard_bytes  # noqa: F401
