"""Multi-GPU execution: communicators, ledger sharding, distributed stage drivers."""
from .comm import DistComm, LocalComm
from .ledger import shard_by_k, worker_filter
