"""Data parallelism over MI355X GPUs: one process per GPU, RCCL collectives.

* :mod:`.comm`     - process-group bootstrap and packed collectives.
* :mod:`.sharding` - row-sharded datasets (:class:`ShardedArray`).
"""

from .comm import Comm, init_distributed, shard_bounds, env_world
from .sharding import ShardedArray, shard_rows

__all__ = ["Comm", "init_distributed", "shard_bounds", "env_world", "ShardedArray", "shard_rows"]
