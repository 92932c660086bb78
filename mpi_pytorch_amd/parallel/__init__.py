from .dist import World, init_world, get_world, shutdown, barrier, env_rank_info  # noqa: F401
from .arena import ParamArena, weight_of, grad_sink, grad_done  # noqa: F401
from .ddp import GradBucketer  # noqa: F401
from .comm import (num_processes, mpi_all_reduce, mpi_sum, mpi_avg_grads,  # noqa: F401
                   mpi_broadcast, sync_params, scatter_object, broadcast_object,
                   reduce_scalar, all_gather_object, replica_checksum,
                   agree_tuned_tiles)
from .sharding import array_split_sizes, shard_bounds, shard_dataframe  # noqa: F401
from .watchdog import Watchdog  # noqa: F401
