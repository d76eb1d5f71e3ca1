from . import comm, env
from .comm import (GradAggregator, allgather_average_gradients, allreduce_average_gradients,
                   average_gradients, dist_init, init_parameters)
from .ddp import DDP, DistributedDataParallel
from .straggler import Straggler

__all__ = ["env", "comm", "GradAggregator", "dist_init", "init_parameters",
           "allreduce_average_gradients", "allgather_average_gradients", "average_gradients",
           "DistributedDataParallel", "DDP", "Straggler"]
