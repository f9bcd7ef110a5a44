"""Distributed training: RCCL communicator, DistOpt (sync DP), EASGD and
RandomSync asynchronous-style exchange, layer/data partitioning."""
from .communicator import Communicator, init_distributed, get_communicator  # noqa: F401
from .distopt import DistOpt  # noqa: F401
