"""Reference-compatible config-driven runtime: layers, NeuralNet, Worker."""
from .layers import REGISTRY, create_layer  # noqa: F401
from .neuralnet import NeuralNet  # noqa: F401
from .worker import Worker, Performance, make_updater  # noqa: F401
