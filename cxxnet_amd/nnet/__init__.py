"""Graph executor and trainer (reference src/nnet/)."""
from .arena import ParamArena  # noqa: F401
from .neural_net import NeuralNet  # noqa: F401
from .trainer import NetTrainer, parse_devices  # noqa: F401


def create_net(net_type: int = 0) -> NetTrainer:
    """Reference CreateNet<xpu>(net_type) (src/nnet/nnet.h:99-100)."""
    return NetTrainer(net_type)
