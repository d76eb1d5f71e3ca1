from .lenet import LeNet, Net, SubNetConv, SubNetFC
from .mlp import MLP, ForwardNN
from .resnet import ResNet18

MODELS = {"lenet": Net, "mlp": ForwardNN, "resnet18": ResNet18}


def build_model(name: str, **kw):
    return MODELS[name](**kw)


__all__ = ["Net", "LeNet", "SubNetConv", "SubNetFC", "ForwardNN", "MLP", "ResNet18",
           "MODELS", "build_model"]
