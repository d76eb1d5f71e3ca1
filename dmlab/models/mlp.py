"""The MindSpore lab-1 MLP ``ForwardNN`` (codes/task1/mindspore/model.ipynb):
Dense 784→512→256→128→64→32→10 with ReLU (576,810 params).

The notebook ends the network with a softmax and then applies
``SoftmaxCrossEntropyWithLogits`` (double softmax); by default
this model emits logits, ``reference_compat=True`` restores the softmax."""
from __future__ import annotations

from dmlab.nn.layers import Flatten, Linear, Softmax
from dmlab.nn.program import Program


class ForwardNN(Program):
    DIMS = (784, 512, 256, 128, 64, 32, 10)

    def __init__(self, dims=DIMS, reference_compat: bool = False):
        super().__init__()
        layers = [Flatten()]
        self.fcs = []
        for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
            fc = Linear(a, b, relu=i < len(dims) - 2)
            setattr(self, f"fc{i + 1}", fc)
            layers.append(fc)
        self.flatten = layers[0]
        if reference_compat:
            self.softmax = Softmax()
            layers.append(self.softmax)
        self.build(layers)


MLP = ForwardNN
