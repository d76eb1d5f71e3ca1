from .flat import FlatParams
from .layers import (BasicBlock, Conv2d, ConvBN, ConvBNPool, Flatten, GlobalAvgPool, Linear,
                     MaxPool, Softmax)
from .loss import CrossEntropyLoss, count_correct, cross_entropy
from .program import Ctx, Layer, Program

__all__ = ["FlatParams", "Program", "Layer", "Ctx", "Conv2d", "Linear", "Flatten", "Softmax",
           "ConvBN", "ConvBNPool", "BasicBlock", "MaxPool", "GlobalAvgPool", "CrossEntropyLoss",
           "cross_entropy", "count_correct"]
