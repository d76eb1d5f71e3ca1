from .datasets import (MNIST, SyntheticImageNet, SyntheticMNIST, TensorDataset, input_affine,
                       load_mnist, normalize_input, synthetic_classification)
from .loader import DeviceCursor, DeviceLoader, Gathered
from .samplers import MySampler, PartitionSampler, RandomSampleSampler, make_sampler

__all__ = ["MNIST", "SyntheticMNIST", "SyntheticImageNet", "TensorDataset", "load_mnist",
           "synthetic_classification", "input_affine", "normalize_input", "DeviceLoader", "DeviceCursor", "Gathered", "MySampler", "PartitionSampler",
           "RandomSampleSampler", "make_sampler"]
