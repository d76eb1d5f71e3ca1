from .datasets import (MNIST, SyntheticImageNet, SyntheticMNIST, TensorDataset, load_mnist,
                       synthetic_classification)
from .loader import DeviceLoader
from .samplers import MySampler, PartitionSampler, RandomSampleSampler, make_sampler

__all__ = ["MNIST", "SyntheticMNIST", "SyntheticImageNet", "TensorDataset", "load_mnist",
           "synthetic_classification", "DeviceLoader", "MySampler", "PartitionSampler",
           "RandomSampleSampler", "make_sampler"]
