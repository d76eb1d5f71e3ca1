from .optimizers import AdamOptimizer, BaseOptimizer, GdOptimizer, SGD

Adam = AdamOptimizer
GD = GdOptimizer
MyOptimizer = BaseOptimizer

__all__ = ["BaseOptimizer", "GdOptimizer", "AdamOptimizer", "SGD", "Adam", "GD"]
