from .summary import ScalarWriter, getSummaryWriter, read_events
from .timers import PhaseTimer, Wall

__all__ = ["ScalarWriter", "getSummaryWriter", "read_events", "PhaseTimer", "Wall"]
