"""dmlab: an MI355X-native distributed-training lab harness (see README.md)."""
import os as _os

# HIP hardware queues per process.  HIP maps every stream onto one of GPU_MAX_HW_QUEUES
# hardware queues (default 4) and two streams on one queue execute their kernels in
# submission order, i.e. serially.  A data-parallel ResNet-18 step uses the main stream,
# the weight-gradient side stream, the downsample stream and RCCL's streams: with 4 queues
# the side stream can land on the main stream's queue (measured: the whole step on one
# queue, 22.7 vs 20.4 ms, profiles/hw_queue_collision_r4.txt).  8 queues give every stream
# its own.  Must be set before the HIP runtime initialises (the first device call), so it is
# set at import; an explicit larger value, or DMLAB_HW_QUEUES, wins.
_want = int(_os.environ.get("DMLAB_HW_QUEUES", "8"))
if int(_os.environ.get("GPU_MAX_HW_QUEUES", "4")) < _want:
    _os.environ["GPU_MAX_HW_QUEUES"] = str(min(_want, 32))
