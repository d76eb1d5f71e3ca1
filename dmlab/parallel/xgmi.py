"""One-/two-shot all-reduce over xGMI peer memory (``csrc/comm_xgmi.hip``).

SURVEY §2.7 / build plan step 4: RCCL's ring all-reduce takes 2(W-1) latency-bound steps,
which dominates for the labs' small gradient messages (LeNet: 51,902 floats).  Every rank
allocates one IPC-shareable, uncached device buffer ([2][cap] floats of data in two parity
halves + a [64][8] flag array), exchanges its ``hipIpcMemHandle`` through the process
group (``all_gather_object``) and opens every peer's.  A call is ONE kernel: copy the
slice in, flag every peer, wait for every peer's flag, sum the W slices in rank order
(identical bits on every rank).  Large messages take the two-shot kernel instead: reduce-scatter of W rank slices (each
rank sums ITS slice from all W buffers) then all-gather of the reduced slices, two flag
phases, 2(W-1)/W of the bytes per rank over all W-1 links at once.  Waits are bounded: a
missing peer raises
:class:`RuntimeError` on :meth:`check` (synchronous) or :meth:`poll` (asynchronous: DDP
calls it at the end of every backward; it never blocks) instead of hanging the GPU.

The call epoch (flag value and parity half) is a device-side counter the kernel advances
itself, so a captured hipGraph replays correctly: each replay is a new epoch.

Requirements: one process per GPU on one node (or several processes sharing one GPU, as
the tests do), ``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf IPC), fp32 contiguous tensors of
at most ``cap`` elements.  RCCL stays the default everywhere; this path is opted into
(``DistributedDataParallel(..., small_allreduce="xgmi")``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from dmlab.ops._native import lib

_FLAG_BYTES = 2 * 256 * 8 * 4  # [2 phases][256 blocks][8 ranks] uint32
# auto: two-shot from 1 MB up with >= 3 ranks (at W = 2 both read n remote floats)
_TWO_SHOT_MIN = 1 << 18
_ALGOS = {"one_shot": 0, "two_shot": 1}


def _device_key(device) -> str:
    """Identity of the physical GPU behind ``device`` (UUID or PCI location when the runtime
    reports them; host + index otherwise)."""
    import socket

    if torch.device(device).type != "cuda":
        return f"{socket.gethostname()}:{device}"
    p = torch.cuda.get_device_properties(device)
    uuid = getattr(p, "uuid", None)
    if uuid:
        return str(uuid)
    pci = tuple(getattr(p, a, None) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if any(v is not None for v in pci):
        return f"{socket.gethostname()}:{pci}"
    return f"{socket.gethostname()}:{torch.device(device).index}"


class XGMIAllReduce:
    def __init__(self, cap: int = 1 << 20, group=None, device=None, algo: str = "auto"):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("xGMI all-reduce supports up to 8 ranks (one node)")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        # multiple of 4 floats: keeps both parity halves 16-B aligned for the float4 path
        self.cap = (int(cap) + 3) // 4 * 4
        if algo not in ("auto", *_ALGOS):
            raise ValueError("algo: 'auto' | 'one_shot' | 'two_shot'")
        self.algo = algo
        # every step below can fail on one rank only; failures are exchanged in the two
        # all_gather_object calls every rank makes, so all ranks raise together
        L, self._base, handle, err = None, 0, None, None
        try:
            L = lib()
            self._base = L.xgmi_alloc(8 * self.cap + _FLAG_BYTES)
            handle = L.xgmi_get_handle(self._base)
        except Exception as e:
            err = f"rank {self.rank} alloc: {type(e).__name__}: {e}"
        handles = [None] * self.world
        dist.all_gather_object(handles, (handle, err), group=group)
        errs0 = [e for _, e in handles if e]
        handles = [h for h, _ in handles]
        self._opened = []
        bases = []
        try:
            if errs0:
                raise RuntimeError("; ".join(errs0))
            for q, h in enumerate(handles):
                if q == self.rank:
                    bases.append(self._base)
                else:
                    p = L.xgmi_open_handle(h)
                    self._opened.append(p)
                    bases.append(p)
        except Exception as e:  # reported to every rank below, so all fail together
            err = f"rank {self.rank}: {type(e).__name__}: {e}"
        self._data = bases
        self._flags = [b + 8 * self.cap for b in bases]
        # ranks whose kernels share one physical GPU (1 on a node with one rank per GPU; the
        # single-GPU rehearsals run W ranks on one device): the spinning grids shrink by it so
        # every rank's blocks are resident together.  The kernels split the data by gridDim
        # and match flags by block index, so EVERY rank must launch the same grid: the divisor
        # is the most crowded device's count, identical on all ranks.  The same exchange
        # carries each rank's handle-open status: one failed open fails every rank (no rank
        # is left waiting in a later collective).
        keys = [None] * self.world
        dist.all_gather_object(keys, (_device_key(self.device), err), group=group)
        errs = [e for _, e in keys if e]
        if errs:
            for p in self._opened:
                L.xgmi_close_handle(p)
            self._opened = []
            dist.barrier(group=group)
            if self._base:
                L.xgmi_free(self._base)
            self._base = 0
            raise RuntimeError("xGMI all-reduce: peer memory mapping failed: " + "; ".join(errs))
        keys = [k for k, _ in keys]
        self._share = max(1, max(keys.count(k) for k in keys))
        # [timeout flag, last published epoch, done-block counter, pad] (device side)
        self._state = torch.zeros(4, dtype=torch.int32, device=self.device)
        self._calls = 0
        # asynchronous error poll: a pinned copy of the flag plus the event that completes it
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._err_event = None
        dist.barrier(group=group)

    def _algo(self, n: int, algo: str | None) -> int:
        algo = algo or self.algo
        if algo == "auto":
            algo = "two_shot" if (self.world >= 3 and n >= _TWO_SHOT_MIN) else "one_shot"
        return _ALGOS[algo]

    def __call__(self, t: torch.Tensor, scale: float = 1.0, out: torch.Tensor | None = None,
                 algo: str | None = None):
        """out (default: t, in place) = scale * Σ_ranks t.  Stream-ordered on the current
        stream; returns ``out``.  ``algo`` overrides the instance's choice for this call
        (every rank must pass the same)."""
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() > self.cap:
            raise ValueError("xGMI all-reduce: fp32 contiguous tensor of <= cap elements")
        out = t if out is None else out
        self._calls += 1
        lib().xgmi_allreduce(t, out, self.cap, self._data, self._flags, self.rank, float(scale),
                             self._state, self._algo(t.numel(), algo), self._share)
        return out

    @property
    def epoch(self) -> int:
        """Calls completed on the device so far (synchronises)."""
        return int(self._state[1].item())

    def _raise(self):
        raise RuntimeError("xGMI all-reduce: a peer never arrived (timed out); this rank's "
                           "bucket kept its local gradient, so the replicas have diverged")

    def check(self):
        """Raise if any call so far timed out waiting for a peer (synchronises)."""
        if int(self._state[0].item()):
            self._raise()

    def poll(self):
        """Non-blocking error check on the current stream: raises if an earlier poll's copy of
        the timeout flag has landed and is set, then queues the next copy.  Never
        synchronises; skipped while a hipGraph is being captured."""
        if torch.cuda.is_current_stream_capturing():
            return
        ev = self._err_event
        if ev is not None:
            if not ev.query():
                return  # the previous copy is still in flight: look again next time
            if int(self._err_host[0]):
                self._raise()
        self._err_host.copy_(self._state[:1], non_blocking=True)
        self._err_event = torch.cuda.Event()
        self._err_event.record()

    def close(self):
        L = lib()
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        for p in self._opened:
            L.xgmi_close_handle(p)
        self._opened = []
        dist.barrier(group=self.group)
        if self._base:
            L.xgmi_free(self._base)
            self._base = 0
