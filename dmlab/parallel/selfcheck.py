"""Startup self-checks of the device communication paths a multi-GPU run depends on.

The reference's data parallelism is NCCL collectives between ranks on different GPUs
(codes/task2/dist_utils.py:39-49, codes/task3/dist_utils.py:40-46) and its lab-4 pipeline
moves activations stage to stage (codes/task4/model.py:57-60).  On this project's one-GPU
test pool none of those device paths can cross a GPU boundary, so the first multi-GPU run
must prove them itself, cheaply and before anything is timed:

* :func:`allreduce_selfcheck` -- an all-reduce of a rank-coded tensor checked against its
  CLOSED-FORM sum on every rank (equal-but-wrong replicas fail it, which a replica
  consistency check cannot see);
* :func:`xgmi_selfcheck` -- one call of the one-shot peer-memory kernel
  (:class:`~dmlab.parallel.xgmi.XGMIAllReduce`) on the same data as RCCL, exact equality
  required; any error, kernel timeout (its bounded flag wait) or mismatch on ANY rank
  selects RCCL on every rank;
* :func:`p2p_selfcheck` -- one ping-pong over a pipeline transport (activation direction,
  then gradient direction), payload checked both ways.

Every verdict is agreed over the group (MIN of the per-rank results), so all ranks take
the same path.  ``corrupt=r`` (tests; ``DMLAB_SELFCHECK_CORRUPT=<check>:<rank>`` for a live
run) perturbs rank r's data so the check must fail.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def _corrupt_rank(name: str, corrupt):
    if corrupt is not None:
        return corrupt
    spec = os.environ.get("DMLAB_SELFCHECK_CORRUPT", "")
    for item in spec.split(","):
        if ":" in item:
            k, r = item.split(":", 1)
            if k.strip() == name:
                return int(r)
    return None


def _flag_device(device, group):
    return device if dist.get_backend(group) == "nccl" else torch.device("cpu")


def agree(ok: bool, device, group=None) -> bool:
    """True iff ``ok`` holds on every rank of ``group``."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=_flag_device(device, group))
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def _coded(n: int, rank: int, device):
    """x[i] = (rank + 1) * (i % 4093 + 1): every partial sum over <= 8 ranks is an integer
    below 2^24, so fp32 sums are exact in any order."""
    base = (torch.arange(n, dtype=torch.float32, device=device) % 4093) + 1
    return base * (rank + 1), base


def allreduce_selfcheck(device, group=None, n: int = 1 << 18, corrupt=None) -> dict:
    rank, ws = dist.get_rank(group), dist.get_world_size(group)
    dv = _flag_device(device, group)
    x, base = _coded(n, rank, dv)
    if _corrupt_rank("allreduce", corrupt) == rank:
        x[n // 2] += 1.0
    dist.all_reduce(x, group=group)
    expect = base * float(ws * (ws + 1) // 2)
    ok = bool(torch.equal(x, expect))
    err = float((x - expect).abs().max())
    ok_all = agree(ok, device, group)
    return {"allreduce_selfcheck": "pass" if ok_all else "FAIL",
            "allreduce_selfcheck_elems": n, "allreduce_selfcheck_max_err": err}


def xgmi_selfcheck(device, group=None, n: int = 51902, cap: int | None = None,
                   corrupt=None) -> dict:
    """One xGMI all-reduce of ``n`` floats (default: LeNet's 51,902 gradients) vs RCCL.
    Returns the report; ``report["small_allreduce_used"]`` is "xgmi" only if every rank
    passed."""
    rank = dist.get_rank(group)
    ok, why, xg = False, "", None
    try:
        from dmlab.parallel import xgmi

        if torch.device(device).type != "cuda":
            raise RuntimeError("not a GPU device")
        xg = xgmi.XGMIAllReduce(cap=cap or max(n, 1 << 16), group=group, device=device)
        x, _ = _coded(n, rank, device)
        ref = x.clone()
        dist.all_reduce(ref, group=group)
        xg(x)
        torch.cuda.synchronize(device)
        xg.check()  # raises if a peer's flag never arrived (the kernel's bounded wait)
        if _corrupt_rank("xgmi", corrupt) == rank:
            x[n // 3] += 1.0
        ok = bool(torch.equal(x, ref))
        if not ok:
            why = f"mismatch (max err {float((x - ref).abs().max())})"
    except Exception as e:  # the path is optional: any failure selects RCCL
        ok, why = False, f"{type(e).__name__}: {e}"[:200]
    ok_all = agree(ok, device, group)
    if xg is not None:
        try:
            xg.close()
        except Exception:
            pass
    rep = {"xgmi_selfcheck": "pass" if ok_all else "fail",
           "small_allreduce_used": "xgmi" if ok_all else "rccl"}
    if not ok_all:
        rep["xgmi_selfcheck_reason"] = why or "failed on another rank"
    return rep


def p2p_selfcheck(p2p, rank: int, peer, device, first: bool, numel: int = 32 * 400,
                  corrupt=None, group=None) -> dict:
    """One ping-pong between ``rank`` and ``peer`` over transport ``p2p`` (the pipeline's
    ``send``/``recv`` API): ``first`` sends x on the activation key and expects 2x + 1 back
    on the gradient key; the other side checks x and replies.  Every rank of the default
    group must call it (the verdict is agreed over ``group``); a rank outside the pair passes
    ``peer=None``."""
    # Readiness first: a side that cannot even start (no channel to its peer, a payload it
    # cannot build) must not leave its peer blocked in a receive until the process-group
    # timeout, so every rank agrees before any message is posted.  Past this point both sides
    # post the same messages; a transfer that then fails is bounded by the transport itself
    # (the xGMI channel's flag wait times out; RCCL/gloo by the PG timeout, 120 s in task4).
    ready = True
    try:
        x, _ = _coded(numel, 0, device)
        if peer is not None and hasattr(p2p, "chan"):
            ready = (rank, peer) in p2p.chan and (peer, rank) in p2p.chan
    except Exception:
        ready = False
    if not agree(ready, device, group):
        return {"p2p_selfcheck": "FAIL"}
    ok = True
    try:
        if peer is None:
            raise StopIteration
        if first:
            for w in p2p.send(x, peer, "selfcheck"):
                w.wait()
            buf, h = p2p.recv(peer, "grad_selfcheck", device)
            h.wait()
            buf = buf.to(device)
            ok = bool(torch.equal(buf, 2 * x + 1))
        else:
            buf, h = p2p.recv(peer, "selfcheck", device)
            h.wait()
            buf = buf.to(device)
            ok = bool(torch.equal(buf, x))
            reply = 2 * buf + 1
            if _corrupt_rank("p2p", corrupt) == rank:
                reply[numel // 2] += 1.0
            for w in p2p.send(reply, peer, "grad_selfcheck"):
                w.wait()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if hasattr(p2p, "check"):
            p2p.check()
    except StopIteration:
        pass
    except Exception:
        ok = False
    ok_all = agree(ok, device, group)
    return {"p2p_selfcheck": "pass" if ok_all else "FAIL"}
