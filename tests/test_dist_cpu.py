"""Multi-process (gloo, CPU) tests of the lab-2/3 communication layer and DDP."""
import copy
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F

from dist_helpers import run_dist

pytestmark = pytest.mark.slow


def _make(seed):
    from dmlab.models import Net

    torch.manual_seed(seed)
    return Net()


def _aggregation_equivalence(rank, ws, out):
    from dmlab.parallel import comm

    torch.manual_seed(100 + rank)
    m1 = _make(rank)  # different weights per rank ...
    comm.init_parameters(m1)  # ... until broadcast
    m2 = _make(0)
    comm.init_parameters(m2)
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(a, b)
    x = torch.rand(8, 1, 28, 28)
    y = torch.randint(0, 10, (8,))
    for m in (m1, m2):
        F.cross_entropy(m(x), y).backward()
    local = [p.grad.clone() for p in m1.parameters()]
    comm.allreduce_average_gradients(m1)
    comm.allgather_average_gradients(m2)
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-7)
    # the mean really is the mean of the per-rank gradients
    gathered = [torch.zeros_like(local[0]) for _ in range(ws)]
    dist.all_gather(gathered, local[0])
    torch.testing.assert_close(m1.conv1.weight.grad, torch.stack(gathered).mean(0),
                               rtol=1e-5, atol=1e-7)
    # per-parameter (reference call pattern) gives the same answer
    m3 = _make(0)
    F.cross_entropy(m3(x), y).backward()
    comm.allreduce_average_gradients(m3, granularity="per_param")
    for a, b in zip(m1.parameters(), m3.parameters()):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("ws", [2, 3])
def test_allreduce_equals_allgather(ws):
    run_dist(_aggregation_equivalence, ws, None)


def _reference_bug(rank, ws, out):
    from dmlab.parallel import comm

    m = _make(0)
    x = torch.rand(4, 1, 28, 28) + rank
    F.cross_entropy(m(x), torch.zeros(4, dtype=torch.long)).backward()
    mine = m.fc2.bias.grad.clone()
    last = mine.clone()
    dist.broadcast(last, ws - 1)
    comm.allgather_average_gradients_reference_compat(m)
    # every rank ends up with the LAST rank's gradient, not the mean
    torch.testing.assert_close(m.fc2.bias.grad, last)


def test_reference_allgather_bug_reproduced():
    run_dist(_reference_bug, 2, None)


def _ddp_equivalence(rank, ws, path):
    """DDP on ws ranks with batch b each == one process on the concatenated batch."""
    from dmlab.models import Net
    from dmlab.optim import SGD
    from dmlab.parallel import DDP

    torch.manual_seed(0)
    model = Net()
    ref = Net()
    ref.load_state_dict(model.state_dict())
    g = torch.Generator().manual_seed(7)
    X = torch.rand(ws * 6, 1, 28, 28, generator=g)
    Y = torch.randint(0, 10, (ws * 6,), generator=g)
    ddp = DDP(model, bucket_cap_mb=0.05, first_bucket_mb=0.01)  # several buckets
    assert len(ddp.buckets) >= 2
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9)
    ddp.fold_average_into(opt)
    opt_ref = SGD(ref.parameters(), lr=0.1, momentum=0.9)
    for step in range(3):
        xs, ys = X[rank * 6:(rank + 1) * 6], Y[rank * 6:(rank + 1) * 6]
        loss = F.cross_entropy(ddp(xs), ys)
        opt.zero_grad()
        loss.backward()
        opt.step()
        lr = F.cross_entropy(ref(X), Y)
        opt_ref.zero_grad()
        lr.backward()
        opt_ref.step()
    for (n, a), (_, b) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5, msg=n)


@pytest.mark.parametrize("ws", [2, 4])
def test_ddp_matches_single_process_big_batch(ws):
    run_dist(_ddp_equivalence, ws, None)


def _ddp_generic_module(rank, ws, path):
    """The hook-based reducer on a plain nn.Module (no Program)."""
    from dmlab.models.reference import TorchLeNet
    from dmlab.parallel import DDP

    torch.manual_seed(0)
    model = TorchLeNet()
    ref = TorchLeNet()
    ref.load_state_dict(model.state_dict())
    ddp = DDP(model, bucket_cap_mb=0.05, first_bucket_mb=0.01)
    g = torch.Generator().manual_seed(3)
    X = torch.rand(ws * 4, 1, 28, 28, generator=g)
    Y = torch.randint(0, 10, (ws * 4,), generator=g)
    F.cross_entropy(ddp(X[rank * 4:(rank + 1) * 4]), Y[rank * 4:(rank + 1) * 4]).backward()
    F.cross_entropy(ref(X), Y).backward()
    for (n, a), (_, b) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-4, atol=1e-6, msg=n)


def test_ddp_generic_module():
    run_dist(_ddp_generic_module, 2, None)


def _no_sync(rank, ws, path):
    from dmlab.models import Net
    from dmlab.parallel import DDP

    torch.manual_seed(0)
    model = Net()
    ref = Net()
    ref.load_state_dict(model.state_dict())
    ddp = DDP(model)
    xs = [torch.rand(4, 1, 28, 28) + rank for _ in range(2)]
    y = torch.zeros(4, dtype=torch.long)
    with ddp.no_sync():
        F.cross_entropy(ddp(xs[0]), y).backward()
    F.cross_entropy(ddp(xs[1]), y).backward()  # accumulates, then reduces
    for x in xs:
        for r in range(ws):
            F.cross_entropy(ref(x - rank + r), y).backward()
    for a, b in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(a.grad, b.grad / ws, rtol=1e-4, atol=1e-6)


def test_ddp_no_sync_accumulation():
    run_dist(_no_sync, 2, None)


def _straggler(rank, ws, path):
    from dmlab.parallel import GradAggregator, Straggler

    m = _make(0)
    F.cross_entropy(m(torch.rand(2, 1, 28, 28)), torch.zeros(2, dtype=torch.long)).backward()
    agg = GradAggregator(m)
    s = Straggler(rank=1, delay_ms=150)
    for _ in range(3):
        agg()
        s()
    if rank == 0:
        # rank 0 waits for the straggler inside the next collective
        assert agg.comm_time > 0.2, agg.comm_time
    else:
        assert s.injected_ms == 450


def test_straggler_slows_the_other_rank():
    run_dist(_straggler, 2, None)


def _native_vs_python_reducer(rank, ws, path):
    """The C++ bucket reducer (dmlab._C.Reducer) and the Python one give identical
    gradients: Program (layer hooks) and plain-module (param hooks) paths, SUM+1/ws and
    folded averaging, bf16 communication, no_sync accumulation."""
    from dmlab.models import Net
    from dmlab.models.reference import TorchLeNet
    from dmlab.parallel import DDP

    g = torch.Generator().manual_seed(11 + rank)
    X = torch.rand(5, 1, 28, 28, generator=g)
    Y = torch.randint(0, 10, (5,), generator=g)
    for cls in (Net, TorchLeNet):
        for comm_dtype in (None, torch.bfloat16):
            grads = []
            for native in (True, False):
                torch.manual_seed(0)
                m = cls()
                ddp = DDP(m, bucket_cap_mb=0.05, first_bucket_mb=0.01, comm_dtype=comm_dtype,
                          native=native)
                assert (ddp._native is not None) == native
                with ddp.no_sync():  # accumulate locally, no communication
                    F.cross_entropy(ddp(X), Y).backward()
                assert ddp.buckets_launched == 0
                F.cross_entropy(ddp(X * 0.5), Y).backward()
                assert ddp.buckets_launched == len(ddp.buckets)
                grads.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]))
            tol = dict(rtol=0, atol=0) if comm_dtype is None else dict(rtol=1e-2, atol=1e-4)
            torch.testing.assert_close(grads[0], grads[1], **tol)


def test_native_reducer_matches_python():
    run_dist(_native_vs_python_reducer, 2, None)


def _resume_other_world_size(rank, ws, path):
    """A checkpoint written by a DDP run (1/ws folded into the optimiser) resumed by a
    single process: the resumed optimiser must not inherit the 1/ws gradient scale."""
    import os

    from dmlab.models import Net
    from dmlab.optim import SGD
    from dmlab.parallel import DDP
    from dmlab.utils import checkpoint

    torch.manual_seed(0)
    model = Net()
    ddp = DDP(model)
    opt = ddp.fold_average_into(SGD(model.parameters(), lr=0.1, momentum=0.9))
    assert opt.grad_scale == 1.0 / ws
    g = torch.Generator().manual_seed(5)
    X, Y = torch.rand(4, 1, 28, 28, generator=g), torch.randint(0, 10, (4,), generator=g)
    opt.zero_grad()
    F.cross_entropy(ddp(X), Y).backward()
    opt.step()
    ck = os.path.join(path, "ck.pt")
    checkpoint.save(ck, ddp, opt)
    if rank == 0:
        assert "grad_scale" not in torch.load(ck, weights_only=True)["optimizer"]


def test_checkpoint_resume_on_another_world_size(tmp_path):
    from dmlab.models import Net
    from dmlab.optim import SGD
    from dmlab.utils import checkpoint

    run_dist(_resume_other_world_size, 2, str(tmp_path))
    b = Net()
    ob = SGD(b.parameters(), lr=0.5, momentum=0.9)
    checkpoint.load(tmp_path / "ck.pt", b, ob)
    assert ob.grad_scale == 1.0 and ob.lr == 0.1 and ob.step_count == 1


# ---------------------------------------------------------------- eight ranks (one node)
@pytest.mark.parametrize("ws", [8])
def test_ddp_matches_single_process_big_batch_ws8(ws):
    """The full node: 8 gloo ranks (the world size of the driver's scaling run)."""
    run_dist(_ddp_equivalence, ws, None)


def _sampler_disjoint_ws(rank, ws, path):
    """PartitionSampler shards of the 8 ranks, gathered over the process group: disjoint,
    covering the (padded) dataset, and reshuffled by set_epoch identically on every rank."""
    from dmlab.data import PartitionSampler

    ds = list(range(1001))  # not a multiple of 8: padded by wrap-around
    s = PartitionSampler(ds, ws, rank, seed=5)
    for epoch in (0, 1):
        s.set_epoch(epoch)
        mine = s.indices().to(torch.long)
        allg = [torch.zeros_like(mine) for _ in range(ws)]
        dist.all_gather(allg, mine)
        cat = torch.cat(allg)
        assert len(mine) == (1001 + ws - 1) // ws
        assert set(cat.tolist()) == set(range(1001))
        assert len(cat) - len(set(cat.tolist())) == len(mine) * ws - 1001  # only the pad repeats
        if epoch == 0:
            first = cat.clone()
    assert not torch.equal(first, cat)  # set_epoch reshuffles


def test_partition_sampler_disjoint_ws8():
    run_dist(_sampler_disjoint_ws, 8, None)


def _buffers_synced(rank, ws, path):
    """broadcast_buffers: BatchNorm running statistics agree on every rank after 3 DDP
    steps with a different batch per rank (rank 0's buffers are broadcast at each training
    forward; ``sync_buffers()`` on every rank before evaluating brings the last forward's
    update across too -- ``eval()`` itself enters no collective)."""
    from dmlab.parallel import DDP

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(1, 4, 3), torch.nn.BatchNorm2d(4),
                                torch.nn.ReLU(), torch.nn.Flatten(), torch.nn.Linear(4 * 26 * 26, 10))
    for sync in (True, False):
        m = copy.deepcopy(model)
        ddp = DDP(m, broadcast_buffers=sync)
        g = torch.Generator().manual_seed(40 + rank)
        for _ in range(3):
            x = torch.rand(4, 1, 28, 28, generator=g) * (1 + rank)
            F.cross_entropy(ddp(x), torch.zeros(4, dtype=torch.long)).backward()
        ddp.eval()  # no collective here (a rank-0-only evaluation must not deadlock)
        bn = m[1]
        if sync:
            # the flat broadcast issued during each backward already left rank 0's statistics
            # of the last forward on every rank; an explicit sync is idempotent
            assert ddp._buf_flat is not None and ddp._buffers_still_flat()
            rm0 = [torch.zeros_like(bn.running_mean) for _ in range(ws)]
            dist.all_gather(rm0, bn.running_mean)
            assert all(torch.equal(rm0[0], r) for r in rm0), rm0
            ddp.sync_buffers()
        rm = [torch.zeros_like(bn.running_mean) for _ in range(ws)]
        dist.all_gather(rm, bn.running_mean)
        same = all(torch.equal(rm[0], r) for r in rm)
        assert same == sync, (sync, rm)


def test_ddp_broadcast_buffers():
    run_dist(_buffers_synced, 2, None)


def _buffers_sync_every(rank, ws, path):
    """buffer_sync_every=2 (bench.py --buffer-sync-every 2): the running statistics are
    broadcast at the 1st, 3rd, ... training forward only, so the ranks agree after those
    steps and differ (different batch per rank) after the others."""
    from dmlab.parallel import DDP

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Conv2d(1, 4, 3), torch.nn.BatchNorm2d(4),
                            torch.nn.ReLU(), torch.nn.Flatten(), torch.nn.Linear(4 * 26 * 26, 10))
    ddp = DDP(m, broadcast_buffers=True, buffer_sync_every=2)
    g = torch.Generator().manual_seed(40 + rank)
    for step in range(4):
        x = torch.rand(4, 1, 28, 28, generator=g) * (1 + rank)
        F.cross_entropy(ddp(x), torch.zeros(4, dtype=torch.long)).backward()
        rm = [torch.zeros_like(m[1].running_mean) for _ in range(ws)]
        dist.all_gather(rm, m[1].running_mean)
        same = all(torch.equal(rm[0], r) for r in rm)
        assert same == (step % 2 == 0), (step, rm)


def test_ddp_buffer_sync_every():
    run_dist(_buffers_sync_every, 2, None)


def _bf16_comm_side_hooks(rank, ws, path):
    """bf16 gradient communication through the persistent buffer equals the fp32
    communication within bf16 rounding, with the side-stream (stream_ok) hook path."""
    from dmlab.models import Net
    from dmlab.parallel import DDP

    g = torch.Generator().manual_seed(3 + rank)
    X, Y = torch.rand(6, 1, 28, 28, generator=g), torch.randint(0, 10, (6,), generator=g)
    grads = []
    for comm_dtype in (None, torch.bfloat16):
        torch.manual_seed(0)
        m = Net()
        ddp = DDP(m, bucket_cap_mb=0.05, first_bucket_mb=0.01, comm_dtype=comm_dtype)
        assert all(m._hook_stream_ok.get(h, False) for h in m._grad_hooks)
        if comm_dtype is not None:
            assert ddp._comm_flat is not None and ddp._comm_flat.dtype == torch.bfloat16
        for _ in range(2):  # the persistent buffer is reused across steps
            m.flat.grad.zero_()
            F.cross_entropy(ddp(X), Y).backward()
        grads.append(m.flat.grad.clone())
    torch.testing.assert_close(grads[1], grads[0], rtol=2e-2, atol=2e-3)


def test_ddp_bf16_comm_persistent_buffer():
    run_dist(_bf16_comm_side_hooks, 2, None)
