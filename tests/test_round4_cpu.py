"""CPU checks of the round-4 plumbing: forced communication at one rank, the DDP wrapper as a
plain nn.Module, the loader's unmaterialised (``Gathered``) batches and device cursor, the
bench's replica self-check, the p2p shape guard and the aggregator's timing flags."""
import pytest
import torch

from dist_helpers import run_dist


def _force_comm_one_rank(rank, ws):
    from dmlab.models import Net
    from dmlab.nn import cross_entropy
    from dmlab.optim import SGD
    from dmlab.parallel import DDP

    g = torch.Generator().manual_seed(3)
    X = torch.rand(16, 1, 28, 28, generator=g)
    Y = torch.randint(0, 10, (16,), generator=g)
    res = []
    for force in (True, False):
        torch.manual_seed(0)
        m = Net()
        ddp = DDP(m, force_comm=force)
        assert ddp.comm_active == force
        opt = ddp.fold_average_into(SGD(m.parameters(), lr=0.1, momentum=0.9))
        for _ in range(2):
            opt.zero_grad()
            cross_entropy(ddp(X), Y).backward()
            opt.step()
        res.append((m.flat.data.clone(), ddp.buckets_launched, len(ddp.buckets)))
    (p1, launched, nb), (p0, launched0, _) = res
    assert torch.equal(p1, p0)
    assert launched == 2 * nb and launched0 == 0


def test_ddp_force_comm_one_rank_gloo():
    """force_comm at world size 1: every bucket goes through the process group (gloo here,
    RCCL on the GPU box) and training is unchanged bit for bit."""
    run_dist(_force_comm_one_rank, 1)


def test_ddp_force_comm_needs_a_group():
    from dmlab.models import Net
    from dmlab.parallel import DDP

    with pytest.raises(RuntimeError, match="process group"):
        DDP(Net(), force_comm=True)


def test_ddp_is_a_normal_module():
    """the wrapper must keep nn.Module's own buffer registry intact."""
    from dmlab.models import ResNet18
    from dmlab.parallel import DDP

    m = ResNet18(num_classes=10)
    ddp = DDP(m)
    sd = ddp.state_dict()
    assert any(k.endswith("running_mean") for k in sd)
    ddp.to("cpu")
    assert len(list(ddp.buffers())) == len(list(m.buffers())) > 0
    ddp.load_state_dict(sd)
    ddp.eval()  # no collective on eval()
    assert not m.training


def test_gathered_batches_match_materialised():
    from dmlab.data import DeviceLoader, Gathered, MySampler, synthetic_classification

    ds = synthetic_classification(40, (3, 8, 8), 5, seed=1)
    s1 = MySampler(ds, 2, 1, shuffle=True, seed=0)
    s2 = MySampler(ds, 2, 1, shuffle=True, seed=0)
    a = list(DeviceLoader(ds, 8, sampler=s1, drop_last=True))
    b = list(DeviceLoader(ds, 8, sampler=s2, drop_last=True).iter_gathered())
    assert len(a) == len(b) == 2
    for (xa, ya), (gb, yb) in zip(a, b):
        assert isinstance(gb, Gathered) and gb.shape == tuple(xa.shape)
        assert torch.equal(gb.materialize(), xa) and torch.equal(ya, yb)


def test_program_accepts_gathered_input():
    """A Program fed a Gathered batch computes what it computes on the gathered tensor."""
    from dmlab.data import Gathered
    from dmlab.models import Net

    torch.manual_seed(0)
    net = Net()
    im = torch.rand(10, 1, 28, 28)
    idx = torch.tensor([3, 1, 4, 1, 5])
    out_g = net(Gathered(im, idx))
    out_t = net(im.index_select(0, idx))
    assert torch.equal(out_g, out_t)


def test_device_cursor_walks_the_shard():
    from dmlab.data import DeviceLoader, MySampler, synthetic_classification

    ds = synthetic_classification(50, (1, 4, 4), 3, seed=2)
    smp = MySampler(ds, 2, 0, shuffle=True, seed=0)
    ld = DeviceLoader(ds, 4, sampler=smp, drop_last=True)
    cur = ld.cursor()
    assert cur.nbatch == 25 // 4 and cur.order.numel() == cur.nbatch * 4
    assert torch.equal(cur.order, smp.indices()[: cur.order.numel()])
    cur.cursor.fill_(3)
    cur.refill(1)
    smp2 = MySampler(ds, 2, 0, shuffle=True, seed=0)
    smp2.set_epoch(1)
    assert int(cur.cursor) == 0
    assert torch.equal(cur.order, smp2.indices()[: cur.order.numel()])


def _verify(rank, ws, skew):
    import bench
    from dmlab.models import Net

    torch.manual_seed(0)
    m = Net()
    if skew and rank == 1:
        with torch.no_grad():
            m.flat.data[7] += 1e-6
    v = bench.verify_replicas(m, torch.device("cpu"))
    assert v["distinct_gpus"] == 1 and v["rccl_world"] is None
    assert v["replicas_in_sync"] is (not skew), v


@pytest.mark.parametrize("skew", [False, True])
def test_bench_replica_check(skew):
    """bench.py's multi-rank self-check flips replicas_in_sync on a one-element skew."""
    run_dist(_verify, 2, skew)


def test_p2p_header_mismatch_raises():
    from dmlab.parallel.p2p import _ShapeCache

    c = _ShapeCache(group=None, gloo=True)
    c.shapes["act"] = ((4, 400), torch.float32)
    assert c.send(torch.zeros(4, 400), 1, "act") == []
    with pytest.raises(ValueError, match="differs"):
        c.send(torch.zeros(3, 400), 1, "act")


def test_aggregator_timing_flags():
    from dmlab.models import Net
    from dmlab.parallel.comm import GradAggregator

    m = Net()
    assert GradAggregator(m).timing == "events"
    assert GradAggregator(m, sync_timing=True).timing == "sync"
    assert GradAggregator(m, sync_timing=False).timing == "host"


def test_import_raises_hip_hw_queues():
    """`import dmlab` gives each process 8 HIP hardware queues (before the runtime starts) so
    the main, weight-gradient, downsample and RCCL streams do not share a queue; an explicit
    larger value is kept."""
    import os
    import subprocess
    import sys

    code = "import os, dmlab; print(os.environ['GPU_MAX_HW_QUEUES'])"
    for given, want in ((None, "8"), ("4", "8"), ("16", "16")):
        env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
        if given:
            env["GPU_MAX_HW_QUEUES"] = given
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True,
                             text=True, cwd=str(__import__("pathlib").Path(__file__).parent.parent))
        assert out.stdout.strip() == want, (given, out.stdout, out.stderr[-500:])
