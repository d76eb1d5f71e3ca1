"""CPU tests: samplers, TB event writer, optimisers, Program engine parity."""
import math
import os

import pytest
import torch
import torch.nn.functional as F

from dmlab.data import (DeviceLoader, MySampler, PartitionSampler, RandomSampleSampler,
                        SyntheticMNIST, load_mnist)
from dmlab.models import ForwardNN, Net, ResNet18, SubNetConv, SubNetFC
from dmlab.models.reference import TorchLeNet, TorchMLP
from dmlab.optim import SGD, AdamOptimizer, GdOptimizer
from dmlab.utils import getSummaryWriter, read_events

# ---------------------------------------------------------------- samplers


@pytest.mark.parametrize("n,ws", [(100, 3), (60000, 8), (7, 4)])
def test_partition_sampler_disjoint_cover(n, ws):
    ds = list(range(n))
    shards = [PartitionSampler(ds, ws, r, seed=3).indices() for r in range(ws)]
    assert all(len(s) == math.ceil(n / ws) for s in shards)
    allidx = torch.cat(shards)
    assert set(allidx.tolist()) == set(range(n))        # covers the dataset
    if n % ws == 0:
        assert len(set(allidx.tolist())) == n           # disjoint when no padding


def test_partition_sampler_epochs_and_determinism():
    ds = list(range(1000))
    a = PartitionSampler(ds, 4, 1, seed=0)
    b = PartitionSampler(ds, 4, 1, seed=0)
    assert torch.equal(a.indices(), b.indices())
    e0 = a.indices()
    a.set_epoch(1)
    assert not torch.equal(e0, a.indices())              # reshuffled per epoch (B3)


def test_random_sample_sampler():
    ds = list(range(1000))
    s0 = RandomSampleSampler(ds, 4, 0, seed=0)
    s1 = RandomSampleSampler(ds, 4, 1, seed=0)
    i0, i1 = s0.indices(), s1.indices()
    assert len(i0) == 250 and len(set(i0.tolist())) == 250  # no duplicates within a rank
    assert not torch.equal(i0, i1)                           # ranks draw independently
    s0.set_epoch(2)
    assert not torch.equal(i0, s0.indices())
    boot = RandomSampleSampler(ds, 4, 0, seed=0, replacement=True).indices()
    assert boot.max() < 1000 and len(boot) == 250


def test_mysampler_reference_api():
    ds = list(range(10))
    s = MySampler(ds, 2, 1, shuffle=True, seed=1)
    assert len(s) == 5 and len(list(iter(s))) == 5          # reference skeleton raised here (B2)
    s.set_epoch(3)
    assert MySampler(ds, 2, 0, mode="division").mode == "partition"
    with pytest.raises(ValueError):
        MySampler(ds, 2, 0, mode="bogus")


def test_device_loader_batches():
    ds = SyntheticMNIST(train=False, n=100)
    ld = DeviceLoader(ds, 32, sampler=PartitionSampler(ds, 2, 0))
    sizes = [x.shape[0] for x, _ in ld]
    assert sizes == [32, 18] and len(ld) == 2


def test_synthetic_mnist_shape_and_range():
    ds = load_mnist("/nonexistent", train=True, n=256)
    assert ds.images.shape == (256, 1, 28, 28)
    assert ds.images.min() >= 0 and ds.images.max() <= 1
    assert ds.labels.min() >= 0 and ds.labels.max() <= 9


# ---------------------------------------------------------------- TB writer


def test_summary_writer_roundtrip(tmp_path):
    w = getSummaryWriter(3, del_dir=False, root=str(tmp_path) + "/")
    for i in range(5):
        w.add_scalar("Train Loss", 2.0 - 0.1 * i, i * 20)
    w.close()
    files = list(tmp_path.rglob("events.out.tfevents.*"))
    assert len(files) == 1
    assert files[0].parent.name.endswith("-epoch3")          # ./logs/<date>/<time>-epoch<N>/
    ev = read_events(files[0])
    assert ev[0]["file_version"] == "brain.Event:2"
    sc = [e for e in ev if "tag" in e]
    assert [e["step"] for e in sc] == [0, 20, 40, 60, 80]
    assert sc[-1]["tag"] == "Train Loss" and abs(sc[-1]["value"] - 1.6) < 1e-6
    # del_dir wipes the log root
    w2 = getSummaryWriter(1, del_dir=True, root=str(tmp_path) + "/")
    w2.close()
    assert len(list(tmp_path.rglob("events.out.tfevents.*"))) == 1


def test_crc32c_known_vector():
    from dmlab.utils.summary import crc32c

    assert crc32c(b"123456789") == 0xE3069283  # standard CRC-32C check value


# ---------------------------------------------------------------- optimisers


def _lenet_pair():
    torch.manual_seed(0)
    a = Net()
    b = TorchLeNet()
    b.load_state_dict(a.state_dict())
    return a, b


def _loss(m, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(16, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (16,), generator=g)
    return F.cross_entropy(m(x), y)


def test_adam_reference_formula_flat_and_per_tensor():
    a, b = _lenet_pair()
    oa = AdamOptimizer(a.parameters(), lr=0.01)   # flat path (Program)
    ob = AdamOptimizer(b.parameters(), lr=0.01)   # per-tensor path (plain module)
    assert oa.flat is not None and ob.flat is None
    for s in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            _loss(m, s).backward()
            o.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)


def test_sgd_matches_torch_optim():
    a, b = _lenet_pair()
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4, nesterov=True)
    ob = torch.optim.SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4, nesterov=True)
    for s in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            _loss(m, s).backward()
            o.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)


def test_gd_is_plain_gradient_step():
    a, b = _lenet_pair()
    before = [p.detach().clone() for p in a.parameters()]
    o = GdOptimizer(a.parameters(), lr=0.1)
    o.zero_grad()
    _loss(a).backward()
    grads = [p.grad.clone() for p in a.parameters()]
    o.step()
    for p, p0, g in zip(a.parameters(), before, grads):
        torch.testing.assert_close(p, p0 - 0.1 * g)


def test_torch_optimizer_on_program_with_set_to_none():
    """torch.optim + zero_grad(set_to_none=True) re-attaches flat grad views."""
    a, b = _lenet_pair()
    oa = torch.optim.SGD(a.parameters(), lr=0.05, momentum=0.9)
    ob = torch.optim.SGD(b.parameters(), lr=0.05, momentum=0.9)
    for s in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad(set_to_none=True)
            _loss(m, s).backward()
            o.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
    assert a.flat.attached()


# ---------------------------------------------------------------- program engine


def test_mlp_param_count_and_parity():
    torch.manual_seed(0)
    a = ForwardNN()
    b = TorchMLP()
    b.load_state_dict(_mlp_sd(a))
    assert sum(p.numel() for p in a.parameters()) == 576_810
    x = torch.rand(8, 1, 28, 28)
    torch.testing.assert_close(a(x), b(x))


def _mlp_sd(a):
    sd = {}
    for k, v in a.state_dict().items():
        i = int(k[2:k.index(".")]) - 1
        sd[f"layers.{i}.{k.split('.')[1]}"] = v
    return sd


def test_reference_compat_softmax():
    m = ForwardNN(reference_compat=True)
    out = m(torch.rand(4, 1, 28, 28))
    torch.testing.assert_close(out.sum(1), torch.ones(4))


def test_pipeline_halves_compose_to_lenet():
    torch.manual_seed(0)
    full = Net()
    a, b = SubNetConv(), SubNetFC()
    a.load_state_dict({k: v for k, v in full.state_dict().items() if k.startswith("conv")})
    b.load_state_dict({k: v for k, v in full.state_dict().items() if k.startswith("fc")})
    x = torch.rand(5, 1, 28, 28)
    torch.testing.assert_close(b(a(x)), full(x))
    xr = x.clone().requires_grad_(True)
    b(a(xr)).sum().backward()                                # grad flows across programs
    assert xr.grad is not None and a.conv1.weight.grad.abs().sum() > 0


def test_resnet18_cpu_forward_backward():
    torch.manual_seed(0)
    m = ResNet18(num_classes=10)
    assert sum(p.numel() for p in m.parameters()) == 11_181_642
    out = m(torch.rand(2, 3, 32, 32))
    assert out.shape == (2, 10)
    F.cross_entropy(out, torch.tensor([1, 2])).backward()
    assert all(p.grad is not None for p in m.parameters())
    assert int(m.stem.num_batches_tracked) == 1


def test_program_grad_hooks_fire_in_reverse_order():
    m = Net()
    seen = []
    m.register_grad_hook(lambda prog, i: seen.append(i))
    _loss(m).backward()
    assert seen == list(range(len(m.layers) - 1, -1, -1))


def test_program_to_refits_flat_buffer():
    m = Net().to(torch.device("cpu"))
    assert m.flat.attached()
    for p in m.parameters():
        assert p._dm_flat is m.flat


def test_param_groups_lr_is_persistent():
    """`for g in opt.param_groups: g["lr"] = x` (manual LR schedule) reaches step()."""
    m, _ = _lenet_pair()
    o = SGD(m.parameters(), lr=0.1)
    for grp in o.param_groups:
        grp["lr"] = 0.0
    assert o.lr == 0.0
    before = [p.detach().clone() for p in m.parameters()]
    o.zero_grad()
    _loss(m, 0).backward()
    o.step()
    for a, b in zip(before, m.parameters()):
        torch.testing.assert_close(a, b)
    o.lr = 0.3
    assert o.param_groups[0]["lr"] == 0.3


def test_checkpoint_roundtrip(tmp_path):
    from dmlab.utils import checkpoint

    a, _ = _lenet_pair()
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9)
    for s in range(2):
        oa.zero_grad()
        _loss(a, s).backward()
        oa.step()
    checkpoint.save(tmp_path / "ck.pt", a, oa, epoch=3)
    torch.manual_seed(1)
    b = Net()
    ob = SGD(b.parameters(), lr=0.01, momentum=0.9)
    extra = checkpoint.load(tmp_path / "ck.pt", b, ob)
    assert extra == {"epoch": 3} and ob.lr == 0.05 and ob.step_count == 2
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb)
    # one more identical step keeps them identical (momentum restored)
    for m, o in ((a, oa), (b, ob)):
        o.zero_grad()
        _loss(m, 9).backward()
        o.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb)


# ---------------------------------------------------------------- DDP bucket layout
def _sizes(numels, pad=64):
    out, off = [], 0
    for n in numels:
        end = off + (n + pad - 1) // pad * pad
        out.append((off, n, end))
        off = end
    return out


@pytest.mark.parametrize("numels,cap,first,last", [
    ([100, 5000, 70000, 300, 9000, 120000, 64, 64, 200000], 100000, 6000, 20000),
    ([1000], 100, 10, 10),                       # a single parameter: one bucket
    ([10, 10, 10], 10**9, 10**9, 10**9),          # everything fits: one bucket
    ([64] * 40, 640, 128, 256),                   # many small params
    ([5000, 500000], 1000, 1000, 1000),           # tail param larger than every cap: unsplit
])
def test_ddp_make_buckets_invariants(numels, cap, first, last):
    from dmlab.parallel.ddp import DistributedDataParallel as D

    sizes = _sizes(numels)
    bks = D._make_buckets(None, sizes, cap, first, last)
    # contiguous cover of [0, total) in order, boundaries on parameter boundaries
    assert bks[0].lo == 0 and bks[-1].hi == sizes[-1][2]
    for a, b in zip(bks, bks[1:]):
        assert a.hi == b.lo
    starts = {s[0] for s in sizes} | {sizes[-1][2]}
    for b in bks:
        assert b.lo in starts and b.hi in starts
        assert b.params == sorted(b.params)
        assert sizes[b.params[0]][0] == b.lo and sizes[b.params[-1]][2] == b.hi
    # every parameter in exactly one bucket
    ids = [i for b in bks for i in b.params]
    assert sorted(ids) == list(range(len(numels))) and len(ids) == len(set(ids))
    # the last bucket is capped, unless even its final parameter alone exceeds the cap (then
    # it is left unsplit) or it is the only bucket's single parameter
    tail = bks[-1]
    last_alone = sizes[tail.params[-1]][2] - sizes[tail.params[-1]][0]
    if len(tail.params) > 1 and last_alone <= last:
        assert tail.hi - tail.lo <= last


def test_res64_picked_for_layer1():
    """cfg 80 (csrc/conv_res64.hip) only for 64 -> 64 channel 3x3/s1 convs of known width whose
    128-pixel halo fits the kernel's 256-row LDS image."""
    from dmlab.ops.convbn import pick_cfg, dgrad_cfg
    assert pick_cfg(1024 * 56 * 56, 64, 3, 1, 64, W=56) == 80
    assert dgrad_cfg(1024 * 56 * 56, 64, 3, 1, 64, 56, 56) == 80
    assert pick_cfg(1024 * 56 * 56, 64, 3, 1, 64) != 80        # width unknown
    assert pick_cfg(4 * 112 * 112, 64, 3, 1, 64, W=112) != 80  # halo too wide
    assert pick_cfg(1024 * 28 * 28, 128, 3, 1, 128, W=28) != 80
    assert dgrad_cfg(1024 * 56 * 56, 64, 3, 2, 128, 56, 56) != 80  # layer2 c1 data gradient


def test_wgrad_res64_plan():
    """wgrad cfg 8 (csrc/wgrad_res64.hip) for 64 -> 64 channel 3x3/s1 layers of width <= 60,
    one slab per workgroup on 5/8 of the CUs (at most one per image row)."""
    from dmlab.ops.convbn import _wgrad_plan
    cfg, S = _wgrad_plan(1024 * 56 * 56, 64, 576, 3, 1, 64, W=56, rows=1024 * 56)
    assert cfg == 8 and 1 <= S <= 1024 * 56
    assert _wgrad_plan(2 * 5 * 5, 64, 576, 3, 1, 64, W=5, rows=10)[1] <= 10
    assert _wgrad_plan(1024 * 56 * 56, 64, 576, 3, 1, 64)[0] != 8           # width unknown
    assert _wgrad_plan(4 * 112 * 112, 64, 576, 3, 1, 64, W=112, rows=448)[0] != 8
    assert _wgrad_plan(1024 * 28 * 28, 128, 1152, 3, 1, 128, W=28, rows=1024 * 28)[0] != 8


def test_wgrad_s2_plan():
    """wgrad cfg 7 (the stride-2 parity-plane kernel) for 3x3/s2 layers whose output is half
    the input and at most 31 wide; the igemm tile otherwise (1x1 projections included)."""
    from dmlab.ops.convbn import _wgrad_plan
    cfg, S = _wgrad_plan(1024 * 28 * 28, 128, 576, 3, 2, 64, even=28)
    assert cfg == 7 and S >= 1
    assert _wgrad_plan(1024 * 7 * 7, 512, 2304, 3, 2, 256, even=7)[0] == 7
    assert _wgrad_plan(1024 * 28 * 28, 128, 64, 1, 2, 64, even=28)[0] != 7   # 1x1: igemm
    assert _wgrad_plan(64 * 64 * 64, 128, 576, 3, 2, 64, even=64)[0] != 7   # too wide
    assert _wgrad_plan(1024 * 28 * 28, 128, 576, 3, 2, 64)[0] != 7          # odd input
    assert _wgrad_plan(1024 * 28 * 28, 128, 288, 3, 2, 32, even=28)[0] != 7  # channels


def test_dgrad_red_selection(monkeypatch):
    """Which data gradients reduce the consumer BN's backward sums in their epilogue
    (ops/convbn.py _dgrad_red): cfg 80 / 90-93 / 42, stride 1, a ReLU consumer of dx's shape;
    the residual block's 1-bit mask rides along; layer1's masked case (cfg 80 + mask, or the
    stem's pooled grid) is opt-in; the consumer's ctx receives the partial-sum slab."""
    from types import SimpleNamespace as NS
    import torch
    from dmlab.ops import convbn as CB

    L = NS(conv_stats_rows=lambda M, cfg, C: 7)
    dx = torch.zeros(2, 4, 4, 64)

    def ctx(has_res=False, mask=False, pool=False):
        c = dict(y=torch.zeros(2, 4, 4, 64), mean=torch.zeros(64), invstd=torch.ones(64),
                 scale=torch.ones(64), shift=torch.zeros(64), has_res=has_res)
        if mask:
            c["mask"] = torch.zeros(2 * 4 * 4 * 64 // 8, dtype=torch.uint8)
        if pool:
            c["yarg"] = torch.zeros(2, 4, 4, 64)
            c["y"] = torch.zeros(2, 8, 8, 64)
        return c

    relu, stem = NS(relu=True), NS(relu=True, pool_k=3)
    c = ctx()
    kw = CB._dgrad_red(L, (relu, c), 80, 1, dx)
    assert kw["red_y"] is c["y"] and "red_mask" not in kw and kw["red_part"].numel() == 7 * 2 * 64
    assert c["pre_sums"]["pre_rows"] == 7 and c["pre_sums"]["pre_slab"] is kw["red_part"]
    assert CB._dgrad_red(L, (relu, c), 80, 1, dx) == {}            # sums already planned
    assert CB._dgrad_red(L, (relu, ctx()), 80, 2, dx) == {}        # stride-2 dgrad
    assert CB._dgrad_red(L, (relu, ctx()), 39, 1, dx) == {}        # kernel without the epilogue
    assert CB._dgrad_red(L, (NS(relu=False), ctx()), 90, 1, dx) == {}
    assert CB._dgrad_red(L, (relu, ctx()), 90, 1, torch.zeros(2, 4, 4, 128)) == {}
    assert CB._dgrad_red(L, (relu, ctx(has_res=True)), 90, 1, dx) == {}   # no 1-bit mask
    c = ctx(has_res=True, mask=True)
    assert CB._dgrad_red(L, (relu, c), 42, 1, dx)["red_mask"] is c["mask"]
    # res64 with the fused skip add: on by default (round 6), DMLAB_RES64_RED_ADD=0 opts out
    assert CB._dgrad_red(L, (relu, ctx(has_res=True, mask=True)), 80, 1, dx)["red_mask"] is not None
    monkeypatch.setenv("DMLAB_RES64_RED_ADD", "0")
    assert CB._dgrad_red(L, (relu, ctx(has_res=True, mask=True)), 80, 1, dx) == {}
    monkeypatch.delenv("DMLAB_RES64_RED_ADD")
    c = ctx(pool=True)  # the stem's pooled-grid sums: reduced in the last layer-1 dgrad
    assert CB._dgrad_red(L, (stem, c), 80, 1, dx)["red_y"] is c["yarg"]
    c = ctx(has_res=True, mask=True)
    assert CB._dgrad_red(L, (relu, c), 80, 1, dx, allow_res64_add=True)["red_mask"] is c["mask"]
