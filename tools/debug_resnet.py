import copy, sys, torch, torch.nn.functional as F
sys.path.insert(0, '.')
from dmlab.models import ResNet18
from dmlab.nn import cross_entropy
def rel(a, b): return ((a.float()-b.float()).norm()/(b.float().norm()+1e-12)).item()
dev = torch.device('cuda')
for B, R in ((8, 64), (32, 64)):
    torch.manual_seed(0)
    a = ResNet18(num_classes=10).to(dev)
    b = copy.deepcopy(a).set_backend("torch"); b._flatten()
    c = copy.deepcopy(b); c._flatten()
    x = torch.rand(B, 3, R, R, device=dev); y = torch.randint(0, 10, (B,), device=dev)
    oa, ob = a(x), b(x)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        oc = c(x)
    print(B, R, 'logits rel native', rel(oa, ob), 'autocast', rel(oc, ob))
    cross_entropy(oa, y).backward(); F.cross_entropy(ob, y).backward(); F.cross_entropy(oc.float(), y).backward()
    for (n, pa), (_, pb), (_, pc) in zip(a.named_parameters(), b.named_parameters(), c.named_parameters()):
        print(f"  {n:28s} native {rel(pa.grad, pb.grad):.4f}  torch-bf16-autocast {rel(pc.grad, pb.grad):.4f}")
