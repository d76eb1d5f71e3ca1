import sys, torch, torch.nn.functional as F
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from test_stem_fused import _inputs, _x_bf16, _run_fwd, _codes_ref
dev = torch.device("cuda")
torch.manual_seed(0)
H = 64
img = _inputs(dev, torch.float32, 5, H, 1)
idx = torch.tensor([4, 0, 2], device=dev, dtype=torch.long)
w = torch.randn(64, 3, 7, 7, device=dev) * 0.08
gamma = torch.randn(64, device=dev)
pext, code, stats, wk, grid = _run_fwd(img, idx, w, gamma)
xb = _x_bf16(img.index_select(0, idx)).cpu()
y = F.conv2d(xb, w.to(torch.bfloat16).double().cpu(), stride=2, padding=3)
sgn = torch.where(gamma.cpu() < 0, -1.0, 1.0).double().view(1, 64, 1, 1)
yb = y.to(torch.bfloat16).double()
v, cref = _codes_ref(sgn * yb)
pref = (sgn * v).permute(0, 2, 3, 1)
got = pext.double().cpu()
err = (got - pref).abs() > 1e-2 * pref.abs().max()
print("bad frac", err.double().mean().item())
print("by image", err.double().mean((1, 2, 3)).tolist())
print("by row", [round(x, 3) for x in err.double().mean((0, 2, 3)).tolist()])
print("by col", [round(x, 3) for x in err.double().mean((0, 1, 3)).tolist()])
print("by ch", [round(x, 2) for x in err.double().mean((0, 1, 2)).tolist()])
print("neg gamma ch", (gamma < 0).nonzero().flatten().tolist())
# is got equal to the max of plain y (no sign) or of the wrong row?
vmax, _ = _codes_ref(yb)
print("matches plain max", ((got - vmax.permute(0,2,3,1)).abs() < 1e-2).double().mean().item())
print("sample", got[0, 3, 3, :8].tolist(), pref[0, 3, 3, :8].tolist())
# conv values at pooled window 3,3 ch0
print("y window", yb[0, 0, 5:8, 5:8].tolist())
