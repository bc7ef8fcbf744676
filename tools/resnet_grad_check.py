import os, sys, torch, torch.nn.functional as F
sys.path.insert(0, os.getcwd())
from pytorch_distributed_example_amd.models import build_resnet18
dev = "cuda"
res = {}
for mode in ("0", "1"):
    os.environ["PDE_RESNET_FUSED_BLOCK"] = mode
    g = build_resnet18(num_classes=10, seed=0, device=dev)
    c = build_resnet18(num_classes=10, seed=0, dtype=torch.float32)
    with torch.no_grad():
        for pc, pg in zip(c.parameters(), g.parameters()):
            pc.copy_(pg.float())
    torch.manual_seed(2)
    x = torch.randn(8, 3, 64, 64); y = torch.randint(0, 10, (8,))
    lg = F.cross_entropy(g(x.to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)).float(), y.to(dev))
    lc = F.cross_entropy(c(x), y)
    lg.backward(); lc.backward()
    print(mode, "loss", lg.item(), lc.item())
    for (n, pg), pc in zip(g.named_parameters(), c.parameters()):
        res.setdefault(n, []).append(round(F.cosine_similarity(pg.grad.float().flatten().cpu(), pc.grad.flatten(), dim=0).item(), 3))
for n, v in res.items():
    print(n, v)
