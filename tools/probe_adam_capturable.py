import torch, time
dev = torch.device("cuda:0")
ps = [torch.nn.Parameter(torch.randn(256, 256, device=dev)) for _ in range(19)]
for p in ps: p.grad = torch.randn_like(p)
for kw in ({}, {"foreach": True}, {"fused": True}):
    opt = torch.optim.Adam(ps, lr=1e-3, **kw)
    for g in opt.param_groups:
        g["capturable"] = True
        g["lr"] = torch.tensor(1e-3, device=dev)
    try:
        for _ in range(5): opt.step()
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(50): opt.step()
        torch.cuda.synchronize()
        print(kw, opt.param_groups[0].get("foreach"), opt.param_groups[0].get("fused"), round((time.perf_counter()-t)/50*1e3, 3), "ms")
    except Exception as e:
        print(kw, "error", type(e).__name__, str(e)[:200])
