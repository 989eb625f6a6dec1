"""Diagnostic: where one mid-N training step (bench.py's model_dense_A_mid_n:
GraphCNNDropEdge(4369, 53, 6, 256), dense (1, N, 6, N) A, train fwd+bwd) spends
its time -- wall per step, then torch.profiler's top ops by device and host
time.  PROBE_ROOT selects the tree whose package is imported (A/B of two
trees on one box)."""
import os
import sys
import time

ROOT = os.environ.get("PROBE_ROOT", os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(ROOT, "graph-representation-learning_amd"))
import torch  # noqa: E402


def main():
    from gnn.models import GraphCNNDropEdge

    dev = torch.device("cuda:0")
    N = int(os.environ.get("PROBE_N", "512"))
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 256).to(dev)
    model.train()
    lossf = torch.nn.CrossEntropyLoss()
    gen = torch.Generator(device=dev).manual_seed(N)
    A = (torch.rand(1, N, 6, N, generator=gen, device=dev) < 3.0 / (6 * N)).float()
    V = torch.zeros(1, N, 4369, device=dev)
    V[0].scatter_(1, torch.randint(0, 4365, (N, 7), generator=gen, device=dev), 1.0)
    y = torch.randint(0, 53, (1, N), generator=gen, device=dev)

    def step():
        model.zero_grad(set_to_none=True)
        lossf(model.forward([V, A]).reshape(-1, 53), y.reshape(-1)).backward()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    print(f"root {ROOT} N {N}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/step", flush=True)
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(5):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25), flush=True)
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25), flush=True)


if __name__ == "__main__":
    main()
