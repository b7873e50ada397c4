"""Per-launch floor of back-to-back kernels replayed from one hipGraph (tiny elementwise op,
and a 1024 x 256 bf16 row op of the decoder's size).  python tools/launch_floor.py  (GPU)"""
import torch


def per_launch(fn, n=200):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * n) * 1e3


def main():
    a = torch.zeros(1, device="cuda")
    x = torch.randn(1024, 256, device="cuda", dtype=torch.bfloat16)
    y = torch.empty_like(x)
    print(f"1-element add_:            {per_launch(lambda: a.add_(1)):6.2f} us per launch")
    print(f"1024x256 bf16 copy:        {per_launch(lambda: y.copy_(x)):6.2f} us per launch")
    print(f"1024x256 bf16 relu:        {per_launch(lambda: torch.relu(x, out=y) if False else torch.relu_(y)):6.2f} us per launch")


if __name__ == "__main__":
    main()
