import torch, sys
sys.path.insert(0, '.')
import ov3d_import
ov3d_import.load()
from ov3d_amd import gemm
ps = [torch.nn.Parameter(torch.randn(256, 256, device='cuda')) for _ in range(50)]
with torch.autograd.profiler.profile(use_device='cuda') as prof:
    with torch.no_grad():
        for p in ps: p.add_(1)
    xs = [gemm.cast_param(p, torch.bfloat16) for p in ps]
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=8))
