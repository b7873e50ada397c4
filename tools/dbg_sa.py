import sys, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import ov3d_import
ov3d_amd = ov3d_import.load()
from ov3d_amd import _native, synthetic
from ov3d_amd.dataset_config import SunrgbdDatasetConfig
from bench import default_args
cuda = torch.device("cuda", 0)
args = default_args()
cfg = SunrgbdDatasetConfig()
torch.manual_seed(0)
model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
model = model.to(cuda).train()
crit = ov3d_amd.build_criterion(args, cfg).to(cuda)
batch = synthetic.make_batch(8, seed=2, device=cuda)
_native.timing_enable(["ov3d_sa_layer_pool_fwd", "ov3d_sa_layer_dy", "ov3d_sa_pool_bwd"])
with torch.autocast("cuda", dtype=torch.bfloat16):
    out = model({k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
loss, _ = crit(out, batch)
print("loss", loss.item(), loss.requires_grad, loss.grad_fn)
loss.backward()
t = _native.timing_collect()
print({k: len(v) for k, v in t.items()})
w = model.pre_encoder.mlp_module.layer0.conv.weight
print("sa grad", None if w.grad is None else w.grad.abs().sum().item())
for n, p in model.named_parameters():
    if p.requires_grad and p.grad is None:
        print("no grad:", n)
