"""Debug helper: compare StepGraph grads with an eager step on a small model."""
import copy
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ov3d_import
ov3d = ov3d_import.load()
from ov3d_amd import synthetic
from ov3d_amd.dataset_config import SunrgbdDatasetConfig
from ov3d_amd.graphs import StepGraph
from bench import default_args, train_step

args = default_args(enc_dropout=0.0, dec_dropout=0.0, mlp_dropout=0.0, preenc_npoints=512, nqueries=64)
cfg = SunrgbdDatasetConfig()
torch.manual_seed(0)
cuda = torch.device("cuda")
model, _ = ov3d.build_model(args, cfg, text_embedding=synthetic.text_embedding())
model = model.to(cuda).train()
twin = copy.deepcopy(model)
crit = ov3d.build_criterion(args, cfg).to(cuda)
mk = lambda m: torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=args.base_lr,
                                 weight_decay=args.weight_decay, fused=True, capturable=True)
opt_e, opt_g = mk(model), mk(twin)
b1 = synthetic.make_batch(2, seed=4, num_points=4096, device=cuda)
b2 = synthetic.make_batch(2, seed=5, num_points=4096, device=cuda)
sg = StepGraph(twin, crit, opt_g, b1, amp_dtype=torch.bfloat16, clip=args.clip_gradient, warmup_iters=1)
train_step(model, crit, opt_e, b1, args, torch.bfloat16)
le = train_step(model, crit, opt_e, b2, args, torch.bfloat16)
lg = sg.step(b2)
torch.cuda.synchronize()
print("loss", le.item(), lg.item())
ge = dict(model.named_parameters())
for n, p in list(twin.named_parameters())[:12] + list(twin.named_parameters())[-4:]:
    a = p.grad
    b = ge[n].grad
    print(n, None if a is None else float(a.float().norm()), None if b is None else float(b.float().norm()),
          None if (a is None or b is None) else float((a.float() - b.float()).norm()))
