"""Which python lines launch torch glue kernels (zeros / copies / adds / cats) in one eager
training step: the tensor methods are wrapped and every call that produces device work is
counted by caller file:line.  python tools/glue_probe.py"""
import os
import sys
import traceback
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ov3d_import  # noqa: E402

COUNT = Counter()
ON = [False]


def _caller():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "glue_probe" in fr.filename:
            continue
        if "ov3d_amd" in fr.filename or "open-vocabulary" in fr.filename or "bench.py" in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno}"
    return "?"


def wrap(owner, name, produces):
    orig = getattr(owner, name)

    def f(*a, **k):
        out = orig(*a, **k)
        if ON[0]:
            try:
                if produces(a, k, out):
                    COUNT[(name, _caller())] += 1
            except Exception:
                pass
        return out
    setattr(owner, name, f)


def _cuda(out):
    return isinstance(out, torch.Tensor) and out.is_cuda and out.numel() > 0


def _new_storage(a, k, out):
    return _cuda(out) and isinstance(a[0], torch.Tensor) and out.data_ptr() != a[0].data_ptr()


def main():
    ov3d_import.load()
    from ov3d_amd import synthetic
    from bench import build, default_args, train_step
    from ov3d_amd import gemm
    gemm.DEFER_WGRAD = True   # as bench.py's captured step
    args = default_args()
    dev = torch.device("cuda")
    model, crit, opt = build(args, dev)
    batch = synthetic.make_batch(8, seed=1, device=dev)
    for _ in range(2):
        train_step(model, crit, opt, batch, args, torch.bfloat16)
    torch.cuda.synchronize()
    for n in ("zeros", "zeros_like", "ones_like", "full", "cat", "stack"):
        wrap(torch, n, lambda a, k, o: _cuda(o))
    for n in ("reshape", "contiguous", "to", "float", "clone", "repeat", "expand_as"):
        wrap(torch.Tensor, n, _new_storage)
    for n in ("add_", "copy_", "zero_", "fill_", "mul_", "__add__", "__mul__", "__sub__", "add"):
        wrap(torch.Tensor, n, lambda a, k, o: _cuda(o))
    ON[0] = True
    train_step(model, crit, opt, batch, args, torch.bfloat16)
    ON[0] = False
    torch.cuda.synchronize()
    print("glue calls in one step:", sum(COUNT.values()))
    for (n, where), c in COUNT.most_common(80):
        print(f"{c:5d}  {n:12s} {where}")


if __name__ == "__main__":
    main()
