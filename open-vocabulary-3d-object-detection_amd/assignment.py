"""Batched Hungarian matching on the device (ov3d_hungarian).

Replaces the per-scene host loop of the reference matcher (criterion.py:65-86:
cost -> numpy, ``scipy.optimize.linear_sum_assignment(final_cost[b, :, :n])``)
with one kernel launch for all L*B problems of a step.  The kernel restates
scipy 1.15's algorithm with the same float64 arithmetic and tie rule, so the
assignment is scipy's for the same cost; nothing is copied to the host and the
training step has no synchronisation point here.
"""
from collections.abc import Sequence

import torch

from . import _native as nat


def hungarian(cost, nactual):
    """cost (P,Q,G) float, nactual (P,) int (device tensor or list)
    -> gt_inds (P,Q) int64, matched (P,Q) float32, status (P,) int32
    (status: 0 ok, -1 NaN/-inf costs — scipy raises there —, -2 infeasible)."""
    cost = nat.check(cost.detach().float().contiguous(), "cost", torch.float32, 3)
    P, Q, G = cost.shape
    if not isinstance(nactual, torch.Tensor):
        nactual = torch.tensor(list(nactual), dtype=torch.int32)
    nactual = nactual.to(device=cost.device, dtype=torch.int32).contiguous()
    if nactual.shape != (P,):
        raise ValueError(f"nactual must have shape ({P},), got {tuple(nactual.shape)}")
    inds = torch.empty((P, Q), dtype=torch.int64, device=cost.device)
    mask = torch.empty((P, Q), dtype=torch.float32, device=cost.device)
    status = torch.empty((P,), dtype=torch.int32, device=cost.device)
    nat.call("ov3d_hungarian", cost, nactual, P, Q, G, inds, mask, status, like=cost)
    return inds, mask, status


class Assignments(Sequence):
    """The reference's ``assignments`` list (criterion.py:86-89): per problem
    ``[row_ind, col_ind]`` (rows ascending, as scipy returns them) or ``[]``.
    Built from the device result on first access (that access synchronises)."""

    def __init__(self, inds, mask):
        self._inds, self._mask, self._list = inds, mask, None

    def _materialise(self):
        if self._list is None:
            out = []
            for p in range(self._mask.shape[0]):
                rows = torch.nonzero(self._mask[p] > 0).flatten()
                out.append([rows, self._inds[p, rows]] if rows.numel() else [])
            self._list = out
        return self._list

    def __getitem__(self, i):
        return self._materialise()[i]

    def __len__(self):
        return self._mask.shape[0]


def check_status(status):
    """Raise like scipy would for an invalid cost (host sync; call outside the hot loop)."""
    s = status.cpu()
    if (s == -1).any():
        raise ValueError("matrix contains invalid numeric entries")
    if (s == -2).any():
        raise ValueError("cost matrix is infeasible")
