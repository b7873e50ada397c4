"""Fourier / sine 3D position embeddings (mirror of reference
models/position_embedding.py:12-139).  Always evaluated in fp32 (the
reference runs it under no_grad in fp32; a bf16 matmul before sin/cos of
arguments up to ~20 rad would be far outside the 1e-3 feature tolerance)."""
import math

import torch
from torch import nn

from .pc_util import shift_scale_points


class PositionEmbeddingCoordsSine(nn.Module):
    def __init__(self, temperature=10000, normalize=False, scale=None, pos_type="fourier",
                 d_pos=None, d_in=3, gauss_scale=1.0):
        super().__init__()
        if scale is not None and not normalize:
            raise ValueError("normalize should be True if scale is passed")
        if pos_type not in ("sine", "fourier"):
            raise ValueError(pos_type)
        self.temperature = temperature
        self.normalize = normalize
        self.scale = 2 * math.pi if scale is None else scale
        self.pos_type = pos_type
        if pos_type == "fourier":
            if d_pos is None or d_pos % 2:
                raise ValueError("fourier embedding needs an even d_pos")
            self.register_buffer("gauss_B", torch.empty((d_in, d_pos // 2)).normal_() * gauss_scale)
            self.d_pos = d_pos

    def _fourier(self, xyz, num_channels, input_range, seq_first=False):
        d_in, max_d_out = self.gauss_B.shape
        if num_channels is None:
            num_channels = 2 * max_d_out
        d_out = num_channels // 2
        if d_out > max_d_out or d_in != xyz.shape[-1]:
            raise ValueError("bad fourier embedding size")
        B, N = xyz.shape[:2]
        if xyz.is_cuda:
            # one HIP launch (csrc/boxparam.hip ov3d_fourier_pe) instead of ~12 torch kernels
            from . import _native
            x = xyz.float().contiguous()
            rng = [t.float().contiguous() for t in input_range] if self.normalize else [None, None]
            gb = self.gauss_B.float().contiguous()
            shape = (N, B, 2 * d_out) if seq_first else (B, N, 2 * d_out)
            out = torch.empty(shape, dtype=torch.float32, device=xyz.device)
            _native.call("ov3d_fourier_pe", x, B, N, rng[0], rng[1], gb, gb.shape[1], d_out,
                         int(seq_first), out, like=x)
            return out
        x = xyz.float()
        if self.normalize:
            x = shift_scale_points(x, src_range=input_range)
        x = x * (2 * math.pi)
        proj = torch.mm(x.reshape(-1, d_in), self.gauss_B[:, :d_out].float()).view(B, N, d_out)
        out = torch.cat([proj.sin(), proj.cos()], dim=2)   # (B, N, d_pos) channels-last
        return out.transpose(0, 1).contiguous() if seq_first else out

    def _sine(self, xyz, num_channels, input_range):
        x = xyz.float()
        if self.normalize:
            x = shift_scale_points(x, src_range=input_range)
        nd = x.shape[2]
        ndim = num_channels // nd
        ndim -= ndim % 2
        rems = num_channels - ndim * nd
        outs = []
        prev = 0
        dim_t = None
        for d in range(nd):
            cdim = ndim
            if rems > 0:
                cdim += 2
                rems -= 2
            if cdim != prev:
                t = torch.arange(cdim, dtype=torch.float32, device=x.device)
                dim_t = self.temperature ** (2 * (t // 2) / cdim)
            raw = x[:, :, d] * self.scale if self.scale else x[:, :, d]
            pos = raw[:, :, None] / dim_t
            outs.append(torch.stack((pos[:, :, 0::2].sin(), pos[:, :, 1::2].cos()), dim=3).flatten(2))
            prev = cdim
        return torch.cat(outs, dim=2)   # (B, N, d_pos) channels-last

    def rows(self, xyz, num_channels=None, input_range=None, seq_first=False):
        """(B, N, 3) -> (B, N, d_pos) channels-last embedding; seq_first: (N, B, d_pos)
        contiguous (the transformer's row order, written so by the HIP launch)."""
        if xyz.ndim != 3:
            raise ValueError("xyz must be (B, N, 3)")
        with torch.no_grad(), torch.autocast(device_type=xyz.device.type, enabled=False):
            if self.pos_type == "fourier":
                return self._fourier(xyz, num_channels, input_range, seq_first)
            out = self._sine(xyz, num_channels, input_range)
            return out.transpose(0, 1).contiguous() if seq_first else out

    def forward(self, xyz, num_channels=None, input_range=None):
        """Reference layout: (B, d_pos, N)."""
        return self.rows(xyz, num_channels, input_range).permute(0, 2, 1)
