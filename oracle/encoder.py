"""ORACLE (test infrastructure only): torch-fp32 CPU restatement of HumanActionScorer.forward.

Functional form of /root/reference/model.py, reading the reference state_dict keys directly:
  SinusoidalPositionalEmbedding  model.py:8-19  (uses the loaded pos_enc.pe buffer)
  TemporalConvBlock              model.py:21-40  (conv k=5 dil d pad 2d, GELU(erf), residual, GroupNorm(1))
  MovementConvEncoder            model.py:43-58  (stem k=1, 4 blocks dil 1,2,4,8, proj)
  MinimalPerFrameFusion          model.py:61-98  (single-query softmax pool over modalities)
  HumanActionScorer.forward      model.py:162-193 (LN per modality, CLS+PE, post-norm transformer,
                                                   L2-normalised outputs)
Eval mode: dropout is identity.  The transformer is nn.TransformerEncoderLayer (post-norm, ReLU,
LN eps 1e-5, batch_first) restated with explicit q/k/v heads.
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F


class OracleEncoder:
    def __init__(self, sd: Dict[str, np.ndarray], dims_raw: Dict[str, int], dims_diff: Dict[str, int],
                 d_model: int = 256, time_layers: int = 4, time_heads: int = 8):
        self.p = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in sd.items()}
        self.mods: List[str] = list(dims_raw.keys())
        self.dims_raw = dims_raw
        self.dims_diff = dims_diff
        self.d = d_model
        self.L = time_layers
        self.H = time_heads

    def _movement(self, prefix: str, x_btf: torch.Tensor) -> torch.Tensor:
        p = self.p
        y = F.conv1d(x_btf.transpose(1, 2), p[prefix + ".stem.weight"])
        for i, dil in enumerate((1, 2, 4, 8)):
            b = f"{prefix}.blocks.{i}"
            res = y
            z = F.gelu(F.conv1d(y, p[b + ".conv1.weight"], padding=2 * dil, dilation=dil))
            z = F.conv1d(z, p[b + ".conv2.weight"], padding=2 * dil, dilation=dil)
            z = F.gelu(z + res)
            y = F.group_norm(z, 1, p[b + ".norm.weight"], p[b + ".norm.bias"], eps=1e-5)
        return y.transpose(1, 2) @ p[prefix + ".proj.weight"].t()

    def _fusion(self, M_tokens: torch.Tensor) -> torch.Tensor:
        p = self.p
        B, T, M, D = M_tokens.shape
        kv = F.layer_norm(M_tokens, (D,), p["fusion.kv_ln.weight"], p["fusion.kv_ln.bias"]).reshape(B * T, M, D)
        q = F.layer_norm(p["fusion.latent"].expand(B * T, 1, D), (D,), p["fusion.q_ln.weight"],
                         p["fusion.q_ln.bias"])
        Q = q @ p["fusion.Wq.weight"].t()
        K = kv @ p["fusion.Wk.weight"].t()
        V = kv @ p["fusion.Wv.weight"].t()
        logits = (Q @ K.transpose(-2, -1)) / math.sqrt(D)
        tau = F.softplus(p["fusion.logit_temp"]) + 1e-3
        logits = logits / tau.view(1, 1, M) + p["fusion.logit_bias"].view(1, 1, M)
        A = logits.softmax(dim=-1)
        fused = (A @ V).squeeze(1) @ p["fusion.Wo.weight"].t()
        return fused.view(B, T, D)

    def _layer(self, l: int, x: torch.Tensor) -> torch.Tensor:
        p = self.p
        pre = f"temporal.layers.{l}"
        B, S, D = x.shape
        H = self.H
        hd = D // H
        qkv = x @ p[pre + ".self_attn.in_proj_weight"].t() + p[pre + ".self_attn.in_proj_bias"]
        q, k, v = qkv.split(D, dim=-1)
        q = q.view(B, S, H, hd).transpose(1, 2)
        k = k.view(B, S, H, hd).transpose(1, 2)
        v = v.view(B, S, H, hd).transpose(1, 2)
        att = ((q / math.sqrt(hd)) @ k.transpose(-2, -1)).softmax(-1)
        o = (att @ v).transpose(1, 2).reshape(B, S, D)
        o = o @ p[pre + ".self_attn.out_proj.weight"].t() + p[pre + ".self_attn.out_proj.bias"]
        x = F.layer_norm(x + o, (D,), p[pre + ".norm1.weight"], p[pre + ".norm1.bias"], eps=1e-5)
        h = F.relu(x @ p[pre + ".linear1.weight"].t() + p[pre + ".linear1.bias"])
        h = h @ p[pre + ".linear2.weight"].t() + p[pre + ".linear2.bias"]
        return F.layer_norm(x + h, (D,), p[pre + ".norm2.weight"], p[pre + ".norm2.bias"], eps=1e-5)

    @torch.no_grad()
    def forward(self, x: torch.Tensor):
        """x [B,T,D_in] -> (seq_embed [B,d], frame_embeds [B,T+1,d], tokens [B,T+1,d])."""
        B, T, _ = x.shape
        n_raw = sum(self.dims_raw[m] for m in self.mods)
        raw, diff = x[:, :, :n_raw], x[:, :, n_raw:]
        rawp = dict(zip(self.mods, torch.split(raw, [self.dims_raw[m] for m in self.mods], dim=-1)))
        diffp = dict(zip(self.mods, torch.split(diff, [self.dims_diff[m] for m in self.mods], dim=-1)))
        per_mod = []
        for m in self.mods:
            s = self._movement(f"state_enc.{m}", rawp[m])
            if self.dims_diff[m] > 0:
                s = s + self._movement(f"motion_enc.{m}", diffp[m])
            per_mod.append(F.layer_norm(s, (s.size(-1),)).unsqueeze(2))
        frame_tok = self._fusion(torch.cat(per_mod, dim=2))
        tokens = torch.cat([self.p["cls"].expand(B, 1, self.d), frame_tok], dim=1)
        tokens = tokens + self.p["pos_enc.pe"][:, :tokens.size(1), :]
        for l in range(self.L):
            tokens = self._layer(l, tokens)
        return F.normalize(tokens[:, 0, :]), F.normalize(tokens, dim=-1), tokens
