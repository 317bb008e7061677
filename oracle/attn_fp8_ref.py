"""CPU restatement of the fp8 attention forward (test infrastructure only: imported by tests/).

It restates, in plain torch on the CPU, the algorithm of ``attn_fwd_fp8`` (csrc/attention.hip,
``vit_sdpa_fwd_fp8``) so the GPU kernel's quantisation and accumulation can be checked element by
element; the kernel's accuracy against exact attention (F.scaled_dot_product_attention as timm
calls it) is checked separately against ``exact_sdpa``.

fp8 here is OCP e4m3fn with E8M0 (power-of-two) block scales, the MX format of
``v_mfma_scale_f32_32x32x64_f8f6f4``:

  * q, k: one scale per row (all 64 head dims): e = the smallest integer with
    max|x| <= 448 * 2^e, x_q = e4m3(x * 2^-e) (round to nearest even), value = x_q * 2^e;
  * v: one scale per (head-dim column, 64-key tile), same rule;
  * S = q k^T (exact products of the dequantised values, f32 sums) * scale;
  * softmax online over 64-key tiles, as the kernel runs it: running max m, p = exp(s - m)
    quantised as e4m3(p * 2^8) * 2^-8 BEFORE the earlier tiles' accumulators are rescaled by
    exp(m_old - m_new); o = (sum p v) / (sum p) with the row sum over the unquantised p.

The reference itself has no fp8 path (it runs fp16 autocast, VIT:138): fp8 is BASELINE.json
configs[4]'s choice, so parity here is "the same algorithm" plus a stated accuracy bound
(tests/test_gpu_fp8_attention.py), not bit-identity with the reference.
"""
from __future__ import annotations

import math

import torch

E4M3_MAX = 448.0


def e8m0_exp(amax: torch.Tensor) -> torch.Tensor:
    """Smallest integer e with amax <= 448 * 2^e, clamped to [-127, 127] (0 -> -127)."""
    m, E = torch.frexp(amax.double())          # amax = m * 2^E, m in [0.5, 1)
    # amax = (2m) * 2^(E-1) with 2m in [1, 2): e = (E-1) - 8 if 2m <= 1.75 else (E-1) - 7
    e = torch.where(2 * m <= 1.75, E - 9, E - 8)
    e = torch.where(amax > 0, e, torch.full_like(e, -127))
    return e.clamp(-127, 127)


def quant(x: torch.Tensor, e: torch.Tensor) -> torch.Tensor:
    """Dequantised e4m3 value of x with block exponent e (broadcast against x)."""
    s = torch.pow(2.0, e.double()).float()
    return (x / s).to(torch.float8_e4m3fn).float() * s


def quant_rows(x: torch.Tensor) -> torch.Tensor:
    """[..., 64] -> per-row scaled e4m3 values."""
    e = e8m0_exp(x.abs().amax(-1, keepdim=True))
    return quant(x, e)


def sdpa_fp8(q, k, v, scale=None, causal=False):
    """q, k, v [B, H, N, 64] (any float dtype) -> o [B, H, N, 64] f32, lse [B, H, N]."""
    B, H, N, d = q.shape
    assert d == 64
    scale = d ** -0.5 if scale is None else scale
    q, k, v = q.float(), k.float(), v.float()
    nkt = (N + 63) // 64
    pad = nkt * 64 - N
    qq = quant_rows(q)
    kq = quant_rows(torch.nn.functional.pad(k, (0, 0, 0, pad)))
    vp = torch.nn.functional.pad(v, (0, 0, 0, pad)).reshape(B, H, nkt, 64, d)
    ve = e8m0_exp(vp.abs().amax(3, keepdim=True))           # per (tile, column)
    vq = quant(vp, ve).reshape(B, H, nkt * 64, d)
    s = (qq @ kq.transpose(-1, -2)).double() * scale          # [B, H, N, keys]
    keys = torch.arange(nkt * 64)
    mask = keys[None, :] >= N
    if causal:
        mask = mask | (keys[None, :] > torch.arange(N)[:, None])
    s = s.masked_fill(mask, -math.inf)
    m = torch.full((B, H, N, 1), -math.inf, dtype=torch.float64)
    l = torch.zeros(B, H, N, 1, dtype=torch.float64)
    acc = torch.zeros(B, H, N, d, dtype=torch.float64)
    for t in range(nkt):
        st = s[..., t * 64:(t + 1) * 64]
        mn = torch.maximum(m, st.amax(-1, keepdim=True))
        alpha = torch.exp(m - mn)
        p = torch.exp(st - mn)
        l = l * alpha + p.sum(-1, keepdim=True)
        pq = (p.float() * 256.0).to(torch.float8_e4m3fn).double() / 256.0
        acc = acc * alpha + pq @ vq[..., t * 64:(t + 1) * 64, :].double()
        m = mn
    o = (acc / l).float()
    lse = (m + torch.log(l)).squeeze(-1).float()
    return o, lse


def exact_sdpa(q, k, v, scale=None, causal=False):
    """F.scaled_dot_product_attention in float64 (the accuracy yardstick)."""
    q, k, v = q.double(), k.double(), v.double()
    scale = q.shape[-1] ** -0.5 if scale is None else scale
    s = (q @ k.transpose(-1, -2)) * scale
    if causal:
        N = q.shape[2]
        s = s.masked_fill(torch.ones(N, N, dtype=torch.bool).triu(1), -math.inf)
    return (torch.softmax(s, -1) @ v).float()
