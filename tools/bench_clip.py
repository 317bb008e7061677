"""Config C3 step rate: CLIP-HBA ViT-L/14 + DoRA (r=32 on the last 2 visual and the last text
out_proj, NEWP:484-544), bs=64 synthetic images, MSE against synthetic 66-D targets, fused AdamW
(NEWP:994-1001, 1181).  Random-init weights (the reference downloads OpenAI weights: absent
offline), synthetic data (THINGS images absent).  Prints one JSON line.

    python tools/bench_clip.py [--batch 64] [--steps 10] [--warmup 3]

FLOP accounting (per step, analytic): visual tower forward 2 x 81.0 GMAC per image (SURVEY
§8a a15) + the last text block forward (66 x 77 tokens; blocks 0-10 are a frozen prefix whose
output is cached) + backward through the two DoRA visual blocks and the DoRA text block (input
gradients 2x, DoRA weight gradients 1x their forward GEMM FLOPs).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))

import torch  # noqa: E402

PEAK = 256 * 4 * 1024 * 2.4e9 / 1e12
PEAK_F32 = 256 * 4 * 64 * 2.4e9 / 1e12  # v_mfma_f32_16x16x4_f32 / VALU FMA: 64 FLOP/clk/SIMD


def block_flops(tokens, width, seq, heads_dim=64):
    """forward FLOPs of one pre-LN transformer block (qkv, attention, out_proj, MLP 4x)."""
    gemm = 2 * tokens * width * (3 * width + width + 8 * width)
    attn = 4 * tokens * seq * width
    return gemm + attn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32",
                    help="compute dtype: f32 = the reference's precision (NEWP:274), bf16 opt-in")
    a = ap.parse_args()
    import vit_amd
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    T = torch.float32 if a.dtype == "f32" else torch.bfloat16
    m = vit_amd.CLIPHBA(["class%d" % i for i in range(66)], "ViT-L/14", pos_embedding=True, compute_dtype=T)
    vit_amd.apply_dora_to_ViT(m, n_vision_layers=2, n_transformer_layers=1, r=32)
    vit_amd.switch_dora_layers(m, freeze_all=True, dora_state=True)
    m = m.to(dev)
    opt = vit_amd.FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=3e-4)
    x = torch.randn(a.batch, 3, 224, 224, device=dev)
    y = torch.randn(a.batch, 66, device=dev) * 0.5 + 1.0

    def step():
        opt.zero_grad(set_to_none=True)
        loss = vit_amd.mse_loss(m(x), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        loss = step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    B = a.batch
    vis_tok, vis_seq, vis_w = B * 257, 257, 1024
    txt_tok, txt_seq, txt_w = 66 * 77, 77, 768
    fwd = 24 * block_flops(vis_tok, vis_w, vis_seq) + 2 * B * 256 * 588 * 1024 + block_flops(txt_tok, txt_w, txt_seq)
    bwd = 2 * (2 * block_flops(vis_tok, vis_w, vis_seq)) + 2 * block_flops(txt_tok, txt_w, txt_seq)
    step_flop = fwd + bwd
    ips = B * a.steps / el
    tf = step_flop * a.steps / el / 1e12
    print(json.dumps({"metric": "images/sec CLIP-HBA ViT-L/14 + DoRA train step (config C3)", "value": round(ips, 2),
                      "unit": "images/s", "ms_per_step": round(el / a.steps * 1e3, 3), "batch": B,
                      "dtype": a.dtype, "data": "synthetic images / targets, random-init weights",
                      "step_tflop": round(step_flop / 1e12, 3), "achieved_tflops": round(tf, 1),
                      "peak_tflops": PEAK if a.dtype == "bf16" else PEAK_F32,
                      "frac_of_peak": round(tf / (PEAK if a.dtype == "bf16" else PEAK_F32), 4), "final_loss": round(float(loss.item()), 4)}))


if __name__ == "__main__":
    main()
