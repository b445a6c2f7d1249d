"""Generate tests/golden/pyref.npz from the reference's Python implementation.

/root/reference/python_simple_implementation.py is imported from where it lies.  Its
top-level `import soundfile` (line 24) names a package this image does not have; soundfile
is used only by transcribe() to read WAV files (line 727), which is never called here, so
an empty placeholder module is registered under that name before the import.  Everything
the fixtures exercise is the reference's own torch code: RMSNorm (229-240),
compute_rope_freqs / apply_rope (243-278), causal_attention (281-324), causal_conv1d
(327-341), compute_time_embedding (344-350), encoder_forward (355-443), adapter_forward
(446-466) and Decoder.prefill / forward_one (469-667).

The Python reference uses exact (erf) GELU where the C reference (the parity target) uses
the tanh form (voxtral_kernels.c:505-513); the oracle's `gelu_erf` switch reproduces the
Python variant for this cross-check only.  Whole-model fixtures use the TINY shapes with
seeded synthetic weights (vox_weights.synth_weights), rebuilt from the seed by the tests.

Run here (needs /root/reference):  python3 tests/golden/gen_pyref.py
"""
import dataclasses
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "voxtral.c_amd"))
from vox_weights import TINY, quantize_q8, synth_weights  # noqa: E402

REF = "/root/reference/python_simple_implementation.py"
PIPE_CFG = dataclasses.replace(TINY, gelu_erf=1)
PIPE_SEED = 7
PIPE_MEL_FRAMES = 320


def load_pyref():
    sys.modules.setdefault("soundfile", types.ModuleType("soundfile"))
    spec = importlib.util.spec_from_file_location("voxtral_pyref", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class SF:
    """safe_open stand-in over in-memory bf16 tensors (get_tensor only)."""

    def __init__(self, w):
        self.w = w

    def get_tensor(self, name):
        a = np.ascontiguousarray(self.w.bf16(name))
        return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)


class SFQ8:
    """The same over a Q8 checkpoint: every tensor as the reference C code sees it after
    safetensors_get_f32 (voxtral_safetensors.c:393-408: (float)q * scale per row)."""

    def __init__(self, w):
        self.w = w

    def get_tensor(self, name):
        return torch.from_numpy(np.ascontiguousarray(self.w.f32(name)).copy())


def pipeline_mel():
    rng = np.random.default_rng(11)
    return rng.uniform(-0.6, 1.4, size=(PIPE_MEL_FRAMES, 128)).astype(np.float32)


def main():
    torch.manual_seed(0)
    pr = load_pyref()
    rng = np.random.default_rng(2026)
    out = {}
    # ---- RMSNorm ----
    x = rng.standard_normal((6, 96)).astype(np.float32)
    w = (1 + 0.1 * rng.standard_normal(96)).astype(np.float32)
    out["rms_x"], out["rms_w"] = x, w
    out["rms_y"] = pr.RMSNorm(torch.from_numpy(w), 1e-5)(torch.from_numpy(x)).numpy()
    # ---- RoPE ----
    pos = np.array([0, 1, 7, 100, 4095, 20000], np.int64)
    out["rope_pos"] = pos
    for hd in (64, 128):
        c, s = pr.compute_rope_freqs(torch.from_numpy(pos), hd, 1e6)
        out[f"rope_cos_{hd}"], out[f"rope_sin_{hd}"] = c.numpy(), s.numpy()
        xr = rng.standard_normal((6, 2 * hd)).astype(np.float32)
        out[f"rope_x_{hd}"] = xr
        out[f"rope_y_{hd}"] = pr.apply_rope(torch.from_numpy(xr), c, s, 2, hd, is_neox_style=False).numpy()
    # ---- attention (GQA, sliding window, query offset) ----
    for name, sq, sk, qoff, H, KVH, hd, win in [("att_chunk", 5, 12, 7, 4, 2, 16, 6),
                                                 ("att_step", 1, 31, 30, 4, 1, 32, 8),
                                                 ("att_full", 9, 9, 0, 2, 2, 64, 750)]:
        q = rng.standard_normal((sq, H * hd)).astype(np.float32)
        k = rng.standard_normal((sk, KVH * hd)).astype(np.float32)
        v = rng.standard_normal((sk, KVH * hd)).astype(np.float32)
        o = pr.causal_attention(torch.from_numpy(q), torch.from_numpy(k), torch.from_numpy(v), H, KVH,
                                hd, win, q_start_pos=qoff, kv_start_pos=0).numpy()
        out.update({f"{name}_q": q, f"{name}_k": k, f"{name}_v": v, f"{name}_o": o,
                    f"{name}_meta": np.array([sq, sk, qoff, H, KVH, hd, win])})
    # ---- causal conv1d ----
    for stride, L in ((1, 13), (2, 14)):
        xc = rng.standard_normal((8, L)).astype(np.float32)
        wc = (rng.standard_normal((6, 8, 3)) / 5).astype(np.float32)
        bc = rng.standard_normal(6).astype(np.float32)
        yc = pr.causal_conv1d(torch.from_numpy(xc)[None], torch.from_numpy(wc), torch.from_numpy(bc), stride)[0]
        out.update({f"conv{stride}_x": xc, f"conv{stride}_w": wc, f"conv{stride}_b": bc, f"conv{stride}_y": yc.numpy()})
    # ---- time embedding, GELU ----
    out["temb_64"] = pr.compute_time_embedding(6.0, 64).numpy()
    out["temb_3072"] = pr.compute_time_embedding(6.0, 3072).numpy()
    g = np.linspace(-6, 6, 101).astype(np.float32)
    out["gelu_x"], out["gelu_y"] = g, torch.nn.functional.gelu(torch.from_numpy(g)).numpy()

    # ---- whole pipeline on TINY shapes: encoder -> adapter -> decoder (2 greedy tokens) ----
    c = PIPE_CFG
    for k_, v_ in dict(ENC_DIM=c.enc_dim, ENC_LAYERS=c.enc_layers, ENC_HEADS=c.enc_heads,
                       ENC_HEAD_DIM=c.enc_head_dim, ENC_HIDDEN=c.enc_hidden, ENC_KV_HEADS=c.enc_kv_heads,
                       ENC_WINDOW=c.enc_window, DEC_DIM=c.dec_dim, DEC_LAYERS=c.dec_layers,
                       DEC_HEADS=c.dec_heads, DEC_HEAD_DIM=c.dec_head_dim, DEC_HIDDEN=c.dec_hidden,
                       DEC_KV_HEADS=c.dec_kv_heads, DEC_WINDOW=c.dec_window, VOCAB_SIZE=c.vocab,
                       ADA_NORM_DIM=c.ada_dim).items():
        setattr(pr, k_, v_)
    wts = synth_weights(c, seed=PIPE_SEED)
    mel = pipeline_mel()

    def pipeline(sf):
        with torch.no_grad():
            enc = pr.encoder_forward(torch.from_numpy(mel.T.copy()), None, sf)
            ad = pr.adapter_forward(enc, sf)
            dec = pr.Decoder(sf)
            t_cond = pr.compute_time_embedding(6.0, c.dec_dim)
            prompt = [pr.TOKEN_BOS] + [pr.TOKEN_STREAMING_PAD] * (32 + 6)
            L = len(prompt)
            pe = ad[:L] + dec.embed_tokens(torch.tensor(prompt))
            dec.prefill(pe[:-1], t_cond)
            lg0 = dec.forward_one(pe[-1], pos=L - 1, t_cond=t_cond)
            t0 = int(lg0.argmax())
            lg1 = dec.forward_one(ad[L] + dec.embed_token(t0), pos=L, t_cond=t_cond)
            t1 = int(lg1.argmax())
        return enc.numpy(), ad.numpy(), np.stack([lg0.numpy(), lg1.numpy()]), np.array([t0, t1])

    enc, ad, lg, tk = pipeline(SF(wts))
    out.update({"pipe_mel": mel, "pipe_enc": enc, "pipe_adapter": ad, "pipe_logits": lg,
                "pipe_tokens": tk, "pipe_seed": np.array(PIPE_SEED)})
    # Q8 checkpoint of the same weights (quantize.py restatement, pinned by q8_ref.json)
    enc, ad, lg, tk = pipeline(SFQ8(quantize_q8(wts)))
    out.update({"pipeq8_enc": enc, "pipeq8_adapter": ad, "pipeq8_logits": lg, "pipeq8_tokens": tk})
    np.savez_compressed(os.path.join(HERE, "pyref.npz"), **out)
    print("wrote", len(out), "arrays; tokens", out["pipe_tokens"], "q8 tokens", out["pipeq8_tokens"])


if __name__ == "__main__":
    main()
