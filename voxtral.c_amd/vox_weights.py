"""Model configuration, checkpoint tensors and synthetic weights.

Host-side mirror of the reference's weight binding: tensor names and shapes follow the
Voxtral-Mini-4B-Realtime consolidated.safetensors (voxtral_encoder.c:58-146,
voxtral_decoder.c:57-145, voxtral.c:102-125; MODEL.md:154-197).  Matrices stay bf16
(the reference maps them straight out of the mmap, voxtral_safetensors.c:446-451);
norms, biases, conv and ada weights are converted to f32 exactly as `load_f32` does.

The real checkpoint is not available offline, so `synth_weights` builds seeded random
weights of the exact architecture (same bytes and FLOPs) with a counter-based hash
(libvox_synth.so), fast enough to make the full 8.86 GB model in a few seconds.
"""
from __future__ import annotations

import ctypes
import dataclasses
import json
import mmap
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))

CONFIG_FIELDS = [
    ("enc_dim", "i"), ("enc_layers", "i"), ("enc_heads", "i"), ("enc_kv_heads", "i"),
    ("enc_head_dim", "i"), ("enc_hidden", "i"), ("enc_window", "i"),
    ("dec_dim", "i"), ("dec_layers", "i"), ("dec_heads", "i"), ("dec_kv_heads", "i"),
    ("dec_head_dim", "i"), ("dec_hidden", "i"), ("dec_window", "i"),
    ("vocab", "i"), ("mel_bins", "i"), ("downsample", "i"), ("ada_dim", "i"),
    ("rope_theta", "f"), ("enc_eps", "f"), ("dec_eps", "f"), ("gelu_erf", "i"),
]


@dataclasses.dataclass(frozen=True)
class VoxConfig:
    enc_dim: int = 1280
    enc_layers: int = 32
    enc_heads: int = 32
    enc_kv_heads: int = 32
    enc_head_dim: int = 64
    enc_hidden: int = 5120
    enc_window: int = 750
    dec_dim: int = 3072
    dec_layers: int = 26
    dec_heads: int = 32
    dec_kv_heads: int = 8
    dec_head_dim: int = 128
    dec_hidden: int = 9216
    dec_window: int = 8192
    vocab: int = 131072
    mel_bins: int = 128
    downsample: int = 4
    ada_dim: int = 32
    rope_theta: float = 1000000.0
    enc_eps: float = 1e-5
    dec_eps: float = 1e-5
    gelu_erf: int = 0

    def ctypes_struct(self, cls):
        return cls(*[getattr(self, n) for n, _ in CONFIG_FIELDS])


def config_struct_class():
    return type("VoxConfigC", (ctypes.Structure,), {
        "_fields_": [(n, ctypes.c_int if t == "i" else ctypes.c_float) for n, t in CONFIG_FIELDS]})


# voxtral.h:26-50
VOXTRAL_4B = VoxConfig()

# Small model with the same structure and head dims (so every kernel specialisation is
# exercised) and short windows so that the sliding-window / rolling-KV paths trigger.
TINY = VoxConfig(enc_dim=256, enc_layers=2, enc_heads=4, enc_kv_heads=4, enc_head_dim=64,
                 enc_hidden=512, enc_window=24, dec_dim=256, dec_layers=2, dec_heads=4,
                 dec_kv_heads=2, dec_head_dim=128, dec_hidden=512, dec_window=48,
                 vocab=4096, ada_dim=32)

# TINY with the real windows (750 / 8192): long streams exercise the multi-block decode
# attention path (more than 256 visible keys) and the encoder window.
TINY_LONG = dataclasses.replace(TINY, enc_window=750, dec_window=8192)

ENC = "mm_streams_embeddings.embedding_module.whisper_encoder"
EMB = "mm_streams_embeddings.embedding_module"


def tensor_specs(c: VoxConfig):
    """(name, shape, kind) for every checkpoint tensor; kind in {w, b, n}."""
    t = []
    ed, eq = c.enc_dim, c.enc_heads * c.enc_head_dim
    ekv = c.enc_kv_heads * c.enc_head_dim
    t += [(f"{ENC}.conv_layers.0.conv.weight", (ed, c.mel_bins, 3), "w"),
          (f"{ENC}.conv_layers.0.conv.bias", (ed,), "b"),
          (f"{ENC}.conv_layers.1.conv.weight", (ed, ed, 3), "w"),
          (f"{ENC}.conv_layers.1.conv.bias", (ed,), "b")]
    for i in range(c.enc_layers):
        p = f"{ENC}.transformer.layers.{i}"
        t += [(f"{p}.attention.wq.weight", (eq, ed), "w"), (f"{p}.attention.wq.bias", (eq,), "b"),
              (f"{p}.attention.wk.weight", (ekv, ed), "w"),
              (f"{p}.attention.wv.weight", (ekv, ed), "w"), (f"{p}.attention.wv.bias", (ekv,), "b"),
              (f"{p}.attention.wo.weight", (ed, eq), "w"), (f"{p}.attention.wo.bias", (ed,), "b"),
              (f"{p}.attention_norm.weight", (ed,), "n"),
              (f"{p}.feed_forward.w1.weight", (c.enc_hidden, ed), "w"),
              (f"{p}.feed_forward.w2.weight", (ed, c.enc_hidden), "w"),
              (f"{p}.feed_forward.w2.bias", (ed,), "b"),
              (f"{p}.feed_forward.w3.weight", (c.enc_hidden, ed), "w"),
              (f"{p}.ffn_norm.weight", (ed,), "n")]
    t += [(f"{ENC}.transformer.norm.weight", (ed,), "n"),
          (f"{EMB}.audio_language_projection.0.weight", (c.dec_dim, ed * c.downsample), "w"),
          (f"{EMB}.audio_language_projection.2.weight", (c.dec_dim, c.dec_dim), "w"),
          (f"{EMB}.tok_embeddings.weight", (c.vocab, c.dec_dim), "w")]
    dq, dkv = c.dec_heads * c.dec_head_dim, c.dec_kv_heads * c.dec_head_dim
    for i in range(c.dec_layers):
        p = f"layers.{i}"
        t += [(f"{p}.ada_rms_norm_t_cond.0.weight", (c.ada_dim, c.dec_dim), "w"),
              (f"{p}.ada_rms_norm_t_cond.2.weight", (c.dec_dim, c.ada_dim), "w"),
              (f"{p}.attention.wq.weight", (dq, c.dec_dim), "w"),
              (f"{p}.attention.wk.weight", (dkv, c.dec_dim), "w"),
              (f"{p}.attention.wv.weight", (dkv, c.dec_dim), "w"),
              (f"{p}.attention.wo.weight", (c.dec_dim, dq), "w"),
              (f"{p}.attention_norm.weight", (c.dec_dim,), "n"),
              (f"{p}.feed_forward.w1.weight", (c.dec_hidden, c.dec_dim), "w"),
              (f"{p}.feed_forward.w2.weight", (c.dec_dim, c.dec_hidden), "w"),
              (f"{p}.feed_forward.w3.weight", (c.dec_hidden, c.dec_dim), "w"),
              (f"{p}.ffn_norm.weight", (c.dec_dim,), "n")]
    t += [("norm.weight", (c.dec_dim,), "n")]
    return t


_synth = None


def synth_lib():
    global _synth
    if _synth is None:
        path = os.path.join(_HERE, "libvox_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
        lib = ctypes.CDLL(path)
        lib.vox_synth_bf16.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                                       ctypes.c_float, ctypes.c_float]
        lib.vox_synth_f32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                                      ctypes.c_float, ctypes.c_float]
        lib.vox_bf16_to_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        _synth = lib
    return _synth


def bf16_to_f32(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint16)
    out = np.empty(a.shape, dtype=np.float32)
    synth_lib().vox_bf16_to_f32(out.ctypes.data, a.ctypes.data, a.size)
    return out


def f32_to_bf16(a: np.ndarray) -> np.ndarray:
    """round-to-nearest-even (finite inputs)"""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return u.astype(np.uint16)


class Weights:
    """bf16 tensors by checkpoint name (views into one buffer or an mmap) plus the f32
    conversions the reference makes at load time."""

    F32_KINDS = ("conv", "bias", "norm", "ada")

    def __init__(self, cfg: VoxConfig, tensors: dict, keep=None):
        self.cfg = cfg
        self.t = tensors
        self._keep = keep
        self._f32 = {}

    def bf16(self, name):
        return self.t[name]

    def f32(self, name):
        if name not in self._f32:
            self._f32[name] = bf16_to_f32(self.t[name])
        return self._f32[name]

    @property
    def nbytes(self):
        return sum(v.nbytes for v in self.t.values())


def synth_weights(cfg: VoxConfig, seed: int = 0) -> Weights:
    specs = tensor_specs(cfg)
    total = sum(int(np.prod(s)) for _, s, _ in specs)
    buf = np.empty(total, dtype=np.uint16)
    lib = synth_lib()
    off = 0
    tensors = {}
    for idx, (name, shape, kind) in enumerate(specs):
        n = int(np.prod(shape))
        view = buf[off:off + n]
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
        if kind == "w":
            std, mean = 1.0 / np.sqrt(fan_in), 0.0
        elif kind == "b":
            std, mean = 0.01, 0.0
        else:
            std, mean = 0.01, 1.0
        lib.vox_synth_bf16(view.ctypes.data, n, (seed * 1000003 + idx * 7919 + 17) & (2**64 - 1),
                           float(std), float(mean))
        tensors[name] = view.reshape(shape)
        off += n
    return Weights(cfg, tensors, keep=buf)


def load_safetensors(path: str, cfg: VoxConfig = VOXTRAL_4B) -> Weights:
    """mmap a BF16 consolidated.safetensors (voxtral_safetensors.c:205-285, 446-451)."""
    f = open(path, "rb")
    mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    hlen = int.from_bytes(mm[:8], "little")
    hdr = json.loads(mm[8:8 + hlen])
    base = 8 + hlen
    tensors = {}
    for name, meta in hdr.items():
        if name == "__metadata__":
            continue
        if meta["dtype"] != "BF16":
            raise ValueError(f"{name}: dtype {meta['dtype']} unsupported (BF16 only)")
        s, e = meta["data_offsets"]
        tensors[name] = np.frombuffer(mm, dtype=np.uint16, count=(e - s) // 2,
                                      offset=base + s).reshape(meta["shape"])
    return Weights(cfg, tensors, keep=(f, mm))


def write_safetensors(w: Weights, path: str):
    hdr, off = {}, 0
    for name, a in w.t.items():
        hdr[name] = {"dtype": "BF16", "shape": list(a.shape), "data_offsets": [off, off + a.nbytes]}
        off += a.nbytes
    hj = json.dumps(hdr).encode()
    hj += b" " * ((8 - len(hj) % 8) % 8)
    with open(path, "wb") as f:
        f.write(len(hj).to_bytes(8, "little"))
        f.write(hj)
        for a in w.t.values():
            f.write(np.ascontiguousarray(a).tobytes())


# ---------------------------------------------------------------------------
# ctypes weight table (same field order in vox_hip_weights_t and vo_weights_t)
# ---------------------------------------------------------------------------
_P = ctypes.c_void_p
_PP = ctypes.POINTER(ctypes.c_void_p)
WEIGHT_FIELDS = [
    ("conv0_w", _P), ("conv0_b", _P), ("conv1_w", _P), ("conv1_b", _P),
    ("enc_wq", _PP), ("enc_wk", _PP), ("enc_wv", _PP), ("enc_wo", _PP), ("enc_w1", _PP),
    ("enc_w2", _PP), ("enc_w3", _PP),
    ("enc_wq_b", _PP), ("enc_wv_b", _PP), ("enc_wo_b", _PP), ("enc_w2_b", _PP),
    ("enc_attn_norm", _PP), ("enc_ffn_norm", _PP),
    ("enc_norm", _P), ("ad0", _P), ("ad1", _P), ("tok_emb", _P),
    ("dec_wq", _PP), ("dec_wk", _PP), ("dec_wv", _PP), ("dec_wo", _PP), ("dec_w1", _PP),
    ("dec_w2", _PP), ("dec_w3", _PP),
    ("dec_attn_norm", _PP), ("dec_ffn_norm", _PP), ("dec_ada_down", _PP), ("dec_ada_up", _PP),
    ("dec_norm", _P),
]


def weights_struct_class():
    return type("VoxWeightsC", (ctypes.Structure,), {"_fields_": WEIGHT_FIELDS})


def build_weights_struct(w: Weights, cls):
    """Fill a weight-table struct; returns (struct, keepalive list)."""
    c = w.cfg
    keep = []

    def p(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return ctypes.c_void_p(a.ctypes.data)

    def arr(ptrs):
        a = (ctypes.c_void_p * len(ptrs))(*[x.value for x in ptrs])
        keep.append(a)
        return ctypes.cast(a, _PP)

    def enc(l, suffix):
        return f"{ENC}.transformer.layers.{l}.{suffix}"

    def dec(l, suffix):
        return f"layers.{l}.{suffix}"

    L, Ld = range(c.enc_layers), range(c.dec_layers)
    s = cls()
    s.conv0_w = p(w.f32(f"{ENC}.conv_layers.0.conv.weight"))
    s.conv0_b = p(w.f32(f"{ENC}.conv_layers.0.conv.bias"))
    s.conv1_w = p(w.f32(f"{ENC}.conv_layers.1.conv.weight"))
    s.conv1_b = p(w.f32(f"{ENC}.conv_layers.1.conv.bias"))
    for fld, suf in [("enc_wq", "attention.wq.weight"), ("enc_wk", "attention.wk.weight"),
                     ("enc_wv", "attention.wv.weight"), ("enc_wo", "attention.wo.weight"),
                     ("enc_w1", "feed_forward.w1.weight"), ("enc_w2", "feed_forward.w2.weight"),
                     ("enc_w3", "feed_forward.w3.weight")]:
        setattr(s, fld, arr([p(w.bf16(enc(l, suf))) for l in L]))
    for fld, suf in [("enc_wq_b", "attention.wq.bias"), ("enc_wv_b", "attention.wv.bias"),
                     ("enc_wo_b", "attention.wo.bias"), ("enc_w2_b", "feed_forward.w2.bias"),
                     ("enc_attn_norm", "attention_norm.weight"), ("enc_ffn_norm", "ffn_norm.weight")]:
        setattr(s, fld, arr([p(w.f32(enc(l, suf))) for l in L]))
    s.enc_norm = p(w.f32(f"{ENC}.transformer.norm.weight"))
    s.ad0 = p(w.bf16(f"{EMB}.audio_language_projection.0.weight"))
    s.ad1 = p(w.bf16(f"{EMB}.audio_language_projection.2.weight"))
    s.tok_emb = p(w.bf16(f"{EMB}.tok_embeddings.weight"))
    for fld, suf in [("dec_wq", "attention.wq.weight"), ("dec_wk", "attention.wk.weight"),
                     ("dec_wv", "attention.wv.weight"), ("dec_wo", "attention.wo.weight"),
                     ("dec_w1", "feed_forward.w1.weight"), ("dec_w2", "feed_forward.w2.weight"),
                     ("dec_w3", "feed_forward.w3.weight")]:
        setattr(s, fld, arr([p(w.bf16(dec(l, suf))) for l in Ld]))
    for fld, suf in [("dec_attn_norm", "attention_norm.weight"), ("dec_ffn_norm", "ffn_norm.weight"),
                     ("dec_ada_down", "ada_rms_norm_t_cond.0.weight"),
                     ("dec_ada_up", "ada_rms_norm_t_cond.2.weight")]:
        setattr(s, fld, arr([p(w.f32(dec(l, suf))) for l in Ld]))
    s.dec_norm = p(w.f32("norm.weight"))
    return s, keep
