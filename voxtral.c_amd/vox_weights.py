"""Model configuration, checkpoint tensors and synthetic weights.

Host-side mirror of the reference's weight binding: tensor names and shapes follow the
Voxtral-Mini-4B-Realtime consolidated.safetensors (voxtral_encoder.c:58-146,
voxtral_decoder.c:57-145, voxtral.c:102-125; MODEL.md:154-197).  Matrices stay bf16
(the reference maps them straight out of the mmap, voxtral_safetensors.c:446-451);
norms, biases, conv and ada weights are converted to f32 exactly as `load_f32` does.

The real checkpoint is not available offline, so `synth_weights` builds seeded random
weights of the exact architecture (same bytes and FLOPs) with a counter-based hash
(libvox_synth.so), fast enough to make the full 8.86 GB model in a few seconds.

Q8 checkpoints (config 5) are what the reference's quantize.py writes: every 2-D tensor
becomes dtype "Q8" = f32 per-row scales followed by int8 [rows, cols]; everything else
becomes F32 (quantize.py:96-150).  `quantize_q8` restates that quantiser (in C,
libvox_synth.so) and `load_safetensors` reads such files.
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
        lib.vox_quantize_q8_bf16.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong,
                                             ctypes.c_void_p, ctypes.c_void_p]
        lib.vox_dequant_q8.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_longlong, ctypes.c_longlong]
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
    """Checkpoint tensors by name: bf16 tensors (views into one buffer or an mmap), or for
    a Q8 checkpoint (scales, int8) pairs for the matrices and f32 for the rest; plus the
    f32 conversions the reference makes at load time (load_f32 / safetensors_get_f32)."""

    def __init__(self, cfg: VoxConfig, tensors: dict, keep=None, q8=None, f32=None):
        self.cfg = cfg
        self.t = tensors          # name -> uint16 (bf16 bits)
        self.q8 = q8 or {}        # name -> (scales f32 [rows], q int8 [rows, cols])
        self._stored_f32 = dict(f32 or {})  # F32 tensors of a Q8 checkpoint
        self._keep = keep
        self._f32 = {}

    @property
    def is_q8(self):
        return bool(self.q8)

    def bf16(self, name):
        return self.t[name]

    def matrix(self, name):
        """(data, scales): bf16 bits and None, or int8 and per-row f32 scales."""
        if name in self.q8:
            s, q = self.q8[name]
            return q, s
        return self.t[name], None

    def f32(self, name):
        if name in self._stored_f32:
            return self._stored_f32[name]
        if name not in self._f32:
            if name in self.q8:
                s, q = self.q8[name]
                out = np.empty(q.shape, np.float32)
                synth_lib().vox_dequant_q8(out.ctypes.data, np.ascontiguousarray(q).ctypes.data,
                                           np.ascontiguousarray(s).ctypes.data, q.shape[0], q.shape[1])
                self._f32[name] = out
            else:
                self._f32[name] = bf16_to_f32(self.t[name])
        return self._f32[name]

    @property
    def nbytes(self):
        return (sum(v.nbytes for v in self.t.values())
                + sum(s.nbytes + q.nbytes for s, q in self.q8.values())
                + sum(v.nbytes for v in self._stored_f32.values()))


def quantize_q8(w: Weights) -> Weights:
    """quantize.py (main, :96-150) on a bf16 checkpoint: 2-D tensors -> per-row int8 with
    f32 scales (quantize_q8_row, :35-46), other tensors -> f32."""
    lib = synth_lib()
    q8, f32 = {}, {}
    for name, a in w.t.items():
        if a.ndim == 2:
            a = np.ascontiguousarray(a)
            rows, cols = a.shape
            s = np.empty(rows, np.float32)
            q = np.empty((rows, cols), np.int8)
            lib.vox_quantize_q8_bf16(a.ctypes.data, rows, cols, s.ctypes.data, q.ctypes.data)
            q8[name] = (s, q)
        else:
            f32[name] = bf16_to_f32(a)
    return Weights(w.cfg, {}, q8=q8, f32=f32)


def synth_elems(cfg: VoxConfig) -> int:
    """bf16 elements of the whole checkpoint (the buffer synth_weights fills)"""
    return sum(int(np.prod(s)) for _, s, _ in tensor_specs(cfg))


def weights_over_buffer(cfg: VoxConfig, buf) -> Weights:
    """the checkpoint's tensors as views into one bf16 buffer laid out as synth_weights
    fills it (e.g. a read-only mapping another process generated)"""
    off = 0
    tensors = {}
    for name, shape, _ in tensor_specs(cfg):
        n = int(np.prod(shape))
        tensors[name] = buf[off:off + n].reshape(shape)
        off += n
    return Weights(cfg, tensors, keep=buf)


def synth_weights(cfg: VoxConfig, seed: int = 0, buf=None) -> Weights:
    """seeded random weights of the exact architecture; buf (optional): a writable uint16
    buffer of synth_elems(cfg) elements to fill (a shared mapping)"""
    specs = tensor_specs(cfg)
    total = synth_elems(cfg)
    if buf is None:
        buf = np.empty(total, dtype=np.uint16)
    assert buf.dtype == np.uint16 and buf.size == total
    lib = synth_lib()
    off = 0
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
        off += n
    return weights_over_buffer(cfg, buf)


def load_safetensors(path: str, cfg: VoxConfig = VOXTRAL_4B) -> Weights:
    """mmap a consolidated.safetensors: BF16 tensors (voxtral_safetensors.c:205-285,
    446-451), or the Q8 / F32 tensors quantize.py writes (:393-408, 457-468)."""
    f = open(path, "rb")
    mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    hlen = int.from_bytes(mm[:8], "little")
    hdr = json.loads(mm[8:8 + hlen])
    base = 8 + hlen
    tensors, q8, f32 = {}, {}, {}
    for name, meta in hdr.items():
        if name == "__metadata__":
            continue
        s, e = meta["data_offsets"]
        shape = meta["shape"]
        dt = meta["dtype"]
        if dt == "BF16":
            tensors[name] = np.frombuffer(mm, dtype=np.uint16, count=(e - s) // 2,
                                          offset=base + s).reshape(shape)
        elif dt == "F32":
            f32[name] = np.frombuffer(mm, dtype=np.float32, count=(e - s) // 4,
                                      offset=base + s).reshape(shape)
        elif dt == "Q8":
            rows, cols = shape
            if e - s != rows * 4 + rows * cols:
                raise ValueError(f"{name}: Q8 size {e - s} != {rows}*4 + {rows}*{cols}")
            # quantize.py packs tensors back to back, so scales may be unaligned: copy them
            sc = np.frombuffer(mm, dtype=np.uint8, count=rows * 4, offset=base + s).copy().view(np.float32)
            q = np.frombuffer(mm, dtype=np.int8, count=rows * cols, offset=base + s + rows * 4).reshape(rows, cols)
            q8[name] = (sc, q)
        else:
            raise ValueError(f"{name}: dtype {dt} unsupported (BF16, F32, Q8)")
    if q8 and tensors:
        raise ValueError("mixed BF16 and Q8 matrices are not a reference checkpoint layout")
    return Weights(cfg, tensors, keep=(f, mm), q8=q8, f32=f32)


def write_safetensors(w: Weights, path: str):
    """BF16 checkpoint, or (Q8 weights) the layout quantize.py:152-186 writes."""
    items = []
    if w.is_q8:
        for name, (sc, q) in w.q8.items():
            items.append((name, "Q8", list(q.shape), [np.ascontiguousarray(sc), np.ascontiguousarray(q)]))
        for name, a in w._stored_f32.items():
            items.append((name, "F32", list(a.shape), [np.ascontiguousarray(a, np.float32)]))
    else:
        for name, a in w.t.items():
            items.append((name, "BF16", list(a.shape), [np.ascontiguousarray(a)]))
    hdr, off = {}, 0
    for name, dt, shape, parts in items:
        n = sum(p.nbytes for p in parts)
        hdr[name] = {"dtype": dt, "shape": shape, "data_offsets": [off, off + n]}
        off += n
    hj = json.dumps(hdr).encode()
    hj += b" " * ((8 - len(hj) % 8) % 8)
    with open(path, "wb") as f:
        f.write(len(hj).to_bytes(8, "little"))
        f.write(hj)
        for _, _, _, parts in items:
            for p in parts:
                f.write(p.tobytes())


def write_quantize_py_layout(w: Weights, path: str):
    """A Q8 checkpoint byte for byte as quantize.py:152-186 writes it: tensors in the input
    file's data order (tensor_specs), 2-D ones as Q8 (f32 row scales then int8 rows), the
    rest F32; compact JSON header (separators ',' ':'), no padding, data back to back -- so
    scales and rows land at arbitrary (unaligned) offsets.  tests/test_q8_cpu.py pins the
    whole file against the reference quantizer's output (q8_ref.json file_sha256)."""
    assert w.is_q8
    entries = []
    for name, _, _ in tensor_specs(w.cfg):
        if name in w.q8:
            sc, q = w.q8[name]
            entries.append((name, "Q8", list(q.shape), np.ascontiguousarray(sc).tobytes()
                            + np.ascontiguousarray(q).tobytes()))
        else:
            a = np.ascontiguousarray(w._stored_f32[name], np.float32)
            entries.append((name, "F32", list(a.shape), a.tobytes()))
    hdr, off = {}, 0
    for name, dt, shape, data in entries:
        hdr[name] = {"dtype": dt, "shape": shape, "data_offsets": [off, off + len(data)]}
        off += len(data)
    hj = json.dumps(hdr, separators=(",", ":")).encode("utf-8")
    with open(path, "wb") as f:
        f.write(len(hj).to_bytes(8, "little"))
        f.write(hj)
        for _, _, _, data in entries:
            f.write(data)


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
    # Q8 per-row scales (NULL for bf16 matrices)
    ("enc_wq_s", _PP), ("enc_wk_s", _PP), ("enc_wv_s", _PP), ("enc_wo_s", _PP), ("enc_w1_s", _PP),
    ("enc_w2_s", _PP), ("enc_w3_s", _PP),
    ("ad0_s", _P), ("ad1_s", _P), ("tok_emb_s", _P),
    ("dec_wq_s", _PP), ("dec_wk_s", _PP), ("dec_wv_s", _PP), ("dec_wo_s", _PP), ("dec_w1_s", _PP),
    ("dec_w2_s", _PP), ("dec_w3_s", _PP),
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
    q8 = w.is_q8

    def mats(fld, names):
        data = [w.matrix(n) for n in names]
        setattr(s, fld, arr([p(d) for d, _ in data]))
        if q8:
            setattr(s, fld + "_s", arr([p(sc) for _, sc in data]))

    def mat(fld, name):
        d, sc = w.matrix(name)
        setattr(s, fld, p(d))
        if q8:
            setattr(s, fld + "_s", p(sc))

    for fld, suf in [("enc_wq", "attention.wq.weight"), ("enc_wk", "attention.wk.weight"),
                     ("enc_wv", "attention.wv.weight"), ("enc_wo", "attention.wo.weight"),
                     ("enc_w1", "feed_forward.w1.weight"), ("enc_w2", "feed_forward.w2.weight"),
                     ("enc_w3", "feed_forward.w3.weight")]:
        mats(fld, [enc(l, suf) for l in L])
    for fld, suf in [("enc_wq_b", "attention.wq.bias"), ("enc_wv_b", "attention.wv.bias"),
                     ("enc_wo_b", "attention.wo.bias"), ("enc_w2_b", "feed_forward.w2.bias"),
                     ("enc_attn_norm", "attention_norm.weight"), ("enc_ffn_norm", "ffn_norm.weight")]:
        setattr(s, fld, arr([p(w.f32(enc(l, suf))) for l in L]))
    s.enc_norm = p(w.f32(f"{ENC}.transformer.norm.weight"))
    mat("ad0", f"{EMB}.audio_language_projection.0.weight")
    mat("ad1", f"{EMB}.audio_language_projection.2.weight")
    mat("tok_emb", f"{EMB}.tok_embeddings.weight")
    for fld, suf in [("dec_wq", "attention.wq.weight"), ("dec_wk", "attention.wk.weight"),
                     ("dec_wv", "attention.wv.weight"), ("dec_wo", "attention.wo.weight"),
                     ("dec_w1", "feed_forward.w1.weight"), ("dec_w2", "feed_forward.w2.weight"),
                     ("dec_w3", "feed_forward.w3.weight")]:
        mats(fld, [dec(l, suf) for l in Ld])
    for fld, suf in [("dec_attn_norm", "attention_norm.weight"), ("dec_ffn_norm", "ffn_norm.weight"),
                     ("dec_ada_down", "ada_rms_norm_t_cond.0.weight"),
                     ("dec_ada_up", "ada_rms_norm_t_cond.2.weight")]:
        setattr(s, fld, arr([p(w.f32(dec(l, suf))) for l in Ld]))
    s.dec_norm = p(w.f32("norm.weight"))
    return s, keep
