"""Python host-side mirror of the voxtral.c streaming API over the MI355X backend.

Loads libvoxtral_hip.so (built in-tree by __graft_entry__.build()) and exposes the same
objects the reference's C API has (voxtral.h:251-337): a model loaded once, streams fed
incrementally, greedy token ids out.  Streams take log-mel frames (host or device
arrays), or raw 16 kHz samples through AudioSession, whose incremental log-mel (Mel,
vox_mel_ctx_t) runs on the device.

There is no CPU fallback: if the HIP library or a GPU is missing every entry point
raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from vox_weights import (VoxConfig, Weights, build_weights_struct, config_struct_class,
                         weights_struct_class)

_HERE = os.path.dirname(os.path.abspath(__file__))
# VOX_HIP_LIB: another build of the same library (developer A/B of two builds on one box)
LIB_PATH = os.environ.get("VOX_HIP_LIB") or os.path.join(_HERE, "libvoxtral_hip.so")

TOKEN_BOS, TOKEN_EOS, TOKEN_STREAMING_PAD = 1, 2, 32
STREAM_FIRST_CHUNK_MIN_MEL = 312          # voxtral.c:405
STREAM_DEFAULT_INTERVAL = 2.0             # voxtral.c:408
RAW_AUDIO_LENGTH_PER_TOK = 1280           # voxtral.c:400
OFFLINE_STREAMING_BUFFER_TOKENS = 10      # voxtral.c:401

ConfigC = config_struct_class()
WeightsC = weights_struct_class()

# exported symbols, as declared in include/voxtral_hip.h
EXPORTS = [
    "vox_hip_init", "vox_hip_available", "vox_hip_shutdown", "vox_hip_memory_used",
    "vox_hip_last_error", "vox_hip_clear_error", "vox_hip_set_device", "vox_hip_config_voxtral_4b",
    "vox_hip_model_create", "vox_hip_model_free", "vox_hip_model_set_delay",
    "vox_hip_model_ada_scale", "vox_hip_model_set_kv_fp16", "vox_hip_stream_kv_fp16",
    "vox_hip_set_gemm_planes", "vox_hip_gemm_planes", "vox_hip_set_gemmf_wait",
    "vox_hip_stream_create", "vox_hip_stream_free",
    "vox_hip_stream_reset", "vox_hip_stream_reset_decoder", "vox_hip_stream_encode_mel",
    "vox_hip_stream_adapter_tokens", "vox_hip_stream_read_adapter", "vox_hip_stream_decode",
    "vox_hip_batch_create", "vox_hip_batch_free", "vox_hip_batch_decode", "vox_hip_batch_decode_rows",
    "vox_hip_batch_begin_rows", "vox_hip_batch_finish",
    "vox_hip_batch_read_logits",
    "vox_hip_batch_stats",
    "vox_hip_stream_state", "vox_hip_stream_set_alt", "vox_hip_stream_read_alts", "vox_hip_sgemm_bf16", "vox_hip_sgemm_q8", "vox_hip_fused_qkv_bf16",
    "vox_hip_fused_ffn_bf16", "vox_hip_encoder_attention", "vox_hip_encoder_full_step",
    "vox_hip_decoder_prefill_step", "vox_hip_decoder_start", "vox_hip_decoder_end",
    "vox_hip_decoder_full_step", "vox_hip_stream_set_profiling", "vox_hip_stream_profile",
    "vox_hip_stream_sync", "vox_hip_stream_set_async_encode", "vox_hip_stream_encode_mel_batch", "vox_hip_device_upload", "vox_hip_device_free",
    "vox_hip_mel_create", "vox_hip_mel_feed", "vox_hip_mel_finish", "vox_hip_mel_frames",
    "vox_hip_mel_frame_ptr", "vox_hip_mel_discard_before", "vox_hip_mel_read", "vox_hip_mel_free", "vox_hip_mel_reset",
]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    fp = ctypes.POINTER(ctypes.c_float)
    ip = ctypes.POINTER(ctypes.c_int)
    sig = {
        "vox_hip_init": (I, []), "vox_hip_available": (I, []), "vox_hip_shutdown": (None, []),
        "vox_hip_memory_used": (ctypes.c_size_t, []), "vox_hip_last_error": (ctypes.c_char_p, []),
        "vox_hip_clear_error": (None, []),
        "vox_hip_set_device": (I, [I]),
        "vox_hip_config_voxtral_4b": (None, [P]),
        "vox_hip_model_create": (P, [P, P, I]), "vox_hip_model_free": (None, [P]),
        "vox_hip_model_set_delay": (I, [P, I]), "vox_hip_model_ada_scale": (I, [P, fp]),
        "vox_hip_model_set_kv_fp16": (I, [P, I]), "vox_hip_stream_kv_fp16": (I, [P]),
        "vox_hip_set_gemm_planes": (I, [I]), "vox_hip_gemm_planes": (I, []),
        "vox_hip_set_gemmf_wait": (I, [I]),
        "vox_hip_stream_create": (P, [P]), "vox_hip_stream_free": (None, [P]),
        "vox_hip_stream_reset": (I, [P]), "vox_hip_stream_reset_decoder": (I, [P]),
        "vox_hip_stream_encode_mel": (I, [P, P, I, I]),
        "vox_hip_stream_adapter_tokens": (I, [P]),
        "vox_hip_stream_read_adapter": (I, [P, I, I, fp]),
        "vox_hip_stream_decode": (I, [P, I, I, ip, fp]),
        "vox_hip_stream_state": (I, [P, ip]),
        "vox_hip_batch_create": (P, [P, I]), "vox_hip_batch_free": (None, [P]),
        "vox_hip_batch_decode": (I, [P, ctypes.POINTER(ctypes.c_void_p), I, I, I, ip, ip]),
        "vox_hip_batch_decode_rows": (I, [P, ctypes.POINTER(ctypes.c_void_p), I, ip, I, I, ip, ip]),
        "vox_hip_batch_begin_rows": (I, [P, ctypes.POINTER(ctypes.c_void_p), I, ip, I, I, ip, ip]),
        "vox_hip_batch_finish": (I, [P]),
        "vox_hip_batch_read_logits": (I, [P, P, fp]),
        "vox_hip_batch_stats": (I, [P, ctypes.POINTER(ctypes.c_longlong)]),
        "vox_hip_stream_set_alt": (I, [P, I, F]),
        "vox_hip_stream_read_alts": (I, [P, I, I, ip, fp]),
        "vox_hip_sgemm_bf16": (None, [I, I, I, fp, P, fp]),
        "vox_hip_sgemm_q8": (None, [I, I, I, fp, P, fp, fp]),
        "vox_hip_fused_qkv_bf16": (None, [I, I, fp, P, I, P, I, P, I, fp, fp, fp]),
        "vox_hip_fused_ffn_bf16": (None, [I, I, I, fp, P, P, P, fp]),
        "vox_hip_encoder_attention": (None, [fp, fp, fp, fp, I, I, I, I, I, F, I, I]),
        "vox_hip_encoder_full_step": (I, [P, fp, I, fp, I]),
        "vox_hip_decoder_prefill_step": (I, [P, fp, I, fp, I]),
        "vox_hip_decoder_start": (None, [P, fp, I]), "vox_hip_decoder_end": (None, [P]),
        "vox_hip_decoder_full_step": (I, [P, fp, I, fp]),
        "vox_hip_stream_set_profiling": (I, [P, I]),
        "vox_hip_stream_profile": (I, [P, ctypes.POINTER(ctypes.c_double)]),
        "vox_hip_stream_sync": (I, [P]),
        "vox_hip_stream_set_async_encode": (I, [P, I]),
        "vox_hip_stream_encode_mel_batch": (I, [P, P, P, I, I, P]),
        "vox_hip_device_upload": (P, [P, ctypes.c_size_t]),
        "vox_hip_device_free": (I, [P]),
        "vox_hip_mel_create": (P, [P, I]), "vox_hip_mel_feed": (I, [P, fp, I]),
        "vox_hip_mel_finish": (I, [P, I]), "vox_hip_mel_frames": (I, [P, ip]),
        "vox_hip_mel_frame_ptr": (P, [P, I]), "vox_hip_mel_discard_before": (I, [P, I]),
        "vox_hip_mel_read": (I, [P, I, I, fp]), "vox_hip_mel_free": (None, [P]), "vox_hip_mel_reset": (I, [P, I]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def fptr(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _err(what):
    msg = lib().vox_hip_last_error()
    raise RuntimeError(f"{what}: {msg.decode() if msg else 'unknown error'}")


def set_gemm_planes(planes: int):
    """bf16 activation planes of the M > 1 GEMMs: 3 (default, exact f32 activations) or 2 (hi + lo)"""
    if lib().vox_hip_set_gemm_planes(int(planes)) != 0:
        _err("set_gemm_planes")


def gemm_planes() -> int:
    return lib().vox_hip_gemm_planes()


def set_gemmf_wait(ticks: int) -> int:
    """the encoder GEMM owner's wait per partial tile (100 MHz ticks; < 0: always recompute);
    returns the previous value (a diagnostic knob for the tests)"""
    return lib().vox_hip_set_gemmf_wait(int(ticks))


def init(device: int | None = None):
    L = lib()
    if device is not None and L.vox_hip_set_device(device) != 0:
        _err("set_device")
    if not L.vox_hip_init():
        _err("vox_hip_init (no GPU?)")


class Model:
    """vox_load (voxtral.c:131-383) for the HIP backend: weights uploaded once into HBM."""

    def __init__(self, cfg: VoxConfig, weights: Weights, delay_tokens: int = 6):
        init()
        self.cfg = cfg
        self.delay_tokens = delay_tokens
        self._cfg_c = cfg.ctypes_struct(ConfigC)
        wstruct, keep = build_weights_struct(weights, WeightsC)
        self.h = lib().vox_hip_model_create(ctypes.byref(self._cfg_c), ctypes.byref(wstruct), delay_tokens)
        if not self.h:
            _err("vox_hip_model_create")

    def set_delay(self, delay_ms: int):
        """vox_set_delay (voxtral.c:1681-1687)"""
        delay_ms = min(max(delay_ms, 80), 2400)
        self.delay_tokens = delay_ms // 80
        if lib().vox_hip_model_set_delay(self.h, self.delay_tokens) != 0:
            _err("set_delay")

    def set_kv_fp16(self, on: bool):
        """VOX_DECODER_KV_FP16 (voxtral.c:189-190): streams created afterwards keep their
        decoder K/V rings in IEEE half"""
        if lib().vox_hip_model_set_kv_fp16(self.h, int(on)) != 0:
            _err("set_kv_fp16")

    def ada_scale(self):
        c = self.cfg
        out = np.empty(c.dec_layers * c.dec_dim, np.float32)
        lib().vox_hip_model_ada_scale(self.h, fptr(out))
        return out.reshape(c.dec_layers, c.dec_dim)

    def close(self):
        if self.h:
            lib().vox_hip_model_free(self.h)
            self.h = None


def encode_mel_batch(streams, mels):
    """vox_hip_stream_encode_mel_batch: each stream's new host mel frames, one encoder pass
    over all of their rows; returns the adapter rows added per stream."""
    n = len(streams)
    assert n == len(mels) and n > 0
    arrs = [np.ascontiguousarray(m, dtype=np.float32) for m in mels]
    for s, a in zip(streams, arrs):
        # the C side copies n * mel_bins floats per stream: shapes are checked here
        assert a.ndim == 2 and a.shape[1] == s.cfg.mel_bins, (a.shape, s.cfg.mel_bins)
        assert s.model is streams[0].model, "encode_mel_batch: streams of one model"
    hs = (ctypes.c_void_p * n)(*[s.h for s in streams])
    ps = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    ns = np.array([a.shape[0] for a in arrs], np.int32)
    added = np.zeros(n, np.int32)
    if lib().vox_hip_stream_encode_mel_batch(hs, ps, ns.ctypes.data, n, 0, added.ctypes.data) != 0:
        _err("encode_mel_batch")
    return added.tolist()


class Stream:
    """Per-stream device state (rolling KV, conv tails, adapter buffer) + decode loop."""

    def __init__(self, model: Model):
        self.model = model
        self.cfg = model.cfg
        self.h = lib().vox_hip_stream_create(model.h)
        if not self.h:
            _err("vox_hip_stream_create")

    def reset(self):
        if lib().vox_hip_stream_reset(self.h) != 0:
            _err("reset")

    @property
    def kv_fp16(self) -> bool:
        return bool(lib().vox_hip_stream_kv_fp16(self.h))

    def encode_mel(self, mel: np.ndarray) -> int:
        mel = np.ascontiguousarray(mel, dtype=np.float32)
        assert mel.ndim == 2 and mel.shape[1] == self.cfg.mel_bins
        n = lib().vox_hip_stream_encode_mel(self.h, mel.ctypes.data, mel.shape[0], 0)
        if n < 0:
            _err("encode_mel")
        return n

    def encode_mel_device(self, dev_ptr: int, n_frames: int) -> int:
        n = lib().vox_hip_stream_encode_mel(self.h, ctypes.c_void_p(dev_ptr), n_frames, 1)
        if n < 0:
            _err("encode_mel")
        return n

    def set_async_encode(self, on: bool):
        """encode_mel returns once the pass is enqueued (vox_hip_stream_set_async_encode);
        host mel arrays must outlive the next sync()."""
        if lib().vox_hip_stream_set_async_encode(self.h, int(on)) != 0:
            _err("set_async_encode")

    def sync(self):
        if lib().vox_hip_stream_sync(self.h) != 0:
            _err("sync")

    @property
    def adapter_tokens(self) -> int:
        return lib().vox_hip_stream_adapter_tokens(self.h)

    def read_adapter(self, first: int = 0, n: int | None = None) -> np.ndarray:
        if n is None:
            n = self.adapter_tokens - first
        out = np.empty((n, self.cfg.dec_dim), np.float32)
        if n and lib().vox_hip_stream_read_adapter(self.h, first, n, fptr(out)) != 0:
            _err("read_adapter")
        return out

    def decode(self, max_steps: int = 1 << 30, stop_at_eos: bool = True, want_logits: bool = False):
        max_steps = min(max_steps, 1 << 20)
        cap = min(max_steps, max(self.adapter_tokens + 1, 1))
        toks = np.zeros(cap, np.int32)
        logits = np.zeros((cap, self.cfg.vocab), np.float32) if want_logits else None
        n = lib().vox_hip_stream_decode(self.h, cap, int(stop_at_eos),
                                        toks.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                        fptr(logits) if want_logits else None)
        if n < 0:
            _err("decode")
        return (toks[:n], logits[:n]) if want_logits else toks[:n]

    def state(self):
        o = np.zeros(6, np.int32)
        lib().vox_hip_stream_state(self.h, o.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        return dict(zip(["kv_pos", "gen_pos", "prev_token", "started", "eos_seen", "generated"], o.tolist()))

    def set_alt(self, n_alt: int, cutoff: float):
        """vox_stream_set_alt: keep up to n_alt candidates per step (1 = off)."""
        if lib().vox_hip_stream_set_alt(self.h, n_alt, cutoff) != 0:
            _err("set_alt")

    def read_alts(self, first: int, n: int):
        """(ids [n, 4] with -1 for none, probs [n, 4]) for generated steps [first, first+n)."""
        ids = np.empty((n, 4), np.int32)
        pr = np.empty((n, 4), np.float32)
        if lib().vox_hip_stream_read_alts(self.h, first, n, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                          fptr(pr)) != 0:
            _err("read_alts")
        return ids, pr

    # ---- reference-boundary twins on this stream's device state (host arrays in / out;
    # the calls INTEGRATION.md sections 4-5 bind into voxtral_encoder.c / voxtral_decoder.c)
    def twin_encoder_full_step(self, x: np.ndarray, rope: np.ndarray, logical_start: int) -> np.ndarray:
        """vox_metal_encoder_full_step twin: all encoder layers + final norm on x [n, enc_dim]
        (a copy is returned), K/V appended at logical positions logical_start.."""
        x = np.array(x, np.float32, copy=True, order="C")
        rope = np.ascontiguousarray(rope, np.float32)
        if lib().vox_hip_encoder_full_step(self.h, fptr(x), x.shape[0], fptr(rope), logical_start) != 0:
            _err("encoder_full_step")
        return x

    def twin_decoder_prefill_step(self, x: np.ndarray, rope: np.ndarray, logical_start: int) -> np.ndarray:
        """vox_metal_decoder_prefill_step twin: decoder layers on x [n, dec_dim], KV written."""
        x = np.array(x, np.float32, copy=True, order="C")
        rope = np.ascontiguousarray(rope, np.float32)
        if lib().vox_hip_decoder_prefill_step(self.h, fptr(x), x.shape[0], fptr(rope), logical_start) != 0:
            _err("decoder_prefill_step")
        return x

    def twin_decoder_step(self, x: np.ndarray, rope_row: np.ndarray, logical_pos: int, want_logits=True):
        """decoder_start + decoder_full_step + decoder_end, as voxtral_decoder.c:686-699
        drives the Metal twins: returns (token, logits or None)."""
        x = np.ascontiguousarray(x, np.float32)
        rope_row = np.ascontiguousarray(rope_row, np.float32)
        L = lib()
        L.vox_hip_clear_error()
        L.vox_hip_decoder_start(self.h, fptr(x), x.shape[-1])
        if L.vox_hip_last_error():
            _err("decoder_start")
        logits = np.empty(self.cfg.vocab, np.float32) if want_logits else None
        tok = L.vox_hip_decoder_full_step(self.h, fptr(rope_row), logical_pos,
                                          fptr(logits) if want_logits else None)
        L.vox_hip_decoder_end(self.h)
        if tok < 0:
            _err("decoder_full_step")
        return tok, logits

    def set_profiling(self, on: bool):
        lib().vox_hip_stream_set_profiling(self.h, int(on))

    def profile(self):
        o = (ctypes.c_double * 8)()
        lib().vox_hip_stream_profile(self.h, o)
        # kind 0: the events bracket the W1|W3 GEMV of every layer
        return {"ms": o[0], "bytes": o[1], "launches": int(o[2]), "avg_ms": o[3], "kind": int(o[4]),
                "bytes_per_launch": o[5], "gemmf_recomputes": int(o[6])}

    def sync(self):
        lib().vox_hip_stream_sync(self.h)

    def close(self):
        if self.h:
            lib().vox_hip_stream_free(self.h)
            self.h = None


class Session:
    """vox_stream_t's chunk scheduling over log-mel input (voxtral.c:827-851, 1242-1316,
    1640-1667).  The caller supplies the mel frames produced so far (vox_mel_feed /
    vox_mel_finish output); the session decides when the encoder runs and drains the
    decoder, exactly as stream_run_encoder / stream_run_decoder do."""

    def __init__(self, stream: Stream, interval_s: float = STREAM_DEFAULT_INTERVAL):
        self.s = stream
        self.mel_cursor = 0
        self.conv_started = False
        self.finished = False
        self.min_new_mel = max(1, int(interval_s * 100.0))
        self.tokens: list[int] = []
        self.chunks: list[int] = []

    def _run_encoder(self, mel_all, min_new: int):
        """stream_run_encoder's chunk decision (voxtral.c:827-851); mel_all is the host
        frame array so far, or a device Mel (frames stay in HBM, discarded once encoded)."""
        dev = isinstance(mel_all, Mel)
        total = mel_all.total if dev else mel_all.shape[0]
        if dev:
            self.mel_cursor = max(self.mel_cursor, mel_all.offset)
        new = total - self.mel_cursor
        need = STREAM_FIRST_CHUNK_MIN_MEL if not self.conv_started else min_new
        if new < need and not self.finished:
            return
        if new <= 0:
            return
        self.chunks.append(new)
        if dev:
            self.s.encode_mel_device(mel_all.ptr(self.mel_cursor), new)
        else:
            self.s.encode_mel(mel_all[self.mel_cursor:total])
        self.conv_started = True
        self.mel_cursor = total
        if dev:
            mel_all.discard_before(self.mel_cursor)

    def _run_decoder(self, stop_at_eos=True):
        self.tokens += self.s.decode(stop_at_eos=stop_at_eos).tolist()

    def feed(self, mel_all: np.ndarray, stop_at_eos=True):
        """vox_stream_feed after vox_mel_feed produced mel_all (all frames so far)."""
        self._run_encoder(mel_all, self.min_new_mel)
        self._run_decoder(stop_at_eos)

    def flush(self, mel_all: np.ndarray, stop_at_eos=True):
        """vox_stream_flush (mel_all includes the right-pad frames)."""
        self._run_encoder(mel_all, 1)
        self._run_decoder(stop_at_eos)

    def finish(self, mel_all: np.ndarray, stop_at_eos=True):
        """vox_stream_finish's final pass after vox_mel_finish."""
        self.finished = True
        self._run_encoder(mel_all, self.min_new_mel)
        self._run_decoder(stop_at_eos)


class Mel:
    """Incremental log-mel on the device (vox_mel_ctx_t twin, voxtral_audio.c:405-671):
    samples in, frames kept in HBM for encode_mel_device.  Frame indices are global."""

    def __init__(self, stream: Stream, left_pad_samples: int = 32 * 1280):
        self.h = lib().vox_hip_mel_create(stream.h, left_pad_samples)
        if not self.h:
            _err("vox_hip_mel_create")

    def feed(self, samples: np.ndarray) -> int:
        samples = np.ascontiguousarray(samples, dtype=np.float32)
        n = lib().vox_hip_mel_feed(self.h, fptr(samples), samples.shape[0])
        if n < 0:
            _err("mel_feed")
        return n

    def finish(self, right_pad: int = 0) -> int:
        n = lib().vox_hip_mel_finish(self.h, right_pad)
        if n < 0:
            _err("mel_finish")
        return n

    @property
    def offset(self) -> int:
        off = ctypes.c_int(0)
        lib().vox_hip_mel_frames(self.h, ctypes.byref(off))
        return off.value

    @property
    def total(self) -> int:
        off = ctypes.c_int(0)
        n = lib().vox_hip_mel_frames(self.h, ctypes.byref(off))
        return off.value + n

    def ptr(self, frame: int) -> int:
        p = lib().vox_hip_mel_frame_ptr(self.h, frame)
        if not p:
            _err("mel_frame_ptr")
        return p

    def discard_before(self, frame: int):
        if lib().vox_hip_mel_discard_before(self.h, frame) != 0:
            _err("mel_discard_before")

    def read(self, first: int, n: int) -> np.ndarray:
        out = np.empty((n, 128), np.float32)
        if n and lib().vox_hip_mel_read(self.h, first, n, fptr(out)) != 0:
            _err("mel_read")
        return out

    def close(self):
        if self.h:
            lib().vox_hip_mel_free(self.h)
            self.h = None


class AudioSession(Session):
    """vox_stream_feed / vox_stream_flush / vox_stream_finish (voxtral.c:1288-1316,
    1640-1667) over raw 16 kHz samples: the log-mel is computed on the device (Mel) and
    encoded from HBM, so only the samples cross PCIe."""

    def __init__(self, stream: Stream, interval_s: float = STREAM_DEFAULT_INTERVAL):
        super().__init__(stream, interval_s)
        self.mel = Mel(stream, 32 * RAW_AUDIO_LENGTH_PER_TOK)
        self.real_samples = 0

    def feed_samples(self, samples: np.ndarray, stop_at_eos=True):
        self.mel.feed(samples)
        self.real_samples += int(samples.shape[0])
        self.feed(self.mel, stop_at_eos)

    def flush_samples(self, stop_at_eos=True):
        pad = right_pad_samples(self.real_samples, self.s.model.delay_tokens)
        self.mel.feed(np.zeros(pad, np.float32))
        self.flush(self.mel, stop_at_eos)

    def finish_samples(self, stop_at_eos=True):
        self.flush_samples(stop_at_eos)
        self.mel.finish(0)
        self.finish(self.mel, stop_at_eos)

    def close(self):
        self.mel.close()


def right_pad_samples(n_real_samples: int, delay_tokens: int) -> int:
    """vox_stream_flush padding (voxtral.c:1645-1649)."""
    align = (RAW_AUDIO_LENGTH_PER_TOK - (n_real_samples % RAW_AUDIO_LENGTH_PER_TOK)) % RAW_AUDIO_LENGTH_PER_TOK
    return align + ((delay_tokens + 1) + OFFLINE_STREAMING_BUFFER_TOKENS) * RAW_AUDIO_LENGTH_PER_TOK


class DeviceArray:
    """A host array copied once into HBM (inputs resident before a timed region)."""

    def __init__(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        self.shape, self.dtype = a.shape, a.dtype
        self.ptr = lib().vox_hip_device_upload(a.ctypes.data, a.nbytes)
        if not self.ptr:
            _err("device_upload")

    def free(self):
        if self.ptr:
            lib().vox_hip_device_free(self.ptr)
            self.ptr = None


# ---------------------------------------------------------------------------
# reference-boundary twins (voxtral_metal.h), host arrays in / out
# ---------------------------------------------------------------------------
class Batch:
    """Cross-stream batched greedy decoding (C4): one weight read per step for all streams."""

    def __init__(self, model: "Model", max_streams: int):
        self.h = lib().vox_hip_batch_create(model.h, max_streams)
        if not self.h:
            _err("vox_hip_batch_create")

    def decode(self, streams, max_steps: int, stop_at_eos: bool = True, rows=None):
        """Returns one int32 token array per stream.  rows: each stream reads only its first
        rows[i] adapter rows (vox_hip_batch_decode_rows; the streams' queues are not waited for)."""
        n = len(streams)
        arr = (ctypes.c_void_p * n)(*[s.h for s in streams])
        toks = np.zeros((n, max(1, max_steps)), np.int32)
        cnt = np.zeros(n, np.int32)
        tp = toks.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
        cp = cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
        if rows is None:
            r = lib().vox_hip_batch_decode(self.h, arr, n, max_steps, int(stop_at_eos), tp, cp)
        else:
            rw = np.ascontiguousarray(rows, np.int32)
            assert rw.shape == (n,), "one row bound per stream"
            r = lib().vox_hip_batch_decode_rows(self.h, arr, n, rw.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                                max_steps, int(stop_at_eos), tp, cp)
        if r < 0:
            _err("vox_hip_batch_decode")
        return [toks[i, :cnt[i]].copy() for i in range(n)]

    def read_logits(self, stream: "Stream") -> np.ndarray:
        """logits of the last batched step for a stream that step advanced"""
        out = np.empty(stream.cfg.vocab, np.float32)
        if lib().vox_hip_batch_read_logits(self.h, stream.h, fptr(out)) != 0:
            _err("vox_hip_batch_read_logits")
        return out

    def stats(self) -> dict:
        """vox_hip_batch_stats: counters since creation"""
        out = (ctypes.c_longlong * 6)()
        if lib().vox_hip_batch_stats(self.h, out) != 0:
            _err("vox_hip_batch_stats")
        keys = ("calls", "replays", "rows", "captures", "prefill_passes", "prefilled")
        return dict(zip(keys, (int(v) for v in out)))

    def close(self):
        if self.h:
            lib().vox_hip_batch_free(self.h)
            self.h = None


def _void_call(what, fn, *args):
    """The reference-boundary twins return void (voxtral_metal.h); a failure is reported
    through vox_hip_last_error(), cleared before the call."""
    L = lib()
    L.vox_hip_clear_error()
    fn(*args)
    msg = L.vox_hip_last_error()
    if msg:
        raise RuntimeError(f"{what}: {msg.decode()}")


def sgemm_bf16(A: np.ndarray, B_bf16: np.ndarray) -> np.ndarray:
    """C = A @ B^T (vox_metal_sgemm_bf16 twin); B is cached on the device by host pointer
    and shape, so keep it alive and unmodified."""
    A = np.ascontiguousarray(A, np.float32)
    B_bf16 = np.ascontiguousarray(B_bf16, np.uint16)
    M, K = A.shape
    N = B_bf16.shape[0]
    assert B_bf16.shape[1] == K
    C = np.empty((M, N), np.float32)
    _void_call("sgemm_bf16", lib().vox_hip_sgemm_bf16, M, N, K, fptr(A), B_bf16.ctypes.data, fptr(C))
    return C


def sgemm_q8(A: np.ndarray, B_q8: np.ndarray, scales: np.ndarray) -> np.ndarray:
    """C = A @ (scales[:, None] * B_q8)^T (vox_metal_sgemm_q8 twin); B/scales are cached
    on the device by host pointer, so keep them alive and unmodified."""
    A = np.ascontiguousarray(A, np.float32)
    M, K = A.shape
    N = B_q8.shape[0]
    C = np.empty((M, N), np.float32)
    _void_call("sgemm_q8", lib().vox_hip_sgemm_q8, M, N, K, fptr(A), B_q8.ctypes.data, fptr(scales), fptr(C))
    return C


def fused_qkv_bf16(x: np.ndarray, wq: np.ndarray, wk: np.ndarray, wv: np.ndarray):
    """vox_metal_fused_qkv_bf16 twin: (x wq^T, x wk^T, x wv^T), biases left to the caller."""
    x = np.ascontiguousarray(x, np.float32)
    M, K = x.shape
    outs = [np.empty((M, w.shape[0]), np.float32) for w in (wq, wk, wv)]
    _void_call("fused_qkv_bf16", lib().vox_hip_fused_qkv_bf16, M, K, fptr(x), wq.ctypes.data, wq.shape[0],
               wk.ctypes.data, wk.shape[0], wv.ctypes.data, wv.shape[0], *[fptr(o) for o in outs])
    return tuple(outs)


def fused_ffn_bf16(x: np.ndarray, w1: np.ndarray, w3: np.ndarray, w2: np.ndarray) -> np.ndarray:
    """vox_metal_fused_ffn_bf16 twin: (silu(x w1^T) * x w3^T) w2^T, w2 bias left to the caller."""
    x = np.ascontiguousarray(x, np.float32)
    M, dim = x.shape
    hidden = w1.shape[0]
    out = np.empty((M, dim), np.float32)
    _void_call("fused_ffn_bf16", lib().vox_hip_fused_ffn_bf16, M, dim, hidden, fptr(x), w1.ctypes.data,
               w3.ctypes.data, w2.ctypes.data, fptr(out))
    return out


def encoder_attention(Q, K, V, n_heads, n_kv_heads, head_dim, window, q_offset):
    Q, K, V = (np.ascontiguousarray(x, np.float32) for x in (Q, K, V))
    out = np.empty_like(Q)
    _void_call("encoder_attention", lib().vox_hip_encoder_attention, fptr(out), fptr(Q), fptr(K), fptr(V),
               Q.shape[0], K.shape[0], n_heads, n_kv_heads, head_dim, float(1.0 / np.sqrt(head_dim)),
               window, q_offset)
    return out


# ---------------------------------------------------------------------------
# the C host side (include/vox_hip_host.h, libvox_hip_host.so): vh_stream_* and the per-GPU
# stream scheduler, over a model this process created
# ---------------------------------------------------------------------------
HOST_LIB_PATH = os.path.join(_HERE, "libvox_hip_host.so")
_host = None


class SchedStats(ctypes.Structure):
    _fields_ = [("runs", ctypes.c_int), ("prefills", ctypes.c_int), ("batch_calls", ctypes.c_int),
                ("tokens", ctypes.c_longlong), ("run_ms", ctypes.c_double), ("batch_ms", ctypes.c_double),
                ("enc_batches", ctypes.c_int), ("steps", ctypes.c_longlong), ("captures", ctypes.c_longlong),
                ("prefill_passes", ctypes.c_longlong), ("enc_ms", ctypes.c_double)]


def host_lib():
    global _host
    if _host is not None:
        return _host
    lib()  # the C ABI library first (the host library links it)
    if not os.path.exists(HOST_LIB_PATH):
        raise RuntimeError(f"{HOST_LIB_PATH} not built (run __graft_entry__.build())")
    H = ctypes.CDLL(HOST_LIB_PATH)
    P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    ip = ctypes.POINTER(ctypes.c_int)
    sig = {
        "vh_ctx_wrap": (P, [P, P, I]), "vh_free": (None, [P]), "vh_last_error": (ctypes.c_char_p, []),
        "vh_stream_init": (P, [P]), "vh_stream_free": (None, [P]), "vh_stream_reset": (I, [P]),
        "vh_set_processing_interval": (None, [P, F]), "vh_stream_set_continuous": (None, [P, I]),
        "vh_stream_feed": (I, [P, ctypes.POINTER(ctypes.c_float), I]), "vh_stream_flush": (I, [P]),
        "vh_stream_finish": (I, [P]), "vh_stream_get": (I, [P, ip, I]),
        "vh_stream_get_alt": (I, [P, ip, I]), "vh_stream_set_alt": (I, [P, I, F]),
        "vh_sched_create": (P, [P, I]), "vh_sched_free": (None, [P]), "vh_sched_attach": (I, [P, P]),
        "vh_sched_detach": (I, [P, P]), "vh_sched_run": (I, [P]),
        "vh_sched_stats": (None, [P, ctypes.POINTER(SchedStats)]),
        "vh_sched_set_step_cap": (None, [P, I]), "vh_stream_pending": (I, [P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(H, name)
        fn.restype = res
        fn.argtypes = args
    _host = H
    return H


def _herr(what):
    msg = host_lib().vh_last_error()
    raise RuntimeError(f"{what}: {msg.decode() if msg else 'unknown error'}")


class HostCtx:
    """vh_ctx_t over a Model of this process (vh_ctx_wrap: the model stays the Model's)."""

    def __init__(self, model: Model):
        self.model = model
        self.h = host_lib().vh_ctx_wrap(model.h, ctypes.byref(model._cfg_c), model.delay_tokens)
        if not self.h:
            _herr("vh_ctx_wrap")

    def close(self):
        if self.h:
            host_lib().vh_free(self.h)
            self.h = None


class HostStream:
    """vh_stream_t: vox_stream_feed / flush / finish / get of the C host (voxtral.c:1242-1327)."""

    def __init__(self, ctx: HostCtx, interval_s: float = STREAM_DEFAULT_INTERVAL, continuous: bool = False):
        H = host_lib()
        self.h = H.vh_stream_init(ctx.h)
        if not self.h:
            _herr("vh_stream_init")
        H.vh_set_processing_interval(self.h, interval_s)
        H.vh_stream_set_continuous(self.h, int(continuous))

    def feed(self, samples: np.ndarray):
        samples = np.ascontiguousarray(samples, np.float32)
        if host_lib().vh_stream_feed(self.h, fptr(samples), samples.shape[0]) != 0:
            _herr("vh_stream_feed")

    def flush(self):
        if host_lib().vh_stream_flush(self.h) != 0:
            _herr("vh_stream_flush")

    def finish(self):
        if host_lib().vh_stream_finish(self.h) != 0:
            _herr("vh_stream_finish")

    def reset(self):
        """vh_stream_reset: new audio on this (detached) stream, its buffers and settings kept"""
        if host_lib().vh_stream_reset(self.h) != 0:
            _herr("vh_stream_reset")

    def get(self) -> list[int]:
        out, buf = [], np.empty(4096, np.int32)
        while True:
            n = host_lib().vh_stream_get(self.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), 4096)
            out += buf[:n].tolist()
            if n < 4096:
                return out

    def set_alt(self, n_alt: int, cutoff: float):
        """vox_stream_set_alt (voxtral.c:1329-1337)"""
        if host_lib().vh_stream_set_alt(self.h, n_alt, cutoff) != 0:
            _herr("vh_stream_set_alt")

    def pending(self) -> int:
        """adapter rows not decoded yet (vh_stream_pending)"""
        return host_lib().vh_stream_pending(self.h)

    def get_alt(self) -> np.ndarray:
        """queued records [n, 4]: the chosen id, then the accepted alternatives, -1 padded"""
        out, buf = [], np.empty((1024, 4), np.int32)
        while True:
            n = host_lib().vh_stream_get_alt(self.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), 1024)
            out.append(buf[:n].copy())
            if n < 1024:
                return np.concatenate(out)

    def close(self):
        if self.h:
            host_lib().vh_stream_free(self.h)
            self.h = None


class Scheduler:
    """vh_sched_t: up to 32 HostStreams (VH_SCHED_MAX) of one model on this GPU; run() decodes every
    attached stream's pending adapter rows with batched greedy steps."""

    def __init__(self, ctx: HostCtx, max_streams: int):
        self.h = host_lib().vh_sched_create(ctx.h, max_streams)
        if not self.h:
            _herr("vh_sched_create")

    def attach(self, s: HostStream):
        if host_lib().vh_sched_attach(self.h, s.h) != 0:
            _herr("vh_sched_attach")

    def detach(self, s: HostStream):
        if host_lib().vh_sched_detach(self.h, s.h) != 0:
            _herr("vh_sched_detach")

    def run(self) -> int:
        n = host_lib().vh_sched_run(self.h)
        if n < 0:
            _herr("vh_sched_run")
        return n

    def set_step_cap(self, cap: int):
        """vh_sched_set_step_cap: at most `cap` steps per stream and run (0: drain every run)"""
        host_lib().vh_sched_set_step_cap(self.h, int(cap))

    def stats(self) -> dict:
        st = SchedStats()
        host_lib().vh_sched_stats(self.h, ctypes.byref(st))
        return {f: getattr(st, f) for f, _ in SchedStats._fields_}

    def close(self):
        if self.h:
            host_lib().vh_sched_free(self.h)
            self.h = None
