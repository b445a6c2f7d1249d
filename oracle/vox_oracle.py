"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the CPU restatement (libvox_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
It is the checker the HIP path is compared against, never part of the product.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "voxtral.c_amd"))
from vox_weights import (VoxConfig, Weights, build_weights_struct,  # noqa: E402
                         config_struct_class, weights_struct_class)

LIB_PATH = os.path.join(_HERE, "libvox_oracle.so")
REF_AUDIO_PATH = os.path.join(_HERE, "_ref", "librefaudio.so")

ConfigC = config_struct_class()
WeightsC = weights_struct_class()
_lib = None

fp = ctypes.POINTER(ctypes.c_float)
ip = ctypes.POINTER(ctypes.c_int)


def f(a):
    return a.ctypes.data_as(fp)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built (make -C oracle)")
        L = ctypes.CDLL(LIB_PATH)
        P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        sig = {
            "vo_set_threads": (None, [I]), "vo_set_no_compaction": (None, [I]),
            "vo_set_kv_fp16": (None, [I]), "vo_f16_round": (None, [fp, I, fp]),
            "vo_linear_bf16": (None, [fp, fp, P, fp, I, I, I]),
            "vo_linear_q8": (None, [fp, fp, P, fp, fp, I, I, I]),
            "vo_rms_norm": (None, [fp, fp, fp, I, I, F]),
            "vo_gelu": (None, [fp, I, I]), "vo_silu": (None, [fp, I]),
            "vo_causal_conv1d": (None, [fp, fp, fp, fp, I, I, I, I, I]),
            "vo_causal_attention": (None, [fp, fp, fp, fp, I, I, I, I, I, F, I, I]),
            "vo_rope_freqs": (None, [fp, ip, I, I, F]),
            "vo_apply_rope": (None, [fp, fp, I, I, I]),
            "vo_time_embedding": (None, [fp, I, F]),
            "vo_model_create": (P, [P, P, I]), "vo_model_free": (None, [P]),
            "vo_model_ada_scale": (fp, [P]), "vo_model_set_delay": (None, [P, I]),
            "vo_stream_create": (P, [P]), "vo_stream_free": (None, [P]),
            "vo_conv_stem": (I, [P, fp, I, fp, I]),
            "vo_encoder_incremental": (I, [P, fp, I]),
            "vo_adapter": (I, [P, fp, I, fp]),
            "vo_stream_encode_mel": (I, [P, fp, I]),
            "vo_stream_adapter_tokens": (I, [P]), "vo_stream_adapter": (fp, [P]),
            "vo_decoder_prefill": (None, [P, fp, I]),
            "vo_decoder_forward": (I, [P, fp, fp]),
            "vo_stream_decode": (I, [P, I, I, ip, fp]),
            "vo_stream_state": (None, [P, ip]),
            "vo_stream_reset_decoder": (None, [P]), "vo_stream_reset_full": (None, [P]),
            "vo_mel_create": (P, [I]), "vo_mel_feed": (I, [P, fp, I]),
            "vo_mel_finish": (I, [P, I]), "vo_mel_data": (fp, [P, ip]), "vo_mel_free": (None, [P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def set_threads(n: int):
    lib().vo_set_threads(n)


def set_no_compaction(on: bool):
    """test-only: grow the KV caches instead of compacting them (invariance tests)"""
    lib().vo_set_no_compaction(int(on))


def set_kv_fp16(on: bool):
    """the reference's fp16 decoder KV cache (VOX_DECODER_KV_FP16): every decoder K/V append
    rounded to IEEE half (process-wide, like set_no_compaction)"""
    lib().vo_set_kv_fp16(int(on))


def f16_round(x):
    x = np.ascontiguousarray(x, np.float32).ravel()
    out = np.empty_like(x)
    lib().vo_f16_round(f(x), x.size, f(out))
    return out


# ---- per-op restatements -------------------------------------------------
def linear_bf16(x, W_bf16, bias=None):
    x = np.ascontiguousarray(x, np.float32)
    M, K = x.shape
    N = W_bf16.shape[0]
    y = np.empty((M, N), np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, np.float32)
    lib().vo_linear_bf16(f(y), f(x), np.ascontiguousarray(W_bf16).ctypes.data,
                         None if b is None else f(b), M, K, N)
    return y


def linear_q8(x, W_q8, scales, bias=None):
    x = np.ascontiguousarray(x, np.float32)
    M, K = x.shape
    N = W_q8.shape[0]
    y = np.empty((M, N), np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, np.float32)
    lib().vo_linear_q8(f(y), f(x), np.ascontiguousarray(W_q8, np.int8).ctypes.data,
                       f(np.ascontiguousarray(scales, np.float32)), None if b is None else f(b), M, K, N)
    return y


def rms_norm(x, w, eps=1e-5):
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    lib().vo_rms_norm(f(out), f(x), f(np.ascontiguousarray(w, np.float32)), x.shape[0], x.shape[1], eps)
    return out


def gelu(x, erf_mode=0):
    x = np.array(x, np.float32, copy=True)
    lib().vo_gelu(f(x), x.size, erf_mode)
    return x


def silu(x):
    x = np.array(x, np.float32, copy=True)
    lib().vo_silu(f(x), x.size)
    return x


def causal_conv1d(x_cl, w, b, stride):
    """x_cl [C_in, L], w [C_out, C_in, 3] -> [C_out, L_out]"""
    x_cl = np.ascontiguousarray(x_cl, np.float32)
    cin, L = x_cl.shape
    cout, _, ks = w.shape
    n_frames = (float(L) - ks + (ks - stride)) / float(stride) + 1.0
    lout = int(np.ceil(np.float32(n_frames)))
    out = np.zeros((cout, lout), np.float32)
    lib().vo_causal_conv1d(f(out), f(x_cl), f(np.ascontiguousarray(w, np.float32)),
                           f(np.ascontiguousarray(b, np.float32)), cin, cout, L, ks, stride)
    return out


def causal_attention(Q, K, V, n_heads, n_kv_heads, head_dim, window, q_offset):
    Q, K, V = (np.ascontiguousarray(a, np.float32) for a in (Q, K, V))
    out = np.zeros_like(Q)
    lib().vo_causal_attention(f(out), f(Q), f(K), f(V), Q.shape[0], K.shape[0], n_heads, n_kv_heads,
                              head_dim, float(np.float32(1.0) / np.sqrt(np.float32(head_dim))),
                              window, q_offset)
    return out


def rope_freqs(positions, dim, theta=1e6):
    pos = np.ascontiguousarray(positions, np.int32)
    out = np.empty((len(pos), dim), np.float32)
    lib().vo_rope_freqs(f(out), pos.ctypes.data_as(ip), len(pos), dim, theta)
    return out


def apply_rope(x, freqs, heads, head_dim):
    x = np.array(x, np.float32, copy=True)
    lib().vo_apply_rope(f(x), f(np.ascontiguousarray(freqs, np.float32)), x.shape[0], heads, head_dim)
    return x


def time_embedding(dim, t):
    out = np.empty(dim, np.float32)
    lib().vo_time_embedding(f(out), dim, float(t))
    return out


# ---- model / stream --------------------------------------------------------
class OracleModel:
    def __init__(self, cfg: VoxConfig, weights: Weights, delay_tokens: int = 6):
        self.cfg = cfg
        self.weights = weights
        self.delay_tokens = delay_tokens
        self._cfg_c = cfg.ctypes_struct(ConfigC)
        self._w, self._keep = build_weights_struct(weights, WeightsC)
        self.h = lib().vo_model_create(ctypes.byref(self._cfg_c), ctypes.byref(self._w), delay_tokens)

    def ada_scale(self):
        c = self.cfg
        p = lib().vo_model_ada_scale(self.h)
        return np.ctypeslib.as_array(p, (c.dec_layers * c.dec_dim,)).reshape(c.dec_layers, c.dec_dim).copy()

    def set_delay(self, delay_tokens):
        self.delay_tokens = delay_tokens
        lib().vo_model_set_delay(self.h, delay_tokens)

    def close(self):
        if self.h:
            lib().vo_model_free(self.h)
            self.h = None


class OracleStream:
    def __init__(self, model: OracleModel):
        self.model = model
        self.cfg = model.cfg
        self.h = lib().vo_stream_create(model.h)

    def conv_stem(self, mel):
        mel = np.ascontiguousarray(mel, np.float32)
        cap = mel.shape[0] // 2 + 4
        out = np.zeros((cap, self.cfg.enc_dim), np.float32)
        n = lib().vo_conv_stem(self.h, f(mel), mel.shape[0], f(out), cap)
        return out[:n]

    def encoder_incremental(self, x):
        x = np.array(x, np.float32, copy=True)
        lib().vo_encoder_incremental(self.h, f(x), x.shape[0])
        return x

    def encode_mel(self, mel):
        mel = np.ascontiguousarray(mel, np.float32)
        return lib().vo_stream_encode_mel(self.h, f(mel), mel.shape[0])

    def decoder_prefill(self, embeds):
        """vox_decoder_prefill (voxtral_decoder.c:447-612) on embeds [n, dec_dim]"""
        e = np.ascontiguousarray(embeds, np.float32)
        lib().vo_decoder_prefill(self.h, f(e), e.shape[0])

    def decoder_forward(self, embed):
        """vox_decoder_forward (voxtral_decoder.c:640-780): (argmax id, logits)"""
        e = np.ascontiguousarray(embed, np.float32)
        logits = np.empty(self.cfg.vocab, np.float32)
        tok = lib().vo_decoder_forward(self.h, f(e), f(logits))
        return tok, logits

    @property
    def adapter_tokens(self):
        return lib().vo_stream_adapter_tokens(self.h)

    def read_adapter(self):
        n = self.adapter_tokens
        if n == 0:
            return np.zeros((0, self.cfg.dec_dim), np.float32)
        p = lib().vo_stream_adapter(self.h)
        return np.ctypeslib.as_array(p, (n * self.cfg.dec_dim,)).reshape(n, self.cfg.dec_dim).copy()

    def decode(self, max_steps=1 << 30, stop_at_eos=True, want_logits=False):
        cap = min(max_steps, max(self.adapter_tokens + 1, 1))
        toks = np.zeros(cap, np.int32)
        logits = np.zeros((cap, self.cfg.vocab), np.float32) if want_logits else None
        n = lib().vo_stream_decode(self.h, cap, int(stop_at_eos), toks.ctypes.data_as(ip),
                                   f(logits) if want_logits else None)
        return (toks[:n], logits[:n]) if want_logits else toks[:n]

    def reset_decoder(self):
        lib().vo_stream_reset_decoder(self.h)

    def reset_full(self):
        lib().vo_stream_reset_full(self.h)

    def state(self):
        o = np.zeros(8, np.int32)
        lib().vo_stream_state(self.h, o.ctypes.data_as(ip))
        return dict(zip(["enc_len", "enc_off", "dec_len", "dec_off", "adapter", "gen_pos",
                         "enc_res", "conv0_res"], o.tolist()))

    def close(self):
        if self.h:
            lib().vo_stream_free(self.h)
            self.h = None


def fill_alts(logits, best_token, n_alt, cutoff, text_min=1000, max_alt=4):
    """stream_fill_alts (voxtral.c:955-1010) on one step's logits: softmax in f32 (max,
    exp(l - max), sum, * 1/sum), then repeated scans over ids >= TOKEN_TEXT_MIN for the most
    probable unused id, accepted while 1 - p / p_best <= cutoff.  Returns (ids, probs),
    length max_alt, -1 / 0 padded."""
    ids = [-1] * max_alt
    probs = [0.0] * max_alt
    ids[0] = int(best_token)
    if n_alt <= 1:
        return ids, probs
    lg = np.asarray(logits, np.float32)
    e = np.exp(lg - lg.max()).astype(np.float32)
    p = e * np.float32(np.float32(1.0) / e.sum(dtype=np.float32))
    best_prob = float(p[best_token])
    probs[0] = best_prob
    if best_prob <= 0:
        return ids, probs
    cand = p.copy()
    cand[:text_min] = -1.0
    cand[best_token] = -1.0
    for k in range(1, n_alt):
        i = int(np.argmax(cand))          # first index of the maximum, as the strict '>' scan
        if cand[i] < 0:
            break
        if 1.0 - float(cand[i]) / best_prob > cutoff:
            break
        ids[k], probs[k] = i, float(cand[i])
        cand[i] = -1.0
    return ids, probs


class OracleMel:
    """Incremental log-mel (voxtral_audio.c:405-633)."""

    def __init__(self, left_pad_samples=32 * 1280):
        self.h = lib().vo_mel_create(left_pad_samples)

    def feed(self, samples):
        s = np.ascontiguousarray(samples, np.float32)
        return lib().vo_mel_feed(self.h, f(s), len(s))

    def finish(self, right_pad=0):
        return lib().vo_mel_finish(self.h, right_pad)

    def data(self):
        n = ctypes.c_int(0)
        p = lib().vo_mel_data(self.h, ctypes.byref(n))
        if n.value == 0:
            return np.zeros((0, 128), np.float32)
        return np.ctypeslib.as_array(p, (n.value * 128,)).reshape(n.value, 128).copy()

    def close(self):
        if self.h:
            lib().vo_mel_free(self.h)
            self.h = None


def read_wav(path):
    """16-bit PCM WAV -> float32 [-1,1] mono at 16 kHz (voxtral_audio.c:49-141)."""
    data = open(path, "rb").read()
    assert data[:4] == b"RIFF" and data[8:12] == b"WAVE"
    p, ch, sr, bits, fmt, pcm = 12, 0, 0, 0, 0, None
    while p + 8 <= len(data):
        cid, size = data[p:p + 4], int.from_bytes(data[p + 4:p + 8], "little")
        if cid == b"fmt ":
            fmt = int.from_bytes(data[p + 8:p + 10], "little")
            ch = int.from_bytes(data[p + 10:p + 12], "little")
            sr = int.from_bytes(data[p + 12:p + 16], "little")
            bits = int.from_bytes(data[p + 22:p + 24], "little")
        elif cid == b"data":
            pcm = data[p + 8:p + 8 + size]
            break
        p += 8 + size + (size & 1)
    assert fmt == 1 and bits == 16 and pcm is not None
    x = np.frombuffer(pcm[:len(pcm) // (2 * ch) * 2 * ch], np.int16).reshape(-1, ch)
    if ch == 1:
        s = x[:, 0].astype(np.float32) / np.float32(32768.0)
    else:
        s = (x.astype(np.float32).sum(1) / np.float32(ch)) / np.float32(32768.0)
    assert sr == 16000, "resampling not needed for the bundled fixtures"
    return s


class OracleSession:
    """stream_run_encoder gating + stream_run_decoder over the oracle (voxtral.c:827-851).
    Independent re-statement of vox_hip.Session (kept separate on purpose)."""

    def __init__(self, stream: OracleStream, interval_s=2.0):
        self.s = stream
        self.cursor = 0
        self.started = False
        self.finished = False
        self.min_new = max(1, int(interval_s * 100.0))
        self.tokens = []
        self.chunks = []

    def _enc(self, mel_all, min_new):
        total = mel_all.shape[0]
        new = total - self.cursor
        need = 312 if not self.started else min_new
        if (new < need and not self.finished) or new <= 0:
            return
        self.chunks.append(new)
        self.s.encode_mel(mel_all[self.cursor:total])
        self.started = True
        self.cursor = total

    def feed(self, mel_all, stop_at_eos=True):
        self._enc(mel_all, self.min_new)
        self.tokens += self.s.decode(stop_at_eos=stop_at_eos).tolist()

    def flush(self, mel_all, stop_at_eos=True):
        self._enc(mel_all, 1)
        self.tokens += self.s.decode(stop_at_eos=stop_at_eos).tolist()

    def finish(self, mel_all, stop_at_eos=True):
        self.finished = True
        self._enc(mel_all, self.min_new)
        self.tokens += self.s.decode(stop_at_eos=stop_at_eos).tolist()


def transcribe_mel_schedule(samples, delay_tokens=6, feed_size=None):
    """Mel frames as vox_transcribe_audio / `-I` streaming would see them: returns a
    list of (kind, mel_all) events, kind in {feed, flush, finish}.  feed_size=None feeds
    all samples at once (vox_transcribe_audio, voxtral.c:1396-1401)."""
    m = OracleMel(32 * 1280)
    events = []
    n = len(samples)
    step = n if not feed_size else feed_size
    for i in range(0, n, step):
        m.feed(samples[i:i + step])
        events.append(("feed", m.data()))
    align = (1280 - (n % 1280)) % 1280
    pad = align + ((delay_tokens + 1) + 10) * 1280
    zeros = np.zeros(pad, np.float32)
    for i in range(0, pad, 4096):
        m.feed(zeros[i:i + 4096])
    events.append(("flush", m.data()))
    m.finish(0)
    events.append(("finish", m.data()))
    m.close()
    return events


class OracleAudioSession:
    """vox_stream_feed / flush / finish over raw 16 kHz samples (voxtral.c:1288-1316,
    1640-1667) with stream_run_encoder's gating (voxtral.c:827-851), stream_run_decoder's
    drain (voxtral.c:1013-1145) and, with continuous=True, its live-mode restarts
    (voxtral.c:1189-1239, limits :410-420).  Token classes as vh_token_class: EOS, control
    (< 1000), invalid (1000: Tekken's empty raw byte), text.  Records every generated id and
    the restarts (kind 1 EOS, 2 KV, 3 non-text streak, 4 no-decode watchdog; full reset)."""

    def __init__(self, stream: OracleStream, interval_s=2.0, continuous=False, delay_tokens=6):
        self.s = stream
        self.interval = interval_s
        self.min_new = max(1, int(interval_s * 100.0))
        self.continuous = continuous
        self.delay_tokens = delay_tokens
        self.mel = OracleMel(32 * 1280)
        self.cursor = 0
        self.started = False
        self.finished = False
        self.real = 0
        self.last_decode = 0
        self.streak = 0
        self.text_since = False
        self.empty_restarts = 0
        self.tokens = []
        self.restarts = []

    def _enc(self, min_new):
        mel = self.mel.data()
        new = mel.shape[0] - self.cursor
        need = 312 if not self.started else min_new
        if (new < need and not self.finished) or new <= 0:
            return
        self.s.encode_mel(mel[self.cursor:])
        self.started = True
        self.cursor = mel.shape[0]

    def _dec(self):
        st = self.s.state()
        prompt = 1 + 32 + self.delay_tokens
        started = lib_started(self.s)
        if not started and self.s.adapter_tokens < prompt:
            return
        toks = self.s.decode(stop_at_eos=True).tolist()
        eos = False
        for t in toks:
            if t == 2:
                eos = True
            elif t < 1000 or t == 1000:
                self.streak += 1
            else:
                self.streak = 0
                self.text_since = True
                self.empty_restarts = 0
        if toks:
            self.last_decode = self.real
        self.tokens += toks
        if not self.continuous:
            return
        st = self.s.state()
        started = lib_started(self.s)
        need = 0
        if eos:
            need = 1
        elif started and st["dec_len"] + st["dec_off"] > 2000:
            need = 2
        elif started and self.streak >= 64:
            need = 3
        elif not self.finished and self.real - self.last_decode >= 16000 * 20:
            need = 4
        if not need:
            return
        if self.text_since:
            self.empty_restarts = 0
        else:
            self.empty_restarts += 1
        full = need >= 2 or self.empty_restarts >= 2
        self.restarts.append((need, full, len(self.tokens)))
        if full:
            self.mel.close()
            self.mel = OracleMel(32 * 1280)
            self.cursor = 0
            self.started = False
            self.s.reset_full()
            self.empty_restarts = 0
        else:
            self.s.reset_decoder()
        self.streak = 0
        self.text_since = False
        self.last_decode = self.real

    def feed(self, samples):
        self.mel.feed(samples)
        self.real += len(samples)
        self._enc(self.min_new)
        self._dec()

    def flush(self):
        align = (1280 - (self.real % 1280)) % 1280
        pad = align + ((self.delay_tokens + 1) + 10) * 1280
        self.mel.feed(np.zeros(pad, np.float32))
        self._enc(1)
        self._dec()

    def finish(self):
        self.flush()
        self.finished = True
        self.mel.finish(0)
        self._enc(self.min_new)
        self._dec()

    def close(self):
        self.mel.close()


def lib_started(stream: OracleStream) -> bool:
    """the oracle stream's decoder has run its prefill (vo_stream_state has no flag for it:
    a started decoder has generated at least one token since its last reset)"""
    return stream.state()["gen_pos"] > 0
