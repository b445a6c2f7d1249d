"""The C host side (include/vox_hip_host.h, voxtral.c_amd/host/): the reference's loader and
streaming API in C99 over the C ABI, and the main.c-style CLI.

CPU: the safetensors header parser derives the model dimensions from a checkpoint written by
vox_weights.write_safetensors (bf16 and the quantize.py Q8 layout), and the WAV reader
returns the samples the oracle's reader does.  GPU: the CLI transcribes jfk.wav from a
TINY_LONG checkpoint file with the ids of the Python AudioSession and of the CPU oracle."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

PKG = os.path.join(ROOT, "voxtral.c_amd")
HOSTLIB = os.path.join(PKG, "libvox_hip_host.so")
CLI = os.path.join(PKG, "vox_hip_transcribe")


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory, tiny_weights):
    from vox_weights import write_safetensors
    d = tmp_path_factory.mktemp("ckpt")
    path = str(d / "consolidated.safetensors")
    write_safetensors(tiny_weights, path)
    return path


def _host():
    import vox_hip
    L = ctypes.CDLL(HOSTLIB)
    L.vh_inspect.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    L.vh_load_wav.restype = ctypes.POINTER(ctypes.c_float)
    L.vh_load_wav.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    return L, vox_hip.ConfigC


@pytest.mark.cpu
@pytest.mark.parametrize("q8", [False, True])
def test_inspect_derives_the_config(ckpt, tiny_weights, tmp_path, q8):
    from vox_weights import TINY_LONG, quantize_q8, write_safetensors
    path = ckpt
    if q8:
        path = str(tmp_path / "q8.safetensors")
        write_safetensors(quantize_q8(tiny_weights), path)
    L, ConfigC = _host()
    c = ConfigC()
    assert L.vh_inspect(path.encode(), ctypes.byref(c)) == 0
    want = TINY_LONG.ctypes_struct(ConfigC)
    for name, _ in ConfigC._fields_:
        assert getattr(c, name) == pytest.approx(getattr(want, name)), name


@pytest.mark.cpu
def test_wav_reader_matches(jfk_samples):
    L, _ = _host()
    n = ctypes.c_int(0)
    p = L.vh_load_wav(os.path.join(GOLDEN, "jfk.wav").encode(), ctypes.byref(n))
    got = np.ctypeslib.as_array(p, (n.value,)).copy()
    assert np.array_equal(got, jfk_samples)


def _ref_parse_wav(pcm, rate, ch):
    """vox_parse_wav_buffer (voxtral_audio.c:49-141) in float32 numpy, the reference's
    operation order: mean of the channels' int16 values / 32768, then linear interpolation at
    src_pos = (float)i * rate / 16000 (float32 product, then the division)"""
    pcm = pcm.reshape(-1, ch)
    if ch == 1:
        x = pcm[:, 0].astype(np.float32) / np.float32(32768.0)
    else:
        s = np.zeros(pcm.shape[0], np.float32)
        for c in range(ch):
            s = (s + pcm[:, c].astype(np.float32)).astype(np.float32)
        x = (s / np.float32(ch)).astype(np.float32) / np.float32(32768.0)
    if rate == 16000:
        return x.astype(np.float32)
    n = x.shape[0]
    m = n * 16000 // rate
    i = np.arange(m)
    pos = (i.astype(np.float32) * np.float32(rate)).astype(np.float32) / np.float32(16000)
    k = pos.astype(np.int64)
    fr = (pos - k.astype(np.float32)).astype(np.float32)
    y = np.zeros(m, np.float32)
    ok = k + 1 < n
    y[ok] = x[k[ok]] * (np.float32(1.0) - fr[ok]) + x[k[ok] + 1] * fr[ok]
    last = ~ok & (k < n)
    y[last] = x[k[last]]
    return y


@pytest.mark.cpu
@pytest.mark.parametrize("rate,ch,ffmpeg", [(44100, 2, False), (8000, 1, False), (48000, 3, True)])
def test_wav_reader_resamples_like_reference(tmp_path, rate, ch, ffmpeg):
    """vh_load_wav mirrors vox_load_wav beyond 16 kHz mono (VERDICT r3 missing 3): channels
    mixed by their mean, linear resampling to 16 kHz, an extra chunk before "data", and piped
    ffmpeg's 0xFFFFFFFF data size."""
    import struct
    rng = np.random.default_rng(rate + ch)
    pcm = rng.integers(-32768, 32767, size=(rate // 3) * ch, dtype=np.int16)
    fmt = struct.pack("<HHIIHH", 1, ch, rate, rate * 2 * ch, 2 * ch, 16)
    data = pcm.tobytes()
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt
    body += b"LIST" + struct.pack("<I", 5) + b"abcde" + b"\0"          # odd chunk, padded
    body += b"data" + struct.pack("<I", 0xFFFFFFFF if ffmpeg else len(data)) + data
    path = tmp_path / "x.wav"
    path.write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)
    L, _ = _host()
    n = ctypes.c_int(0)
    p = L.vh_load_wav(str(path).encode(), ctypes.byref(n))
    assert p, "vh_load_wav failed"
    got = np.ctypeslib.as_array(p, (n.value,)).copy()
    want = _ref_parse_wav(pcm, rate, ch)
    assert got.shape == want.shape
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("interval", [None, 0.5])
def test_cli_transcribes_like_python_and_oracle(ckpt, tiny_weights, jfk_samples, interval):
    import vox_hip
    import vox_oracle
    from vox_weights import TINY_LONG
    cmd = [CLI, "-d", ckpt, "-i", os.path.join(GOLDEN, "jfk.wav")]
    if interval:
        cmd += ["-I", str(interval)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ids = [int(t) for t in r.stdout.split()]
    assert "Encoder:" in r.stderr and "Decoder:" in r.stderr and "Audio: 176000 samples" in r.stderr
    # the same schedule through the Python mirror and the CPU oracle (EOS stops both)
    piece = int(min(interval or 1.0, 1.0) * 16000)
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    hs = vox_hip.Stream(hm)
    sess = vox_hip.AudioSession(hs, interval_s=interval or 2.0)
    for i in range(0, len(jfk_samples), piece):
        sess.feed_samples(jfk_samples[i:i + piece])
    sess.finish_samples()
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    os_ = vox_oracle.OracleStream(om)
    osess = vox_oracle.OracleSession(os_, interval_s=interval or 2.0)
    for kind, mel in vox_oracle.transcribe_mel_schedule(jfk_samples, feed_size=piece):
        getattr(osess, kind)(mel)
    assert len(ids) > 0
    assert ids == sess.tokens == osess.tokens
    sess.close()
    hs.close(); hm.close(); os_.close(); om.close()


@pytest.mark.gpu
def test_cli_q8_checkpoint_in_quantize_py_layout(tmp_path, tiny_weights, jfk_samples):
    """Config 5 from a file: the TINY_LONG weights quantised and written exactly as the
    reference's quantize.py writes them (unpadded header, unaligned f32 scales and int8 rows;
    the layout is pinned byte for byte in test_q8_cpu), loaded by the C loader (vh_load:
    scales copied aligned, int8 handed over as is, voxtral_safetensors.c:457-468) and
    transcribed by the CLI on the GPU: ids equal the CPU oracle's q8 path."""
    import vox_oracle
    from vox_weights import TINY_LONG, quantize_q8, write_quantize_py_layout
    q8 = quantize_q8(tiny_weights)
    path = str(tmp_path / "consolidated.safetensors")
    write_quantize_py_layout(q8, path)
    assert (8 + int.from_bytes(open(path, "rb").read(8), "little")) % 4 != 0
    r = subprocess.run([CLI, "-d", path, "-i", os.path.join(GOLDEN, "jfk.wav"), "-I", "0.5"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ids = [int(t) for t in r.stdout.split()]
    om = vox_oracle.OracleModel(TINY_LONG, q8)
    os_ = vox_oracle.OracleStream(om)
    osess = vox_oracle.OracleSession(os_, interval_s=0.5)
    for kind, mel in vox_oracle.transcribe_mel_schedule(jfk_samples, feed_size=8000):
        getattr(osess, kind)(mel)
    assert len(ids) > 0
    assert ids == osess.tokens
    os_.close(); om.close()


def _write_wav(path, samples):
    import wave
    pcm = np.clip(np.round(samples * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(pcm.tobytes())


def _text_biased(w):
    """TINY weights whose control-range embedding rows (ids <= 1000, tied LM head) are
    scaled down: greedy decoding then emits text ids, so a live stream runs into the KV
    limit instead of the non-text streak limit."""
    import copy
    from vox_weights import EMB, bf16_to_f32, f32_to_bf16
    w2 = copy.copy(w)
    w2.t = dict(w.t)
    name = EMB + ".tok_embeddings.weight"
    e = bf16_to_f32(w.t[name]).copy()
    e[:1001] *= 0.05
    w2.t[name] = f32_to_bf16(e)
    w2._f32 = {}
    return w2


@pytest.mark.gpu
@pytest.mark.parametrize("bias", ["streak", "kv"])
def test_cli_continuous_mode_restarts_like_the_reference(tiny_weights, jfk_samples, tmp_path, bias):
    """Live mode (vox_stream_set_continuous; voxtral.c:1189-1239) on 200 s of audio (jfk
    repeated) through the C host with --continuous.  "streak": the random TINY model emits
    runs of control ids, so the decoder restarts on the 64-token non-text streak; "kv":
    control ids suppressed, so it passes 2000 KV positions.  Both are full resets (new mel
    context, conv stem, encoder KV).  The ids and the restart count equal the oracle's
    audio session run with the reference's restart rules."""
    import vox_oracle
    from vox_weights import TINY_LONG, write_safetensors
    w = tiny_weights if bias == "streak" else _text_biased(tiny_weights)
    ck = tmp_path / "consolidated.safetensors"
    write_safetensors(w, str(ck))
    audio = np.concatenate([jfk_samples] * 19)
    wav = tmp_path / "long.wav"
    _write_wav(wav, audio)
    audio = vox_oracle.read_wav(str(wav))
    r = subprocess.run([CLI, "-d", str(ck), "-i", str(wav), "--continuous"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    ids = [int(t) for t in r.stdout.split()]
    line = next(l for l in r.stderr.splitlines() if l.startswith("Restarts:"))
    restarts = int(line.split()[1])
    om = vox_oracle.OracleModel(TINY_LONG, w)
    os_ = vox_oracle.OracleStream(om)
    sess = vox_oracle.OracleAudioSession(os_, interval_s=2.0, continuous=True)
    for i in range(0, len(audio), 16000):
        sess.feed(audio[i:i + 16000])
    sess.finish()
    print(bias, "oracle restarts", sess.restarts)
    assert ids == sess.tokens
    assert restarts == len(sess.restarts) > 0
    assert any(k == (3 if bias == "streak" else 2) for k, _, _ in sess.restarts)
    sess.close(); os_.close(); om.close()


@pytest.mark.gpu
def test_cli_alternatives_like_stream_fill_alts(ckpt, tiny_weights, jfk_samples):
    """--alt 0.5 (main.c:149-154 / vox_stream_set_alt(s, 3, cutoff)): each printed record is
    the chosen id and the alternatives stream_fill_alts accepts (voxtral.c:955-1010), for
    text tokens only; checked against the reference rule applied to the oracle's logits."""
    import vox_oracle
    from vox_weights import TINY_LONG
    r = subprocess.run([CLI, "-d", ckpt, "-i", os.path.join(GOLDEN, "jfk.wav"), "--alt", "0.5"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    recs = [[int(x) for x in t.split("|")] for t in r.stdout.split()]
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    os_ = vox_oracle.OracleStream(om)
    toks, logits = [], []
    sess = vox_oracle.OracleSession(os_, interval_s=2.0)
    for kind, mel in vox_oracle.transcribe_mel_schedule(jfk_samples, feed_size=16000):
        if kind == "finish":
            sess.finished = True
        sess._enc(mel, 1 if kind == "flush" else sess.min_new)
        t, lg = os_.decode(stop_at_eos=True, want_logits=True)
        toks += t.tolist()
        logits.append(lg)
    logits = np.concatenate(logits)
    assert [rr[0] for rr in recs] == toks
    n_alt = 0
    for i, t in enumerate(toks):
        want, _ = vox_oracle.fill_alts(logits[i], t, 3, 0.5)
        want = [w for w in want[:3] if w >= 0]
        if t < 1001 or t == 2:
            want = [t]
        assert recs[i] == want, (i, recs[i], want)
        n_alt += len(want) > 1
    assert n_alt > 0
    os_.close(); om.close()
