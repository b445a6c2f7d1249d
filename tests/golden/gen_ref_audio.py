"""Generate tests/golden/ref_mel.npz from the reference's own voxtral_audio.c.

The reference's mel front-end needs only libm, so `make -C oracle ref` compiles
/root/reference/voxtral_audio.c in place into oracle/_ref/librefaudio.so (nothing is
copied).  This script drives its incremental API (vox_mel_ctx_init / vox_mel_feed /
vox_mel_finish, voxtral_audio.h:42-71) exactly as vox_transcribe_audio does
(voxtral.c:1255, 1288-1316, 1640-1667) on samples/jfk.wav (kept as tests/golden/jfk.wav)
and on a short synthetic chirp fed in ragged pieces, and stores the frames.

Run here (needs /root/reference):  python3 tests/golden/gen_ref_audio.py
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import vox_oracle  # noqa: E402  (read_wav only)

LIB = os.path.join(ROOT, "oracle", "_ref", "librefaudio.so")


def ref_lib():
    L = ctypes.CDLL(LIB)
    L.vox_mel_ctx_init.restype = ctypes.c_void_p
    L.vox_mel_ctx_init.argtypes = [ctypes.c_int]
    L.vox_mel_feed.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    L.vox_mel_finish.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.vox_mel_data.restype = ctypes.POINTER(ctypes.c_float)
    L.vox_mel_data.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    L.vox_mel_free.argtypes = [ctypes.c_void_p]
    return L


def run(L, samples, pieces, delay_tokens=6):
    """Returns the mel frames after feed / flush / finish (cumulative, as the stream sees them)."""
    ctx = L.vox_mel_ctx_init(32 * 1280)
    out = {}

    def data():
        n = ctypes.c_int(0)
        p = L.vox_mel_data(ctx, ctypes.byref(n))
        return np.ctypeslib.as_array(p, (n.value * 128,)).reshape(n.value, 128).copy()

    pos = 0
    for k in pieces:
        seg = np.ascontiguousarray(samples[pos:pos + k], np.float32)
        L.vox_mel_feed(ctx, seg.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(seg))
        pos += k
    out["feed"] = data()
    n = len(samples)
    pad = (1280 - n % 1280) % 1280 + ((delay_tokens + 1) + 10) * 1280
    zeros = np.zeros(4096, np.float32)
    rem = pad
    while rem > 0:
        c = min(4096, rem)
        L.vox_mel_feed(ctx, zeros.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), c)
        rem -= c
    out["flush"] = data()
    L.vox_mel_finish(ctx, 0)
    out["finish"] = data()
    L.vox_mel_free(ctx)
    return out


def main():
    L = ref_lib()
    jfk = vox_oracle.read_wav(os.path.join(HERE, "jfk.wav"))
    a = run(L, jfk, [len(jfk)])
    t = np.arange(24000, dtype=np.float64) / 16000.0
    chirp = (0.3 * np.sin(2 * np.pi * (200 + 900 * t) * t)).astype(np.float32)
    b = run(L, chirp, [1000, 1, 4095, 333, 16000, 2571])
    # frames are never recomputed, so feed/flush outputs are prefixes of the finish output
    for r in (a, b):
        assert np.array_equal(r["finish"][:len(r["flush"])], r["flush"][:len(r["finish"])])
        assert np.array_equal(r["flush"][:len(r["feed"])], r["feed"])
    np.savez_compressed(os.path.join(HERE, "ref_mel.npz"),
                        jfk_finish=a["finish"], jfk_counts=np.array([len(a[k]) for k in ("feed", "flush", "finish")]),
                        chirp=chirp, chirp_pieces=np.array([1000, 1, 4095, 333, 16000, 2571]),
                        chirp_finish=b["finish"],
                        chirp_counts=np.array([len(b[k]) for k in ("feed", "flush", "finish")]))
    print({k: v.shape for k, v in a.items()}, {k: v.shape for k, v in b.items()})


if __name__ == "__main__":
    main()
