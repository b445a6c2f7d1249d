"""Single-stream decode across the short-context attention's range and out of it:
voxtral_decoder.c:709-733 (QKV, RoPE, KV append, attention over the last min(pos + 1,
window) keys).  Contexts up to 256 keys run k_attn_short (one 1024-thread block per query
head, keys 64.. loaded after the position read), longer ones the split attention with the
merging block.

TINY_LONG keeps Voxtral's head_dim 128 and the 8192-key window, so a stream's greedy steps
go from the prompt across 64 / 128 / 192 / 256 keys into the split path, with the f32 and
the 16-bit ring.  Oracle: the CPU restatement; every id equal, logits of every step within
5e-5 of the largest magnitude (1e-4 with the 16-bit ring, tests/test_gpu_kv16.py).  (Round
6 also ran this test on the attention folded into the QKV launch)"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOGIT_TOL = 5e-5
LOGIT_TOL16 = 1e-4
CHUNK = 4096


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))


def _mel(seed, n):
    rng = np.random.default_rng(seed)
    return rng.uniform(-0.6, 1.4, size=(n, 128)).astype(np.float32)


@pytest.fixture(scope="module")
def models(tiny_weights):
    import vox_hip
    import vox_oracle
    from vox_weights import TINY_LONG
    vox_oracle.set_threads(min(16, os.cpu_count() or 1))
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    yield hm, om
    vox_oracle.set_kv_fp16(False)
    hm.close()
    om.close()


@pytest.mark.parametrize("kv16", [False, True])
def test_short_attention_into_split_vs_oracle(models, kv16):
    """prefill + 300 greedy steps (contexts from the prompt to past 256 keys): ids equal to
    the oracle's on every step, logits of every step within the bar."""
    import vox_hip
    import vox_oracle
    hm, om = models
    n = 300
    mel = _mel(23 if kv16 else 17, 8 * 400)
    hm.set_kv_fp16(kv16)
    s = vox_hip.Stream(hm)
    hm.set_kv_fp16(False)
    for i in range(0, mel.shape[0], CHUNK):
        s.encode_mel(mel[i:i + CHUNK])
    ids, lg = s.decode(max_steps=n, stop_at_eos=False, want_logits=True)
    st = s.state()
    s.close()
    vox_oracle.set_kv_fp16(kv16)
    try:
        o = vox_oracle.OracleStream(om)
        for i in range(0, mel.shape[0], CHUNK):
            o.encode_mel(mel[i:i + CHUNK])
        ref, rlg = o.decode(max_steps=n, stop_at_eos=False, want_logits=True)
        o.close()
    finally:
        vox_oracle.set_kv_fp16(False)
    assert st["kv_pos"] > 256, st
    ids, ref = list(ids), list(ref)
    first = next((i for i in range(n) if ids[i] != ref[i]), None)
    assert first is None, (first, ids[first], ref[first])
    r = rel(np.asarray(lg), np.asarray(rlg))
    print(f"short + split attention ({'16-bit' if kv16 else 'f32'} ring): {n} ids equal, logits rel err {r:.2e}, "
          f"kv_pos {st['kv_pos']}")
    assert r < (LOGIT_TOL16 if kv16 else LOGIT_TOL), r
