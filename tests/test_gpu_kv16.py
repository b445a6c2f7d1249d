"""The reference's fp16 decoder KV cache (VOX_DECODER_KV_FP16, voxtral.c:189-190; the Metal
path's dual-format cache, voxtral_decoder.c:180-243, measured in SPEED.md:24-38) as the
opt-in 16-bit mode of the HIP decoder rings (vox_hip_model_set_kv_fp16).

Oracle: the CPU restatement with every decoder K/V append rounded to IEEE half
(vox_oracle.set_kv_fp16, the f32 -> half -> f32 of oracle/vox_oracle.c f16_round, checked
bit-exact against numpy in tests/test_oracle_kv16.py).  The GPU rounds its own f32 K/V,
which differ from the oracle's in summation order (~1e-7), so an element close to a
rounding boundary can land one half-ulp (2^-11 relative) away: the logit bar of this mode
is LOGIT_TOL16 = 1e-4 of the largest logit magnitude (twice the f32 ring's 5e-5; measured
1.5e-5 on 120 TINY_LONG steps), and greedy ids must be identical.  TINY_LONG: Voxtral's head dims (the 16-bit mode is head_dim 128
only) and the real 8192-key window."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOGIT_TOL16 = 1e-4
CHUNK = 4096


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))


def _mel(seed, n):
    rng = np.random.default_rng(seed)
    return rng.uniform(-0.6, 1.4, size=(n, 128)).astype(np.float32)


def _encode(s, mel):
    for i in range(0, mel.shape[0], CHUNK):
        s.encode_mel(mel[i:i + CHUNK])


@pytest.fixture(scope="module")
def kv(tiny_weights):
    import os

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


def _oracle(om, mel, n, kv16, logits_from=0):
    import vox_oracle
    vox_oracle.set_kv_fp16(kv16)
    try:
        st = vox_oracle.OracleStream(om)
        _encode(st, mel)
        a = st.decode(max_steps=logits_from, stop_at_eos=False) if logits_from else np.zeros(0, np.int32)
        b, lg = st.decode(max_steps=n - logits_from, stop_at_eos=False, want_logits=True)
        st.close()
    finally:
        vox_oracle.set_kv_fp16(False)
    return np.concatenate([a, b]).tolist(), lg


def _gpu(hm, mel, n, kv16, logits_from=0):
    import vox_hip
    hm.set_kv_fp16(kv16)
    s = vox_hip.Stream(hm)
    hm.set_kv_fp16(False)
    assert s.kv_fp16 == kv16
    _encode(s, mel)
    a = s.decode(max_steps=logits_from, stop_at_eos=False) if logits_from else np.zeros(0, np.int32)
    b, lg = s.decode(max_steps=n - logits_from, stop_at_eos=False, want_logits=True)
    st = s.state()
    s.close()
    return np.concatenate([a, b]).tolist(), lg, st


def test_kv16_stream_decode_vs_oracle(kv):
    """prefill + 120 greedy steps with the 16-bit ring: ids equal to the rounded-KV oracle,
    logits within LOGIT_TOL16 and closer to it than to the f32 oracle (the rounding is
    applied), and the ring memory halves."""
    import vox_hip
    hm, om = kv
    mel = _mel(11, 8 * 170)
    ids, lg, _ = _gpu(hm, mel, 120, True)
    ref, rlg = _oracle(om, mel, 120, True)
    assert ids == ref
    r = rel(lg, rlg)
    _, flg = _oracle(om, mel, 120, False)
    r32 = rel(lg, flg)
    print(f"kv16 single stream: logits rel err {r:.2e} vs the rounded-KV oracle, {r32:.2e} vs the f32 one")
    assert r < LOGIT_TOL16, r
    assert r32 > r
    # ring bytes: the 16-bit stream allocates half the decoder K/V of the f32 one
    L = vox_hip.lib()
    m0 = L.vox_hip_memory_used()
    s32 = vox_hip.Stream(hm)
    m1 = L.vox_hip_memory_used()
    hm.set_kv_fp16(True)
    s16 = vox_hip.Stream(hm)
    hm.set_kv_fp16(False)
    m2 = L.vox_hip_memory_used()
    c = hm.cfg
    ring32 = 2 * c.dec_layers * (c.dec_window + 64) * c.dec_kv_heads * c.dec_head_dim * 4
    assert (m1 - m0) - (m2 - m1) == ring32 // 2, (m1 - m0, m2 - m1, ring32)
    s32.close()
    s16.close()


def test_kv16_through_ring_wrap_vs_oracle(kv):
    """8330 greedy steps (graph replays, every attention split bucket, the ring wrap at
    8256) with the 16-bit ring: ids equal to the rounded-KV oracle on every step, logits of
    the last 230 steps within LOGIT_TOL16."""
    hm, om = kv
    n, plain = 8330, 8100
    mel = _mel(81, 8 * 8400)
    ref = {}

    def run():
        ref["ids"], ref["lg"] = _oracle(om, mel, n, True, logits_from=plain)
    th = threading.Thread(target=run)
    th.start()
    ids, lg, st = _gpu(hm, mel, n, True, logits_from=plain)
    th.join()
    assert st["kv_pos"] > 8256 + 64, st
    first_diff = next((i for i in range(n) if ids[i] != ref["ids"][i]), None)
    assert first_diff is None, (first_diff, ids[first_diff], ref["ids"][first_diff])
    r = rel(lg, ref["lg"])
    print(f"kv16 ring: {n} ids equal, logits rel err {r:.2e}")
    assert r < LOGIT_TOL16, r


def test_kv16_batch_vs_single(kv):
    """batched decode (fused RoPE / KV append attention over half rings) of 3 streams at
    different positions: ids equal to each stream's single-stream 16-bit decode, logits
    within LOGIT_TOL16 (the two paths sum K/V in different orders before rounding), and a
    batch mixing element types is refused."""
    import vox_hip
    hm, om = kv
    mels = [_mel(91 + k, 8 * (300 + 40 * k)) for k in range(3)]
    hm.set_kv_fp16(True)
    ss = [vox_hip.Stream(hm) for _ in mels]
    hm.set_kv_fp16(False)
    for s, mel in zip(ss, mels):
        _encode(s, mel)
    out = [[] for _ in ss]
    out[1] += ss[1].decode(max_steps=23, stop_at_eos=False).tolist()
    b = vox_hip.Batch(hm, 4)
    for k, t in enumerate(b.decode(ss, max_steps=150, stop_at_eos=False)):
        out[k] += t.tolist()
    lgs = [[] for _ in ss]
    for _ in range(20):
        for k, t in enumerate(b.decode(ss, max_steps=1, stop_at_eos=False)):
            out[k] += t.tolist()
            lgs[k].append(b.read_logits(ss[k]))
    for k, mel in enumerate(mels):
        n = len(out[k])
        ids, lg, _ = _gpu(hm, mel, n, True, logits_from=n - 20)
        assert out[k] == ids, k
        r = rel(np.stack(lgs[k]), lg)
        print(f"kv16 batch stream {k}: {n} ids equal, logits rel err {r:.2e}")
        assert r < LOGIT_TOL16, (k, r)
    s32 = vox_hip.Stream(hm)
    s32.encode_mel(mels[0][:800])
    with pytest.raises(RuntimeError):
        b.decode([ss[0], s32], max_steps=1, stop_at_eos=False)
    s32.close()
    for s in ss:
        s.close()
    b.close()
