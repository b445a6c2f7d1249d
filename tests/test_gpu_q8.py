"""Q8 checkpoints (config 5: quantize.py output) on the HIP path against the CPU oracle's
q8 path (q8 matvec for M=1, dequantise + sgemm for M>1, q8 token embeddings;
voxtral_kernels.c:277-393, voxtral.c:443-451; oracle pinned in tests/test_q8_cpu.py).

The HIP kernels compute scale * sum(x * q) (int8 exact in bf16 / f32); the reference's
M>1 path sums x * (q * scale) after rounding each dequantised weight to f32, so results
agree to f32 rounding, not bitwise.  Tolerances: greedy ids identical; adapter rows and
logits within 5e-5 of the largest magnitude (as the bf16 tests)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 5e-5


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))


@pytest.fixture(scope="module")
def q8_models(tiny_cfg, tiny_weights):
    import vox_hip
    import vox_oracle
    from vox_weights import quantize_q8
    w = quantize_q8(tiny_weights)
    hm = vox_hip.Model(tiny_cfg, w)
    om = vox_oracle.OracleModel(tiny_cfg, w)
    yield w, hm, om
    hm.close()
    om.close()


def test_q8_ada_scale_matches(q8_models):
    """ada_scale is host math on both sides (voxtral.c:47-80) over dequantised f32 weights
    with full 24-bit mantissas: gcc -ffast-math (oracle) and hipcc round a few sums
    differently, so 1 ulp of the largest value is allowed."""
    _, hm, om = q8_models
    assert rel(hm.ada_scale(), om.ada_scale()) < 1e-6


def test_q8_sgemm_twin(q8_models):
    """vox_hip_sgemm_q8 (GEMV for M=1, MFMA GEMM for M>1) against the oracle's q8 linear."""
    import vox_hip
    import vox_oracle
    w, _, _ = q8_models
    sc, q = w.q8["layers.0.feed_forward.w2.weight"]
    rng = np.random.default_rng(9)
    for M in (1, 3, 70):
        A = rng.standard_normal((M, q.shape[1])).astype(np.float32)
        got = vox_hip.sgemm_q8(A, q, sc)
        ref = vox_oracle.linear_q8(A, q, sc)
        assert rel(got, ref) < 1e-5, (M, rel(got, ref))


def test_q8_encode_and_decode_match(q8_models, tiny_cfg, jfk_samples):
    """jfk.wav one-shot schedule (1355 / 140 / 1 mel frames) on the Q8 TINY model."""
    import vox_hip
    import vox_oracle
    _, hm, om = q8_models
    events = vox_oracle.transcribe_mel_schedule(jfk_samples)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    ht, ot, hl, ol = [], [], [], []
    done = 0
    for kind, mel in events:
        for s, toks, logs in ((hs, ht, hl), (os_, ot, ol)):
            s.encode_mel(mel[done:])
            t, lg = s.decode(stop_at_eos=False, want_logits=True)
            toks += t.tolist()
            logs.append(lg)
        done = mel.shape[0]
    ra = rel(hs.read_adapter(), os_.read_adapter())
    assert ra < TOL, ra
    rl = rel(np.concatenate(hl), np.concatenate(ol))
    assert rl < TOL, rl
    assert len(ot) > 100 and ht == ot
    hs.close()
    os_.close()


@pytest.mark.slow
def test_q8_full_jfk_transcription(jfk_samples):
    """Full Voxtral-4B shapes, Q8 weights (4.43 GB int8 + scales) quantised from the seeded
    synthetic bf16 checkpoint."""
    import vox_hip
    import vox_oracle
    from vox_weights import VOXTRAL_4B, quantize_q8, synth_weights
    w = quantize_q8(synth_weights(VOXTRAL_4B, seed=0))
    hm = vox_hip.Model(VOXTRAL_4B, w)
    om = vox_oracle.OracleModel(VOXTRAL_4B, w)
    vox_oracle.set_threads(min(16, os.cpu_count() or 1))
    events = vox_oracle.transcribe_mel_schedule(jfk_samples)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    ht, ot, hl, ol = [], [], [], []
    done = 0
    for kind, mel in events:
        for s, toks, logs in ((hs, ht, hl), (os_, ot, ol)):
            s.encode_mel(mel[done:])
            t, lg = s.decode(stop_at_eos=False, want_logits=True)
            toks += t.tolist()
            logs.append(lg)
        done = mel.shape[0]
    assert hs.adapter_tokens == os_.adapter_tokens == 187
    ra = rel(hs.read_adapter(), os_.read_adapter())
    rl = rel(np.concatenate(hl), np.concatenate(ol))
    print(f"q8 adapter rel err {ra:.2e}, logits rel err {rl:.2e}")
    assert ra < TOL and rl < TOL, (ra, rl)
    assert len(ot) == 149 and ht == ot
    hs.close()
    os_.close()
    hm.close()
    om.close()


def test_q8_streaming_skinny_encoder_and_batch(q8_models, tiny_cfg, jfk_samples):
    """Q8 through the short-chunk paths: raw samples at -I 0.5 (device mel, 25-row encoder
    chunks on the skinny int8 GEMMs) against the oracle's q8 path, then the same streams
    decoded as one batch (int8 fragment-major weights) against single-stream decoding."""
    import vox_hip
    import vox_oracle
    _, hm, om = q8_models
    hs = vox_hip.Stream(hm)
    sess = vox_hip.AudioSession(hs, interval_s=0.5)
    for i in range(0, len(jfk_samples), 8000):
        sess.feed_samples(jfk_samples[i:i + 8000], stop_at_eos=False)
    sess.finish_samples(stop_at_eos=False)
    os_ = vox_oracle.OracleStream(om)
    osess = vox_oracle.OracleSession(os_, interval_s=0.5)
    for kind, mel in vox_oracle.transcribe_mel_schedule(jfk_samples, feed_size=8000):
        getattr(osess, kind)(mel, stop_at_eos=False)
    ha, oa = hs.read_adapter(), os_.read_adapter()
    assert ha.shape == oa.shape and rel(ha, oa) < TOL, rel(ha, oa)
    assert sess.tokens == osess.tokens and len(sess.tokens) > 100
    sess.close(); hs.close(); os_.close()
    # batch: 3 streams at different lengths, decoded together, vs each alone
    rng = np.random.default_rng(21)
    mels = [rng.uniform(-0.6, 1.4, size=(n, tiny_cfg.mel_bins)).astype(np.float32) for n in (420, 500, 460)]
    ss = [vox_hip.Stream(hm) for _ in mels]
    for s, mel in zip(ss, mels):
        s.encode_mel(mel)
    b = vox_hip.Batch(hm, 4)
    got = b.decode(ss, max_steps=1000, stop_at_eos=False)
    for i, mel in enumerate(mels):
        one = vox_hip.Stream(hm)
        one.encode_mel(mel)
        assert got[i].tolist() == one.decode(stop_at_eos=False).tolist(), i
        one.close()
    for s in ss:
        s.close()
    b.close()
