"""End-to-end parity of the HIP path against the CPU oracle on the TINY configuration
(same structure and head dims as Voxtral-4B, short windows so the rolling KV wraps).

Tolerances: greedy ids must be identical; logits within 5e-5 relative to the largest
logit magnitude (f32 arithmetic with a different summation order; the MFMA GEMMs use the
exact 3-term bf16 split of the activations)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOGIT_TOL = 5e-5
ADAPTER_TOL = 5e-5


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))


@pytest.fixture(scope="module")
def models(tiny_cfg, tiny_weights):
    import vox_hip
    import vox_oracle
    hm = vox_hip.Model(tiny_cfg, tiny_weights)
    om = vox_oracle.OracleModel(tiny_cfg, tiny_weights)
    yield hm, om
    hm.close()
    om.close()


def test_ada_scale_matches(models):
    hm, om = models
    np.testing.assert_array_equal(hm.ada_scale(), om.ada_scale())


def test_encode_chunks_match(models, tiny_cfg):
    import vox_hip
    import vox_oracle
    hm, om = models
    rng = np.random.default_rng(3)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    # ragged chunk sizes incl. 1-frame and odd chunks (conv stride residual paths)
    for n in [313, 1, 2, 7, 50, 1, 1, 200, 3]:
        mel = rng.uniform(-0.6, 1.4, size=(n, tiny_cfg.mel_bins)).astype(np.float32)
        a = hs.encode_mel(mel)
        b = os_.encode_mel(mel)
        assert a == b, (n, a, b)
    ha, oa = hs.read_adapter(), os_.read_adapter()
    assert ha.shape == oa.shape
    assert rel(ha, oa) < ADAPTER_TOL, rel(ha, oa)
    hs.close()
    os_.close()


def test_async_encode_interleaved_streams(models, tiny_cfg):
    """vox_hip_stream_set_async_encode as the scheduler uses it: three streams' ragged chunks
    enqueued round-robin without a sync in between (several passes in flight on their own
    queues), then each stream decoded; adapter rows and ids equal the oracle's per stream."""
    import vox_hip
    import vox_oracle
    hm, om = models
    rng = np.random.default_rng(11)
    sizes = [[313, 50, 7, 1, 200], [300, 120, 33], [400, 2, 2, 90]]  # each past the 39-row prompt
    hs = [vox_hip.Stream(hm) for _ in sizes]
    os_ = [vox_oracle.OracleStream(om) for _ in sizes]
    mels = [[rng.uniform(-0.6, 1.4, size=(n, tiny_cfg.mel_bins)).astype(np.float32) for n in sz] for sz in sizes]
    for h in hs:
        h.set_async_encode(True)
    counts = [[], [], []]
    for k in range(max(len(sz) for sz in sizes)):
        for i in range(len(hs)):
            if k < len(mels[i]):
                counts[i].append(hs[i].encode_mel(mels[i][k]))
    for i in range(len(hs)):
        oc = [os_[i].encode_mel(m) for m in mels[i]]
        assert counts[i] == oc, (i, counts[i], oc)
        hs[i].sync()
        ra = rel(hs[i].read_adapter(), os_[i].read_adapter())
        assert ra < ADAPTER_TOL, (i, ra)
        ht, hl = hs[i].decode(max_steps=12, stop_at_eos=False, want_logits=True)
        ot, ol = os_[i].decode(max_steps=12, stop_at_eos=False, want_logits=True)
        assert len(ot) > 0 and np.array_equal(ht, ot), (i, len(ot))
        assert rel(hl, ol) < LOGIT_TOL, (i, rel(hl, ol))
        hs[i].set_async_encode(False)
        hs[i].close()
        os_[i].close()


def test_encode_mel_batch_matches_oracle(models, tiny_cfg):
    """vox_hip_stream_encode_mel_batch: three streams' ragged chunks (1-frame and odd chunks
    included, one stream idle in some rounds) through shared encoder passes; every stream's
    adapter-row counts and rows, then its greedy ids and logits, equal its own oracle session."""
    import vox_hip
    import vox_oracle
    hm, om = models
    rng = np.random.default_rng(17)
    rounds = [[313, 300, 400], [50, 0, 2], [7, 120, 2], [1, 33, 90], [200, 1, 0]]
    hs = [vox_hip.Stream(hm) for _ in range(3)]
    os_ = [vox_oracle.OracleStream(om) for _ in range(3)]
    for r in rounds:
        mels = [rng.uniform(-0.6, 1.4, size=(n, tiny_cfg.mel_bins)).astype(np.float32) for n in r]
        got = vox_hip.encode_mel_batch(hs, mels)
        want = [os_[i].encode_mel(mels[i]) if r[i] else 0 for i in range(3)]
        assert got == want, (r, got, want)
    for i in range(3):
        assert hs[i].adapter_tokens == os_[i].adapter_tokens
        ra = rel(hs[i].read_adapter(), os_[i].read_adapter())
        assert ra < ADAPTER_TOL, (i, ra)
        ht, hl = hs[i].decode(max_steps=12, stop_at_eos=False, want_logits=True)
        ot, ol = os_[i].decode(max_steps=12, stop_at_eos=False, want_logits=True)
        assert len(ot) > 0 and np.array_equal(ht, ot), (i, len(ot))
        assert rel(hl, ol) < LOGIT_TOL, (i, rel(hl, ol))
        hs[i].close()
        os_[i].close()


def test_encode_mel_batch_rejects_duplicate_stream(models, tiny_cfg):
    """a stream listed twice in one batched encoder pass would append its K/V
    twice at the same positions; the call refuses it and leaves the stream untouched."""
    import vox_hip
    hm, _ = models
    s = vox_hip.Stream(hm)
    mel = np.zeros((40, tiny_cfg.mel_bins), np.float32)
    with pytest.raises(RuntimeError, match="twice"):
        vox_hip.encode_mel_batch([s, s], [mel, mel])
    assert s.adapter_tokens == 0
    s.close()


def test_window_256_decodes_past_256(tiny_weights, jfk_samples):
    """with a decoder window of exactly 256 the short-context attention kernel (keys
    = ring slots 0..lp, valid only while nothing has left the window) must not serve contexts
    at or past 256 positions; decoding ~400 positions on TINY with dec_window = 256 gives the
    oracle's ids."""
    import dataclasses
    import vox_hip
    import vox_oracle
    from vox_weights import TINY
    cfg = dataclasses.replace(TINY, dec_window=256)
    samples = np.concatenate([jfk_samples] * 3)
    events = vox_oracle.transcribe_mel_schedule(samples)
    hm = vox_hip.Model(cfg, tiny_weights)
    om = vox_oracle.OracleModel(cfg, tiny_weights)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    hsess, osess = vox_hip.Session(hs), vox_oracle.OracleSession(os_)
    for kind, mel in events:
        getattr(hsess, kind)(mel, stop_at_eos=False)
        getattr(osess, kind)(mel, stop_at_eos=False)
    assert len(osess.tokens) > 300
    assert hsess.tokens == osess.tokens
    hs.close(); os_.close(); hm.close(); om.close()


def test_jfk_transcribe_tokens_match(models, jfk_samples):
    """vox_transcribe_audio schedule on jfk.wav (1355 / 140 / 1 mel-frame chunks)."""
    import vox_hip
    import vox_oracle
    hm, om = models
    events = vox_oracle.transcribe_mel_schedule(jfk_samples)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    hsess, osess = vox_hip.Session(hs), vox_oracle.OracleSession(os_)
    for kind, mel in events:
        getattr(hsess, kind)(mel, stop_at_eos=False)
        getattr(osess, kind)(mel, stop_at_eos=False)
    assert hsess.chunks == osess.chunks == [1355, 140, 1]
    assert len(osess.tokens) == 149
    assert hsess.tokens == osess.tokens
    hs.close()
    os_.close()


def test_streaming_interval_and_logits(models, jfk_samples):
    """`-I 0.5` style feeding (1 s feeds, 50-frame encoder chunks), logits per step."""
    import vox_hip
    import vox_oracle
    hm, om = models
    events = vox_oracle.transcribe_mel_schedule(jfk_samples[:80000], feed_size=16000)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    hsess, osess = vox_hip.Session(hs, 0.5), vox_oracle.OracleSession(os_, 0.5)
    hl, ol = [], []
    for kind, mel in events:
        hsess._run_encoder(mel, 1 if kind == "flush" else hsess.min_new_mel) if kind != "finish" else None
        if kind == "finish":
            hsess.finished = True
            hsess._run_encoder(mel, hsess.min_new_mel)
        t, l = hs.decode(stop_at_eos=False, want_logits=True)
        hl.append(l)
        hsess.tokens += t.tolist()
        getattr(osess, "_enc")(mel, 1 if kind == "flush" else osess.min_new) if kind != "finish" else None
        if kind == "finish":
            osess.finished = True
            osess._enc(mel, osess.min_new)
        t, l = os_.decode(stop_at_eos=False, want_logits=True)
        ol.append(l)
        osess.tokens += t.tolist()
    assert hsess.chunks == osess.chunks
    assert hsess.tokens == osess.tokens
    hl, ol = np.concatenate(hl), np.concatenate(ol)
    assert hl.shape == ol.shape and hl.shape[0] > 0
    assert rel(hl, ol) < LOGIT_TOL, rel(hl, ol)
    hs.close()
    os_.close()


def test_long_stream_multiblock_attention(tiny_weights):
    """~33 s of audio (jfk x3) on TINY_LONG: 560 decoder positions, so the decode
    attention runs on up to 3 key blocks (> 256 keys) and merges them."""
    import vox_hip
    import vox_oracle
    from vox_weights import TINY_LONG
    samples = np.concatenate([vox_oracle.read_wav(__import__("conftest").GOLDEN + "/jfk.wav")] * 3)
    events = vox_oracle.transcribe_mel_schedule(samples)
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    hsess, osess = vox_hip.Session(hs), vox_oracle.OracleSession(os_)
    for kind, mel in events:
        getattr(hsess, kind)(mel, stop_at_eos=False)
        getattr(osess, kind)(mel, stop_at_eos=False)
    assert len(osess.tokens) > 400
    assert hsess.tokens == osess.tokens
    # logits of a late step (window > 256 keys)
    assert hs.state()["kv_pos"] == os_.state()["dec_len"]
    hs.close(); os_.close(); hm.close(); om.close()


def test_alternatives_match_stream_fill_alts(models, jfk_samples):
    """--alt (voxtral.c:955-1010): candidates kept on the device per step agree with the
    reference's softmax + repeated scan applied to the oracle's logits (ids exact, probs
    within what the logit bar allows), for several n_alt / cutoff settings."""
    import vox_hip
    import vox_oracle
    hm, om = models
    events = vox_oracle.transcribe_mel_schedule(jfk_samples)
    for n_alt, cutoff in ((3, 1.0), (4, 0.5), (2, 0.0), (1, 1.0)):
        hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
        hs.set_alt(n_alt, cutoff)
        ht, ol = [], []
        done = 0
        for kind, mel in events:
            hs.encode_mel(mel[done:])
            os_.encode_mel(mel[done:])
            done = mel.shape[0]
            ht += hs.decode(stop_at_eos=False).tolist()
            t, lg = os_.decode(stop_at_eos=False, want_logits=True)
            ol.append(lg)
        ol = np.concatenate(ol)
        ids, pr = hs.read_alts(0, len(ht))
        n_with_alts = 0
        for i, tok in enumerate(ht):
            rid, rpr = vox_oracle.fill_alts(ol[i], tok, n_alt, cutoff)
            assert ids[i].tolist() == rid, (i, ids[i], rid)
            # a logit error e moves p by a factor exp(e) (numerator) and the normaliser alike:
            # the logit bar (LOGIT_TOL of the largest logit) bounds the probability's relative error
            np.testing.assert_allclose(pr[i], rpr, rtol=2 * LOGIT_TOL * float(np.max(np.abs(ol[i]))), atol=1e-9)
            n_with_alts += ids[i][1] >= 0
        if n_alt > 1 and cutoff >= 0.5:
            assert n_with_alts > 0
        hs.close()
        os_.close()
