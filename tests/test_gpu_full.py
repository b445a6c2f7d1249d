"""Full Voxtral-4B shapes (seeded synthetic weights, 8.86 GB): the HIP path against the
CPU oracle on the reference's jfk.wav one-shot transcription (vox_transcribe_audio):
1355/140/1 mel-frame encoder chunks, 38-row prefill, 149 greedy tokens.

Tolerances (north_star: "identical greedy token ids and logits within a stated fp
tolerance"): token ids identical; adapter rows and logits within 5e-5 of the largest
magnitude (f32 arithmetic, different summation order)."""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

TOL = 5e-5


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))


@pytest.fixture(scope="module")
def full():
    import vox_hip
    import vox_oracle
    from vox_weights import VOXTRAL_4B, synth_weights
    w = synth_weights(VOXTRAL_4B, seed=0)
    hm = vox_hip.Model(VOXTRAL_4B, w)
    om = vox_oracle.OracleModel(VOXTRAL_4B, w)
    vox_oracle.set_threads(min(16, os.cpu_count() or 1))
    yield VOXTRAL_4B, hm, om
    hm.close()
    om.close()


def test_full_jfk_transcription(full, jfk_samples):
    import vox_hip
    import vox_oracle
    cfg, hm, om = full
    events = vox_oracle.transcribe_mel_schedule(jfk_samples)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    h_tok, o_tok, h_log, o_log = [], [], [], []
    for kind, mel in events:
        prev = 0 if not h_tok else None
        for s, toks, logs in ((hs, h_tok, h_log), (os_, o_tok, o_log)):
            cur = {"feed": 0, "flush": events[0][1].shape[0], "finish": events[1][1].shape[0]}[kind]
            s.encode_mel(mel[cur:])
            t, l = s.decode(stop_at_eos=False, want_logits=True)
            toks += t.tolist()
            logs.append(l[:, :].copy())
    assert hs.adapter_tokens == os_.adapter_tokens == 187
    ra = rel(hs.read_adapter(), os_.read_adapter())
    assert ra < TOL, ra
    assert len(o_tok) == 149
    h_log, o_log = np.concatenate(h_log), np.concatenate(o_log)
    rl = rel(h_log, o_log)
    print(f"adapter rel err {ra:.2e}, logits rel err {rl:.2e}")
    assert rl < TOL, rl
    assert h_tok == o_tok
    hs.close()
    os_.close()


def test_full_gemmf_recompute_backstop_bit_identical(full):
    """k_gemmf's stream-K hand-off (csrc/vox_hip_gemmf.hip): when a tile's owner does not see
    a later part published in time it computes that stage range itself.  Forcing that path
    for every partial (vox_hip_set_gemmf_wait(-1)) must give the same bits as the normal
    hand-off: the jfk first chunk (M = 677 encoder rows, every projection on k_gemmf) encoded
    both ways, adapter rows compared exactly, and the device counter records the recomputes
    (zero on the normal path, > 0 when forced)."""
    import vox_hip
    cfg, hm, om = full
    rng = np.random.default_rng(17)
    mel = rng.uniform(-0.6, 1.4, size=(1355, cfg.mel_bins)).astype(np.float32)
    out, rec = [], []
    for ticks in (5000, -1):
        old = vox_hip.set_gemmf_wait(ticks)
        st = vox_hip.Stream(hm)
        try:
            n = st.encode_mel(mel)
            out.append(st.read_adapter(0, n))
            rec.append(st.profile()["gemmf_recomputes"])
        finally:
            vox_hip.set_gemmf_wait(old)
            st.close()
    assert out[0].shape[0] > 100
    np.testing.assert_array_equal(out[0], out[1])
    assert rec[1] > 0, rec
    print(f"gemmf recomputes normal / forced: {rec}")


def test_full_night1968_5s_transcription(full):
    """C2's shortest benchmark clip, the reference's samples/benchmark/night1968/
    5s_dont_worry_about_him.wav (a recording, not synthetic audio; kept as a fixture like
    jfk.wav): one-shot schedule, every greedy step's id and logits against the oracle."""
    import vox_hip
    import vox_oracle
    cfg, hm, om = full
    samples = vox_oracle.read_wav(os.path.join(os.path.dirname(__file__), "golden", "night1968_5s.wav"))
    assert abs(len(samples) / 16000.0 - 5.0) < 0.01
    events = vox_oracle.transcribe_mel_schedule(samples)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    h_tok, o_tok, h_log, o_log = [], [], [], []
    for kind, mel in events:
        cur = {"feed": 0, "flush": events[0][1].shape[0], "finish": events[1][1].shape[0]}[kind]
        for s, toks, logs in ((hs, h_tok, h_log), (os_, o_tok, o_log)):
            s.encode_mel(mel[cur:])
            t, lg = s.decode(stop_at_eos=False, want_logits=True)
            toks += t.tolist()
            logs.append(lg.copy())
    assert hs.adapter_tokens == os_.adapter_tokens
    ra = rel(hs.read_adapter(), os_.read_adapter())
    rl = rel(np.concatenate(h_log), np.concatenate(o_log))
    print(f"night1968 5 s: {hs.adapter_tokens} adapter rows rel err {ra:.2e}, {len(o_tok)} ids, logits rel err {rl:.2e}")
    assert ra < TOL, ra
    assert len(o_tok) > 50
    assert h_tok == o_tok
    assert rl < TOL, rl
    hs.close()
    os_.close()


def test_full_encode_mel_batch_streaming_chunks(full):
    """The batched encoder pass at full size on the shape the scheduler feeds it: 6 streams,
    a first chunk each, then -I 0.5-sized chunks (50 mel frames -> 25 encoder rows per
    stream, 150 stacked rows per pass: the stream-K MFMA projections), one stream skipping a
    round; adapter-row counts per stream exact, rows within TOL of each stream's oracle."""
    import vox_hip
    import vox_oracle
    cfg, hm, om = full
    rng = np.random.default_rng(23)
    rounds = [[300, 260, 330, 300, 290, 310]] + [[50, 50, 50, 0 if k == 1 else 50, 50, 51] for k in range(4)]
    hs = [vox_hip.Stream(hm) for _ in range(6)]
    os_ = [vox_oracle.OracleStream(om) for _ in range(6)]
    for r in rounds:
        mels = [rng.uniform(-0.6, 1.4, size=(n, cfg.mel_bins)).astype(np.float32) for n in r]
        got = vox_hip.encode_mel_batch(hs, mels)
        want = [os_[i].encode_mel(mels[i]) if r[i] else 0 for i in range(6)]
        assert got == want, (r, got, want)
    worst = 0.0
    for i in range(6):
        ra = rel(hs[i].read_adapter(), os_[i].read_adapter())
        worst = max(worst, ra)
        assert ra < TOL, (i, ra)
        hs[i].close()
        os_[i].close()
    print(f"batched encoder, 6 full-size streams: adapter rows worst rel err {worst:.2e}")


def synth_audio(seconds, seed):
    """Speech-band synthetic audio (no recording offline; the path's work depends only on
    the length): noise bursts under a slow envelope plus drifting tones."""
    rng = np.random.default_rng(seed)
    n = int(seconds * 16000)
    t = np.arange(n) / 16000.0
    env = 0.5 + 0.5 * np.sin(2 * np.pi * 0.7 * t) * np.sin(2 * np.pi * 0.13 * t)
    x = 0.05 * rng.standard_normal(n) * env + 0.1 * env * np.sin(2 * np.pi * (180 + 60 * np.sin(0.5 * t)) * t)
    return x.astype(np.float32)


def test_full_long_clip_one_shot(full):
    """C2's longest clip (59.75 s, vox_transcribe_audio one-shot, voxtral.c:1388-1401): the
    first encoder call takes every frame fed so far -- over 3000 encoder rows, run in passes
    of <= 1024 rows through all 32 layers -- then the flush and finish chunks.  Adapter rows
    against the oracle, then 8 greedy steps (ids and logits)."""
    import vox_hip
    import vox_oracle
    cfg, hm, om = full
    events = vox_oracle.transcribe_mel_schedule(synth_audio(59.75, 7))
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    cur = 0
    for kind, mel in events:
        assert hs.encode_mel(mel[cur:]) == os_.encode_mel(mel[cur:])
        cur = mel.shape[0]
    assert events[0][1].shape[0] // 2 > 3000  # encoder rows of the one-shot chunk (3 passes)
    assert hs.adapter_tokens == os_.adapter_tokens
    ra = rel(hs.read_adapter(), os_.read_adapter())
    assert ra < TOL, ra
    ht, hl = hs.decode(max_steps=8, stop_at_eos=False, want_logits=True)
    ot, ol = os_.decode(max_steps=8, stop_at_eos=False, want_logits=True)
    rl = rel(hl, ol)
    print(f"59.75 s one-shot: {hs.adapter_tokens} adapter rows rel err {ra:.2e}, 8 steps logits rel err {rl:.2e}")
    assert np.array_equal(ht, ot) and len(ht) == 8
    assert rl < TOL, rl
    hs.close()
    os_.close()


def test_full_streaming_decode_vs_oracle(full):
    """C3's decode at full size: 24 s of audio fed in -I 0.5 pieces (main.c file mode), the
    decoder drained after every piece (stream_run_decoder, voxtral.c:1013-1145) on both
    sides; over 200 greedy steps interleaved with ~50 encoder chunks, every id identical and
    every step's logits within TOL of the oracle's."""
    import vox_hip
    import vox_oracle
    cfg, hm, om = full
    audio = synth_audio(24.0, 13)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    ha = vox_hip.AudioSession(hs, interval_s=0.5)
    oa = vox_oracle.OracleAudioSession(os_, interval_s=0.5)
    hl, ol, ot = [], [], []

    def hdec(stop_at_eos=True):
        t, lg = hs.decode(stop_at_eos=False, want_logits=True)
        ha.tokens += t.tolist()
        hl.append(lg)

    def odec():
        t, lg = os_.decode(stop_at_eos=False, want_logits=True)
        ot.extend(t.tolist())
        ol.append(lg)
    ha._run_decoder = hdec
    oa._dec = odec
    for i in range(0, len(audio), 8000):
        ha.feed_samples(audio[i:i + 8000])
        oa.feed(audio[i:i + 8000])
    ha.finish_samples()
    oa.finish()
    assert len(ha.chunks) > 40
    assert len(ot) > 200, len(ot)
    assert ha.tokens == ot
    hl, ol = np.concatenate(hl), np.concatenate(ol)
    rl = rel(hl, ol)
    print(f"24 s -I 0.5 full decode: {len(ha.chunks)} chunks, {len(ot)} ids equal, logits rel err {rl:.2e}")
    assert rl < TOL, rl
    ha.close()
    oa.close()
    hs.close()
    os_.close()


def test_full_streaming_60s_encoder(full):
    """C3 scale: 60 s of audio fed in -I 0.5 pieces (main.c file mode) through the device
    log-mel and the chunked encoder (~25-row chunks over the rolling 750-row window, KV ring
    vs the reference's compaction) against the oracle's session on host mel; the decoder is
    left out on both sides (the oracle's single-threaded decode would take minutes).  Every
    chunk size and every adapter row is compared."""
    import vox_hip
    import vox_oracle
    cfg, hm, om = full
    audio = synth_audio(60.0, 11)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    ha = vox_hip.AudioSession(hs, interval_s=0.5)
    ha._run_decoder = lambda stop_at_eos=True: None
    oa = vox_oracle.OracleAudioSession(os_, interval_s=0.5)
    oa._dec = lambda: None
    ochunks = []
    enc = oa._enc

    def counted(min_new):
        before = oa.cursor
        enc(min_new)
        if oa.cursor != before:
            ochunks.append(oa.cursor - before)
    oa._enc = counted
    for i in range(0, len(audio), 8000):
        ha.feed_samples(audio[i:i + 8000])
        oa.feed(audio[i:i + 8000])
    ha.finish_samples()
    oa.finish()
    assert len(ha.chunks) > 100
    assert ha.chunks == ochunks, (ha.chunks[:8], ochunks[:8])
    assert hs.adapter_tokens == os_.adapter_tokens
    ra = rel(hs.read_adapter(), os_.read_adapter())
    print(f"60 s -I 0.5: {len(ha.chunks)} chunks, {hs.adapter_tokens} adapter rows rel err {ra:.2e}")
    assert ra < TOL, ra
    ha.close()
    oa.close()
    hs.close()
    os_.close()
