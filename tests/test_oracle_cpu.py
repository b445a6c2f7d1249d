"""CPU: pin the oracle (oracle/vox_oracle.c) against the reference's own outputs.

* ref_mel.npz  -- frames produced by the reference's voxtral_audio.c, compiled in place
                  (tests/golden/gen_ref_audio.py).  Tolerance 2e-7 absolute (1 ulp at the
                  mel value range; 98.6 % of frames are bit-identical: gcc flags differ).
* pyref.npz    -- the reference's Python implementation (tests/golden/gen_pyref.py): per-op
                  vectors and a whole TINY pipeline.  Tolerance: 2e-5 relative per op,
                  1e-4 relative for the 2-layer encoder/decoder pipeline (torch and OpenBLAS
                  sum in different orders), identical greedy tokens.
"""
import dataclasses
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.cpu


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1e-12, float(np.max(np.abs(b)))))


@pytest.fixture(scope="module")
def pyref():
    return np.load(os.path.join(GOLDEN, "pyref.npz"))


@pytest.fixture(scope="module")
def refmel():
    return np.load(os.path.join(GOLDEN, "ref_mel.npz"))


def test_mel_matches_reference_audio_c_jfk(refmel, jfk_samples):
    import vox_oracle
    ev = vox_oracle.transcribe_mel_schedule(jfk_samples)
    counts = refmel["jfk_counts"]
    ref = refmel["jfk_finish"]
    for (kind, mel), n in zip(ev, counts):
        assert mel.shape[0] == n, (kind, mel.shape, n)
        m = min(n, ref.shape[0])
        np.testing.assert_allclose(mel[:m], ref[:m], rtol=0, atol=2e-7)


def test_mel_matches_reference_audio_c_ragged_feeds(refmel):
    import vox_oracle
    chirp, pieces = refmel["chirp"], refmel["chirp_pieces"]
    m = vox_oracle.OracleMel(32 * 1280)
    pos = 0
    for k in pieces:
        m.feed(chirp[pos:pos + k])
        pos += k
    assert m.data().shape[0] == refmel["chirp_counts"][0]
    n = len(chirp)
    pad = (1280 - n % 1280) % 1280 + 17 * 1280
    z = np.zeros(pad, np.float32)
    for i in range(0, pad, 4096):
        m.feed(z[i:i + 4096])
    assert m.data().shape[0] == refmel["chirp_counts"][1]
    m.finish(0)
    got = m.data()
    assert got.shape[0] == refmel["chirp_counts"][2]
    np.testing.assert_allclose(got, refmel["chirp_finish"], rtol=0, atol=2e-7)
    m.close()


def test_rms_norm(pyref):
    import vox_oracle
    y = vox_oracle.rms_norm(pyref["rms_x"], pyref["rms_w"], 1e-5)
    assert rel(y, pyref["rms_y"]) < 2e-6


@pytest.mark.parametrize("hd", [64, 128])
def test_rope(pyref, hd):
    import vox_oracle
    f = vox_oracle.rope_freqs(pyref["rope_pos"], hd, 1e6)
    np.testing.assert_allclose(f[:, 0::2], pyref[f"rope_cos_{hd}"], atol=2e-6)
    np.testing.assert_allclose(f[:, 1::2], pyref[f"rope_sin_{hd}"], atol=2e-6)
    y = vox_oracle.apply_rope(pyref[f"rope_x_{hd}"], f, 2, hd)
    np.testing.assert_allclose(y, pyref[f"rope_y_{hd}"], atol=1e-5)


@pytest.mark.parametrize("name", ["att_chunk", "att_step", "att_full"])
def test_causal_attention(pyref, name):
    import vox_oracle
    sq, sk, qoff, H, KVH, hd, win = pyref[f"{name}_meta"].tolist()
    o = vox_oracle.causal_attention(pyref[f"{name}_q"], pyref[f"{name}_k"], pyref[f"{name}_v"],
                                    H, KVH, hd, win, qoff)
    assert rel(o, pyref[f"{name}_o"]) < 2e-5


@pytest.mark.parametrize("stride", [1, 2])
def test_causal_conv1d(pyref, stride):
    import vox_oracle
    y = vox_oracle.causal_conv1d(pyref[f"conv{stride}_x"], pyref[f"conv{stride}_w"], pyref[f"conv{stride}_b"], stride)
    assert y.shape == pyref[f"conv{stride}_y"].shape
    assert rel(y, pyref[f"conv{stride}_y"]) < 2e-6


def test_time_embedding_and_gelu(pyref):
    import vox_oracle
    for d in (64, 3072):
        np.testing.assert_allclose(vox_oracle.time_embedding(d, 6.0), pyref[f"temb_{d}"], atol=2e-6)
    np.testing.assert_allclose(vox_oracle.gelu(pyref["gelu_x"], erf_mode=1), pyref["gelu_y"], atol=2e-6)
    # the C path's tanh GELU (voxtral_kernels.c:505-513) differs from erf by < 1e-3
    assert np.max(np.abs(vox_oracle.gelu(pyref["gelu_x"], 0) - pyref["gelu_y"])) < 1e-3


def test_pipeline_matches_python_reference(pyref):
    """conv stem -> 2-layer encoder -> adapter -> decoder prefill + 2 greedy steps."""
    import vox_oracle
    from vox_weights import TINY, synth_weights
    cfg = dataclasses.replace(TINY, gelu_erf=1)
    w = synth_weights(cfg, seed=int(pyref["pipe_seed"]))
    om = vox_oracle.OracleModel(cfg, w, delay_tokens=6)
    st = vox_oracle.OracleStream(om)
    conv = st.conv_stem(pyref["pipe_mel"])
    enc = st.encoder_incremental(conv)
    assert rel(enc, pyref["pipe_enc"]) < 1e-4, rel(enc, pyref["pipe_enc"])
    st2 = vox_oracle.OracleStream(om)
    assert st2.encode_mel(pyref["pipe_mel"]) == pyref["pipe_adapter"].shape[0]
    assert rel(st2.read_adapter(), pyref["pipe_adapter"]) < 1e-4
    toks, logits = st2.decode(max_steps=2, stop_at_eos=False, want_logits=True)
    assert rel(logits, pyref["pipe_logits"]) < 1e-4, rel(logits, pyref["pipe_logits"])
    assert toks.tolist() == pyref["pipe_tokens"].tolist()
    st.close(); st2.close(); om.close()


def _oracle_run(cfg, w, events, interval=None):
    """tokens, per-step logits and adapter rows of one oracle stream over mel events"""
    import vox_oracle
    om = vox_oracle.OracleModel(cfg, w)
    st = vox_oracle.OracleStream(om)
    sess = vox_oracle.OracleSession(st, interval_s=interval or 2.0)
    logits = []
    for kind, mel in events:
        if kind == "finish":
            sess.finished = True
        sess._enc(mel, 1 if kind == "flush" else sess.min_new)
        t, lg = st.decode(stop_at_eos=False, want_logits=True)
        sess.tokens += t.tolist()
        logits.append(lg)
    out = (sess.tokens, np.concatenate(logits), st.read_adapter(), sess.chunks)
    st.close()
    om.close()
    return out


def test_invariance_compaction_vs_none(tiny_cfg, tiny_weights, jfk_samples):
    """the window semantics do not depend on the physical KV
    compaction (voxtral_encoder.c:431-449, voxtral_decoder.c:354-384).  TINY's windows
    (24 / 48) compact the encoder and decoder caches many times over jfk; a run that only
    grows the caches gives bit-identical adapter rows, logits and ids."""
    import vox_oracle
    events = vox_oracle.transcribe_mel_schedule(jfk_samples)
    a = _oracle_run(tiny_cfg, tiny_weights, events)
    vox_oracle.set_no_compaction(True)
    try:
        b = _oracle_run(tiny_cfg, tiny_weights, events)
    finally:
        vox_oracle.set_no_compaction(False)
    assert len(a[0]) == 149
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[1], b[1])


def test_invariance_chunked_vs_one_shot(tiny_cfg, tiny_weights, jfk_samples):
    """the causal encoder with its conv-stem tails and 4-row carry
    (voxtral.c:581-759, 868-934) gives the same adapter rows whether the audio arrives in one
    chunk (vox_transcribe_audio) or in -I 0.5 chunks (main.c file mode), up to f32
    summation order; greedy ids equal (the reference's own -I 2 / -I 0.5 runs on jfk gave
    identical ids)."""
    import vox_oracle
    one = _oracle_run(tiny_cfg, tiny_weights, vox_oracle.transcribe_mel_schedule(jfk_samples))
    chk = _oracle_run(tiny_cfg, tiny_weights, vox_oracle.transcribe_mel_schedule(jfk_samples, feed_size=8000), 0.5)
    assert len(one[3]) == 3 and len(chk[3]) > 10
    assert one[2].shape == chk[2].shape
    assert rel(one[2], chk[2]) < 1e-5, rel(one[2], chk[2])
    assert one[0] == chk[0]
