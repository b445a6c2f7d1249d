"""GPU parity of the reference-boundary twins: the functions INTEGRATION.md sections 4-6 bind
into voxtral_kernels.c / voxtral_encoder.c / voxtral_decoder.c in place of the Metal backend
(voxtral_metal.h:38-41 sgemm_bf16, :59-64 fused_qkv_bf16, :86-91 fused_ffn_bf16,
:245-246 encoder_full_step, :254-255 decoder_prefill_step, :161-164 decoder_start/end,
:219 decoder_full_step; q8: :262-265).  Each is driven the way the reference's call sites
drive the Metal twin and compared with the CPU oracle (oracle/, restating
voxtral_kernels.c / voxtral_encoder.c / voxtral_decoder.c).

Tolerance: identical greedy ids; every output within TOL = 5e-5 of the reference output's
largest magnitude (f32 arithmetic on exact bf16 / int8 weights, different summation order;
measured errors are ~1e-6)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 5e-5
BOS, PAD = 1, 32


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-30, float(np.max(np.abs(b)))))


# The twins cache device weights by host pointer and shape, as the Metal backend does
# (voxtral_metal.m:165-201: weights are mmap views that live for the process): a weight must
# stay alive and unmodified while in use, so every test weight is kept for the session (a
# freed array's address could come back for a new weight of the same shape).
_KEEP = []


def rand_bf16(rng, n, k):
    from vox_weights import f32_to_bf16
    w = f32_to_bf16(rng.standard_normal((n, k), dtype=np.float32) / np.float32(np.sqrt(k)))
    _KEEP.append(w)
    return w


def rand_x(rng, m, k):
    return rng.uniform(-2, 2, size=(m, k)).astype(np.float32)


@pytest.fixture(scope="module")
def hip():
    import vox_hip
    vox_hip.init()
    return vox_hip


# ---------------------------------------------------------------------------
# single GEMMs (voxtral_kernels.c:199-204, 218-229, 249-254; q8 :316-320, 342-353, 373-377)
# ---------------------------------------------------------------------------
RAGGED = [(1, 1001, 333), (5, 77, 129), (1, 4096, 256), (38, 768, 256), (25, 512, 256),
          (677, 1001, 333), (3, 130, 9), (1, 7, 8), (17, 3, 1000), (2, 130, 100)]


@pytest.mark.parametrize("M,N,K", RAGGED)
def test_sgemm_bf16_ragged(hip, M, N, K):
    import vox_oracle
    rng = np.random.default_rng(M * 7919 + N * 31 + K)
    W, x = rand_bf16(rng, N, K), rand_x(rng, M, K)
    got = hip.sgemm_bf16(x, W)
    ref = vox_oracle.linear_bf16(x, W)
    assert got.shape == ref.shape
    assert rel(got, ref) < TOL, rel(got, ref)


# every projection shape of Voxtral-4B: encoder wq|wk|wv (2048x1280), wo, w1/w3, w2; adapter
# 0/1; decoder wq, wk/wv, wo, w1/w3, w2
FULL_SHAPES = [(2048, 1280), (1280, 2048), (5120, 1280), (1280, 5120), (3072, 5120), (3072, 3072),
               (4096, 3072), (1024, 3072), (3072, 4096), (9216, 3072), (3072, 9216)]


@pytest.mark.slow
@pytest.mark.parametrize("N,K", FULL_SHAPES)
def test_sgemm_bf16_full_shapes(hip, N, K):
    import vox_oracle
    vox_oracle.set_threads(min(16, os.cpu_count() or 1))
    rng = np.random.default_rng(N + K)
    W = rand_bf16(rng, N, K)
    for M in (1, 25, 38, 677):
        x = rand_x(rng, M, K)
        got, ref = hip.sgemm_bf16(x, W), vox_oracle.linear_bf16(x, W)
        assert rel(got, ref) < TOL, (M, N, K, rel(got, ref))


@pytest.mark.slow
def test_sgemm_bf16_lm_head(hip):
    """vox_matmul_t_bf16 M=1 (voxtral_kernels.c:242-264): logits over the 131072 x 3072
    tied embeddings, argmax equal."""
    import vox_oracle
    rng = np.random.default_rng(5)
    W, x = rand_bf16(rng, 131072, 3072), rand_x(rng, 1, 3072)
    got, ref = hip.sgemm_bf16(x, W), vox_oracle.linear_bf16(x, W)
    assert rel(got, ref) < TOL
    assert int(np.argmax(got)) == int(np.argmax(ref))


@pytest.mark.parametrize("M,N,K", [(1, 1001, 333), (25, 1001, 336), (38, 3072, 1280), (1, 4096, 256), (7, 130, 16)])
def test_sgemm_q8(hip, M, N, K):
    import vox_oracle
    rng = np.random.default_rng(M + N + K)
    q = rng.integers(-127, 128, size=(N, K), dtype=np.int8)
    s = (rng.uniform(0.5, 1.5, N) / 127 / np.sqrt(K)).astype(np.float32)
    _KEEP.extend([q, s])
    x = rand_x(rng, M, K)
    got, ref = hip.sgemm_q8(x, q, s), vox_oracle.linear_q8(x, q, s)
    assert rel(got, ref) < TOL, rel(got, ref)


def _ffn_ref(x, w1, w3, w2):
    import vox_oracle
    g = vox_oracle.silu(vox_oracle.linear_bf16(x, w1))
    return vox_oracle.linear_bf16(g * vox_oracle.linear_bf16(x, w3), w2)


@pytest.mark.parametrize("dims", [(256, 512, 256, 128, 128), (1280, 5120, 2048, 2048, 2048),
                                  (3072, 9216, 4096, 1024, 1024), (100, 333, 70, 30, 30)])
def test_fused_qkv_ffn(hip, dims):
    """fused_qkv_bf16 at the encoder's call sites (voxtral_encoder.c:240-245, 570-575) and the
    decoder prefill's (voxtral_decoder.c:511-516); fused_ffn_bf16 at voxtral_encoder.c:311-314,
    652-655 and voxtral_decoder.c:574-577; plus a ragged shape."""
    import vox_oracle
    dim, hidden, nq, nk, nv = dims
    rng = np.random.default_rng(dim + hidden)
    wq, wk, wv = rand_bf16(rng, nq, dim), rand_bf16(rng, nk, dim), rand_bf16(rng, nv, dim)
    w1, w3, w2 = rand_bf16(rng, hidden, dim), rand_bf16(rng, hidden, dim), rand_bf16(rng, dim, hidden)
    for M in (1, 38, 25 if dim > 256 else 3):
        x = rand_x(rng, M, dim)
        q, k, v = hip.fused_qkv_bf16(x, wq, wk, wv)
        for got, w in ((q, wq), (k, wk), (v, wv)):
            ref = vox_oracle.linear_bf16(x, w)
            assert rel(got, ref) < TOL, (M, dims, rel(got, ref))
        got = hip.fused_ffn_bf16(x, w1, w3, w2)
        ref = _ffn_ref(x, w1, w3, w2)
        assert rel(got, ref) < TOL, (M, dims, rel(got, ref))


def test_twin_errors_are_reported(hip):
    """void twins report failures through vox_hip_last_error() (no silent no-op)."""
    x = np.ones((2, 8), np.float32)
    with pytest.raises(RuntimeError):
        hip.sgemm_bf16(x[:, :0], np.zeros((4, 0), np.uint16))
    y = hip.sgemm_bf16(x, rand_bf16(np.random.default_rng(0), 4, 8))   # and the next call is clean
    assert y.shape == (2, 4)


# ---------------------------------------------------------------------------
# encoder_full_step (voxtral_encoder.c:551-560) driven with the chunk sequence of
# vox_encoder_forward_incremental: conv-stem rows of each stream chunk, logical positions
# ---------------------------------------------------------------------------
def _encoder_twin_case(cfg, w, mel_chunks):
    import vox_hip
    import vox_oracle
    hm = vox_hip.Model(cfg, w)
    om = vox_oracle.OracleModel(cfg, w)
    stem = vox_oracle.OracleStream(om)   # conv stem only: produces each chunk's encoder input rows
    enc = vox_oracle.OracleStream(om)    # the reference encoder (physical KV compaction)
    hs = vox_hip.Stream(hm)
    pos, worst = 0, 0.0
    rng = np.random.default_rng(11)
    for n in mel_chunks:
        mel = rng.uniform(-0.6, 1.4, size=(n, cfg.mel_bins)).astype(np.float32)
        x = stem.conv_stem(mel)
        if x.shape[0] == 0:
            continue
        rope = vox_oracle.rope_freqs(np.arange(pos, pos + x.shape[0]), cfg.enc_head_dim, cfg.rope_theta)
        got = hs.twin_encoder_full_step(x, rope, pos)
        ref = enc.encoder_incremental(x)
        worst = max(worst, rel(got, ref))
        assert rel(got, ref) < TOL, (n, pos, rel(got, ref))
        pos += x.shape[0]
    hs.close(); stem.close(); enc.close(); hm.close(); om.close()
    return pos, worst


def test_encoder_full_step_tiny(tiny_cfg, tiny_weights):
    # TINY's 24-row window: the rolling cache wraps within the first chunk
    pos, worst = _encoder_twin_case(tiny_cfg, tiny_weights, [355, 50, 50, 1, 2, 7, 200, 3, 50])
    assert pos > 300
    print(f"encoder twin TINY: {pos} rows, worst rel {worst:.2e}")


@pytest.mark.slow
def test_encoder_full_step_full():
    """Voxtral-4B shapes: a 177-row first chunk, 25-row -I 0.5 chunks, a flush-sized chunk
    and a 1-row final chunk (355 mel -> 177, 50 -> 25, ..., 1)."""
    import vox_oracle
    from vox_weights import VOXTRAL_4B, synth_weights
    vox_oracle.set_threads(min(16, os.cpu_count() or 1))
    pos, worst = _encoder_twin_case(VOXTRAL_4B, synth_weights(VOXTRAL_4B, seed=0),
                                    [355, 50, 50, 50, 180, 3])
    print(f"encoder twin full: {pos} rows, worst rel {worst:.2e}")


# ---------------------------------------------------------------------------
# decoder_prefill_step + decoder_start / decoder_full_step / decoder_end, driven as
# voxtral_decoder.c:486-492 and :686-699
# ---------------------------------------------------------------------------
def _embed(w, cfg, adapter_row, tok):
    from vox_weights import EMB, bf16_to_f32
    return adapter_row + bf16_to_f32(w.bf16(EMB + ".tok_embeddings.weight")[tok])


def _decoder_twin_case(cfg, w, adapter, n_steps, delay_tokens=6, check_every=1):
    import vox_hip
    import vox_oracle
    hm = vox_hip.Model(cfg, w, delay_tokens)
    om = vox_oracle.OracleModel(cfg, w, delay_tokens)
    hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
    prompt = [BOS] + [PAD] * (32 + delay_tokens)
    npf = len(prompt) - 1
    x = np.stack([_embed(w, cfg, adapter[i], prompt[i]) for i in range(npf)])
    rope = vox_oracle.rope_freqs(np.arange(npf), cfg.dec_head_dim, cfg.rope_theta)
    hs.twin_decoder_prefill_step(x, rope, 0)
    os_.decoder_prefill(x)
    prev, toks, worst = prompt[-1], [], 0.0
    for pos in range(npf, npf + n_steps):
        e = _embed(w, cfg, adapter[pos], prev)
        r = vox_oracle.rope_freqs([pos], cfg.dec_head_dim, cfg.rope_theta)[0]
        want = (pos - npf) % check_every == 0
        ht, hl = hs.twin_decoder_step(e, r, pos, want_logits=want)
        ot, ol = os_.decoder_forward(e)
        assert ht == ot, (pos, ht, ot)
        if want:
            worst = max(worst, rel(hl, ol))
            assert rel(hl, ol) < TOL, (pos, rel(hl, ol))
        toks.append(ot)
        prev = ot
    hs.close(); os_.close(); hm.close(); om.close()
    return toks, worst


def test_decoder_twins_tiny(tiny_cfg, tiny_weights, jfk_samples):
    """TINY (window 48, ring of 112 slots): the 149 jfk steps wrap the decoder KV ring."""
    import vox_oracle
    om = vox_oracle.OracleModel(tiny_cfg, tiny_weights)
    st = vox_oracle.OracleStream(om)
    done = 0
    for kind, mel in vox_oracle.transcribe_mel_schedule(jfk_samples):
        st.encode_mel(mel[done:])
        done = mel.shape[0]
    adapter = st.read_adapter()
    st.close(); om.close()
    n = adapter.shape[0] - 38
    toks, worst = _decoder_twin_case(tiny_cfg, tiny_weights, adapter, n)
    assert len(toks) == n > 100
    print(f"decoder twins TINY: {n} steps, worst logit rel {worst:.2e}")


def test_decoder_twins_window_wrap_8192(tiny_weights):
    """TINY_LONG (the real 8192-key window): 8300 greedy steps, so the decoder passes the
    8256-slot ring and the 8192-key window slides; the oracle compacts its cache physically
    (voxtral_decoder.c:354-384, 668-677).  Logits checked every 97 steps and at the end."""
    from vox_weights import TINY_LONG
    rng = np.random.default_rng(8192)
    n = 8300
    adapter = (rng.standard_normal((n + 40, TINY_LONG.dec_dim)) * 0.5).astype(np.float32)
    toks, worst = _decoder_twin_case(TINY_LONG, tiny_weights, adapter, n, check_every=97)
    assert len(toks) == n
    print(f"decoder twins TINY_LONG: {n} steps past the 8192 window, worst logit rel {worst:.2e}")


@pytest.mark.slow
def test_decoder_twins_full(jfk_samples):
    """Voxtral-4B: prefill + the 149 jfk greedy steps through the twins, ids and logits
    against the oracle (adapter rows from the oracle's own encoder)."""
    import vox_oracle
    from vox_weights import VOXTRAL_4B, synth_weights
    vox_oracle.set_threads(min(16, os.cpu_count() or 1))
    w = synth_weights(VOXTRAL_4B, seed=0)
    om = vox_oracle.OracleModel(VOXTRAL_4B, w)
    st = vox_oracle.OracleStream(om)
    done = 0
    for kind, mel in vox_oracle.transcribe_mel_schedule(jfk_samples):
        st.encode_mel(mel[done:])
        done = mel.shape[0]
    adapter = st.read_adapter()
    st.close(); om.close()
    assert adapter.shape[0] == 187
    toks, worst = _decoder_twin_case(VOXTRAL_4B, w, adapter, 149, check_every=1)
    print(f"decoder twins full: 149 steps, worst logit rel {worst:.2e}")
