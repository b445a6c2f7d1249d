"""CPU checks of the oracle's fp16 decoder KV restatement (VOX_DECODER_KV_FP16,
voxtral.c:189-190; voxtral_decoder.c:151-178 widens the stored halves back to f32).

f16_round (oracle/vox_oracle.c) is f32 -> IEEE half (round to nearest even, subnormals,
overflow to inf) -> f32; numpy's float16 cast is the same IEEE conversion, so the two must
agree bit for bit.  The reference's own fp16 path is Metal-only (no fixture covers it): the
mode's decode parity is pinned by this rounding plus the f32 oracle, and the GPU tests
(tests/test_gpu_kv16.py) hold the HIP rings to it."""
import numpy as np


def test_f16_round_bit_exact_vs_numpy():
    import vox_oracle
    rng = np.random.default_rng(5)
    x = rng.standard_normal(300000).astype(np.float32)
    x *= (np.float32(10.0) ** rng.integers(-9, 6, x.size)).astype(np.float32)
    edges = np.array([65504, 65519.99, 65520, 65536, 1e9, -1e9, 6.1e-5, 6.103515625e-05, 5.96e-8,
                      2.98e-8, 2.99e-8, 0.0, -0.0, np.inf, -np.inf, 1.0009765625, 1.00048828125,
                      1.000732421875, 2049.0, 2051.0], np.float32)
    x = np.concatenate([x, edges]).astype(np.float32)
    with np.errstate(over="ignore"):
        want = x.astype(np.float16).astype(np.float32)
    got = vox_oracle.f16_round(x)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    nan = vox_oracle.f16_round(np.array([np.nan], np.float32))
    assert np.isnan(nan[0])


def test_oracle_kv16_decode_differs_and_is_deterministic(tiny_cfg, tiny_weights):
    """the rounding is applied (logits move) and only to the decoder cache (the encoder /
    adapter output is untouched); two runs agree exactly"""
    import vox_oracle
    om = vox_oracle.OracleModel(tiny_cfg, tiny_weights)
    mel = np.random.default_rng(3).uniform(-0.6, 1.4, size=(480, tiny_cfg.mel_bins)).astype(np.float32)

    def run(kv16):
        vox_oracle.set_kv_fp16(kv16)
        try:
            st = vox_oracle.OracleStream(om)
            st.encode_mel(mel)
            ad = st.read_adapter()
            ids, lg = st.decode(max_steps=12, stop_at_eos=False, want_logits=True)
            st.close()
        finally:
            vox_oracle.set_kv_fp16(False)
        return ad, ids, lg
    a32, i32, l32 = run(False)
    a16, i16, l16 = run(True)
    b16 = run(True)
    assert np.array_equal(a32, a16)
    assert not np.array_equal(l32, l16)
    assert np.array_equal(l16, b16[2]) and np.array_equal(i16, b16[1])
    om.close()
