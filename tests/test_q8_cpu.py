"""CPU: Q8 checkpoints (config 5) -- quantizer, file format and the oracle's q8 path.

* q8_ref.json  -- output of the reference's own quantize.py on a TINY synthetic checkpoint
                  (tests/golden/gen_q8.py); vox_weights.quantize_q8 must reproduce every
                  tensor bit for bit (sha256), including an all-zero row and .5 ties.
* pyref.npz    -- pipeq8_*: the reference's Python model run on the dequantized Q8
                  weights (what safetensors_get_f32 yields); the oracle's q8 path
                  (q8 matvec for M=1, dequantize + sgemm for M>1, q8 embeddings) must match
                  within 1e-4 relative with identical greedy tokens.
"""
import dataclasses
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.cpu


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1e-12, float(np.max(np.abs(b)))))


def digest(parts):
    h = hashlib.sha256()
    for p in parts:
        h.update(np.ascontiguousarray(p).tobytes())
    return h.hexdigest()


@pytest.fixture(scope="module")
def ref():
    with open(os.path.join(GOLDEN, "q8_ref.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def q8w(ref):
    import gen_q8
    import vox_weights as vw
    assert gen_q8.SEED == ref["seed"]
    return vw.quantize_q8(gen_q8.fixture_weights())


def test_quantizer_matches_reference_quantize_py(ref, q8w):
    got = {}
    for name, (sc, q) in q8w.q8.items():
        got[name] = {"dtype": "Q8", "shape": list(q.shape), "sha256": digest([sc, q])}
    for name, a in q8w._stored_f32.items():
        got[name] = {"dtype": "F32", "shape": list(a.shape), "sha256": digest([a])}
    assert set(got) == set(ref["tensors"])
    bad = [n for n in got if got[n] != ref["tensors"][n]]
    assert not bad, bad[:5]
    sc, q = q8w.q8[ref["edge_tensor"]]
    assert sc[ref["zero_row"]] == 0.0 and not q[ref["zero_row"]].any()
    assert float(sc[ref["tie_row"]]) == ref["tie_row_scale"]
    assert q[ref["tie_row"], :len(ref["tie_row_q"])].tolist() == ref["tie_row_q"]


def test_q8_safetensors_round_trip(tmp_path, q8w):
    import vox_weights as vw
    p = str(tmp_path / "consolidated.safetensors")
    vw.write_safetensors(q8w, p)
    back = vw.load_safetensors(p, vw.TINY)
    assert back.is_q8 and set(back.q8) == set(q8w.q8)
    for n, (sc, q) in q8w.q8.items():
        assert np.array_equal(back.q8[n][0], sc) and np.array_equal(back.q8[n][1], q)
    for n, a in q8w._stored_f32.items():
        assert np.array_equal(back.f32(n), a)


@pytest.mark.parametrize("M", [1, 5])
def test_oracle_linear_q8(q8w, M):
    """vo_linear_q8 vs the dequantized matrix (safetensors_get_f32) in float64."""
    import vox_oracle
    name = "layers.1.feed_forward.w2.weight"
    sc, q = q8w.q8[name]
    rng = np.random.default_rng(M)
    x = rng.standard_normal((M, q.shape[1])).astype(np.float32)
    b = rng.standard_normal(q.shape[0]).astype(np.float32)
    y = vox_oracle.linear_q8(x, q, sc, b)
    ref = x.astype(np.float64) @ q8w.f32(name).astype(np.float64).T + b
    assert rel(y, ref) < 1e-5


def test_oracle_q8_pipeline_matches_python_reference():
    import vox_oracle
    from vox_weights import TINY, quantize_q8, synth_weights
    pr = np.load(os.path.join(GOLDEN, "pyref.npz"))
    cfg = dataclasses.replace(TINY, gelu_erf=1)
    w = quantize_q8(synth_weights(cfg, seed=int(pr["pipe_seed"])))
    om = vox_oracle.OracleModel(cfg, w, delay_tokens=6)
    st = vox_oracle.OracleStream(om)
    enc = st.encoder_incremental(st.conv_stem(pr["pipe_mel"]))
    assert rel(enc, pr["pipeq8_enc"]) < 1e-4, rel(enc, pr["pipeq8_enc"])
    st2 = vox_oracle.OracleStream(om)
    assert st2.encode_mel(pr["pipe_mel"]) == pr["pipeq8_adapter"].shape[0]
    assert rel(st2.read_adapter(), pr["pipeq8_adapter"]) < 1e-4
    toks, logits = st2.decode(max_steps=2, stop_at_eos=False, want_logits=True)
    assert rel(logits, pr["pipeq8_logits"]) < 1e-4, rel(logits, pr["pipeq8_logits"])
    assert toks.tolist() == pr["pipeq8_tokens"].tolist()
    st.close(); st2.close(); om.close()


def test_quantize_py_file_layout_byte_identical(ref, q8w, tmp_path):
    """vox_weights.write_quantize_py_layout writes the reference quantizer's output file
    byte for byte (unpadded compact header, tensors back to back: unaligned scales/rows),
    so the GPU test that loads it through the C loader (vh_load) reads exactly what
    quantize.py produces."""
    import vox_weights as vw
    path = tmp_path / "consolidated.safetensors"
    vw.write_quantize_py_layout(q8w, str(path))
    raw = path.read_bytes()
    assert len(raw) == ref["file_bytes"]
    assert int.from_bytes(raw[:8], "little") == ref["header_bytes"]
    assert (8 + ref["header_bytes"]) % 4 != 0       # the data section starts unaligned
    assert hashlib.sha256(raw).hexdigest() == ref["file_sha256"]
