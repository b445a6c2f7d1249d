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
