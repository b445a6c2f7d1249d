"""CPU: host-side scheduling of vox_hip.Session (the mirror of stream_run_encoder's gating,
voxtral.c:827-851) against the reference's chunk schedule, with a recording stub stream."""
import numpy as np
import pytest

pytestmark = pytest.mark.cpu


class RecStream:
    def __init__(self):
        self.calls = []

    def encode_mel(self, mel):
        self.calls.append(mel.shape[0])
        return 0

    def decode(self, stop_at_eos=True):
        return np.zeros(0, np.int32)


def run(events, interval):
    import vox_hip
    import vox_oracle
    rec = RecStream()
    s = vox_hip.Session(rec, interval)
    o = vox_oracle.OracleSession(rec, interval)  # same stub: the oracle's own gating
    for kind, mel in events:
        getattr(s, kind)(mel)
    a = list(rec.calls)
    rec.calls.clear()
    for kind, mel in events:
        getattr(o, kind)(mel)
    return a, list(rec.calls)


def test_one_shot_schedule(jfk_samples):
    import vox_oracle
    a, b = run(vox_oracle.transcribe_mel_schedule(jfk_samples), 2.0)
    assert a == b == [1355, 140, 1]  # one-shot jfk


def test_streaming_schedule(jfk_samples):
    import vox_oracle
    ev = vox_oracle.transcribe_mel_schedule(jfk_samples, feed_size=16000)
    a, b = run(ev, 0.5)
    assert a == b
    assert a[0] >= 312 and sum(a) == ev[-1][1].shape[0]


def test_right_pad_samples():
    import vox_hip
    # voxtral.c:1645-1649: align to 1280 + (delay+1+10) tokens
    assert vox_hip.right_pad_samples(176000, 6) == (1280 - 176000 % 1280) % 1280 + 17 * 1280
    assert vox_hip.right_pad_samples(1280 * 5, 6) == 17 * 1280
