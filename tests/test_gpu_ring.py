"""The 8192-slot rolling decoder KV through the PRODUCT fast paths (north_star's "8192-slot
rolling KV cache"; reference: voxtral_decoder.c:354-384 compaction, :668-677 the window,
README.md:7 / :328 the long-transcription risk).

TINY_LONG keeps Voxtral's head dims and the real 8192-key window, so ~8330 greedy steps
take the decoder past
  * position 8191 (the window fills: the oldest key starts leaving the attention),
  * position 8256 (the HIP ring, capacity window + 64, wraps onto slot 0),
through
  * vox_hip_stream_decode: hipGraph replays, the position held in device state, every
    attention split bucket (1 .. 32 blocks of 256 keys) captured on the way;
  * vox_hip_batch_decode: 4 streams at different positions, the batched step graph with
    the fused RoPE / KV-append attention and its combine kernel.

Bars: greedy ids identical to the CPU oracle over all steps; logits within 5e-5 of the
largest magnitude (f32, different summation order) on every step from 8100 on (positions
8138..8367, both boundaries included)."""
import threading

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

TOL = 5e-5
N_STEPS = 8330          # greedy steps: last position 38 + 8329 = 8367 > 8256
N_PLAIN = 8100          # steps decoded before the per-step logits
CHUNK = 4096            # mel frames per encoder call
N_MEL = 8 * 8400        # 8400 adapter rows


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))


def _mel(seed, n=N_MEL):
    rng = np.random.default_rng(seed)
    return rng.uniform(-0.6, 1.4, size=(n, 128)).astype(np.float32)


def _encode(s, mel):
    for i in range(0, mel.shape[0], CHUNK):
        s.encode_mel(mel[i:i + CHUNK])


def _oracle_run(om, mel, out):
    import vox_oracle
    st = vox_oracle.OracleStream(om)
    _encode(st, mel)
    a = st.decode(max_steps=N_PLAIN, stop_at_eos=False)
    b, lg = st.decode(max_steps=N_STEPS - N_PLAIN, stop_at_eos=False, want_logits=True)
    out["ids"] = np.concatenate([a, b]).tolist()
    out["logits"] = lg
    out["state"] = st.state()
    st.close()


@pytest.fixture(scope="module")
def ring(tiny_weights):
    """HIP + oracle models on TINY_LONG, and the oracle's run on stream A (started in a
    thread: ctypes releases the GIL, so the GPU work of the tests overlaps it)."""
    import os

    import vox_hip
    import vox_oracle
    from vox_weights import TINY_LONG
    vox_oracle.set_threads(min(16, os.cpu_count() or 1))
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    melA = _mel(71)
    ref = {}
    th = threading.Thread(target=_oracle_run, args=(om, melA, ref))
    th.start()

    def oracle():
        th.join()
        assert "ids" in ref, "oracle run failed"
        return ref
    yield hm, melA, oracle
    th.join()
    hm.close()
    om.close()


def _single(hm, mel):
    """vox_hip_stream_decode over the ring: graph-replayed batches of 16 steps, then one
    step per call with its logits."""
    import vox_hip
    s = vox_hip.Stream(hm)
    _encode(s, mel)
    a = s.decode(max_steps=N_PLAIN, stop_at_eos=False)
    b, lg = s.decode(max_steps=N_STEPS - N_PLAIN, stop_at_eos=False, want_logits=True)
    st = s.state()
    s.close()
    return np.concatenate([a, b]).tolist(), lg, st


def test_stream_decode_through_ring_wrap(ring):
    hm, melA, oracle = ring
    ids, lg, st = _single(hm, melA)
    assert len(ids) == N_STEPS
    assert st["kv_pos"] == 39 + N_STEPS - 1 > 8256 + 64, st
    ref = oracle()
    assert ref["state"]["dec_len"] + ref["state"]["dec_off"] == st["kv_pos"]
    first_diff = next((i for i in range(N_STEPS) if ids[i] != ref["ids"][i]), None)
    assert first_diff is None, (first_diff, ids[first_diff], ref["ids"][first_diff])
    r = rel(lg, ref["logits"])
    print(f"ring single stream: {N_STEPS} ids equal, logits rel err {r:.2e} over positions "
          f"{38 + N_PLAIN}..{38 + N_STEPS - 1}")
    assert r < TOL, r


def test_batch_decode_through_ring_wrap(ring):
    """4 streams (A = the oracle's stream, B-D other audio) batched past the ring wrap, at
    different positions: C runs 37 steps alone first, D joins after the batch has run 500
    steps.  Per step logits for the last steps of every stream; A against the oracle, all
    four against their own single-stream decode (ids over every step, logits 5e-5)."""
    import vox_hip
    hm, melA, oracle = ring
    mels = [melA, _mel(72), _mel(73), _mel(74, N_MEL - 8 * 40)]   # D: 40 adapter rows fewer
    ss = [vox_hip.Stream(hm) for _ in mels]
    for s, mel in zip(ss, mels):
        _encode(s, mel)
    b = vox_hip.Batch(hm, 4)
    out = [[] for _ in ss]
    # C alone first; A, B, C batched; then D joins (prefilled on entry); graph replays
    out[2] += ss[2].decode(max_steps=37, stop_at_eos=False).tolist()
    for k, t in enumerate(b.decode(ss[:3], max_steps=500, stop_at_eos=False)):
        out[k] += t.tolist()
    for k, t in enumerate(b.decode(ss, max_steps=N_PLAIN - 537, stop_at_eos=False)):
        out[k] += t.tolist()
    assert [len(o) for o in out] == [N_PLAIN - 37, N_PLAIN - 37, N_PLAIN, N_PLAIN - 537]
    # one batched step per call to the end, logits of every step from N_PLAIN on; the active
    # set changes as streams catch up, reach N_STEPS or run out of adapter rows (D)
    logits = [[] for _ in ss]
    while True:
        act = [k for k in range(4) if len(out[k]) < min(N_STEPS, ss[k].adapter_tokens - 38)]
        if not act:
            break
        toks = b.decode([ss[k] for k in act], max_steps=1, stop_at_eos=False)
        for k, t in zip(act, toks):
            assert len(t) == 1
            out[k] += t.tolist()
            if len(out[k]) > N_PLAIN:
                logits[k].append(b.read_logits(ss[k]))
    for s in ss:
        s.close()
    b.close()
    ref = oracle()
    assert out[0] == ref["ids"]
    rA = rel(np.stack(logits[0]), ref["logits"])
    assert rA < TOL, rA
    worst = rA
    for k in range(1, 4):
        ids, lg, st = _single(hm, mels[k])
        n = len(out[k])
        assert n == len(ids) and n > 8256 - 38, (k, n, len(ids))   # past the ring wrap
        assert out[k] == ids, (k, next(i for i in range(n) if out[k][i] != ids[i]))
        got = np.stack(logits[k])
        assert got.shape == lg.shape, (k, got.shape, lg.shape)
        r = rel(got, lg)
        worst = max(worst, r)
        assert r < TOL, (k, r)
    print(f"ring batch: 4 streams, ids equal, worst logits rel err {worst:.2e}")
