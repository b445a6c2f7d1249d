"""The per-GPU stream scheduler of the C host (vh_sched_*, include/vox_hip_host.h; SURVEY.md
8f#1: the per-stream token loop of voxtral.c:1105-1145 and the feed path of :1288-1316
turned into a serving loop).  Streams of different lengths start at staggered times and are
fed in -I 0.5 pieces; after every round of feeds vh_sched_run prefills the streams whose
prompt is complete and advances all running streams with batched steps.  Every stream's ids
must equal its own single-stream CPU-oracle run on the same pieces (the reference's
vox_stream_feed / flush / finish, voxtral.c:1288-1316, 1640-1667)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PIECE = 8000   # 0.5 s of 16 kHz samples per feed


def _oracle_ids(om, audio, interval, continuous=False):
    import vox_oracle
    os_ = vox_oracle.OracleStream(om)
    sess = vox_oracle.OracleAudioSession(os_, interval_s=interval, continuous=continuous)
    for i in range(0, len(audio), PIECE):
        sess.feed(audio[i:i + PIECE])
    sess.finish()
    ids, restarts = sess.tokens, sess.restarts
    sess.close()
    os_.close()
    return ids, restarts


def _serve(hm, audios, starts, interval, continuous=False, max_streams=8, step_cap=0):
    """One serving loop on one GPU: at tick t every stream that has started feeds its next
    piece (flush + finish after its last one), then one vh_sched_run for all of them (with a
    step cap, runs go on until every stream has drained)."""
    import vox_hip
    ctx = vox_hip.HostCtx(hm)
    q = vox_hip.Scheduler(ctx, max_streams)
    q.set_step_cap(step_cap)
    ss = [vox_hip.HostStream(ctx, interval_s=interval, continuous=continuous) for _ in audios]
    for s in ss:
        q.attach(s)
    pos = [0] * len(audios)
    done = [False] * len(audios)
    ids = [[] for _ in audios]
    tick = 0
    while not all(done) or any(s.pending() for s in ss):
        for k, (a, s) in enumerate(zip(audios, ss)):
            if done[k] or tick < starts[k]:
                continue
            if pos[k] < len(a):
                s.feed(a[pos[k]:pos[k] + PIECE])
                pos[k] += PIECE
            else:
                s.finish()   # vox_stream_finish: flush padding, mel finish, last chunk
                done[k] = True
        q.run()
        for k, s in enumerate(ss):
            ids[k] += s.get()
        tick += 1
    st = q.stats()
    for s in ss:
        s.close()
    q.close()
    ctx.close()
    return ids, st


def test_scheduler_staggered_streams_match_oracle(tiny_weights, jfk_samples):
    """6 streams, 6 audio lengths (2.5 .. 33 s, jfk-derived, different offsets), starts
    staggered by 3 ticks; ids per stream equal the oracle's; the batched steps really ran
    (more tokens from batched steps than from prefills)."""
    import vox_hip
    import vox_oracle
    from vox_weights import TINY_LONG
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    long = np.concatenate([jfk_samples] * 3)
    lens = [2.5, 11.0, 5.0, 33.0, 7.3, 19.0]
    audios = [np.ascontiguousarray(long[int(k * 24000) % 16000:][:int(s * 16000)]) for k, s in enumerate(lens)]
    starts = [3 * k for k in range(len(audios))]
    ids, st = _serve(hm, audios, starts, 0.5)
    for k, a in enumerate(audios):
        ref, _ = _oracle_ids(om, a, 0.5)
        assert len(ref) > 0
        assert ids[k] == ref, (k, len(ids[k]), len(ref))
    assert st["tokens"] > st["prefills"] > 0 and st["batch_calls"] > 0
    print("scheduler stats", st)
    hm.close()
    om.close()


def test_scheduler_step_cap_spreads_bursts(tiny_weights, jfk_samples):
    """vh_sched_set_step_cap(3): each run advances a stream by at most 3 steps, so prompts and
    flush paddings drain over later runs inside the batched steps; every stream's ids still
    equal its oracle session, and more runs than feeds were needed to drain."""
    import vox_hip
    import vox_oracle
    from vox_weights import TINY_LONG
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    long = np.concatenate([jfk_samples] * 2)
    lens = [3.0, 9.0, 5.5, 12.0]
    audios = [np.ascontiguousarray(long[int(k * 17000) % 16000:][:int(s * 16000)]) for k, s in enumerate(lens)]
    ids, st = _serve(hm, audios, [0, 2, 3, 5], 0.5, step_cap=3)
    for k, a in enumerate(audios):
        ref, _ = _oracle_ids(om, a, 0.5)
        assert ids[k] == ref, (k, len(ids[k]), len(ref))
    assert st["steps"] > 0 and st["tokens"] / st["steps"] > 1.0, st
    print("step-capped scheduler stats", st)
    hm.close()
    om.close()


@pytest.mark.parametrize("overlap", ["1", "0"])
def test_scheduler_finish_then_one_run_drains(tiny_weights, jfk_samples, monkeypatch, overlap):
    """without a step cap one vh_sched_run drains every stream, including the rows
    of the chunk vh_stream_finish queued for that run's encoder pass (with the pass beside
    the steps, VOX_HIP_SCHED_OVERLAP=1, and sequentially): feed everything, finish, run once,
    and every stream's ids equal its oracle session with nothing pending."""
    import vox_hip
    from vox_weights import TINY_LONG
    monkeypatch.setenv("VOX_HIP_SCHED_OVERLAP", overlap)
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    import vox_oracle
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    audios = [np.ascontiguousarray(jfk_samples[:int(s * 16000)]) for s in (3.0, 6.5)]
    ctx = vox_hip.HostCtx(hm)
    q = vox_hip.Scheduler(ctx, 4)
    ss = [vox_hip.HostStream(ctx, interval_s=0.5) for _ in audios]
    for s in ss:
        q.attach(s)
    ids = [[] for _ in audios]
    for a, s in zip(audios, ss):
        for i in range(0, len(a), PIECE):
            s.feed(a[i:i + PIECE])
    q.run()
    for k, s in enumerate(ss):
        ids[k] += s.get()
    for s in ss:
        s.finish()
    q.run()   # exactly one run after finish
    for k, s in enumerate(ss):
        ids[k] += s.get()
        assert s.pending() == 0
    for k, a in enumerate(audios):
        ref, _ = _oracle_ids(om, a, 0.5)
        assert ids[k] == ref, (k, len(ids[k]), len(ref))
    for s in ss:
        s.close()
    q.close()
    ctx.close()
    hm.close()
    om.close()


def test_scheduler_continuous_restarts_per_stream(tiny_weights, jfk_samples):
    """Live mode (vh_stream_set_continuous) on two scheduled streams of 88 s: each stream's
    restarts (64-token non-text streaks on the random TINY model, voxtral.c:1189-1239) stay
    its own, and its ids equal the oracle's live-mode session on the same pieces."""
    import vox_hip
    import vox_oracle
    from vox_weights import TINY_LONG
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    a = np.concatenate([jfk_samples] * 8)
    audios = [a, np.ascontiguousarray(-a[5000:])]
    ids, _ = _serve(hm, audios, [0, 7], 2.0, continuous=True)
    n_restarts = 0
    for k, au in enumerate(audios):
        ref, restarts = _oracle_ids(om, au, 2.0, continuous=True)
        n_restarts += len(restarts)
        assert ids[k] == ref, (k, len(ids[k]), len(ref))
    assert n_restarts > 0
    hm.close()
    om.close()


def test_scheduler_free_with_pending_chunk(tiny_weights, jfk_samples):
    """freeing the scheduler while an attached stream holds a deferred encoder
    chunk.  vh_sched_free detaches like vh_sched_detach (the chunk encoded in order, async
    encoding off), so the stream goes on unscheduled -- its later feeds decode on its own
    path -- and its ids equal the oracle's session on the same pieces."""
    import vox_hip
    from vox_weights import TINY_LONG
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    import vox_oracle
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    audio = np.ascontiguousarray(np.concatenate([jfk_samples] * 2)[:16000 * 9])
    ctx = vox_hip.HostCtx(hm)
    q = vox_hip.Scheduler(ctx, 4)
    s = vox_hip.HostStream(ctx, interval_s=0.5)
    q.attach(s)
    ids, pos = [], 0
    for tick in range(6):           # scheduled ticks
        s.feed(audio[pos:pos + PIECE])
        pos += PIECE
        q.run()
        ids += s.get()
    s.feed(audio[pos:pos + PIECE])  # a chunk deferred for a run that never comes
    pos += PIECE
    q.close()
    while pos < len(audio):         # unscheduled from here on
        s.feed(audio[pos:pos + PIECE])
        pos += PIECE
    s.finish()
    ids += s.get()
    s.close()
    ctx.close()
    ref, _ = _oracle_ids(om, audio, 0.5)
    assert ids == ref, (len(ids), len(ref))
    hm.close()
    om.close()


def test_scheduler_alt_stream_stays_batched(tiny_weights, jfk_samples):
    """A stream with alternatives (--alt, vox_stream_set_alt(3, 0.5)) is served by the batched
    steps with the others (no single-stream fallback): its records -- chosen id + accepted
    alternatives -- equal those of the same stream decoded alone (the single-stream path the CLI
    tests pin to stream_fill_alts), and the batched steps produced every id."""
    import vox_hip
    from vox_weights import TINY_LONG
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    a = np.concatenate([jfk_samples] * 2)
    audios = [np.ascontiguousarray(a[:16000 * 8]), np.ascontiguousarray(-a[3000:3000 + 16000 * 6]),
              np.ascontiguousarray(a[9000:9000 + 16000 * 7])]
    ctx = vox_hip.HostCtx(hm)
    q = vox_hip.Scheduler(ctx, 4)
    ss = [vox_hip.HostStream(ctx, interval_s=0.5) for _ in audios]
    ss[1].set_alt(3, 0.5)
    for s in ss:
        q.attach(s)
    recs = [[] for _ in audios]
    pos = [0] * len(audios)
    done = [False] * len(audios)
    while not all(done) or any(s.pending() for s in ss):
        for k, s in enumerate(ss):
            if done[k]:
                continue
            if pos[k] < len(audios[k]):
                s.feed(audios[k][pos[k]:pos[k] + PIECE])
                pos[k] += PIECE
            else:
                s.finish()
                done[k] = True
        q.run()
        for k, s in enumerate(ss):
            recs[k].append(s.get_alt())
    st = q.stats()
    for s in ss:
        q.detach(s)
        s.close()
    q.close()
    got = np.concatenate(recs[1])
    solo = vox_hip.HostStream(ctx, interval_s=0.5)
    solo.set_alt(3, 0.5)
    for i in range(0, len(audios[1]), PIECE):
        solo.feed(audios[1][i:i + PIECE])
    solo.finish()
    want = solo.get_alt()
    solo.close()
    ctx.close()
    assert got.shape == want.shape and got.shape[0] > 0, (got.shape, want.shape)
    np.testing.assert_array_equal(got, want)
    assert (got[:, 1] >= 0).any()
    assert st["tokens"] == sum(len(np.concatenate(r)) for r in recs), st
    hm.close()


@pytest.mark.slow
def test_scheduler_full_size_matches_oracle(jfk_samples):
    """The served composite at full Voxtral-4B shapes: three streams of
    3-5 s fed in 0.5 s pieces with staggered starts through one scheduler (cross-stream encoder
    passes, stacked prefills, slot-table batched steps, a step cap of 4 so prompts and flush
    paddings drain over later runs); every stream's ids equal its own oracle session on the
    same pieces."""
    import vox_hip
    import vox_oracle
    from vox_weights import VOXTRAL_4B, synth_weights
    w = synth_weights(VOXTRAL_4B, seed=0)
    hm = vox_hip.Model(VOXTRAL_4B, w)
    a = np.concatenate([jfk_samples] * 2)
    audios = [np.ascontiguousarray(a[:16000 * 5]), np.ascontiguousarray(-a[20000:20000 + 16000 * 4]),
              np.ascontiguousarray(a[70000:70000 + 16000 * 3])]
    ids, st = _serve(hm, audios, [0, 2, 3], 0.5, step_cap=4)
    hm.close()
    om = vox_oracle.OracleModel(VOXTRAL_4B, w)
    import os
    vox_oracle.set_threads(min(16, os.cpu_count() or 1))
    for k, au in enumerate(audios):
        ref, _ = _oracle_ids(om, au, 0.5)
        assert len(ref) > 20
        assert ids[k] == ref, (k, len(ids[k]), len(ref), next((i for i in range(min(len(ref), len(ids[k])))
                                                               if ids[k][i] != ref[i]), None))
    om.close()
    assert st["prefill_passes"] >= 1 and st["steps"] > 0
    print("full-size scheduler stats", st)


def test_host_stream_reset_reuses_like_fresh(tiny_weights, jfk_samples):
    """vh_stream_reset: a stream that served one clip, was detached and reset serves the next
    clip (scheduled, with another stream beside it) with the ids of a fresh stream -- the
    oracle's for that clip; bench.py --stagger reuses its streams this way."""
    import vox_hip
    import vox_oracle
    from vox_weights import TINY_LONG
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    long = np.concatenate([jfk_samples] * 2)
    clip1 = np.ascontiguousarray(long[:int(7.3 * 16000)])
    clip2 = np.ascontiguousarray(long[8000:8000 + int(9.1 * 16000)])
    other = np.ascontiguousarray(long[3000:3000 + int(6.0 * 16000)])
    ctx = vox_hip.HostCtx(hm)
    q = vox_hip.Scheduler(ctx, 4)
    q.set_step_cap(8)

    def serve(pairs):
        """pairs of (stream, audio): fed together, one vh_sched_run per tick, drained"""
        pos = [0] * len(pairs)
        fin = [False] * len(pairs)
        ids = [[] for _ in pairs]
        while not all(fin) or any(s.pending() for s, _ in pairs):
            for k, (s, a) in enumerate(pairs):
                if fin[k]:
                    continue
                if pos[k] < len(a):
                    s.feed(a[pos[k]:pos[k] + PIECE])
                    pos[k] += PIECE
                else:
                    s.finish()
                    fin[k] = True
            q.run()
            for k, (s, _) in enumerate(pairs):
                ids[k] += s.get()
        return ids

    a = vox_hip.HostStream(ctx, interval_s=0.5)
    b = vox_hip.HostStream(ctx, interval_s=0.5)
    q.attach(a)
    q.attach(b)
    got1, _ = serve([(a, clip1), (b, other)])
    q.detach(a)
    a.reset()
    b2 = vox_hip.HostStream(ctx, interval_s=0.5)
    q.detach(b)
    b.close()
    q.attach(a)
    q.attach(b2)
    got2, _ = serve([(a, clip2), (b2, other)])
    want1, _ = _oracle_ids(om, clip1, 0.5)
    want2, _ = _oracle_ids(om, clip2, 0.5)
    assert got1 == want1
    assert got2 == want2, (len(got2), len(want2))
    for s in (a, b2):
        q.detach(s)
        s.close()
    q.close()
    ctx.close()
    hm.close()
    om.close()


def _single_stream_ids(ctx, audio, interval):
    """The same pieces through one vh_stream_t with no scheduler: its own encoder chunks and the
    single-stream decode path (vox_hip_stream_decode, pinned to the oracle by test_gpu_full)."""
    import vox_hip
    s = vox_hip.HostStream(ctx, interval_s=interval)
    ids = []
    for i in range(0, len(audio), PIECE):
        s.feed(audio[i:i + PIECE])
        ids += s.get()
    s.finish()
    ids += s.get()
    s.close()
    return ids


def test_scheduler_full_size_16_streams_match_single_stream(jfk_samples):
    """The served mix the C4 bench runs, at full Voxtral-4B shapes (the
    full-size served parity had covered 3 short streams): 16 streams of 6-22 s, starts staggered
    by one tick, a step cap of 8 (bench.py --stagger), cross-stream encoder passes beside the
    slot-table batched steps; every stream's ids equal the same audio run alone through the
    single-stream path -- itself pinned to the CPU oracle at full size -- so the batched,
    stacked-prefill and overlapped machinery adds nothing of its own at this scale (an oracle
    run of all ~200 s of audio would take the CPU most of an hour).  The two shortest streams
    (6 s and 7 s) are also pinned to the CPU oracle directly."""
    import vox_hip
    import vox_oracle
    from vox_weights import VOXTRAL_4B, synth_weights
    w = synth_weights(VOXTRAL_4B, seed=0)
    hm = vox_hip.Model(VOXTRAL_4B, w)
    om = vox_oracle.OracleModel(VOXTRAL_4B, w)
    del w
    long = np.concatenate([jfk_samples] * 3)
    rng = np.random.default_rng(5)
    audios = []
    for k in range(16):
        n = int(16000 * (6 + (k * 7) % 17))
        off = int(rng.integers(0, len(long) - n))
        sign = -1.0 if k % 3 == 1 else 1.0
        audios.append(np.ascontiguousarray(sign * long[off:off + n] * (0.6 + 0.05 * (k % 8))))
    ids, st = _serve(hm, audios, list(range(16)), 0.5, max_streams=16, step_cap=8)
    ctx = vox_hip.HostCtx(hm)
    for k, au in enumerate(audios):
        ref = _single_stream_ids(ctx, au, 0.5)
        assert len(ref) > 40, (k, len(ref))
        assert ids[k] == ref, (k, len(ids[k]), len(ref), next((i for i in range(min(len(ref), len(ids[k])))
                                                               if ids[k][i] != ref[i]), None))
    ctx.close()
    hm.close()
    lens = [len(a) for a in audios]
    for k in sorted(range(16), key=lambda i: lens[i])[:2]:
        ref, _ = _oracle_ids(om, audios[k], 0.5)
        assert ids[k] == ref, ("oracle", k, len(ids[k]), len(ref))
    om.close()
    assert st["steps"] > 0 and st["tokens"] / st["steps"] > 4, st
    print("16-stream full-size scheduler stats", st)


def test_scheduler_32_streams_match_oracle(tiny_weights, jfk_samples):
    """32 streams on one scheduler (VH_SCHED_MAX; the batched steps' second 16-row block, the
    cross-stream encoder pass over 32 streams' chunks, stacked prefills in groups): two streams
    start per tick, 8-12 s each, so all 32 are live together; a step cap of 8 as bench.py
    --stagger; every stream's ids = its oracle session."""
    import vox_hip
    import vox_oracle
    from vox_weights import TINY_LONG
    hm = vox_hip.Model(TINY_LONG, tiny_weights)
    om = vox_oracle.OracleModel(TINY_LONG, tiny_weights)
    long = np.concatenate([jfk_samples] * 2)
    audios = []
    for k in range(32):
        n = int(16000 * (8.0 + 0.5 * (k % 9)))
        off = (k * 7919) % (len(long) - n)
        audios.append(np.ascontiguousarray(long[off:off + n]))
    ids, st = _serve(hm, audios, [k // 2 for k in range(32)], 0.5, max_streams=32, step_cap=8)
    for k, a in enumerate(audios):
        ref, _ = _oracle_ids(om, a, 0.5)
        assert len(ref) > 0
        assert ids[k] == ref, (k, len(ids[k]), len(ref))
    assert st["tokens"] / max(1, st["steps"]) > 8, st
    print("32-stream scheduler stats", st)
    hm.close()
    om.close()
