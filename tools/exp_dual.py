"""Experiment (round 6): C4 pre-encoded batched decode as one batch of S rows against two
batches of S/2 rows decoded concurrently from two host threads (two batch queues), so that one
half's latency-bound phases (row kernels, attention, launch ramps) can overlap the other half's
weight streaming.  Prints one JSON line per mode: ids, wall, tok/s, and whether the ids equal
the single-batch ids.  Usage: python tools/exp_dual.py [S] [reps]"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "voxtral.c_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import vox_hip  # noqa: E402
from vox_weights import VOXTRAL_4B, synth_weights  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    vox_hip.init(device=0)
    cfg = VOXTRAL_4B
    w = synth_weights(cfg, seed=0)
    model = vox_hip.Model(cfg, w)
    del w
    rng = np.random.default_rng(1234)
    streams = [vox_hip.Stream(model) for _ in range(S)]
    mels = [vox_hip.DeviceArray(rng.uniform(-0.6, 1.4, size=(sum(bench.JFK_CHUNKS), cfg.mel_bins)).astype(np.float32))
            for _ in range(S)]

    def prep():
        for st, md in zip(streams, mels):
            st.reset()
            off = 0
            for n in bench.JFK_CHUNKS:
                st.encode_mel_device(md.ptr + off * cfg.mel_bins * 4, n)
                off += n
        for st in streams:
            st.decode(max_steps=1, stop_at_eos=False)
        for st in streams:
            st.sync()

    full = vox_hip.Batch(model, S)
    halves = [vox_hip.Batch(model, S // 2), vox_hip.Batch(model, S // 2)]
    ref = None

    def run_single():
        prep()
        t0 = time.perf_counter()
        r = full.decode(streams, max_steps=1 << 16, stop_at_eos=False)
        return time.perf_counter() - t0, r

    def run_dual():
        prep()
        out = [None, None]
        go = threading.Barrier(3)

        def worker(i):
            go.wait()
            out[i] = halves[i].decode(streams[i * (S // 2):(i + 1) * (S // 2)], max_steps=1 << 16, stop_at_eos=False)

        th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        return time.perf_counter() - t0, out[0] + out[1]

    warm = set()
    for mode, fn in (("single", run_single), ("dual", run_dual)) * (reps + 1):
        dt, r = fn()
        ids = sum(len(x) for x in r)
        if ref is None:
            ref = r
        if mode not in warm:
            warm.add(mode)
            continue  # warm-up (graph captures)
        same = all(np.array_equal(a, b) for a, b in zip(r, ref))
        print(json.dumps({"mode": mode, "S": S, "ids": ids, "wall_s": round(dt, 4),
                          "tok_s": round(ids / dt, 1), "ms_per_row_step": round(dt * 1000 * S / ids, 4),
                          "ids_equal_single": same}), flush=True)
    for b in [full] + halves:
        b.close()
    for m in mels:
        m.free()
    for s in streams:
        s.close()
    model.close()


if __name__ == "__main__":
    main()
