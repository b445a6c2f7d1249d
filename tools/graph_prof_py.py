"""Which graph replays does rocprofv3 --kernel-trace survive?  (the C2 bench
ends in SIGSEGV under rocprofv3 inside hipGraphLaunch.)  One mode per process, TINY shapes:
  plain  -- single-stream decode, step graphs replayed, no profiling events
  prof   -- the same with Stream.set_profiling(True): the last step of each batch launched
            eagerly through hipExtLaunchKernel with dispatch-recorded events, as bench.py does
  batch  -- the batched decode's slot-table step graphs
  full   -- plain at the full Voxtral-4B shapes (synthetic weights, 200 graph-replayed steps)
  fullbatch -- the batched decode at the full shapes: 16 streams of a 1355-frame chunk each,
            148 graph-replayed batched steps (C4's pre-encoded step)
  fullprof -- full with Stream.set_profiling(True) (bench.py's roofline pass)
Run: rocprofv3 --kernel-trace --stats -d DIR -o x -- python3 tools/graph_prof_py.py MODE"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "voxtral.c_amd"))
import vox_hip  # noqa: E402
from vox_weights import TINY, VOXTRAL_4B, synth_weights  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
# the process's mappings, so a crash's frame addresses can be put to library + offset and
# symbolised afterwards (llvm-symbolizer --obj=LIB OFFSET on the same image)
maps_out = os.environ.get("VOX_GP_MAPS")
cfg = VOXTRAL_4B if mode.startswith("full") else TINY
w = synth_weights(cfg, seed=1)
m = vox_hip.Model(cfg, w)
del w
rng = np.random.default_rng(0)
nst, nfr = (16, 1355) if mode == "fullbatch" else (4, 900)
mels = [rng.uniform(-0.5, 1.5, size=(nfr, cfg.mel_bins)).astype(np.float32) for _ in range(nst)]


def dump_maps():
    if maps_out:
        with open("/proc/self/maps") as f, open(maps_out, "w") as o:
            o.write(f.read())


dump_maps()
if mode in ("batch", "fullbatch"):
    ss = [vox_hip.Stream(m) for _ in mels]
    for s, mel in zip(ss, mels):
        s.encode_mel(mel)
    b = vox_hip.Batch(m, len(ss))
    n = sum(len(t) for t in b.decode(ss, max_steps=148 if mode == "fullbatch" else 1000, stop_at_eos=False))
    b.close()
    for s in ss:
        s.close()
else:
    st = vox_hip.Stream(m)
    st.encode_mel(mels[0])
    if mode in ("prof", "fullprof"):
        st.set_profiling(True)
    dump_maps()  # every library the decode loads is mapped by now
    n = len(st.decode(max_steps=200, stop_at_eos=False)) if mode.startswith("full") else len(st.decode(stop_at_eos=False))
    st.close()
m.close()
print(f"{mode}: {n} tokens, exited cleanly", flush=True)
