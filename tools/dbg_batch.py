import sys, numpy as np
sys.path.insert(0, "voxtral.c_amd")
import vox_hip
from vox_weights import VOXTRAL_4B, synth_weights
w = synth_weights(VOXTRAL_4B, seed=0)
hm = vox_hip.Model(VOXTRAL_4B, w)
rng = np.random.default_rng(42)
mels = [rng.uniform(-0.6, 1.4, size=(n, 128)).astype(np.float32) for n in (1496, 1496, 1200)]
def fresh(mel):
    s = vox_hip.Stream(hm); s.encode_mel(mel); a = s.read_adapter(); t = s.decode(stop_at_eos=False).tolist(); s.close(); return t, a
ref = [fresh(m) for m in mels]
print("fresh", [(len(r[0]), r[0][:3]) for r in ref], flush=True)
ss = [vox_hip.Stream(hm) for _ in mels]
for s, m in zip(ss, mels): s.encode_mel(m)
b = vox_hip.Batch(hm, 4)
got = b.decode(ss, max_steps=1000, stop_at_eos=False)
print("batch", [(len(g), g[:3].tolist(), g.tolist() == r[0]) for g, r in zip(got, ref)], flush=True)
for i, m in enumerate(mels):
    t, a = fresh(m)
    print("after", i, len(t), t[:3], t == ref[i][0], float(np.abs(a - ref[i][1]).max()), flush=True)
for s in ss: s.close()
b.close()
for i, m in enumerate(mels):
    t, a = fresh(m)
    print("after close", i, len(t), t[:3], t == ref[i][0], float(np.abs(a - ref[i][1]).max()), flush=True)
