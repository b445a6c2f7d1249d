"""Debug: device mel vs reference fixture, error by frame."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "voxtral.c_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import vox_hip, vox_oracle
from vox_weights import TINY, synth_weights
from test_gpu_mel import _run_device_mel
ref = np.load(os.path.join(ROOT, "tests/golden/ref_mel.npz"))
jfk = vox_oracle.read_wav(os.path.join(ROOT, "tests/golden/jfk.wav"))
hm = vox_hip.Model(TINY, synth_weights(TINY, seed=1)); st = vox_hip.Stream(hm)
got, counts = _run_device_mel(st, jfk, [len(jfk)])
r = ref["jfk_finish"]
e = np.abs(got - r)
print("max", e.max(), "argmax frame/bin", np.unravel_index(e.argmax(), e.shape))
pf = e.max(axis=1)
for t in np.argsort(-pf)[:10]:
    b = e[t].argmax()
    print(t, b, got[t, b], r[t, b], pf[t])
print("frames with err>2e-6:", int((pf > 2e-6).sum()), "of", len(pf))
print("bins with err>2e-6:", np.unique(np.where(e > 2e-6)[1])[:40])
