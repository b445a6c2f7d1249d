"""The opt-in persistent decode step (VOX_HIP_PSTEP=1, csrc/vox_hip_pstep.hip: every decoder
layer of a step in one launch) against the CPU oracle: TINY weights, a decode long enough
for the 48-key window to wrap, and TINY_LONG up to the 256-key in-launch attention limit
(the per-operation graph takes over past it).  The switch is read once per process, so the
check runs in a child process.  Bars as test_gpu_tiny: identical greedy ids, logits within
5e-5 of the largest magnitude."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, {pkg!r})
sys.path.insert(0, {orc!r})
import vox_hip, vox_oracle
from vox_weights import TINY, TINY_LONG, synth_weights

def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))

for cfg, frames, steps in ((TINY, 400, 60), (TINY_LONG, 1100, 200)):
    w = synth_weights(cfg, seed=1)
    mel = np.random.default_rng(0).uniform(-0.5, 1.5, size=(frames, cfg.mel_bins)).astype(np.float32)
    hm = vox_hip.Model(cfg, w)
    hs = vox_hip.Stream(hm)
    hs.encode_mel(mel)
    toks, logits = hs.decode(max_steps=steps, stop_at_eos=False, want_logits=True)
    om = vox_oracle.OracleModel(cfg, w)
    os_ = vox_oracle.OracleStream(om)
    os_.encode_mel(mel)
    otoks, ologits = os_.decode(max_steps=steps, stop_at_eos=False, want_logits=True)
    assert len(toks) == len(otoks) > 0, (len(toks), len(otoks))
    assert np.array_equal(toks, otoks), (cfg.dec_window, toks, otoks)
    err = rel(logits, ologits)
    assert err < 5e-5, err
    print("pstep", cfg.dec_window, len(toks), "tokens match, max rel logit err", err)
    hs.close(); hm.close(); os_.close(); om.close()
"""


def test_persistent_step_matches_oracle():
    code = CHILD.format(pkg=os.path.join(ROOT, "voxtral.c_amd"), orc=os.path.join(ROOT, "oracle"))
    env = dict(os.environ, VOX_HIP_PSTEP="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("tokens match") == 2, r.stdout
