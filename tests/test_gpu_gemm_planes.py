"""The M > 1 GEMMs' activation planes (csrc/vox_hip_kernels.hip, gemm_planes): the default
exact three-plane split (hi + mid + lo = the f32 value, so only summation order differs from
the reference's sgemm, voxtral_kernels.c:197-240) and the approximate two-plane split
(VOX_HIP_GEMM_PLANES=2: hi + lo, ~2^-18 relative per activation).  The switch is read once per process, so
each mode runs in a child process: the sgemm twin at encoder / prefill shapes against an f64
statement of the same product, and the TINY jfk transcription against the oracle.  Bars:
identical ids; 2e-6 (sgemm) and 1e-5 (pipeline) for the exact default, 5e-5 of the largest
magnitude for the two-plane split."""
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
from vox_weights import TINY, synth_weights

def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))

rng = np.random.default_rng(3)
worst = 0.0
for M, N, K in ((677, 2048, 1280), (38, 3072, 3072), (100, 1280, 5120)):
    A = rng.standard_normal((M, K)).astype(np.float32)
    Wf = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
    Wb = (Wf.view(np.uint32) >> 16).astype(np.uint16)
    ref = A.astype(np.float64) @ (Wb.astype(np.uint32) << 16).view(np.float32).astype(np.float64).T
    got = vox_hip.sgemm_bf16(A, Wb)
    worst = max(worst, rel(got, ref))
print("sgemm", worst)
assert worst < {sgemm_tol}, worst

w = synth_weights(TINY, seed=1)
hm = vox_hip.Model(TINY, w)
om = vox_oracle.OracleModel(TINY, w)
samples = vox_oracle.read_wav({wav!r})
events = vox_oracle.transcribe_mel_schedule(samples)
hs, os_ = vox_hip.Stream(hm), vox_oracle.OracleStream(om)
h_tok, o_tok, h_log, o_log = [], [], [], []
for kind, mel in events:
    for s, toks, logs in ((hs, h_tok, h_log), (os_, o_tok, o_log)):
        cur = {{"feed": 0, "flush": events[0][1].shape[0], "finish": events[1][1].shape[0]}}[kind]
        s.encode_mel(mel[cur:])
        t, l = s.decode(stop_at_eos=False, want_logits=True)
        toks += t.tolist()
        logs.append(l.copy())
assert h_tok == o_tok and len(o_tok) > 0
ra = rel(hs.read_adapter(), os_.read_adapter())
err = rel(np.concatenate(h_log), np.concatenate(o_log))
print("pipeline", len(h_tok), "tokens match, adapter", ra, "logits", err)
assert ra < {pipe_tol} and err < {pipe_tol}, (ra, err)
hs.close(); os_.close(); hm.close(); om.close()
"""


@pytest.mark.parametrize("planes,sgemm_tol,pipe_tol", [("2", 5e-5, 5e-5), ("3", 2e-6, 1e-5)])
def test_gemm_planes_mode(planes, sgemm_tol, pipe_tol):
    code = CHILD.format(pkg=os.path.join(ROOT, "voxtral.c_amd"), orc=os.path.join(ROOT, "oracle"),
                        wav=os.path.join(ROOT, "tests", "golden", "jfk.wav"), sgemm_tol=sgemm_tol, pipe_tol=pipe_tol)
    env = dict(os.environ, VOX_HIP_GEMM_PLANES=planes)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "tokens match" in r.stdout, r.stdout
    print(r.stdout)
