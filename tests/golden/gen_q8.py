"""Generate tests/golden/q8_ref.json with the reference's own quantizer.

/root/reference/quantize.py is run unmodified, as a subprocess, on a TINY synthetic bf16
checkpoint written by vox_weights.write_safetensors.  Two rows of one matrix are set by
hand so that the quantizer's edge cases appear: an all-zero row (scale 0, quantize.py:38-40)
and a row whose scaled values fall exactly on .5 ties (np.round is round-half-to-even,
quantize.py:43).  The fixture keeps, per output tensor, its dtype, shape and the sha256 of
its data bytes (Q8: f32 scales then int8 rows, quantize.py:121; F32: the values), the two
crafted rows in full, and the sha256 / length of the whole output file (the unaligned
quantize.py layout, :152-186).  tests/test_q8_cpu.py rebuilds the same checkpoint from the seed
and checks vox_weights.quantize_q8 against every hash.

Run here (needs /root/reference):  python3 tests/golden/gen_q8.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "voxtral.c_amd"))
import vox_weights as vw  # noqa: E402

REF = "/root/reference/quantize.py"
SEED = 5
EDGE_TENSOR = "layers.0.attention.wk.weight"
ZERO_ROW, TIE_ROW = 3, 4
# scale = 127 * 2^-6 / 127 = 2^-6 exactly, so row / scale lands on these values
TIE_VALUES = [127.0, 0.5, 1.5, 2.5, -0.5, -1.5, -2.5, 126.5, -126.5, -127.0, 3.5, -3.5]


def fixture_weights():
    w = vw.synth_weights(vw.TINY, seed=SEED)
    a = w.t[EDGE_TENSOR]
    a[ZERO_ROW, :] = 0
    row = np.zeros(a.shape[1], np.float32)
    row[:len(TIE_VALUES)] = np.array(TIE_VALUES, np.float32) * 2.0 ** -6
    a[TIE_ROW, :] = vw.f32_to_bf16(row)
    return w


def tensor_digest(dtype, parts):
    h = hashlib.sha256()
    for p in parts:
        h.update(np.ascontiguousarray(p).tobytes())
    return h.hexdigest()


def main():
    w = fixture_weights()
    with tempfile.TemporaryDirectory() as td:
        src, dst = os.path.join(td, "bf16"), os.path.join(td, "q8")
        os.makedirs(src)
        vw.write_safetensors(w, os.path.join(src, "consolidated.safetensors"))
        subprocess.run([sys.executable, REF, src, dst], check=True, stdout=subprocess.DEVNULL)
        qpath = os.path.join(dst, "consolidated.safetensors")
        q = vw.load_safetensors(qpath, vw.TINY)
        raw = open(qpath, "rb").read()
        out = {"seed": SEED, "edge_tensor": EDGE_TENSOR, "zero_row": ZERO_ROW, "tie_row": TIE_ROW,
               "tensors": {}, "file_sha256": hashlib.sha256(raw).hexdigest(), "file_bytes": len(raw),
               "header_bytes": int.from_bytes(raw[:8], "little")}
        for name, (sc, qq) in q.q8.items():
            out["tensors"][name] = {"dtype": "Q8", "shape": list(qq.shape),
                                    "sha256": tensor_digest("Q8", [sc, qq])}
        for name, a in q._stored_f32.items():
            out["tensors"][name] = {"dtype": "F32", "shape": list(a.shape),
                                    "sha256": tensor_digest("F32", [a])}
        sc, qq = q.q8[EDGE_TENSOR]
        out["zero_row_scale"] = float(sc[ZERO_ROW])
        out["tie_row_scale"] = float(sc[TIE_ROW])
        out["tie_row_q"] = qq[TIE_ROW, :len(TIE_VALUES)].tolist()
    with open(os.path.join(HERE, "q8_ref.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(len(out["tensors"]), "tensors; tie row", out["tie_row_q"])


if __name__ == "__main__":
    main()
