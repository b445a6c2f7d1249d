"""The M > 1 attention kernel (k_attn_mf, f32 MFMA; with the key-range split + combine for
few query rows) through the vox_hip_encoder_attention twin, against a plain PyTorch fp32
statement of vox_causal_attention (voxtral_kernels.c:541-611: query i at position
q_offset + i sees keys max(0, qp - window + 1) .. qp; GQA head h reads kv head
h / (n_heads / n_kv_heads)) and against the CPU oracle.  Tolerance: 2e-5 of the largest
output magnitude (f32 products in both; only the summation order differs)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def torch_attention(Q, K, V, n_heads, n_kv, hd, window, q_offset):
    import torch
    q = torch.from_numpy(Q).view(-1, n_heads, hd).transpose(0, 1)          # [H, Mq, hd]
    k = torch.from_numpy(K).view(-1, n_kv, hd).transpose(0, 1)             # [KV, Mk, hd]
    v = torch.from_numpy(V).view(-1, n_kv, hd).transpose(0, 1)
    rep = n_heads // n_kv
    k = k.repeat_interleave(rep, 0)
    v = v.repeat_interleave(rep, 0)
    s = (q @ k.transpose(1, 2)) * (1.0 / np.sqrt(hd))
    qp = torch.arange(Q.shape[0])[:, None] + q_offset
    kp = torch.arange(K.shape[0])[None, :]
    lo = qp - window + 1 if window > 0 else torch.zeros_like(qp) - (1 << 30)
    ok = (kp <= qp) & (kp >= lo)
    s = s.masked_fill(~ok, float("-inf"))
    o = torch.softmax(s, dim=-1) @ v                                       # [H, Mq, hd]
    return o.transpose(0, 1).reshape(Q.shape[0], n_heads * hd).numpy()


CASES = [
    # (seq_q, seq_k, n_heads, n_kv, head_dim, window, q_offset)
    (1, 1, 4, 4, 64, 0, 0),
    (5, 40, 4, 2, 64, 0, 35),          # GQA, short range, one block
    (25, 775, 32, 32, 64, 750, 750),   # streaming encoder chunk: key-range splits + combine
    (26, 800, 8, 8, 64, 750, 774),     # ragged rows, window cut
    (70, 300, 8, 8, 64, 750, 230),     # several 16-query blocks
    (70, 819, 4, 4, 64, 750, 749),     # 70 rows over a full 750 window: the most key splits (12) + combine
    (38, 38, 32, 8, 128, 8192, 0),     # decoder prefill shape (head_dim 128, GQA 4)
    (17, 600, 32, 8, 128, 0, 583),     # head_dim 128 with splits
    (200, 200, 4, 4, 64, 24, 0),       # window much shorter than the rows
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "q%d_k%d_h%d_kv%d_d%d_w%d" % c[:6])
def test_attention_matches_torch_and_oracle(case):
    import vox_hip
    import vox_oracle
    mq, mk, h, kv, hd, window, q_off = case
    rng = np.random.default_rng(mq * 1000 + mk)
    Q = rng.standard_normal((mq, h * hd), dtype=np.float32)
    K = rng.standard_normal((mk, kv * hd), dtype=np.float32)
    V = rng.standard_normal((mk, kv * hd), dtype=np.float32)
    got = vox_hip.encoder_attention(Q, K, V, h, kv, hd, window, q_off)
    ref = torch_attention(Q, K, V, h, kv, hd, window, q_off)
    tol = 2e-5 * float(np.abs(ref).max())
    assert np.abs(got - ref).max() <= tol
    orc = vox_oracle.causal_attention(Q, K, V, h, kv, hd, window, q_off)
    assert np.abs(got - orc).max() <= tol
