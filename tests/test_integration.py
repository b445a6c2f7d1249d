"""The call-site patch of INTEGRATION.md against the reference's own headers: the binding
(integration/voxtral_hip_glue.c) must compile as C99 with -Wall -Wextra -Werror against
voxtral.h / voxtral_kernels.h where they lie, and reference nothing but the C ABI of
include/voxtral_hip.h, the reference's vox_compute_rope_freqs and libc.  Skipped where the
reference tree is absent (the GPU box)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "voxtral.h")), reason="reference tree absent")
def test_glue_compiles_against_reference_headers(tmp_path):
    obj = tmp_path / "glue.o"
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-DUSE_HIP", f"-I{REF}",
                    f"-I{ROOT}/include", "-c", f"{ROOT}/integration/voxtral_hip_glue.c", "-o", str(obj)],
                   check=True)
    out = subprocess.run(["nm", str(obj)], check=True, capture_output=True, text=True).stdout
    defined = set(re.findall(r" T (\w+)", out))
    undef = set(re.findall(r" U (\w+)", out))
    header = open(os.path.join(ROOT, "integration", "voxtral_hip_glue.h")).read()
    declared = set(re.findall(r"\b(vox_hip_bind_\w+)\s*\(", header))
    assert declared and declared == defined, (declared, defined)
    abi = open(os.path.join(ROOT, "include", "voxtral_hip.h")).read()
    abi_funcs = set(re.findall(r"\b(vox_hip_\w+)\s*\(", abi))
    foreign = {u for u in undef if u.startswith("vox_") and u not in abi_funcs}
    assert foreign == {"vox_compute_rope_freqs"}, foreign
    assert {"vox_hip_model_create", "vox_hip_encoder_full_step", "vox_hip_decoder_prefill_step",
            "vox_hip_decoder_full_step", "vox_hip_model_set_kv_fp16"} <= undef
