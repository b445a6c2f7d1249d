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
            "vox_hip_decoder_full_step", "vox_hip_model_set_kv_fp16", "vox_hip_sgemm_bf16",
            "vox_hip_sgemm_q8"} <= undef
    # no per-process state: the weight tables of a load live on the heap
    assert not re.search(r" [bBdD] ", out), out


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "voxtral_kernels.c")), reason="reference tree absent")
def test_kernels_hunks_call_the_glue(tmp_path):
    """Every `USE_HIP` hunk INTEGRATION.md adds to voxtral_kernels.c sits right after one of the
    six `USE_METAL` branches it mirrors, and its call type-checks: each hunk's statement is
    compiled inside a function with the reference function's own parameter list (taken from
    voxtral_kernels.h), against the glue header."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    hunks = re.findall(r"--- voxtral_kernels.c\s+\((\w+), after its USE_METAL block, :(\d+)\)\n@@[^\n]*\n"
                       r"\+#ifdef USE_HIP\n\+(.*?)\n\+#endif", doc)
    names = [h[0] for h in hunks]
    assert names == ["vox_linear_nobias_bf16", "vox_linear_bf16", "vox_matmul_t_bf16", "vox_linear_nobias_q8",
                     "vox_linear_q8", "vox_matmul_t_q8"], names
    src = open(os.path.join(REF, "voxtral_kernels.c")).read().splitlines()
    hdr = open(os.path.join(REF, "voxtral_kernels.h")).read()
    lines = ['#include "voxtral_hip_glue.h"', '#include "voxtral_kernels.h"']
    for name, line, stmt in hunks:
        # the anchor line closes that function's USE_METAL block
        body = "\n".join(src[:int(line)])
        assert src[int(line) - 1].strip() == "#endif", (name, line)
        assert re.findall(r"^void\s+(\w+)\s*\(", body, re.M)[-1] == name, (name, line)
        proto = re.search(r"void\s+" + name + r"\s*\(([^)]*)\)\s*;", hdr, re.S)
        assert proto, name
        lines.append(f"void hunk_{name}({proto.group(1)}) {{\n{stmt}\n}}")
    c = tmp_path / "hunks.c"
    c.write_text("\n".join(lines) + "\n")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "-DUSE_HIP",
                    f"-I{REF}", f"-I{ROOT}/include", f"-I{ROOT}/integration", "-c", str(c), "-o",
                    str(tmp_path / "hunks.o")], check=True)
