"""CPU: the C-ABI library loads and exports every entry point include/voxtral_hip.h declares
(no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

pytestmark = pytest.mark.cpu
HEADER = os.path.join(ROOT, "include", "voxtral_hip.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vox_hip_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared()
    # the reference-boundary twins of voxtral_metal.h must all be there
    for n in ["vox_hip_init", "vox_hip_available", "vox_hip_shutdown", "vox_hip_sgemm_bf16",
              "vox_hip_fused_qkv_bf16", "vox_hip_fused_ffn_bf16", "vox_hip_encoder_attention",
              "vox_hip_encoder_full_step", "vox_hip_decoder_prefill_step", "vox_hip_decoder_start",
              "vox_hip_decoder_full_step", "vox_hip_decoder_end", "vox_hip_memory_used"]:
        assert n in names, n


def test_library_exports_every_declared_symbol():
    import vox_hip
    lib = ctypes.CDLL(vox_hip.LIB_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(vox_hip.EXPORTS) == declared()


def test_library_is_gfx950_code_object():
    import vox_hip
    data = open(vox_hip.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_host_library_exports_vox_hip_host_h():
    """libvox_hip_host.so (the C host side) exports every vh_* entry point its header declares."""
    src = open(os.path.join(ROOT, "include", "vox_hip_host.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = sorted(set(re.findall(r"\b(vh_[a-z0-9_]+)\s*\(", src)))
    assert len(names) >= 12
    lib = ctypes.CDLL(os.path.join(ROOT, "voxtral.c_amd", "libvox_hip_host.so"))
    assert not [n for n in names if not hasattr(lib, n)]
