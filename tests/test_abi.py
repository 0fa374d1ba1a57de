"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports
every entry point include/roms_gpu.h declares, and its field table matches the
header enum.  No compute calls (no GPU in this container)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "roms_gpu.h")
LIB = os.path.join(ROOT, "ucla-roms_amd", "libromsgpu.so")


def _declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"\b(roms_gpu_\w+)\s*\(", src)))


def test_header_declares_routine_entries():
    names = _declared()
    for r in ("rho_eos", "set_huv", "omega", "lmd_vmix", "prsgrd", "pre_step3d", "set_huv1", "step3d_uv1",
              "visc3d", "step2d", "step3d_uv2", "step3d_t", "t3dmix", "set_depth", "step", "init", "finalize",
              "register", "upload", "download"):
        assert "roms_gpu_" + r in names


@pytest.mark.skipif(not os.path.exists(LIB), reason="libromsgpu.so not built")
def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    missing = [n for n in _declared() if n not in exported]
    assert not missing, missing
    L = ctypes.CDLL(LIB)
    assert L.roms_gpu_abi_version() == 4


@pytest.mark.skipif(not os.path.exists(LIB), reason="libromsgpu.so not built")
def test_field_table_matches_header():
    import romsgpu
    src = open(HDR).read()
    body = src[src.index("enum roms_field"):src.index("ROMS_NFIELDS")]
    ids = re.findall(r"ROMS_(\w+)", body)
    ids = [i for i in ids if i != "ALL"]
    assert ids == romsgpu.FIELDS


@pytest.mark.skipif(not os.path.exists(LIB), reason="libromsgpu.so not built")
def test_uninitialised_calls_fail_loudly():
    import romsgpu
    m = romsgpu.Model()
    with pytest.raises(romsgpu.RomsGpuError):
        m.omega()
