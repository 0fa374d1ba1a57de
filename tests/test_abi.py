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
    want = int(re.search(r"#define ROMS_GPU_ABI_VERSION (\d+)", open(HDR).read()).group(1))
    assert L.roms_gpu_abi_version() == want


def test_ctypes_structs_match_header_layout(tmp_path):
    """The Python mirrors (romsgpu.Dims/Cfg/Tlev/Case) have the C structs'
    size and field offsets (compiled against include/roms_gpu.h here)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "ucla-roms_amd"))
    import romsgpu
    structs = {"roms_dims": romsgpu.Dims, "roms_cfg": romsgpu.Cfg, "roms_tlev": romsgpu.Tlev,
               "roms_case": romsgpu.Case}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "roms_gpu.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append('  printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for fname, _ in py._fields_:
            lines.append('  printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, fname, cname, fname))
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n") if l)
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got["%s.%s" % (cname, fname)]) == getattr(py, fname).offset, (cname, fname)


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


def test_fortran_module_abi_version_matches_header():
    """fortran/roms_gpu_mod.F90's ROMS_GPU_ABI must follow ROMS_GPU_ABI_VERSION."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    h = open(os.path.join(root, "include", "roms_gpu.h")).read()
    f = open(os.path.join(root, "fortran", "roms_gpu_mod.F90")).read()
    vh = int(re.search(r"#define ROMS_GPU_ABI_VERSION (\d+)", h).group(1))
    vf = int(re.search(r"ROMS_GPU_ABI = (\d+)", f).group(1))
    assert vh == vf


@pytest.mark.skipif(not os.path.exists(LIB), reason="libromsgpu.so not built")
def test_init_refuses_subdomain_beyond_buffer_offsets():
    """The buffer-addressed kernels use 32-bit byte offsets below 2 GiB per
    field (k_common.h BufF64): roms_gpu_init refuses a rank whose w-point
    field reaches that (2048^2 x 100 on one rank: 3.4 GiB) with a clear error,
    before touching the device, instead of dropping accesses."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "ucla-roms_amd"))
    import romsgpu
    L = romsgpu.load_library()
    cfg = romsgpu.Cfg()
    cfg.nfast, cfg.ndtfast, cfg.dt = 82, 60, 300.0
    for (n, ok) in ((2048, False), (1024, True)):
        dims = romsgpu.Dims(Lm=n, Mm=n, N=100, NT=2, LLm=n, MMm=n, np_xi=1, np_eta=1)
        rc = L.roms_gpu_init(ctypes.byref(dims), ctypes.byref(cfg), 0, None)
        err = L.roms_gpu_last_error().decode()
        if ok:   # gets past the guard; without a GPU the device call then fails
            assert "2 GiB" not in err, err
        else:
            assert rc == -1 and "2 GiB" in err, (rc, err)
