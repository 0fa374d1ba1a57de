"""Fortran host side (fortran/): the iso_c_binding module and a driver
program over the C ABI build with amdflang (CPU), and on the GPU the driver
reproduces the reference Filament golden log (benchmark.result_github_gnu)
within the reduction-order tolerance of a single-rank run."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FDIR = os.path.join(ROOT, "fortran")


def test_fortran_module_and_driver_build():
    r = subprocess.run(["make", "-C", FDIR], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.exists(os.path.join(FDIR, "filament_driver"))


def test_dropins_keep_reference_signatures():
    """Every hot-path routine has a drop-in with the reference's name and
    argument list (no-arg / tile / tidx / tind)."""
    want = {"step2d": "", "prsgrd": "", "omega": "", "set_HUV": "", "visc3d": "", "t3dmix": "",
            "pre_step3d": "tile", "set_HUV1": "tile", "step3d_uv1": "tile", "step3d_uv2": "tile",
            "step3d_t": "tile", "set_depth": "tile", "rho_eos": "tidx", "lmd_vmix": "tind",
            "swr_frac": "tile"}
    for name, arg in want.items():
        src = open(os.path.join(FDIR, "dropin", name + ".F")).read()
        head = "subroutine %s%s" % (name, "(%s)" % arg if arg else "")
        assert head in src, name
        assert "roms_gpu_%s(" % name.lower() in src, name


@pytest.mark.gpu
def test_fortran_driver_matches_golden():
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "filament_github_gnu.json")))["rows"]
    exe = os.path.join(FDIR, "filament_driver")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", FDIR], check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe, "20"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    rows = [list(map(float, ln.split()[1:])) for ln in r.stdout.strip().splitlines()]
    assert len(rows) == 21
    for s, (g, row) in enumerate(zip(gold, rows)):
        for key, val in zip(("ke", "ke2b", "cu_adv"), row[:3]):
            ref = float(g[key])
            assert abs(val - ref) <= 1e-11 * abs(ref), (s, key, val, ref)
