"""netCDF classic (CDF-2) files of the restart/history writer, on the CPU.

The reference writes its restart/history files through the netCDF library
(basic_output.F, roms_read_write.F:1161-1208) and reads them with nf90_open
(get_init.F), which accepts every netCDF format.  The library writes the
64-bit-offset classic format natively (ucla-roms_amd/csrc/ncio.cpp); an
independent reader of that format -- scipy.io.netcdf_file -- checks the files
it writes, and files scipy writes are read back through ncio's reader.
"""
import os
import subprocess

import numpy as np
import pytest
from scipy.io import netcdf_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def tool(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("ncio") / "ncio_roundtrip")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "ncio_roundtrip.cpp"),
                    os.path.join(ROOT, "ucla-roms_amd", "csrc", "ncio.cpp")], check=True)
    return exe


def val(rec, idx):
    return rec * 1000.0 + idx + 0.25


def test_written_file_reads_with_scipy(tool, tmp_path):
    p = str(tmp_path / "rt.nc")
    subprocess.run([tool, "write", p], check=True)
    with open(p, "rb") as f:
        assert f.read(4) == b"CDF\x02"
    with netcdf_file(p, "r", mmap=False) as nc:
        assert nc.version_byte == 2
        assert nc.dimensions["xi_rho"] == 5 and nc.dimensions["eta_rho"] == 3 and nc.dimensions["s_rho"] == 2
        assert nc.dimensions["time"] is None          # the record dimension
        assert list(nc.partition) == [1, 4, 7, 9]
        assert nc.title == b"ncio round trip" and nc.dt == 300.0
        assert np.array_equal(nc.variables["h"][:], 100.0 + np.arange(15.0).reshape(3, 5))
        assert nc.variables["h"].units == b"meter"
        assert nc.variables["ocean_time"][:].tolist() == [0.0, 300.0, 600.0, 900.0]
        ts = nc.variables["time_step"][:]
        assert ts.shape == (4, 6) and ts[:, 0].tolist() == [1, 2, 3, 4]
        z = nc.variables["zeta"][:]
        u = nc.variables["u"][:]
        assert z.shape == (4, 3, 5) and u.shape == (4, 2, 3, 5)
        for r in range(4):   # records 0-2 at creation, 3 appended after reopening
            assert np.array_equal(z[r].ravel(), val(r, np.arange(15)))
            assert np.array_equal(u[r].ravel(), -val(r, np.arange(30)))
        assert nc.variables["zeta"].long_name == b"free-surface elevation"


def test_reads_files_written_by_scipy(tool, tmp_path):
    p = str(tmp_path / "sc.nc")
    rng = np.random.default_rng(7)
    a = rng.standard_normal((3, 4, 6))
    with netcdf_file(p, "w", version=2) as nc:
        nc.createDimension("time", None)
        nc.createDimension("eta_rho", 4)
        nc.createDimension("xi_rho", 6)
        nc.createDimension("auxil", 6)
        t = nc.createVariable("ocean_time", "d", ("time",))
        z = nc.createVariable("zeta", "d", ("time", "eta_rho", "xi_rho"))
        s = nc.createVariable("time_step", "i", ("time", "auxil"))
        t[:] = [10.0, 20.0, 30.0]
        z[:] = a
        s[:] = np.arange(18).reshape(3, 6)
    for r in range(3):
        out = subprocess.run([tool, "read", p, "zeta", str(r)], check=True, capture_output=True, text=True).stdout.split()
        assert out[-2:] == ["numrecs", "3"]
        got = np.array([float(x) for x in out[:-2]])
        assert np.array_equal(got, a[r].ravel())   # %.17g round-trips doubles exactly
    out = subprocess.run([tool, "read", p, "time_step", "2"], check=True, capture_output=True, text=True).stdout.split()
    assert [int(x) for x in out[:-2]] == list(range(12, 18))


def test_record_out_of_range_is_an_error(tool, tmp_path):
    p = str(tmp_path / "rt.nc")
    subprocess.run([tool, "write", p], check=True)
    r = subprocess.run([tool, "read", p, "zeta", "4"], capture_output=True, text=True)
    assert r.returncode != 0
