"""Restart and history files on the GPU.

* History records written from the device snapshot (wrt_his_ocean_vars,
  basic_output.F:273-419) hold exactly the device state of the written step:
  zeta/ubar/vbar(knew), u/v/tracers(nnew) on the partition's i0:i1/j0:j1
  ranges (dimensions.F:40-45), read back with scipy's independent netCDF
  reader; the write returns before the file is on disk and the model keeps
  stepping meanwhile.
* EXACT_RESTART (main.F:244-248, get_init.F, basic_output.F:568-682): a run
  that writes its restart file at steps M-1 and M, and a second run that
  restarts from that file (get_init(rec-1, 2), get_init(rec, 1), then the
  roms_init sequence) and steps on, equal the uninterrupted run bitwise.
* PARALLEL_FILES: the per-rank history files of a 2x2 decomposition, joined by
  their 'partition' attributes as the reference's ncjoin does, equal the
  single-domain file bitwise.
"""
import os
import threading

import numpy as np
import pytest
from scipy.io import netcdf_file

import romsgpu

pytestmark = pytest.mark.gpu

FIL = dict(case_id=0, LLm=40, MMm=30, N=12, NT=1, salinity=False, nonlin_eos=False, dt=5.0, ndtfast=60,
           sizex=8.0e3, sizey=1.5e3)
BASIN_LMD = dict(case_id=1, LLm=36, MMm=28, N=16, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                 sizex=72e3, sizey=56e3, lmd=True, surf_flux=True)
PASSIVE = dict(BASIN_LMD, NT=4)


def read(path):
    with netcdf_file(path, "r", mmap=False) as nc:
        out = {k: np.array(v[:]) for k, v in nc.variables.items()}
        out["_attrs"] = dict(nc._attributes)
        out["_dims"] = dict(nc.dimensions)
    return out


def slab(a, g, Lm, Mm):
    """Single-rank partition of a (.., Mm+4, Lm+4) field: rho i,j = 0..L+1, u i from 1, v j from 1."""
    i0 = 1 if g == "u" else 0
    j0 = 1 if g == "v" else 0
    return a[..., j0 + 1:Mm + 3, i0 + 1:Lm + 3]


def state(m):
    t = m.t
    z = m.get("zeta")[t.knew - 1]
    ub = m.get("ubar")[t.knew - 1]
    vb = m.get("vbar")[t.knew - 1]
    N = m.N
    u = m.get("u")[(t.nnew - 1) * N:t.nnew * N]
    v = m.get("v")[(t.nnew - 1) * N:t.nnew * N]
    tr = m.get("t").reshape(m.NT, 3, N, *m.shape2)[:, t.nnew - 1]
    return dict(zeta=z, ubar=ub, vbar=vb, u=u, v=v, t=tr)


def test_history_records_equal_device_state(tmp_path):
    p = str(tmp_path / "fil_his.nc")
    m = romsgpu.Model.from_case(**FIL)
    snaps = []
    for rec in (1, 2):
        m.step(3)
        m.wrt_his(p, rec, rec, m.time(FIL["dt"]), mask=romsgpu.WRT_DEFAULT | romsgpu.WRT["O"])
        # history omega is pm*pn*(We+Wi) in m/s (basic_output.F:374-384)
        om = m.get("pm")[0] * m.get("pn")[0] * (m.get("We") + m.get("Wi"))
        snaps.append((state(m), om, m.t.iic))
        m.step(1)   # keeps stepping while the writer drains the snapshot
    m.io_wait()
    L, M = m.Lm, m.Mm
    m.close()
    d = read(p)
    assert d["_attrs"]["type"] == b"ROMS history file"
    assert d["_dims"]["xi_rho"] == L + 2 and d["_dims"]["xi_u"] == L + 1 and d["_dims"]["eta_v"] == M + 1
    assert d["ocean_time"].tolist() == [3 * 5.0, 7 * 5.0]
    for r, (s, we, iic) in enumerate(snaps):
        assert d["time_step"][r].tolist() == [iic, r + 1, r + 1, 0, 0, 0]
        assert np.array_equal(d["zeta"][r], slab(s["zeta"], "r", L, M))
        assert np.array_equal(d["ubar"][r], slab(s["ubar"], "u", L, M))
        assert np.array_equal(d["vbar"][r], slab(s["vbar"], "v", L, M))
        assert np.array_equal(d["u"][r], slab(s["u"], "u", L, M))
        assert np.array_equal(d["v"][r], slab(s["v"], "v", L, M))
        assert np.array_equal(d["temp"][r], slab(s["t"][0], "r", L, M))
        assert np.array_equal(d["omega"][r], slab(we, "r", L, M))


@pytest.mark.parametrize("case", [FIL, BASIN_LMD, PASSIVE], ids=["filament", "basin_lmd", "basin_nt4"])
def test_exact_restart_is_bitwise(case, tmp_path):
    M = 4
    a = romsgpu.Model.from_case(**case)
    a.step(2 * M)
    ref = state(a)
    ref_h = (a.get("hbls"), a.get("hbbl")) if case.get("lmd") else None
    a.close()

    p = str(tmp_path / "rst.nc")
    b = romsgpu.Model.from_case(**case)
    b.step(M - 1)
    b.wrt_rst(p, 1, 1, b.time(case["dt"]))   # EXACT_RESTART: the step before the period ...
    b.step(1)
    b.wrt_rst(p, 2, 2, b.time(case["dt"]))   # ... and the period
    b.io_wait()
    b.close()
    d = read(p)
    assert d["_attrs"]["type"] == b"ROMS restart file"
    assert d["time_step"][:, 0].tolist() == [M - 1, M]
    names = {"temp", "DU_avg1", "DV_avg_bak", "riv_umask"} | ({"hbls", "hbbl"} if case.get("lmd") else set())
    names |= {"salt"} if case["salinity"] else set()
    names |= {"trc%02d" % q for q in range(3, case["NT"] + 1)}
    assert names <= set(d), names - set(d)

    c = romsgpu.Model.from_case(**case)
    c.restart(p)
    assert c.t.forw_start == 1 and c.t.ntstart == M + 1 and c.t.iic == M   # exact restart (get_init.F:383)
    c.step(M)
    got = state(c)
    got_h = (c.get("hbls"), c.get("hbbl")) if case.get("lmd") else None
    c.close()
    for k in ref:
        assert np.array_equal(got[k], ref[k]), k
    if ref_h:
        assert np.array_equal(got_h[0], ref_h[0]) and np.array_equal(got_h[1], ref_h[1])


def test_restart_without_second_record_is_approximate(tmp_path):
    p = str(tmp_path / "rst1.nc")
    b = romsgpu.Model.from_case(**FIL)
    b.step(3)
    b.wrt_rst(p, 1, 1, b.time(FIL["dt"]))
    b.io_wait()
    b.close()
    c = romsgpu.Model.from_case(**FIL)
    c.restart(p)
    assert c.t.ntstart == 4 and c.t.forw_start == 4   # forward first step (get_init.F:383-385)
    c.step(2)
    c.sync()
    assert np.isfinite(c.get("zeta")).all()
    c.close()


def test_restart_file_of_another_grid_is_an_error(tmp_path):
    p = str(tmp_path / "rst.nc")
    b = romsgpu.Model.from_case(**FIL)
    b.step(1)
    b.wrt_rst(p, 1, 1, 5.0)
    b.io_wait()
    b.close()
    c = romsgpu.Model.from_case(**dict(FIL, LLm=32))
    with pytest.raises(romsgpu.RomsGpuError, match="partition"):
        c.get_init(p, 1, 1)
    c.close()


def join(paths):
    """ncjoin: place every partition file's slabs by its 'partition' attribute."""
    parts = [read(p) for p in paths]
    LL, MM = int(parts[0]["_attrs"]["global_x"]), int(parts[0]["_attrs"]["global_y"])
    out = {}
    for d in parts:
        _, _, is_, js = [int(x) for x in d["_attrs"]["partition"]]
        sr, tr = is_ - 1, js - 1
        for name, a in d.items():
            if name.startswith("_") or a.ndim < 3:
                continue
            g = "u" if name in ("u", "ubar") else "v" if name in ("v", "vbar") else "r"
            nx = LL + 1 if g == "u" else LL + 2
            ny = MM + 1 if g == "v" else MM + 2
            x0 = max(sr - 1, 0) if g == "u" else sr
            y0 = max(tr - 1, 0) if g == "v" else tr
            if name not in out:
                out[name] = np.full(a.shape[:-2] + (ny, nx), np.nan)
            out[name][..., y0:y0 + a.shape[-2], x0:x0 + a.shape[-1]] = a
    return out


def test_partitioned_history_joins_to_single_domain(tmp_path):
    single = str(tmp_path / "single.nc")
    m = romsgpu.Model.from_case(**FIL)
    m.step(3)
    m.wrt_his(single, 1, 1, m.time(FIL["dt"]))
    m.io_wait()
    m.close()
    npx, npe = 2, 2
    paths = [str(tmp_path / ("his.%d.nc" % r)) for r in range(npx * npe)]
    errs = []

    def work(rank):
        try:
            h = romsgpu.comm_create_local(777, npx * npe, rank)
            mm = romsgpu.Model.from_case(np_xi=npx, np_eta=npe, comm=h, rank=rank, **FIL)
            mm.step(3)
            mm.wrt_his(paths[rank], 1, 1, mm.time(FIL["dt"]))
            mm.io_wait()
            mm.close()
            romsgpu.comm_destroy(h)
        except Exception as e:
            errs.append((rank, repr(e)))

    th = [threading.Thread(target=work, args=(r,)) for r in range(npx * npe)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not errs, errs
    a = read(paths[3])["_attrs"]
    assert list(a["partition"])[:2] == [3, 4]
    joined = join(paths)
    ref = read(single)
    for name in ("zeta", "ubar", "vbar", "u", "v", "temp"):
        assert np.array_equal(joined[name], ref[name]), name
