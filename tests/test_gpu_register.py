"""The drop-in host path of the C ABI: a host that owns
its module arrays -- as the Fortran driver does after init_arrays -- calls
roms_gpu_init with its dims/cppdefs, roms_gpu_register for every array,
roms_gpu_upload, then the per-routine entries / roms_gpu_step, and
roms_gpu_download before it reads results.  No analytic case builder of the
library is involved: the state comes from the oracle's own ana_grid /
ana_init + roms_init (main.F:85-321), so this is the contract a Fortran host
sees, checked against the oracle after 20 steps (field RMS < 1e-10).

Also: TIDES with pot_tides -- the surface tidal potential ptide (tides.F:26)
enters prsgrd's surface pressure (prsgrd.F:209-211); the host writes ptide
and uploads it like any forcing field.
"""
import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_parity import PROGNOSTIC, RMS_RUN, RTOL_ROUTINE, basin_cfg, check_fields

pytestmark = pytest.mark.gpu


def dims_cfg(o, c):
    """roms_dims / roms_cfg of an oracle configuration (param.F, cppdefs.opt, roms.in)."""
    D = romsgpu.Dims()
    D.Lm, D.Mm, D.N, D.NT, D.LLm, D.MMm = c.LLm, c.MMm, c.N, c.NT, c.LLm, c.MMm
    D.np_xi = D.np_eta = 1
    D.ew_periodic, D.ns_periodic = c.ew_periodic, c.ns_periodic
    C = romsgpu.Cfg()
    C.nonlin_eos, C.salinity, C.lmd_mixing = c.nonlin_eos, c.salinity, c.lmd
    C.uv_vis2 = C.ts_dif2 = 1
    C.dt, C.ndtfast, C.nfast = c.dt, c.ndtfast, o.nfast()
    w = o.weights()
    for q in range(romsgpu.MAX_FAST):
        C.weight[0][q] = w[0, q]
        C.weight[1][q] = w[1, q]
    C.g, C.rho0, C.rdrg, C.rdrg2, C.Zob, C.gamma2 = 9.81, c.rho0, c.rdrg, c.rdrg2, c.Zob, 1.0
    C.Akv_bak = c.Akv_bak
    C.Akt_bak[0], C.Akt_bak[1] = c.Akt_bak[0], c.Akt_bak[1]
    C.Tcoef, C.T0, C.Scoef, C.S0 = c.Tcoef, c.T0, c.Scoef, c.S0
    C.theta_s, C.theta_b, C.hc = c.theta_s, c.theta_b, c.hc
    C.obc, C.ubind, C.curvgrid = c.obc, c.ubind, c.curvgrid
    C.uv_adv, C.uv_cor, C.pot_tides = c.uv_adv, c.uv_cor, c.pot_tides
    return D, C


def host_model(o, c):
    """Init through roms_gpu_init, register host copies of every oracle array,
    upload them all (ROMS_ALL), and set the time indices the oracle left."""
    D, C = dims_cfg(o, c)
    m = romsgpu.Model.from_dims(D, C)
    host = {}
    for name in romsgpu.FIELDS:
        a = np.ascontiguousarray(o.field(name), dtype=np.float64).copy()
        m.register(name, a)
        host[name] = a
    m.upload()
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, nfast=o.nfast())
    return m, host


def test_register_upload_step_download_matches_oracle():
    """Iceland switch set (OBC, SPONGE, island, CURVGRID, LMD/KPP without
    CONVEC, NONLIN+SPLIT EOS) driven purely through register/upload/download."""
    c = basin_cfg(LLm=40, MMm=32, N=16, nonlin=True)
    c.obc, c.ubind, c.v_sponge, c.island, c.curvgrid = 15, 0.1, 1.0, 1, 1
    c.lmd, c.surf_flux = oracle.LMD_ICELAND, 1
    o = oracle.Oracle(c)
    o.init()
    m, host = host_model(o, c)
    o.step(20)
    m.step(20)
    m.download()           # every registered mirror, as a host before diag / wrt_*
    for n in ("zeta", "ubar", "vbar", "u", "v", "t", "We", "Akv", "Akt"):
        a = host[n].reshape(o.field(n).shape)[..., 2:-2, 2:-2]
        b = o.field(n)[..., 2:-2, 2:-2]
        e = float(np.sqrt(np.mean((a - b) ** 2))) / max(1.0, float(np.sqrt(np.mean(b ** 2))))
        assert e < RMS_RUN, (n, e)
    assert o.tindex() == m.t.as_list()
    m.close()


def _ptide(o, amp=0.3):
    x, y = o.field("xr")[0], o.field("yr")[0]
    Lx, Ly = float(x.max()), float(y.max())
    return amp * np.sin(2 * np.pi * x / Lx) * np.cos(np.pi * y / Ly)


@pytest.mark.parametrize("fused", ["0", "1"])
def test_pot_tides_prsgrd_parity(fused, monkeypatch):
    monkeypatch.setenv("ROMS_GPU_PRSGRD_FUSED", fused)
    c = basin_cfg(nonlin=True)
    c.pot_tides = 1
    o = oracle.Oracle(c)
    o.init()
    o.field("ptide")[...] = _ptide(o)
    o.step(3)
    m, host = host_model(o, c)
    o.call("prsgrd")
    m.prsgrd()
    m.sync()
    check_fields(o, m, ["ru", "rv"], c.LLm, c.MMm, RTOL_ROUTINE)
    m.close()


def test_pot_tides_20_steps():
    c = basin_cfg(LLm=40, MMm=32, N=10, nonlin=True)
    c.pot_tides = 1
    o = oracle.Oracle(c)
    o.init()
    o.field("ptide")[...] = _ptide(o, 0.5)
    m, host = host_model(o, c)
    # the tidal potential drives flow: compare against a run without it
    o.step(20)
    m.step(20)
    m.sync()
    check_fields(o, m, PROGNOSTIC, c.LLm, c.MMm, RMS_RUN, kind="rms")
    c0 = basin_cfg(LLm=40, MMm=32, N=10, nonlin=True)
    o0 = oracle.Oracle(c0)
    o0.init()
    o0.step(20)
    assert float(np.max(np.abs(o.field("zeta") - o0.field("zeta")))) > 1e-6
    m.close()
