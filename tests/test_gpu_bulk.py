"""GPU parity of the BULK_FRC surface fluxes (bulk_frc.F calc_all_bulk_forces,
the COARE-style bulk formulae, the current-feedback stress correction and
the rho->u/v averaging) and of KPP driven by them (lmd_kpp.F u* from
sustr_r/svstr_r under BULK_FRC).

The reference reads the atmosphere from netCDF; the C4 stand-in (SURVEY.md
8(d)) is a synthetic analytic atmosphere over the closed basin (westerly
jet, air a few degC off the sea surface, humid, light rain), set identically
by the oracle (oracle_main.c or_ana_forces) and the host (host_init.cpp).
Parity unpinned against the reference itself: no reference test or golden
log exercises BULK_FRC, so the HIP path is held to the oracle's restatement
(oracle/oracle_bulk.c, bulk_frc.F line by line):
  * the fluxes after init and after one call from a mid-run state (1e-12
    relative; the bulk formulae carry exp/log/sqrt/pow, an ulp apart
    between device libm and glibc);
  * a 40-step basin run with KPP: diag norms and field RMS (north_star 1e-10).
"""
import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_parity import PROGNOSTIC, RMS_RUN, RTOL_ROUTINE, basin_cfg, check_fields, copy_state, interior

pytestmark = pytest.mark.gpu

FLUX_OUT = ["sustr", "svstr", "sustr_r", "svstr_r", "srflx", "stflx", "swflx"]
LMD_OUT = ["Akv", "Akt", "hbls", "hbbl", "ghat"]


def bulk_cfg(**kw):
    c = basin_cfg(nonlin=True, **kw)
    c.lmd = oracle.LMD_ALL
    c.bulk_frc = 1
    return c


def make_pair(cfg):
    o = oracle.Oracle(cfg)
    o.init()
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, lmd=cfg.lmd,
                                bulk_frc=True)
    return o, m


def test_bulk_init_matches_oracle():
    cfg = bulk_cfg(LLm=40, MMm=32, N=16)
    o, m = make_pair(cfg)
    names = [n for n in PROGNOSTIC if n != "Wi"]
    check_fields(o, m, names + FLUX_OUT + ["uwnd", "vwnd", "tair", "qair", "prate", "swrad", "lwrad"],
                 cfg.LLm, cfg.MMm, RTOL_ROUTINE)
    # at rest the only vertical velocity is the surface fresh-water flux
    # (omega.F:116): We carries it, Wi is cancellation noise of order 1e-17,
    # so it is held to the scale of We
    dwi = np.abs(interior(m.get("Wi") - o.field("Wi"), cfg.LLm, cfg.MMm)).max()
    assert dwi <= RTOL_ROUTINE * np.abs(o.field("We")).max()
    # the fluxes are live: wind stress from the jet, net heat and fresh water
    assert np.abs(o.field("sustr")).max() > 1e-5 and np.abs(o.field("stflx")).max() > 1e-6
    m.close()


@pytest.mark.parametrize("nrhs_mode", ["nstp", "corr"])
def test_bulk_flux_routine_parity(nrhs_mode):
    """One calc_all_bulk_forces call from an identical mid-run state (moving
    surface currents feed the CFB correction), at the step's first set_forces
    (nrhs = nstp) and at the second (nrhs = 3, main.F:433)."""
    cfg = bulk_cfg(LLm=40, MMm=32, N=16)
    o, m = make_pair(cfg)
    o.step(4)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    nrhs = nstp if nrhs_mode == "nstp" else 3
    o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
    copy_state(o, m)
    for n in FLUX_OUT:   # start both sides from zeroed outputs
        z = np.zeros_like(o.field(n))
        m.put(n, z)
    m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, iif=1, nfast=o.nfast())
    o.call("bulk_flux")
    m.bulk_flux()
    m.sync()
    check_fields(o, m, FLUX_OUT, cfg.LLm, cfg.MMm, RTOL_ROUTINE)
    m.close()


def test_bulk_kpp_40_steps_vs_oracle():
    cfg = bulk_cfg(LLm=40, MMm=32, N=16)
    o, m = make_pair(cfg)
    for _ in range(40):
        o.step()
        m.step()
        d = m.diag()
        for v, w in zip(d, o.norms()):
            assert abs(v - w) <= 1e-11 * max(abs(w), 1e-300), (d, o.norms())
    check_fields(o, m, PROGNOSTIC + LMD_OUT + FLUX_OUT, cfg.LLm, cfg.MMm, RMS_RUN, kind="rms")
    m.close()


def test_bulk_requires_bulk_case():
    """bulk_flux on a model built without BULK_FRC fails loudly."""
    cfg = basin_cfg(nonlin=True, LLm=24, MMm=20, N=8)
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey)
    with pytest.raises(romsgpu.RomsGpuError):
        m.bulk_flux()
    m.close()


def test_bulk_rain_heat_uses_air_temperature():
    """step3d_t_ISO.F:939-951: under BULK_FRC the heat of rain is
    dt*swflx*tair (2 m air temperature), not dt*swflx*t(N)/Hz(N).  step3d_t
    on identical corrector states with tair as set and shifted by +5 degC:
    each matches the oracle, and the shift moves T in every wet column with
    fresh-water flux while S stays put (this failed before the restatement
    was fixed: tair did not enter step3d_t at all)."""
    cfg = bulk_cfg(LLm=40, MMm=32, N=16)
    res = {}
    for shift in (0.0, 5.0):
        o, m = make_pair(cfg)
        o.step(4)
        iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
        nrhs, nnew = 3, 3 - nstp
        o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
        o.field("tair")[...] += shift
        copy_state(o, m)
        m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, iif=1, nfast=o.nfast())
        o.call("step3d_t")
        m.step3d_t()
        m.sync()
        check_fields(o, m, ["t"], cfg.LLm, cfg.MMm, RTOL_ROUTINE)
        t = m.get("t").reshape(cfg.NT, 3, cfg.N, cfg.MMm + 4, cfg.LLm + 4)[:, nnew - 1]
        res[shift] = (t.copy(), o.field("swflx").reshape(cfg.MMm + 4, cfg.LLm + 4).copy())
        m.close()
    t0, sw = res[0.0]
    t1 = res[5.0][0]
    wet = (np.abs(sw) > 0)[2:-2, 2:-2]
    assert wet.sum() > 0
    dT = (t1[0, -1] - t0[0, -1])[2:-2, 2:-2]
    assert np.all(dT[wet] != 0.0)
    assert np.array_equal(t1[1], t0[1])   # salinity does not see tair
