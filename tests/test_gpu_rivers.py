"""GPU parity of the river sources (river_frc.F and its hooks in
step2d_FB.F:531-554, pre_step3d4S.F:493-522, step3d_uv2.F:689-717 and
compute_horiz_tracer_fluxes.h:217-246) on the reference's Rivers_ana case.

The oracle's river restatement (oracle/oracle_main.c or_ana_grid,
oracle_step.c) follows tests/Rivers_ana; its diag lines are compared with the
golden log in tests/test_oracle_golden.py.  Here the HIP path is compared
with the oracle:
  * each hooked routine from an identical mid-run state (1e-12 relative);
  * a 20-step run: diag norms and field RMS against the oracle (the north_star
    bound, 1e-10);
  * a river update through roms_gpu_set_river_frc (new riv_vol / riv_trc,
    faces kept) changes the GPU run exactly as the oracle's.
"""
import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_parity import PROGNOSTIC, RMS_RUN, RTOL_ROUTINE, check_fields, copy_state

pytestmark = pytest.mark.gpu

LMD_OUT = ["Akv", "Akt", "hbls", "hbbl", "ghat"]


def make_pair(LLm=60, MMm=60):
    cfg = oracle.rivers_cfg(LLm=LLm, MMm=MMm, np_xi=1, np_eta=1)
    o = oracle.Oracle(cfg)
    o.init()
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, lmd=cfg.lmd)
    return cfg, o, m


def test_river_faces_match_calc_river_flux():
    """The host restatement of init_river_frc/calc_river_flux marks the same
    faces as the oracle's: the rivers case after init equals the oracle's."""
    cfg, o, m = make_pair()
    uf, vf = o.field("riv_uflx"), o.field("riv_vflx")
    assert np.count_nonzero(np.abs(vf) > 1e-3) > 0 and np.count_nonzero(np.abs(uf) > 1e-3) == 0
    check_fields(o, m, PROGNOSTIC + ["rmask", "umask", "vmask"], cfg.LLm, cfg.MMm, RTOL_ROUTINE)
    m.close()


@pytest.mark.parametrize("routine,mode,outs", [
    ("step2d", "fast", ["zeta", "ubar", "vbar", "Zt_avg1", "DU_avg1", "DV_avg1"]),
    ("pre_step3d", "pred", ["t", "u", "v"]),
    ("step3d_uv2", "corr", ["u", "v", "ubar", "vbar", "FlxU", "FlxV"]),
    ("step3d_t", "corr", ["t"]),
])
def test_river_routine_parity(routine, mode, outs):
    cfg, o, m = make_pair()
    o.step(3)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    iif = 1
    if mode == "fast":
        kstp, knew = knew, knew % 4 + 1
        nrhs, nnew = 3, 3 - nstp
        o.L.or_set_iif(o.h, 2)
        iif = 2
    elif mode == "corr":
        nrhs, nnew = 3, 3 - nstp
    else:
        nrhs, nnew = nstp, 3
    o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
    copy_state(o, m)
    m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, iif=iif, nfast=o.nfast())
    o.call(routine)
    getattr(m, routine)()
    m.sync()
    check_fields(o, m, outs, cfg.LLm, cfg.MMm, RTOL_ROUTINE)
    m.close()


def test_rivers_20_steps_vs_oracle():
    cfg, o, m = make_pair()
    for _ in range(20):
        o.step()
        m.step()
        d = m.diag()
        for v, w in zip(d, o.norms()):
            assert abs(v - w) <= 1e-11 * max(abs(w), 1e-300), (d, o.norms())
    check_fields(o, m, PROGNOSTIC + LMD_OUT, cfg.LLm, cfg.MMm, RMS_RUN, kind="rms")
    # the river water is in: salinity (t(:,:,:,:,2), levels 3N..6N of the
    # oracle's flattened view) drops below the ocean's 36 in wet cells
    N = cfg.N
    S = o.field("t")[3 * N:6 * N]
    wet = o.field("rmask")[0] > 0.5
    assert int(np.count_nonzero((S < 35.9) & wet[None])) > 0
    m.close()


def test_river_update_riv_vol_trc():
    """set_river_frc with new riv_vol / riv_trc and the faces kept: the GPU
    follows the oracle given the same change."""
    cfg, o, m = make_pair(LLm=40, MMm=40)
    o.step(2)
    m.step(2)
    m.set_river_frc([800.0], [[20.0, 5.0]])
    o.set_river(800.0, [20.0, 5.0])
    o.step(3)
    m.step(3)
    check_fields(o, m, PROGNOSTIC, cfg.LLm, cfg.MMm, RMS_RUN, kind="rms")
    m.close()


def test_river_count_below_face_indices_is_rejected():
    """Faces kept from an earlier call index riv_vol up to their largest river
    number: a smaller nriv without new faces fails loudly instead of reading
    past the new arrays on the device; with the faces passed
    again it is accepted."""
    m = romsgpu.Model.from_case(3, 40, 40, 10, 2, salinity=True, nonlin_eos=True, dt=20.0, ndtfast=30,
                                sizex=10e3, sizey=10e3, lmd=True)
    uf = np.zeros((42 + 2, 42 + 2))
    vf = np.zeros_like(uf)
    uf[10, 5] = 10 * 1 + 0.5   # river 1 through one u face ...
    uf[11, 5] = 10 * 2 + 0.5   # ... river 2 through the next
    m.set_river_frc([500.0, 300.0], [[24.0, 1.0], [20.0, 2.0]], uf, vf)
    with pytest.raises(romsgpu.RomsGpuError, match="largest river index"):
        m.set_river_frc([500.0], [[24.0, 1.0]])
    uf[11, 5] = 0.0
    m.set_river_frc([500.0], [[24.0, 1.0]], uf, vf)   # new faces: accepted
    m.step(1)
    m.close()
