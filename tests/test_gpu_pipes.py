"""GPU parity of several pipe sources (pipe_frc.F set_pipe_frc, omega.F:102-108,
step3d_t_ISO.F:927-934): every pipe cell draws its vertical profile
pipe_prf(pidx,:) and tracer values pipe_trc(pidx,:) through its own pipe
number pidx = pipe_idx.  The Pipes_ana case has one pipe; here a second one,
with a different profile, volume and tracers, is added at another wet spot
through roms_gpu_set_pipe_frc and through the oracle's or_set_pipes, and the
two runs are compared (the oracle's single-pipe diag lines are pinned to the
reference's golden log in tests/test_oracle_golden.py)."""
import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_parity import PROGNOSTIC, RMS_RUN, RTOL_ROUTINE, check_fields

pytestmark = pytest.mark.gpu


def two_pipes(o, cfg):
    idx = o.field("pipe_idx")[0].copy()
    flx = o.field("pipe_flx")[0].copy()
    rmask = o.field("rmask")[0]
    ny, nx = idx.shape
    # pipe 2: a 3x3 patch of wet cells in the north-east quarter, 300 m3/s
    j0, i0 = (3 * ny) // 4, (3 * nx) // 4
    patch = (slice(j0, j0 + 3), slice(i0, i0 + 3))
    assert np.all(rmask[patch] > 0.5) and np.all(idx[patch] == 0)
    idx[patch] = 2.0
    flx[patch] = 300.0 / 9.0
    N, NT = cfg.N, cfg.NT
    prf = np.zeros((2, N))
    prf[0, 0:2] = 0.5                        # ana_pipe_frc.h: bottom two levels
    prf[1, N - 4:N - 1] = [0.2, 0.3, 0.5]    # pipe 2 discharges near the surface
    trc = np.array([[24.0, 1.0], [10.0, 30.0]])
    return idx, flx, prf, trc


@pytest.mark.parametrize("nsteps", [1, 12])
def test_two_pipes_vs_oracle(nsteps):
    cfg = oracle.pipes_cfg(LLm=48, MMm=48, np_xi=1, np_eta=1)
    o = oracle.Oracle(cfg)
    o.init()
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, lmd=cfg.lmd)
    idx, flx, prf, trc = two_pipes(o, cfg)
    o.set_pipes(idx, flx, prf, trc)
    m.set_pipe_frc(idx.astype(np.int32), flx, prf, trc)
    for _ in range(nsteps):
        o.step()
        m.step()
        d = m.diag()
        for v, w in zip(d, o.norms()):
            assert abs(v - w) <= 1e-11 * max(abs(w), 1e-300), (d, o.norms())
    tol, kind = (RTOL_ROUTINE, "rel") if nsteps == 1 else (RMS_RUN, "rms")
    check_fields(o, m, PROGNOSTIC, cfg.LLm, cfg.MMm, tol, kind=kind)
    # pipe 2 is live: the one-pipe run of the same length differs near its patch
    o1 = oracle.Oracle(cfg)
    o1.init()
    o1.step(nsteps)
    j0, i0 = (3 * (cfg.MMm + 4)) // 4, (3 * (cfg.LLm + 4)) // 4
    t2, t1 = o.field("t"), o1.field("t")
    assert np.max(np.abs(t2[:, j0 + 1, i0 + 1] - t1[:, j0 + 1, i0 + 1])) > 1e-6
    m.close()


def test_pipe_index_above_npip_is_rejected():
    cfg = oracle.pipes_cfg(LLm=32, MMm=32, np_xi=1, np_eta=1)
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, lmd=cfg.lmd)
    idx = np.zeros((cfg.MMm + 4, cfg.LLm + 4), dtype=np.int32)
    idx[10, 10] = 3
    with pytest.raises(romsgpu.RomsGpuError, match="pipe_idx"):
        m.set_pipe_frc(idx, np.ones(idx.shape), np.ones((2, cfg.N)) / cfg.N, np.ones((2, cfg.NT)))
    m.close()
