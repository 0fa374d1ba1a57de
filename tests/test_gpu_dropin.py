"""The drop-in deployment run as a sequence (BASELINE C1).

A Fortran host that links the drop-ins (fortran/dropin/*.F) keeps the
reference's roms_step (src/main.F:374-479) and calls the hot-path routines one
by one; each lands in its per-routine C-ABI entry.  `dropin_step` below is that
sequence, entry for entry, with the time indices of module scalars advanced
where main.F advances them:

    nstp = 1 + mod(iic - ntstart, 2); nrhs = nstp; nnew = 3           :377-378
    [set_forces: bulk fluxes]  rho_eos(nrhs)  set_HUV  omega           :386-406
    lmd_vmix(nstp)  prsgrd  pre_step3d(0)  set_HUV1(0)                 :409-423
    nrhs = 3; nnew = 3 - nstp                                          :425
    omega  rho_eos(nrhs)  [set_forces]  lmd_vmix(nrhs)                 :429-436
    prsgrd  step3d_uv1(0)  visc3d                                      :445-449
    do iif = 1, nfast: kstp = knew; knew = kstp + 1 (wrap 4); step2d   :456-464
    step3d_uv2(0)  omega  step3d_t(0)  t3dmix  rho_eos(nnew)           :467-479

The whole-step entry (roms_gpu_step) runs the same routines with fusions
(prsgrd + the horizontal momentum r.h.s., the predictor omega forming
pre_step3d's Hz_bak/Hz_fwd, P formed in rho_eos, the step-opening rho_eos
reused, set_HUV's Hz_u/Hz_v skipped) and replays HIP graphs.  Both must give
the same state bitwise, and the oracle's within the north_star RMS bound:
  * C1: the Filament benchmark's ana_grid/ana_init (SizeX 12.8 km, SizeY
    3.2 km, dt 5 s, ndtfast 60) at 128x128x20 on a 2x2 processor grid
    (subdomains on threads, roms_gpu_comm_create_local), 20 steps, with the
    per-step diag norms equal to the oracle's 2x2 per-rank sums digit for
    digit;
  * the C3 switch set (closed basin, NONLIN+SPLIT EOS, T+S, KPP/BKPP/RIMIX/
    NONLOCAL, dt 300 s, nfast 82) at 64x48x100 on one rank, 20 steps;
  * the C4 Iceland stand-in switch set (open edges, sponge, island, CURVGRID,
    BULK_FRC) at a small size, 10 steps.
"""
import os
import signal
import subprocess
import threading

import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_configs import c3_cfg, c4_cfg, pair
from test_gpu_parity import PROGNOSTIC, RMS_RUN, check_fields

pytestmark = pytest.mark.gpu

STATE = ("zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "FlxV", "We", "Wi", "Hz", "z_r", "z_w", "rho", "rufrc",
         "rvfrc", "DU_avg1", "DV_avg1", "DU_avg2", "DV_avg2", "Zt_avg1")
LMD_STATE = ("Akv", "Akt", "hbls", "hbbl", "ghat")


def dropin_step(m, lmd=False, bulk=False, visc=True, mix=True):
    """One roms_step through the per-routine entries (main.F:374-479)."""
    t = m.t
    t.iic += 1
    t.nstp = 1 + (t.iic - t.ntstart) % 2
    t.nrhs, t.nnew = t.nstp, 3
    if bulk:
        m.bulk_flux()                 # set_forces 'current' (main.F:386)
    m.rho_eos(t.nrhs)
    m.set_HUV()
    m.omega()
    if lmd:
        m.lmd_vmix(t.nstp)
    m.prsgrd()
    m.pre_step3d()
    m.set_HUV1()
    t.nrhs, t.nnew = 3, 3 - t.nstp    # main.F:425
    m.omega()
    m.rho_eos(t.nrhs)
    if bulk:
        m.bulk_flux()                 # set_forces '1/2 fwd' (main.F:433)
    if lmd:
        m.lmd_vmix(t.nrhs)
    m.prsgrd()
    m.step3d_uv1()
    if visc:
        m.visc3d()
    for iif in range(1, t.nfast + 1):
        t.iif = iif
        t.kstp = t.knew
        t.knew = t.kstp + 1 if t.kstp < 4 else 1
        m.step2d()
    m.step3d_uv2()
    m.omega()
    m.step3d_t()
    if mix:
        m.t3dmix()
    m.rho_eos(t.nnew)


def _cfg_flags(cfg):
    return dict(lmd=bool(cfg.lmd), bulk=bool(cfg.bulk_frc))


def _assert_bitwise(a, b, names, what):
    bad = [(n, float(np.max(np.abs(a[n] - b[n])))) for n in names if not np.array_equal(a[n], b[n])]
    assert not bad, (what, bad[:6])


def _single_rank(cfg, nsteps):
    names = STATE + (LMD_STATE if cfg.lmd else ())
    o, m = pair(cfg)
    flags = _cfg_flags(cfg)
    for _ in range(nsteps):
        dropin_step(m, **flags)
    m.sync()
    tl = m.t.as_list()
    got = {n: m.get(n) for n in names}
    # the oracle runs the same sequence as one call per step
    o.step(nsteps)
    assert o.tindex() == tl
    check_fields(o, m, PROGNOSTIC + (["Akv", "Akt", "hbls", "hbbl"] if cfg.lmd else []), cfg.LLm, cfg.MMm, RMS_RUN,
                 kind="rms")
    m.close()
    # the whole-step entry (graph replay) on the same initial state
    _, w = pair(cfg)
    w.step(nsteps)
    w.sync()
    assert w.t.as_list() == tl
    ref = {n: w.get(n) for n in names}
    w.close()
    _assert_bitwise(got, ref, names, "drop-in sequence vs roms_gpu_step")


def test_dropin_sequence_c3_switch_set_n100():
    cfg = c3_cfg()
    _single_rank(cfg, 20)


def test_dropin_sequence_iceland_switch_set():
    cfg = c4_cfg(L=48, sponge=1.0e3, island=1)
    _single_rank(cfg, 10)


C1 = dict(case_id=0, LLm=128, MMm=128, N=20, NT=1, salinity=False, nonlin_eos=False, dt=5.0, ndtfast=60,
          sizex=12.8e3, sizey=3.2e3)


def _run_2x2(case, nsteps, dropin, grp):
    n = 4
    out, errs, norms = [None] * n, [], []

    def work(rank):
        try:
            h = romsgpu.comm_create_local(grp, n, rank)
            m = romsgpu.Model.from_case(np_xi=2, np_eta=2, comm=h, rank=rank, **case)
            d = m.diag()                  # diag is collective: every rank calls it
            if rank == 0:
                norms.append(d)
            for _ in range(nsteps):
                if dropin:
                    dropin_step(m)
                else:
                    m.step()
                d = m.diag()
                if rank == 0:
                    norms.append(d)
            m.sync()
            out[rank] = (m.iSW, m.jSW, m.Lm, m.Mm, m.t.as_list(), {f: m.get(f) for f in STATE})
            m.close()
            romsgpu.comm_destroy(h)
        except Exception as e:  # surfaced in the main thread
            errs.append((rank, repr(e)))

    th = [threading.Thread(target=work, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    return out, norms


def test_dropin_sequence_c1_filament_128_2x2():
    """BASELINE C1 at its stated size and processor grid, driven as the
    Fortran host drives the drop-ins."""
    nsteps = 20
    seq, seq_norms = _run_2x2(C1, nsteps, True, 901)
    whole, whole_norms = _run_2x2(C1, nsteps, False, 902)
    for r in range(4):
        assert seq[r][4] == whole[r][4]
        _assert_bitwise(seq[r][5], whole[r][5], STATE, "rank %d drop-in vs roms_gpu_step" % r)
    assert seq_norms == whole_norms
    # the oracle on the whole grid, diag sums emulating the 2x2 ranks (diag.F:409-535)
    cfg = oracle.filament_cfg(LLm=128, MMm=128, N=20, np_xi=2, np_eta=2)
    o = oracle.Oracle(cfg)
    o.init()
    want = [o.norms()]
    for _ in range(nsteps):
        o.step()
        want.append(o.norms())
    for s, (a, b) in enumerate(zip(seq_norms, want)):
        for x, y in zip(a, b):
            assert abs(x - y) <= 1e-12 * abs(y), (s, a, b)
    exact = sum(("%23.16E" % x) == ("%23.16E" % y) for a, b in zip(seq_norms, want) for x, y in zip(a, b))
    print("C1 diag columns equal to the oracle's digits: %d of %d" % (exact, 4 * (nsteps + 1)))
    # every subdomain's prognostic fields against the oracle's window
    for (iSW, jSW, Lm, Mm, _, got) in seq:
        for f in ("zeta", "ubar", "vbar", "u", "v", "t"):
            w = o.field(f)[..., jSW + 2:jSW + Mm + 2, iSW + 2:iSW + Lm + 2]
            g = got[f][..., 2:Mm + 2, 2:Lm + 2]
            e = float(np.sqrt(np.mean((g - w) ** 2)))
            assert e < RMS_RUN, (f, iSW, jSW, e)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = "/opt/conda/bin/mpiexec"
MPI_DRIVER = os.path.join(ROOT, "fortran", "dropin_mpi_driver")


def _oracle_c1_2x2(nsteps):
    cfg = oracle.filament_cfg(LLm=128, MMm=128, N=20, np_xi=2, np_eta=2)
    o = oracle.Oracle(cfg)
    o.init()
    want = [o.norms()]
    for _ in range(nsteps):
        o.step()
        want.append(o.norms())
    return want


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="MPICH mpiexec not in this image")
def test_fortran_mpi_dropin_c1_2x2_processes():
    """The north_star's deployment as it would run: a Fortran + MPI host
    (fortran/mpi/dropin_mpi_driver.F90) started by mpiexec as 4 processes,
    bootstrapped like the reference (MPI_Init, mpi_setup's 2x2 grid,
    main.F:26-28 / mpi_setup.F:14-211), the library's communicator built by
    roms_gpu_comm_create_host over a Fortran MPI_Allgather callback, and the
    reference's roms_step calling the drop-ins by name.  The processes share
    this box's one GPU; halos move by IPC peer writes between them.  Rank 0's
    per-step diag norms of BASELINE C1 (Filament 128x128x20, 20 steps) equal
    the oracle's 2x2 per-rank sums in every ES23.16 column."""
    assert os.path.exists(MPI_DRIVER), "build() makes fortran/dropin_mpi_driver"
    nsteps = 20
    p = subprocess.Popen([MPIEXEC, "-n", "4", MPI_DRIVER, str(nsteps), "2", "2"], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=300)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        raise
    assert p.returncode == 0, (p.returncode, out[-2000:], err[-3000:])
    head = [ln for ln in out.splitlines() if ln.startswith("#")]
    assert head and "halo transport ipc" in head[0], out[-2000:]
    rows = [ln.split() for ln in out.splitlines() if ln.strip() and not ln.startswith("#")]
    got = {int(r[0]): [float(x) for x in r[1:5]] for r in rows if len(r) == 5 and r[0].isdigit()}
    assert sorted(got) == list(range(nsteps + 1)), out[-2000:]
    want = _oracle_c1_2x2(nsteps)
    exact = 0
    for s_, b in enumerate(want):
        for x, y in zip(got[s_], b):
            assert abs(x - y) <= 1e-12 * abs(y), (s_, got[s_], b)
            exact += ("%23.16E" % x) == ("%23.16E" % y)
    print("Fortran+MPI C1 2x2 (4 processes): diag columns equal to the oracle's digits: %d of %d" %
          (exact, 4 * (nsteps + 1)))
    assert exact == 4 * (nsteps + 1)
