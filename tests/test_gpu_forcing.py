"""Forcing and boundary producers on the device.

* set_frc_data (roms_read_write.F:303-392): two records per field in HBM,
  interpolated to the model time on the device -- equal bitwise to the
  reference's cff1*rec(it1) + cff2*rec(it2) restated in numpy, for a 2-D
  surface field and an open-boundary array, with the kinds filter and the
  out-of-window error (roms_read_write.F:381).
* set_tides (tides.F:86-254): pot_tides' ptide and bry_tides' boundary
  zeta/ubar/vbar sums over the constituents at omT = ftide*(time + dt/2),
  bitwise against the same sums in numpy (the cos/sin are formed once per
  constituent on the host in both).  Parity unpinned against the reference
  itself: its tidal tests need netCDF inputs that are not available offline.
"""
import math

import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_parity import basin_cfg
from test_gpu_register import host_model

pytestmark = pytest.mark.gpu


def open_basin(pot=1):
    c = basin_cfg(LLm=40, MMm=32, N=12, nonlin=True)
    c.obc, c.ubind, c.pot_tides = 15, 0.1, pot
    o = oracle.Oracle(c)
    o.init()
    m, _ = host_model(o, c)
    return c, m


def test_frc_interp_bitwise():
    c, m = open_basin()
    rng = np.random.default_rng(3)
    shp = m.get("sustr").shape
    a, b = rng.standard_normal(shp), rng.standard_normal(shp)
    nb = m.get("zeta_west").size
    za, zb = rng.standard_normal(nb), rng.standard_normal(nb)
    m.frc_record("sustr", 1, 10.5, b)     # slots in either order: it1 is the earlier record
    m.frc_record("sustr", 0, 10.0, a)
    m.frc_record("zeta_west", 0, 10.0, za)
    m.frc_record("zeta_west", 1, 10.5, zb)
    before = m.get("zeta_west").copy()
    t = 10.2
    m.frc_interp(t, m.FRC_SURFACE)
    cff1, cff2 = (10.5 - t) / (10.5 - 10.0), (t - 10.0) / (10.5 - 10.0)
    assert np.array_equal(m.get("sustr"), cff1 * a + cff2 * b)
    assert np.array_equal(m.get("zeta_west"), before)          # not of the requested kind
    m.frc_interp(t, m.FRC_BRY)
    assert np.array_equal(m.get("zeta_west").ravel(), cff1 * za + cff2 * zb)
    with pytest.raises(romsgpu.RomsGpuError, match="outside the forcing records"):
        m.frc_interp(10.0 - 2 * c.dt - 1.0)   # set_frc_data's window check uses dt as is (roms_read_write.F:381)
    with pytest.raises(romsgpu.RomsGpuError, match="past the last forcing record"):
        m.frc_interp(10.6)                    # set_frc_data would read the next record here
    # a third record: past 10.5 the pair is (10.5, 11.0), as after the reference's refresh
    cz = rng.standard_normal(shp)
    m.frc_record("sustr", 2, 11.0, cz)
    t = 10.7
    m.frc_interp(t, m.FRC_SURFACE)
    cff1, cff2 = (11.0 - t) / (11.0 - 10.5), (t - 10.5) / (11.0 - 10.5)
    assert np.array_equal(m.get("sustr"), cff1 * b + cff2 * cz)
    m.close()


def test_set_tides_bitwise():
    c, m = open_basin()
    rng = np.random.default_rng(5)
    nt = 3
    shp = (nt,) + m.get("zeta").shape[1:]
    ftide = np.array([1.405e-4, 1.454e-4, 7.29e-5])
    pr, pi = 0.1 * rng.standard_normal(shp), 0.1 * rng.standard_normal(shp)
    bry = [(rng.standard_normal(shp), rng.standard_normal(shp)) for _ in range(3)]
    m.set_tide_data(ftide, pot=(pr, pi), bry=bry)
    base = {n: m.get(n).copy() for n in ("zeta_west", "ubar_east", "vbar_south", "zeta_north")}
    time = 3600.0 * 7
    m.set_tides(time)
    cs = [math.cos(f * (time + 0.5 * c.dt)) for f in ftide]
    sn = [math.sin(f * (time + 0.5 * c.dt)) for f in ftide]
    # pot_tides over (istrR-1..iendR, jstrR-1..jendR) = (-1..L+1, -1..M+1) on a closed-or-open single domain
    L, M = c.LLm, c.MMm
    want = pr[0] * cs[0] - pi[0] * sn[0]
    for t in range(1, nt):
        want = want + pr[t] * cs[t] - pi[t] * sn[t]
    got = m.get("ptide")[0]
    assert np.array_equal(got[0:M + 3, 0:L + 3], want[0:M + 3, 0:L + 3])
    # bry_tides: western zeta at i = istr-1 = 0, j = jstrR..jendR = 0..M+1
    z = base["zeta_west"].copy()
    for t in range(nt):
        z[0:M + 2] = z[0:M + 2] + bry[0][0][t][1:M + 3, 1] * cs[t] - bry[0][1][t][1:M + 3, 1] * sn[t]
    assert np.array_equal(m.get("zeta_west"), z)
    # eastern ubar at i = iend+1 = L+1, j = 0..M+1
    u = base["ubar_east"].copy()
    for t in range(nt):
        u[0:M + 2] = u[0:M + 2] + bry[1][0][t][1:M + 3, L + 2] * cs[t] - bry[1][1][t][1:M + 3, L + 2] * sn[t]
    assert np.array_equal(m.get("ubar_east"), u)
    # southern vbar at j = jstrV-1 = 1, i = istrR..iendR = 0..L+1
    v = base["vbar_south"].copy()
    for t in range(nt):
        v[0:L + 2] = v[0:L + 2] + bry[2][0][t][2, 1:L + 3] * cs[t] - bry[2][1][t][2, 1:L + 3] * sn[t]
    assert np.array_equal(m.get("vbar_south"), v)
    m.close()


def test_tide_data_needs_pairs():
    c, m = open_basin()
    shp = (1,) + m.get("zeta").shape[1:]
    with pytest.raises(romsgpu.RomsGpuError, match="come together"):
        m.set_tide_data([1e-4], pot=(np.zeros(shp), None))
    m.close()


ATMOS = ("uwnd", "vwnd", "tair", "qair", "prate", "swrad", "lwrad")
BRY = tuple("%s_%s" % (v, e) for v in ("zeta", "ubar", "vbar", "u", "v", "t") for e in ("west", "east", "south", "north"))
PERTURB = dict(uwnd=lambda a: 1.3 * a, vwnd=lambda a: a + 1.0, tair=lambda a: a + 2.0, qair=lambda a: 0.9 * a,
               prate=lambda a: 2.0 * a, swrad=lambda a: 1.2 * a, lwrad=lambda a: a + 10.0,
               zeta=lambda a: a + 0.02, ubar=lambda a: 0.5 * a, vbar=lambda a: 0.5 * a, u=lambda a: 0.5 * a,
               v=lambda a: 0.5 * a, t=lambda a: a + 0.3)


def _clocked_pair(clock, nrec=3):
    """Records [days] at 0, 6 dt and 14 dt.  Step iic's set_frc_data points
    are (iic-1) dt ('current'), (iic-1/2) dt ('1/2 fwd') and (iic+1/2) dt
    ('forward'), so the boundary data move to the second pair at 'forward' of
    step 6 -- between that step's two set_bry_all calls -- and the surface
    fields at '1/2 fwd' of step 7 (a refresh inside a step).  The
    third record is not on the line through the first two."""
    c = basin_cfg(LLm=40, MMm=32, N=12, nonlin=True)
    c.obc, c.ubind, c.lmd, c.bulk_frc = 15, 0.1, oracle.LMD_ICELAND, 1
    o = oracle.Oracle(c)
    o.init()
    m = romsgpu.Model.from_case(c.case_id, c.LLm, c.MMm, c.N, c.NT, salinity=True, nonlin_eos=True, dt=c.dt,
                                ndtfast=c.ndtfast, sizex=c.sizex, sizey=c.sizey, lmd=c.lmd, obc=15, bulk_frc=True)
    day = c.dt / 86400.0
    for name in ATMOS + BRY:
        a = o.field(name).copy()
        b = PERTURB[name.split("_")[0]](a)
        recs = [(0.0, a), (6 * day, b), (14 * day, 0.5 * (a + b))]
        order = (2, 0, 1) if nrec == 3 else (0, 1)   # slots in any order: the pair follows the times
        for side in (o, m):
            for slot in order:
                side.frc_record(name, slot, recs[slot][0], recs[slot][1])
    if clock:
        o.frc_clock(0.0)
        m.frc_clock(0.0)
    return c, o, m


def test_in_step_forcing_records_vs_oracle():
    """Time-varying forcing inside roms_gpu_step: three
    records of every BULK_FRC atmospheric field and of every open-boundary
    array; each step interpolates them at the reference's four points
    (main.F:384-441: surface at 'current' and '1/2 fwd', boundary data at
    '1/2 fwd' and 'forward'), each point on its own record pair, on the device
    (a stateless pair choice per point) and in the oracle (set_frc_data's
    stateful refresh restated in plain C).  12 steps (graph replay from step
    2) against the oracle, RMS < 1e-10; and the result is not that of one
    interpolation per step."""
    from test_gpu_parity import PROGNOSTIC, RMS_RUN, check_fields
    c, o, m = _clocked_pair(True)
    o.step(12)
    m.step(12)
    m.sync()
    check_fields(o, m, PROGNOSTIC + ["stflx", "swflx", "sustr", "uwnd", "tair", "hbls"], c.LLm, c.MMm, RMS_RUN,
                 kind="rms")
    for n in ("u_west", "t_north", "zeta_south"):   # boundary data at 'forward' of step 12
        assert np.array_equal(m.get(n).ravel(), o.field(n).ravel()), n
    got = m.get("t").copy()
    m.close()
    # interpolating once per step at 'current' (the host-driven path) gives another state
    c2, o2, m2 = _clocked_pair(False)
    for k in range(12):
        m2.frc_interp(c2.dt * k / 86400.0)
        m2.step()
    assert not np.array_equal(m2.get("t"), got)
    m2.close()


def test_in_step_forcing_refresh_inside_a_step_bitwise():
    """Step 6's 'forward' boundary point is past the second record: with the
    third record loaded the boundary arrays after step 6 equal
    cff1*rec(2) + cff2*rec(3) at (6 + 1/2) dt exactly (the pair set_frc_data
    holds after its refresh), while '1/2 fwd' of the same step used the first
    pair."""
    c, o, m = _clocked_pair(True)
    m.step(6)
    m.sync()
    day, sec2day = c.dt / 86400.0, 1.0 / 86400.0
    time = 5 * c.dt    # step 6: time = start_time + dt*(iic - ntstart) (main.F:374)
    t1, t2 = 6 * day, 14 * day
    mt = (time + 0.5 * c.dt) * sec2day + c.dt * sec2day   # 'forward' (main.F:438, roms_read_write.F:335)
    cff1, cff2 = (t2 - mt) / (t2 - t1), (mt - t1) / (t2 - t1)
    for n in ("zeta_west", "u_east", "t_north"):
        a = o.field(n).copy()    # the oracle has not stepped: its arrays are record 1
        b = PERTURB[n.split("_")[0]](a)
        want = cff1 * b + cff2 * (0.5 * (a + b))
        assert np.array_equal(m.get(n).ravel(), want.ravel()), n
    m.close()


def test_in_step_forcing_past_last_record_fails_before_queueing():
    """With only two records, step 6's 'forward' point needs the next record
    (the reference refreshes there, roms_read_write.F:341): the step fails
    with -8 before anything is queued, and the state is that of step 5."""
    c, o, m = _clocked_pair(True, nrec=2)
    m.step(5)
    m.sync()
    before = m.get("t").copy()
    with pytest.raises(romsgpu.RomsGpuError, match="past the last forcing record"):
        m.step()
    assert np.array_equal(m.get("t"), before)
    m.close()


def test_in_step_forcing_out_of_window_fails_before_queueing():
    c, o, m = _clocked_pair(True)
    m.frc_clock(-100 * 86400.0)   # far before the records (set_frc_data's window check, :381)
    with pytest.raises(romsgpu.RomsGpuError, match="outside the forcing records"):
        m.step()
    m.close()


def test_boundary_tides_need_interpolated_boundary_data():
    """bry_tides adds onto boundary arrays that set_bry_all has
    just re-set; an open side's zeta/ubar/vbar array that is never
    interpolated in-step would accumulate the sums, so the step refuses."""
    c, m = open_basin(pot=0)
    shp = (1,) + m.get("zeta").shape[1:]
    z = np.zeros(shp)
    m.set_tide_data([1.4e-4], bry=((z, z), (z, z), (z, z)))
    nb = m.get("zeta_west").size
    m.frc_record("zeta_west", 0, 0.0, np.zeros(nb))
    m.frc_record("zeta_west", 1, 1.0, np.zeros(nb))
    m.frc_clock(0.0)
    with pytest.raises(romsgpu.RomsGpuError, match="boundary tides need two records"):
        m.step()
    m.close()
