"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the UCLA-ROMS hot path.

ctypes binding of oracle/liboracle.so (plain-C restatement, see
roms_oracle.h).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package.  Parity pinned against the
reference golden log tests/Filament/benchmark.result_github_gnu.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
CASE_FILAMENT, CASE_BASIN, CASE_PIPES, CASE_RIVERS = 0, 1, 2, 3
LMD_RIMIX, LMD_CONVEC, LMD_NONLOCAL, LMD_DDMIX = 8, 16, 32, 64
LMD_ALL = 63       # LMD_MIXING+KPP+BKPP+RIMIX+CONVEC+NONLOCAL (tests/Pipes_ana/cppdefs.opt)
LMD_ICELAND = 47   # all but LMD_CONVEC (Examples/Iceland/Iceland_parent/cppdefs.opt:41-46)


class OrCfg(ctypes.Structure):
    _fields_ = [("LLm", ctypes.c_int), ("MMm", ctypes.c_int), ("N", ctypes.c_int), ("NT", ctypes.c_int),
                ("ew_periodic", ctypes.c_int), ("ns_periodic", ctypes.c_int),
                ("salinity", ctypes.c_int), ("nonlin_eos", ctypes.c_int), ("lmd", ctypes.c_int),
                ("case_id", ctypes.c_int), ("ntimes", ctypes.c_int),
                ("dt", ctypes.c_double), ("ndtfast", ctypes.c_int),
                ("theta_s", ctypes.c_double), ("theta_b", ctypes.c_double), ("hc", ctypes.c_double),
                ("rho0", ctypes.c_double), ("visc2", ctypes.c_double), ("tnu2", ctypes.c_double),
                ("rdrg", ctypes.c_double), ("rdrg2", ctypes.c_double), ("Zob", ctypes.c_double),
                ("Akv_bak", ctypes.c_double), ("Akt_bak", ctypes.c_double * 2),
                ("Tcoef", ctypes.c_double), ("T0", ctypes.c_double), ("Scoef", ctypes.c_double),
                ("S0", ctypes.c_double), ("sizex", ctypes.c_double), ("sizey", ctypes.c_double),
                ("diag_np_xi", ctypes.c_int), ("diag_np_eta", ctypes.c_int), ("surf_flux", ctypes.c_int),
                ("obc", ctypes.c_int), ("ubind", ctypes.c_double), ("v_sponge", ctypes.c_double),
                ("island", ctypes.c_int), ("curvgrid", ctypes.c_int), ("uv_adv", ctypes.c_int),
                ("uv_cor", ctypes.c_int), ("pot_tides", ctypes.c_int),
                ("bulk_frc", ctypes.c_int), ("adv_isoneutral", ctypes.c_int)]

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        # every reference case defines UV_ADV and UV_COR
        if "uv_adv" not in k:
            self.uv_adv = 1
        if "uv_cor" not in k:
            self.uv_cor = 1


def build():
    """Compile liboracle.so with the committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        L.or_create.restype = ctypes.c_void_p
        L.or_create.argtypes = [ctypes.POINTER(OrCfg)]
        for fn in ("or_init", "or_step"):
            getattr(L, fn).argtypes = [ctypes.c_void_p]
            getattr(L, fn).restype = ctypes.c_int
        L.or_norms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        L.or_field.restype = ctypes.POINTER(ctypes.c_double)
        L.or_field.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t)]
        L.or_iic.argtypes = [ctypes.c_void_p]
        L.or_nfast.argtypes = [ctypes.c_void_p]
        L.or_weights.argtypes = [ctypes.c_void_p]
        L.or_weights.restype = ctypes.POINTER(ctypes.c_double)
        L.or_tindex.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.or_set_tindex.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.or_destroy.argtypes = [ctypes.c_void_p]
        for fn in ("or_set_HUV", "or_omega", "or_prsgrd", "or_pre_step3d", "or_set_HUV1", "or_step3d_uv1",
                   "or_visc3d", "or_step2d", "or_step3d_uv2", "or_step3d_t", "or_t3dmix", "or_set_depth",
                   "or_diag", "or_swr_frac", "or_bulk_flux"):
            getattr(L, fn).argtypes = [ctypes.c_void_p]
        L.or_rho_eos.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.or_lmd_vmix.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.or_set_iif.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.or_set_river.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double)]
        L.or_set_ub.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_double)] * 4
        L.or_frc_record.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_double,
                                    ctypes.POINTER(ctypes.c_double)]
        L.or_frc_clock.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_int]
        L.or_set_pipes.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.POINTER(ctypes.c_double)] * 4
        _lib = L
    return _lib


def filament_cfg(LLm=64, MMm=64, N=32, NT=1, salinity=False, sizex=12.8e3, sizey=3.2e3, np_xi=3, np_eta=2):
    """tests/Filament/{param.opt,benchmark.in,cppdefs.opt} of the reference."""
    c = OrCfg()
    c.LLm, c.MMm, c.N, c.NT = LLm, MMm, N, NT
    c.ew_periodic = c.ns_periodic = 1
    c.salinity = int(salinity)
    c.case_id = CASE_FILAMENT
    c.dt, c.ndtfast = 5.0, 60
    c.theta_s, c.theta_b, c.hc, c.rho0 = 6.0, 2.0, 25.0, 1000.0
    c.rdrg, c.rdrg2, c.Zob = 0.0, 1.0e-3, 1.0e-2
    c.Tcoef, c.T0, c.Scoef, c.S0 = 0.20, 1.0, 0.822, 1.0
    c.sizex, c.sizey = sizex, sizey
    c.diag_np_xi, c.diag_np_eta = np_xi, np_eta
    return c


def pipes_cfg(LLm=100, MMm=100, N=10, np_xi=3, np_eta=2):
    """tests/Pipes_ana/{param.opt,benchmark.in,cppdefs.opt,ana_grid.h,ana_init.h,ana_pipe_frc.h}:
    KPP/BKPP/RIMIX/CONVEC/NONLOCAL, NONLIN+SPLIT EOS, T+S, land mask, one pipe.
    benchmark.in has no vertical_mixing line, so Akv_bak = Akt_bak = 0."""
    c = OrCfg()
    c.LLm, c.MMm, c.N, c.NT = LLm, MMm, N, 2
    c.ew_periodic = c.ns_periodic = 0
    c.salinity, c.nonlin_eos, c.lmd = 1, 1, LMD_ALL
    c.case_id = CASE_PIPES
    c.dt, c.ndtfast = 60.0, 30
    c.theta_s, c.theta_b, c.hc, c.rho0 = 6.0, 6.0, 25.0, 1027.5
    c.visc2, c.tnu2 = 0.0, 0.0
    c.rdrg, c.rdrg2, c.Zob = 0.0, 1.0e-3, 1.0e-2
    c.Akv_bak = 0.0
    c.Akt_bak[0] = c.Akt_bak[1] = 0.0
    c.sizex, c.sizey = 30.0e3, 30.0e3
    c.diag_np_xi, c.diag_np_eta = np_xi, np_eta
    return c


def rivers_cfg(LLm=100, MMm=100, N=10, np_xi=3, np_eta=2):
    """tests/Rivers_ana/{param.opt,benchmark.in,cppdefs.opt,ana_grid.h,ana_init.h,
    ana_frc_river.h,river_frc.opt}: the Pipes_ana physics (KPP/BKPP/RIMIX/CONVEC/
    NONLOCAL, NONLIN+SPLIT EOS, T+S, land mask) on a 10 km shelf (depth 5..100 m,
    f = 0) with one analytic river (river_frc.F: riv_vol = 500 m3/s, T = 24,
    S = 1) entering through the 20 cells of the channel mouth; dt = 20 s."""
    c = pipes_cfg(LLm, MMm, N, np_xi, np_eta)
    c.case_id = CASE_RIVERS
    c.dt, c.ndtfast = 20.0, 30
    c.sizex, c.sizey = 10.0e3, 10.0e3
    return c


class Oracle:
    """One CPU model instance; field() returns Fortran-ordered numpy views."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.L = lib()
        self.h = self.L.or_create(ctypes.byref(cfg))
        self.nx2, self.ny2 = cfg.LLm + 4, cfg.MMm + 4

    def init(self):
        self.L.or_init(self.h)

    def step(self, n=1):
        for _ in range(n):
            self.L.or_step(self.h)

    def norms(self):
        out = (ctypes.c_double * 4)()
        self.L.or_norms(self.h, out)
        return list(out)

    def field(self, name):
        cnt = ctypes.c_size_t()
        p = self.L.or_field(self.h, name.encode(), ctypes.byref(cnt))
        if not p:
            raise KeyError(name)
        a = np.ctypeslib.as_array(p, shape=(cnt.value,))
        n2 = self.nx2 * self.ny2
        return a.reshape((cnt.value // n2, self.ny2, self.nx2)) if cnt.value % n2 == 0 else a

    def tindex(self):
        out = (ctypes.c_int * 6)()
        self.L.or_tindex(self.h, out)
        return list(out)

    def set_tindex(self, t):
        self.L.or_set_tindex(self.h, (ctypes.c_int * 6)(*t))

    def nfast(self):
        return self.L.or_nfast(self.h)

    def weights(self):
        p = self.L.or_weights(self.h)
        w = np.ctypeslib.as_array(p, shape=(2 * 288,)).reshape(2, 288)
        return w.copy()

    def set_river(self, vol, trc):
        """river_frc.F set_river_frc for one river: riv_vol, riv_trc(1:NT)."""
        v = np.ascontiguousarray([vol], dtype=np.float64)
        t = np.ascontiguousarray(trc, dtype=np.float64)
        P = ctypes.POINTER(ctypes.c_double)
        self.L.or_set_river(self.h, 1, v.ctypes.data_as(P), t.ctypes.data_as(P))

    def set_ub(self, ub):
        """SPONGE_TUNE ub_west/east/south/north (sequence of 4 arrays or None)."""
        P = ctypes.POINTER(ctypes.c_double)
        keep = [None if a is None else np.ascontiguousarray(a, dtype=np.float64) for a in ub]
        args = [None if a is None else a.ctypes.data_as(P) for a in keep]
        self.L.or_set_ub(self.h, *args)

    def set_pipes(self, idx, flx, prf, trc):
        """set_pipe_frc (pipe_frc.F:33-80): idx/flx on the (-1:Lm+2,-1:Mm+2) grid
        (pipe number, 0 = none), prf (npip, N), trc (npip, NT)."""
        P = ctypes.POINTER(ctypes.c_double)
        prf = np.asfortranarray(prf, dtype=np.float64)
        trc = np.asfortranarray(trc, dtype=np.float64)
        keep = [np.ascontiguousarray(idx, dtype=np.float64).ravel(), np.ascontiguousarray(flx, dtype=np.float64).ravel(),
                prf.ravel(order="F"), trc.ravel(order="F")]
        assert keep[0].size == self.nx2 * self.ny2 and keep[1].size == self.nx2 * self.ny2
        assert prf.shape[1] == self.cfg.N and trc.shape == (prf.shape[0], self.cfg.NT)
        if self.L.or_set_pipes(self.h, prf.shape[0], *[a.ctypes.data_as(P) for a in keep]) != 0:
            raise ValueError("or_set_pipes")

    def frc_record(self, name, slot, rec_time, arr):
        """set_frc_data record `slot` (0/1/2) of field `name` at rec_time [days]."""
        a = np.ascontiguousarray(arr, dtype=np.float64).ravel()
        if self.L.or_frc_record(self.h, name.encode(), slot, rec_time,
                                a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))) != 0:
            raise KeyError(name)

    def frc_clock(self, start_time, on=True):
        """Interpolate the recorded fields at roms_step's set_forces /
        set_bry_all points (main.F:373-441), time = start + dt*(iic-ntstart)."""
        self.L.or_frc_clock(self.h, start_time, int(on))

    def call(self, routine, *args):
        getattr(self.L, "or_" + routine)(self.h, *args)

    def __del__(self):
        try:
            self.L.or_destroy(self.h)
        except Exception:
            pass
