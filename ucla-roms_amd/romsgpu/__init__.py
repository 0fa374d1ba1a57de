"""romsgpu -- host-side mirror of the UCLA-ROMS hot-path routines on MI355X.

The reference drives its split-explicit step from Fortran (main.F:333-520)
by calling argument-less / (tile) / (tidx) subroutines that operate on module
arrays.  ``Model`` exposes the same routines with the same names and the same
time-index bookkeeping (scalars.F: iic, kstp, knew, nstp, nrhs, nnew), backed
by ``libromsgpu.so`` (HIP kernels for gfx950 behind the C ABI declared in
include/roms_gpu.h).  There is no CPU fallback: constructing a Model without
the built library or without a GPU raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("ROMS_GPU_LIB") or os.path.join(_PKG, "libromsgpu.so")   # ROMS_GPU_LIB: A/B builds only
MAX_FAST = 288

FIELDS = ["h", "hinv", "f", "fomn", "pm", "pn", "dm_r", "dn_r", "dm_u", "dn_u", "dm_v", "dn_v", "dm_p", "dn_p",
          "pmon_u", "pnom_v", "rmask", "pmask", "umask", "vmask", "Cs_w", "Cs_r",
          "zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "FlxV", "We", "Wi", "Hz", "Hz_u", "Hz_v", "z_r", "z_w",
          "rufrc", "rvfrc", "rhoA", "rhoS", "r_D", "Zt_avg1", "DU_avg1", "DV_avg1", "DU_avg2", "DV_avg2",
          "DU_avg_bak", "DV_avg_bak", "rho", "rho1", "qp1", "bvf", "Akv", "Akt", "visc2_r", "visc2_p", "diff2",
          "hbls", "hbbl", "ghat", "swr_frac", "sustr", "svstr", "stflx", "srflx", "swflx", "ru", "rv"] + \
         ["%s_%s" % (v, e) for v in ("zeta", "ubar", "vbar", "u", "v", "t") for e in ("west", "east", "south", "north")] + \
         ["dndx", "dmde", "ptide", "uwnd", "vwnd", "tair", "qair", "prate", "swrad", "lwrad", "sustr_r", "svstr_r"]
FIELD_ID = {n: i for i, n in enumerate(FIELDS)}
CASE_FILAMENT, CASE_BASIN, CASE_PIPES, CASE_RIVERS = 0, 1, 2, 3
# LMD switch bits (ROMS_LMD_* of include/roms_gpu.h)
LMD_MIXING, LMD_KPP, LMD_BKPP, LMD_RIMIX, LMD_CONVEC, LMD_NONLOCAL = 1, 2, 4, 8, 16, 32
LMD_DDMIX = 64    # double diffusion (lmd_vmix.F:279-360), needs salinity
LMD_ALL = 63       # tests/Pipes_ana/cppdefs.opt
LMD_ICELAND = 47   # Examples/Iceland/Iceland_parent/cppdefs.opt: no LMD_CONVEC


def lmd_bits(lmd):
    """True -> every LMD switch (the Pipes_ana set), False -> 0, else the bits."""
    if lmd is True:
        return LMD_ALL
    return int(lmd)


class Dims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("Lm", "Mm", "N", "NT", "LLm", "MMm", "np_xi", "np_eta", "inode", "jnode", "iSW_corn", "jSW_corn",
                 "ew_periodic", "ns_periodic", "west_exchng", "east_exchng", "south_exchng", "north_exchng")]


class Cfg(ctypes.Structure):
    _fields_ = [("nonlin_eos", ctypes.c_int), ("salinity", ctypes.c_int), ("lmd_mixing", ctypes.c_int),
                ("uv_vis2", ctypes.c_int), ("ts_dif2", ctypes.c_int), ("dt", ctypes.c_double),
                ("ndtfast", ctypes.c_int), ("nfast", ctypes.c_int), ("weight", (ctypes.c_double * MAX_FAST) * 2),
                ("g", ctypes.c_double), ("rho0", ctypes.c_double), ("rdrg", ctypes.c_double),
                ("rdrg2", ctypes.c_double), ("Zob", ctypes.c_double), ("gamma2", ctypes.c_double),
                ("Akv_bak", ctypes.c_double), ("Akt_bak", ctypes.c_double * 2), ("Tcoef", ctypes.c_double),
                ("T0", ctypes.c_double), ("Scoef", ctypes.c_double), ("S0", ctypes.c_double),
                ("theta_s", ctypes.c_double), ("theta_b", ctypes.c_double), ("hc", ctypes.c_double),
                ("obc", ctypes.c_int), ("ubind", ctypes.c_double), ("curvgrid", ctypes.c_int),
                ("uv_adv", ctypes.c_int), ("uv_cor", ctypes.c_int), ("pot_tides", ctypes.c_int),
                ("bulk_frc", ctypes.c_int), ("adv_isoneutral", ctypes.c_int)]


class Tlev(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("iic", "ntstart", "forw_start", "iif", "nfast", "kstp", "knew", "nstp", "nrhs", "nnew")]

    def as_list(self):
        return [self.iic, self.kstp, self.knew, self.nstp, self.nrhs, self.nnew]


class Case(ctypes.Structure):
    _fields_ = [("case_id", ctypes.c_int), ("LLm", ctypes.c_int), ("MMm", ctypes.c_int), ("N", ctypes.c_int),
                ("NT", ctypes.c_int), ("salinity", ctypes.c_int), ("nonlin_eos", ctypes.c_int),
                ("lmd_mixing", ctypes.c_int), ("dt", ctypes.c_double), ("ndtfast", ctypes.c_int),
                ("sizex", ctypes.c_double), ("sizey", ctypes.c_double), ("surf_flux", ctypes.c_int),
                ("obc", ctypes.c_int), ("v_sponge", ctypes.c_double), ("island", ctypes.c_int),
                ("curvgrid", ctypes.c_int), ("uv_adv", ctypes.c_int), ("uv_cor", ctypes.c_int),
                ("bulk_frc", ctypes.c_int), ("adv_isoneutral", ctypes.c_int)]


ROUTINES_T = ["set_huv", "omega", "prsgrd", "pre_step3d", "set_huv1", "step3d_uv1", "visc3d", "step2d",
              "step3d_uv2", "step3d_t", "t3dmix", "set_depth", "swr_frac", "step", "init_sequence"]

_lib = None


def load_library(path=LIB_PATH):
    """Load libromsgpu.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError("romsgpu: %s not built -- run __graft_entry__.build()" % path)
    L = ctypes.CDLL(path)
    P = ctypes.POINTER
    L.roms_gpu_last_error.restype = ctypes.c_char_p
    L.roms_gpu_init.argtypes = [P(Dims), P(Cfg), ctypes.c_int, ctypes.c_void_p]
    L.roms_gpu_init_case.argtypes = [P(Case), ctypes.c_int, P(Tlev)]
    L.roms_gpu_field_size.argtypes = [ctypes.c_int]
    L.roms_gpu_field_size.restype = ctypes.c_long
    for fn in ("roms_gpu_copy_in", "roms_gpu_copy_out", "roms_gpu_register"):
        getattr(L, fn).argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_long]
    L.roms_gpu_upload.argtypes = [ctypes.c_int]
    L.roms_gpu_download.argtypes = [ctypes.c_int]
    for fn in ROUTINES_T:
        getattr(L, "roms_gpu_" + fn).argtypes = [P(Tlev)]
    L.roms_gpu_rho_eos.argtypes = [ctypes.c_int, P(Tlev)]
    L.roms_gpu_lmd_vmix.argtypes = [ctypes.c_int, P(Tlev)]
    L.roms_gpu_set_pipe_frc.argtypes = [ctypes.c_int, P(ctypes.c_int), P(ctypes.c_double), P(ctypes.c_double),
                                        P(ctypes.c_double)]
    L.roms_gpu_set_river_frc.argtypes = [ctypes.c_int, P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_double),
                                         P(ctypes.c_double)]
    L.roms_gpu_bulk_flux.argtypes = [P(Tlev)]
    L.roms_gpu_set_ub_tune.argtypes = [P(ctypes.c_double)] * 4
    L.roms_gpu_frc_record.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, P(ctypes.c_double)]
    L.roms_gpu_frc_interp.argtypes = [ctypes.c_double, ctypes.c_int]
    L.roms_gpu_frc_clock.argtypes = [ctypes.c_double, ctypes.c_int]
    L.roms_gpu_set_tide_data.argtypes = [ctypes.c_int] + [P(ctypes.c_double)] * 9
    L.roms_gpu_set_tides.argtypes = [ctypes.c_double]
    L.roms_gpu_diag.argtypes = [P(Tlev), P(ctypes.c_double)]
    L.roms_gpu_time_steps.argtypes = [P(Tlev), ctypes.c_int, P(ctypes.c_double)]
    L.roms_gpu_stream.restype = ctypes.c_void_p
    L.roms_gpu_time_routine.argtypes = [ctypes.c_int, ctypes.c_int, P(Tlev), P(ctypes.c_double), P(ctypes.c_long)]
    L.roms_gpu_init_case_comm.argtypes = [P(Case), ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, P(Tlev)]
    L.roms_gpu_comm_unique_id.argtypes = [ctypes.c_void_p]
    L.roms_gpu_comm_create.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       P(ctypes.c_void_p)]
    L.roms_gpu_comm_create_local.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P(ctypes.c_void_p)]
    L.roms_gpu_comm_create_host.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, HOST_ALLGATHER_FN,
                                            ctypes.c_void_p, P(ctypes.c_void_p)]
    L.roms_gpu_comm_destroy.argtypes = [ctypes.c_void_p]
    L.roms_gpu_halo_plan.argtypes = [ctypes.c_int] * 8 + [P(ctypes.c_int), P(ctypes.c_long), P(ctypes.c_int)]
    L.roms_gpu_halo_map.argtypes = [ctypes.c_int] * 10 + [P(ctypes.c_int), P(ctypes.c_int), ctypes.c_long]
    L.roms_gpu_halo_map.restype = ctypes.c_long
    L.roms_gpu_halo_map_wide.argtypes = [ctypes.c_int] * 11 + [P(ctypes.c_int), P(ctypes.c_int), ctypes.c_long]
    L.roms_gpu_halo_map_wide.restype = ctypes.c_long
    L.roms_gpu_wrt_rst.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_double, P(Tlev)]
    L.roms_gpu_wrt_his.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_double, P(Tlev), ctypes.c_int]
    L.roms_gpu_get_init.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, P(Tlev), P(ctypes.c_double)]
    L.roms_gpu_io_tracer_name.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    _lib = L
    return L


class RomsGpuError(RuntimeError):
    pass


def _check(L, rc, what):
    if rc != 0:
        raise RomsGpuError("%s failed (%d): %s" % (what, rc, L.roms_gpu_last_error().decode()))


def rank_extent(LL, np_, node):
    """(length, SW-corner offset) of a subdomain along one direction (mpi_setup.F:110-154)."""
    base = (LL + np_ - 1) // np_
    off = np_ * base - LL
    sw = 0 if node == 0 else node * base - off // 2
    n = base
    if node == 0:
        n -= off // 2
    if node == np_ - 1:
        n -= (off + 1) // 2
    return n, sw


def halo_plan(Lm, Mm, np_xi, np_eta, inode, jnode, ew_periodic, ns_periodic):
    """Neighbour ranks, per-level message sizes (W,E,S,N,SW,SE,NW,NE) and strip
    extents (i0,i1,j0,j1) of the library's halo exchange (host-only call)."""
    L = load_library()
    peer = (ctypes.c_int * 8)()
    cnt = (ctypes.c_long * 8)()
    strip = (ctypes.c_int * 4)()
    rc = L.roms_gpu_halo_plan(Lm, Mm, np_xi, np_eta, inode, jnode, int(ew_periodic), int(ns_periodic), peer, cnt, strip)
    if rc != 0:
        raise ValueError("bad halo plan arguments")
    return list(peer), list(cnt), tuple(strip)


def halo_map(Lm, Mm, np_xi, np_eta, inode, jnode, ew_periodic, ns_periodic, direction, unpack, width=2):
    """(i, j) arrays of the cells direction `direction` packs (unpack=False) or
    fills (unpack=True), in message order (host-only call); width > 2: the
    fast loop's width-deep exchange (roms_gpu_halo_map_wide)."""
    L = load_library()
    cap = max(width, 2) * (max(Lm, Mm) + 4)
    iv = (ctypes.c_int * cap)()
    jv = (ctypes.c_int * cap)()
    if width == 2:
        n = L.roms_gpu_halo_map(Lm, Mm, np_xi, np_eta, inode, jnode, int(ew_periodic), int(ns_periodic), direction,
                                int(unpack), iv, jv, cap)
    else:
        n = L.roms_gpu_halo_map_wide(Lm, Mm, np_xi, np_eta, inode, jnode, int(ew_periodic), int(ns_periodic), width,
                                     direction, int(unpack), iv, jv, cap)
    if n < 0:
        raise ValueError("bad halo map arguments")
    return np.array(iv[:n]), np.array(jv[:n])


HALO_DIRS = ("W", "E", "S", "N", "SW", "SE", "NW", "NE")
# ROMS_WRT_* of include/roms_gpu.h (ocean_vars.opt wrt_* switches)
WRT = dict(Z=1, Ub=2, Vb=4, U=8, V=16, T=32, R=64, O=128, Akv=256, Akt=512, Aks=1024, Hbls=2048, Hbbl=4096)
WRT_DEFAULT = 63
# enum roms_routine of include/roms_gpu.h
ROUTINES = ("rho_eos", "set_HUV", "omega", "prsgrd", "pre_step3d", "set_HUV1", "step3d_uv1", "visc3d", "step2d",
            "step3d_uv2", "step3d_t", "t3dmix", "lmd_vmix",
            "k_s2d_fb",  # kernel level: the fused barotropic kernel alone
            "k_pre_uv_seg", "k_uv1_seg", "k_step3d_t_seg", "k_prsgrd_uv",  # kernel level: the N > 63 column solvers
            "k_halo_pack", "k_halo_wait", "k_halo_unpack")  # halo path: pack / transport / unpack of every exchange
HALO_OPP = (1, 0, 3, 2, 7, 6, 5, 4)


def comm_unique_id():
    """128-byte RCCL id (rank 0); broadcast it with the host's own collective."""
    L = load_library()
    buf = ctypes.create_string_buffer(128)
    _check(L, L.roms_gpu_comm_unique_id(buf), "roms_gpu_comm_unique_id")
    return buf.raw


def comm_create(uid, nranks, rank, device=0):
    """RCCL communicator handle for roms_gpu_init / init_case_comm."""
    L = load_library()
    h = ctypes.c_void_p()
    buf = ctypes.create_string_buffer(bytes(uid), 128)
    _check(L, L.roms_gpu_comm_create(buf, nranks, rank, device, ctypes.byref(h)), "roms_gpu_comm_create")
    return h


def comm_create_local(group, nranks, rank):
    """Handle for subdomains driven by threads of this process (one per thread)."""
    L = load_library()
    h = ctypes.c_void_p()
    _check(L, L.roms_gpu_comm_create_local(group, nranks, rank, ctypes.byref(h)), "roms_gpu_comm_create_local")
    return h


# roms_host_allgather_fn of include/roms_gpu.h
HOST_ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p)
_host_channels = {}   # comm handle value -> the ctypes callback (kept alive while the handle is)


def comm_create_host(nranks, rank, allgather, device=0):
    """Host-channel communicator: `allgather(data: bytes) -> list of nranks
    bytes objects` is the host's own collective (the MPI_Allgather a Fortran
    host passes); halos then move by IPC peer writes with RCCL out of the loop."""
    L = load_library()

    def fn(_ctx, send, nbytes, recv):
        try:
            parts = allgather(ctypes.string_at(send, nbytes))
            if len(parts) != nranks or any(len(x) != nbytes for x in parts):
                return -1
            ctypes.memmove(recv, b"".join(parts), nbytes * nranks)
            return 0
        except Exception:   # a failed collective is reported as a status, never raised through C
            return -1

    cb = HOST_ALLGATHER_FN(fn)
    h = ctypes.c_void_p()
    _check(L, L.roms_gpu_comm_create_host(nranks, rank, device, cb, None, ctypes.byref(h)), "roms_gpu_comm_create_host")
    _host_channels[h.value] = cb
    return h


class FileAllgather:
    """A host allgather through files in a shared directory (tests and
    single-node runs without MPI): call k of every rank writes its bytes to
    ag<k>.<rank> and reads everyone's.  A rank's file of call k-2 is removed at
    call k: by then every rank has finished reading it."""

    def __init__(self, path, nranks, rank, timeout=120.0):
        self.path, self.n, self.r, self.timeout, self.k = path, nranks, rank, timeout, 0

    def _f(self, k, r):
        return os.path.join(self.path, "ag%d.%d" % (k, r))

    def __call__(self, data):
        import time
        k = self.k
        self.k += 1
        tmp = self._f(k, self.r) + ".tmp"
        with open(tmp, "wb") as fh:
            fh.write(data)
        os.rename(tmp, self._f(k, self.r))
        if k >= 2:
            try:
                os.remove(self._f(k - 2, self.r))
            except OSError:
                pass
        out, t0 = [], time.time()
        for r in range(self.n):
            f = self._f(k, r)
            while not os.path.exists(f):
                if time.time() - t0 > self.timeout:
                    raise TimeoutError("allgather %d: rank %d missing" % (k, r))
                time.sleep(0.001)
            with open(f, "rb") as fh:
                out.append(fh.read())
        return out


def comm_destroy(h):
    load_library().roms_gpu_comm_destroy(h)
    _host_channels.pop(getattr(h, "value", h), None)


class Model:
    """One rank's device-resident model state and the reference's routines."""

    def __init__(self):
        self.L = load_library()
        self.t = Tlev()
        self.shape2 = None

    def _chk(self, rc, what):
        if rc != 0:
            raise RomsGpuError("%s failed (%d): %s" % (what, rc, self.L.roms_gpu_last_error().decode()))

    # ---- construction ----
    @classmethod
    def from_case(cls, case_id, LLm, MMm, N, NT=1, salinity=False, nonlin_eos=False, dt=5.0, ndtfast=60,
                  sizex=12.8e3, sizey=3.2e3, device=0, np_xi=1, np_eta=1, comm=None, rank=0, lmd=False,
                  surf_flux=False, obc=0, v_sponge=0.0, island=False, curvgrid=False, uv_adv=True, uv_cor=True,
                  bulk_frc=False, adv_isoneutral=False):
        """Analytic case on the whole grid, or on subdomain `rank` of an
        np_xi x np_eta processor grid when a communicator is given.
        lmd: False, True (all LMD switches) or ROMS_LMD_* bits."""
        m = cls()
        c = Case(case_id, LLm, MMm, N, NT, int(salinity), int(nonlin_eos), lmd_bits(lmd), dt, ndtfast, sizex, sizey,
                 int(surf_flux), int(obc), float(v_sponge), int(island), int(curvgrid), int(uv_adv), int(uv_cor),
                 int(bulk_frc), int(adv_isoneutral))
        if comm is None and np_xi * np_eta == 1:
            m._chk(m.L.roms_gpu_init_case(ctypes.byref(c), device, ctypes.byref(m.t)), "roms_gpu_init_case")
        else:
            m._chk(m.L.roms_gpu_init_case_comm(ctypes.byref(c), np_xi, np_eta, comm, device, ctypes.byref(m.t)),
                   "roms_gpu_init_case_comm")
        m.LLm, m.MMm, m.N, m.NT = LLm, MMm, N, NT
        m.jnode, m.inode = divmod(rank, np_xi)
        m.Lm, m.iSW = rank_extent(LLm, np_xi, m.inode)
        m.Mm, m.jSW = rank_extent(MMm, np_eta, m.jnode)
        m.shape2 = (m.Mm + 4, m.Lm + 4)
        return m

    @classmethod
    def from_dims(cls, dims, cfg, device=0):
        m = cls()
        m._chk(m.L.roms_gpu_init(ctypes.byref(dims), ctypes.byref(cfg), device, None), "roms_gpu_init")
        m.LLm, m.MMm, m.N, m.NT = dims.Lm, dims.Mm, dims.N, dims.NT
        m.shape2 = (dims.Mm + 4, dims.Lm + 4)
        return m

    def close(self):
        self.L.roms_gpu_finalize()
        self._host = {}

    # ---- host mirrors (roms_gpu_register / upload / download): the way a
    # Fortran host hands its module arrays to the library ----
    def register(self, name, arr):
        """Borrow the host array `arr` (float64, C-contiguous, the field's
        Fortran layout) as the mirror of field `name` until close()."""
        fid = FIELD_ID[name]
        if arr.dtype != np.float64 or not arr.flags["C_CONTIGUOUS"]:
            raise ValueError("register: %s must be a contiguous float64 array" % name)
        self._chk(self.L.roms_gpu_register(fid, arr.ctypes.data, arr.size), "register " + name)
        if not hasattr(self, "_host"):
            self._host = {}
        self._host[name] = arr   # keep the borrowed buffer alive

    def upload(self, name=None):
        self._chk(self.L.roms_gpu_upload(-1 if name is None else FIELD_ID[name]), "upload")

    def download(self, name=None):
        self._chk(self.L.roms_gpu_download(-1 if name is None else FIELD_ID[name]), "download")

    # ---- state access (Fortran layout, returned as (levels, j, i) C arrays) ----
    def get(self, name):
        fid = FIELD_ID[name]
        n = self.L.roms_gpu_field_size(fid)
        a = np.empty(n, dtype=np.float64)
        self._chk(self.L.roms_gpu_copy_out(fid, a.ctypes.data, n), "copy_out " + name)
        n2 = self.shape2[0] * self.shape2[1]
        return a.reshape((n // n2,) + self.shape2) if n % n2 == 0 else a

    def put(self, name, arr):
        fid = FIELD_ID[name]
        a = np.ascontiguousarray(arr, dtype=np.float64).ravel()
        n = self.L.roms_gpu_field_size(fid)
        if a.size != n:
            raise ValueError("%s: expected %d elements, got %d" % (name, n, a.size))
        self._chk(self.L.roms_gpu_copy_in(fid, a.ctypes.data, n), "copy_in " + name)

    def set_tindex(self, iic, kstp, knew, nstp, nrhs, nnew, iif=1, forw_start=1, ntstart=1, nfast=None):
        self.t.iic, self.t.kstp, self.t.knew, self.t.nstp, self.t.nrhs, self.t.nnew = iic, kstp, knew, nstp, nrhs, nnew
        self.t.iif, self.t.forw_start, self.t.ntstart = iif, forw_start, ntstart
        if nfast is not None:
            self.t.nfast = nfast

    def sync(self):
        self._chk(self.L.roms_gpu_sync(), "sync")

    # ---- reference routines ----
    def rho_eos(self, tidx):
        self._chk(self.L.roms_gpu_rho_eos(tidx, ctypes.byref(self.t)), "rho_eos")

    def lmd_vmix(self, tind):
        self._chk(self.L.roms_gpu_lmd_vmix(tind, ctypes.byref(self.t)), "lmd_vmix")

    def set_pipe_frc(self, pipe_idx, pipe_flx, pipe_prf, pipe_trc):
        """pipe_frc.F:set_pipe_frc: pipe_idx/pipe_flx on the (Mm+4, Lm+4) grid,
        pipe_prf (npip, N) and pipe_trc (npip, NT)."""
        prf = np.asarray(pipe_prf, dtype=np.float64)
        npip = prf.shape[0]
        idx = np.ascontiguousarray(pipe_idx, dtype=np.int32).ravel()
        flx = np.ascontiguousarray(pipe_flx, dtype=np.float64).ravel()
        prf = np.asfortranarray(prf).ravel(order="F")
        trc = np.asarray(pipe_trc, dtype=np.float64).ravel(order="F")
        P = ctypes.POINTER
        self._chk(self.L.roms_gpu_set_pipe_frc(npip, idx.ctypes.data_as(P(ctypes.c_int)), flx.ctypes.data_as(P(ctypes.c_double)),
                                               prf.ctypes.data_as(P(ctypes.c_double)), trc.ctypes.data_as(P(ctypes.c_double))),
                  "set_pipe_frc")

    def set_river_frc(self, riv_vol, riv_trc, riv_uflx=None, riv_vflx=None):
        """river_frc.F:set_river_frc: riv_vol (nriv,), riv_trc (nriv, NT) for the
        current time; riv_uflx/riv_vflx on the (Mm+4, Lm+4) grid as
        calc_river_flux leaves them (None: keep the faces already set)."""
        vol = np.ascontiguousarray(riv_vol, dtype=np.float64).ravel()
        nriv = vol.shape[0]
        trc = np.asfortranarray(np.asarray(riv_trc, dtype=np.float64).reshape(nriv, -1)).ravel(order="F")
        P = ctypes.POINTER
        D = P(ctypes.c_double)
        if riv_uflx is None:
            uf = vf = None
        else:
            uf = np.ascontiguousarray(riv_uflx, dtype=np.float64).ravel()
            vf = np.ascontiguousarray(riv_vflx, dtype=np.float64).ravel()
        self._chk(self.L.roms_gpu_set_river_frc(nriv, uf.ctypes.data_as(D) if uf is not None else None,
                                                vf.ctypes.data_as(D) if vf is not None else None,
                                                vol.ctypes.data_as(D), trc.ctypes.data_as(D)), "set_river_frc")

    def set_ub_tune(self, ub):
        """SPONGE_TUNE: ub_west, ub_east (Mm+2), ub_south, ub_north (Lm+2); None = edge off."""
        D = ctypes.POINTER(ctypes.c_double)
        keep = [None if a is None else np.ascontiguousarray(a, dtype=np.float64) for a in ub]
        self._chk(self.L.roms_gpu_set_ub_tune(*[None if a is None else a.ctypes.data_as(D) for a in keep]),
                  "set_ub_tune")

    # ---- forcing / boundary producers on the device (set_frc_data, set_tides) ----
    FRC_SURFACE, FRC_BRY = 1, 2

    def frc_record(self, name, slot, rec_time, arr):
        """One forcing record (time in days) of field `name` into slot 0/1."""
        a = np.ascontiguousarray(arr, dtype=np.float64).ravel()
        if a.size != self.L.roms_gpu_field_size(FIELD_ID[name]):
            raise ValueError("frc_record: %s has %d elements" % (name, a.size))
        self._chk(self.L.roms_gpu_frc_record(FIELD_ID[name], slot, rec_time,
                                             a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))), "frc_record")

    def frc_interp(self, modtime, kinds=3):
        self._chk(self.L.roms_gpu_frc_interp(modtime, kinds), "frc_interp")

    def frc_clock(self, start_time, on=True):
        """In-step forcing: every step interpolates the recorded fields at
        roms_step's set_forces / set_bry_all points (and runs set_tides)."""
        self._chk(self.L.roms_gpu_frc_clock(start_time, int(on)), "frc_clock")

    def set_tide_data(self, ftide, pot=None, bry=None):
        """ftide (ntides,) [1/s]; pot = (re, im), bry = ((zre, zim), (ure, uim), (vre, vim)),
        each (ntides, Mm+4, Lm+4) or None."""
        D = ctypes.POINTER(ctypes.c_double)
        keep = [np.ascontiguousarray(ftide, dtype=np.float64)]
        def ptr(a):
            if a is None:
                return None
            keep.append(np.ascontiguousarray(a, dtype=np.float64))
            return keep[-1].ctypes.data_as(D)
        pr, pi = pot if pot is not None else (None, None)
        (zr, zi), (ur, ui), (vr, vi) = bry if bry is not None else ((None, None),) * 3
        self._chk(self.L.roms_gpu_set_tide_data(len(keep[0]), keep[0].ctypes.data_as(D), ptr(pr), ptr(pi), ptr(zr),
                                                ptr(zi), ptr(ur), ptr(ui), ptr(vr), ptr(vi)), "set_tide_data")

    def set_tides(self, time):
        self._chk(self.L.roms_gpu_set_tides(time), "set_tides")

    def bulk_flux(self):
        """set_bulk_frc -> calc_all_bulk_forces on the device at the current nrhs."""
        self._chk(self.L.roms_gpu_bulk_flux(ctypes.byref(self.t)), "bulk_flux")

    def _r(self, fn):
        self._chk(getattr(self.L, "roms_gpu_" + fn)(ctypes.byref(self.t)), fn)

    def set_HUV(self): self._r("set_huv")
    def omega(self): self._r("omega")
    def prsgrd(self): self._r("prsgrd")
    def pre_step3d(self): self._r("pre_step3d")
    def set_HUV1(self): self._r("set_huv1")
    def step3d_uv1(self): self._r("step3d_uv1")
    def visc3d(self): self._r("visc3d")
    def step2d(self): self._r("step2d")
    def step3d_uv2(self): self._r("step3d_uv2")
    def step3d_t(self): self._r("step3d_t")
    def t3dmix(self): self._r("t3dmix")
    def set_depth(self): self._r("set_depth")
    def swr_frac(self): self._r("swr_frac")
    def init_sequence(self): self._r("init_sequence")

    def step(self, n=1):
        """roms_step (main.F:333-520) n times; updates the time indices."""
        for _ in range(n):
            self._r("step")

    def time_routine(self, routine, nsteps):
        """Mean duration [ms] of one call of `routine` (name in ROUTINES) and
        the number of calls, from HIP events around its launches over
        `nsteps` eager steps (the model advances by nsteps)."""
        ms = ctypes.c_double()
        n = ctypes.c_long()
        self._chk(self.L.roms_gpu_time_routine(ROUTINES.index(routine), nsteps, ctypes.byref(self.t), ctypes.byref(ms),
                                               ctypes.byref(n)), "time_routine")
        return ms.value, n.value

    def selftest_zero_fill(self, n, chunks=1):
        """roms_gpu_selftest_zero_fill: nonzero elements that fresh zero-filled
        allocations (chunks x n doubles, recycled memory) show to the
        library's stream (0 expected)."""
        nz = ctypes.c_long()
        self._chk(self.L.roms_gpu_selftest_zero_fill(ctypes.c_long(n), ctypes.c_int(chunks), ctypes.byref(nz)),
                  "selftest_zero_fill")
        return nz.value

    def halo_transport(self):
        """'ipc', 'rccl' (or single rank / in-process), or 'ipc-timeout'."""
        r = self.L.roms_gpu_halo_transport()
        return {1: "ipc", 0: "rccl", -1: "ipc-timeout"}.get(r, "error")

    def halo_overlap(self):
        """True when whole steps defer 3-D exchanges onto the halo stream
        (roms_gpu_halo_overlap: the default with > 1 rank, one GPU each)."""
        return bool(self.L.roms_gpu_halo_overlap())

    def s2d_window(self):
        """True when the fused fast step reads its 2-D fields through one
        buffer window (roms_gpu_s2d_window; ROMS_GPU_S2D_WIN=0: pointers)."""
        return bool(self.L.roms_gpu_s2d_window())

    def halo_exchanges(self):
        """(exchanges in the last enqueued step, fast-loop exchange interval)
        -- roms_gpu_halo_exchanges."""
        n, k = ctypes.c_long(), ctypes.c_int()
        self._chk(self.L.roms_gpu_halo_exchanges(ctypes.byref(n), ctypes.byref(k)), "halo_exchanges")
        return n.value, k.value

    def diag(self):
        out = (ctypes.c_double * 4)()
        self._chk(self.L.roms_gpu_diag(ctypes.byref(self.t), out), "diag")
        return list(out)

    # ---- on-disk formats (basic_output.F, get_init.F) ----
    def time(self, dt):
        """Model time at the end of the last step (main.F:487, start_time 0)."""
        return dt * (self.t.iic - self.t.ntstart + 1) + getattr(self, "start_time", 0.0)

    def wrt_rst(self, path, rec, total_rec, time):
        """wrt_restart_file: record rec (1-based) of this rank's restart file."""
        self._chk(self.L.roms_gpu_wrt_rst(path.encode(), rec, total_rec, time, ctypes.byref(self.t)), "wrt_rst")

    def wrt_his(self, path, rec, total_rec, time, mask=WRT_DEFAULT):
        """wrt_his_ocean_vars: record rec of this rank's history file."""
        self._chk(self.L.roms_gpu_wrt_his(path.encode(), rec, total_rec, time, ctypes.byref(self.t), mask), "wrt_his")

    def io_wait(self):
        self._chk(self.L.roms_gpu_io_wait(), "io_wait")

    def get_init(self, path, req_rec, tindx):
        """get_init(req_rec, tindx); returns 0 (read) or 1 (exact restart not possible)."""
        st = ctypes.c_double()
        rc = self.L.roms_gpu_get_init(path.encode(), req_rec, tindx, ctypes.byref(self.t), ctypes.byref(st))
        if rc < 0:
            self._chk(rc, "get_init")
        if tindx == 1:
            self.start_time = st.value
        return rc

    def restart(self, path, rec=0, exact=True):
        """main.F:244-288: get_init(rec-1, 2) [EXACT_RESTART], get_init(rec, 1),
        then set_depth, set_HUV, omega, rho_eos(nrhs) (roms_gpu_init_sequence).
        rec 0 = the last record."""
        self.t.forw_start = 0
        if exact:
            nrec = rec if rec > 0 else self._nrecs(path)
            if nrec >= 2:
                self.get_init(path, nrec - 1, 2)
            rec = nrec
        self.get_init(path, rec, 1)
        self.init_sequence()

    @staticmethod
    def _nrecs(path):
        with open(path, "rb") as f:
            h = f.read(8)
        return int.from_bytes(h[4:8], "big")

    def time_steps(self, n):
        ms = ctypes.c_double()
        self._chk(self.L.roms_gpu_time_steps(ctypes.byref(self.t), n, ctypes.byref(ms)), "time_steps")
        return ms.value
