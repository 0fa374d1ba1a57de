! roms_gpu_mod.F90 -- Fortran (iso_c_binding) interface to libromsgpu.so,
! the MI355X hot path of the split-explicit step (include/roms_gpu.h).
!
! A reference build uses it from drop-in replacements of the hot-path
! routines (fortran/dropin/*.F): each keeps the reference's signature
! (src/main.F:397-479 calls) and forwards to roms_gpu_<routine> with the
! time indices of module `scalars` packed into a roms_tlev.
module roms_gpu_mod
  use iso_c_binding
  implicit none

  integer, parameter :: ROMS_MAX_FAST = 288

  type, bind(c) :: roms_dims
    integer(c_int) :: Lm, Mm, N, NT, LLm, MMm
    integer(c_int) :: np_xi, np_eta, inode, jnode, iSW_corn, jSW_corn
    integer(c_int) :: ew_periodic, ns_periodic
    integer(c_int) :: west_exchng, east_exchng, south_exchng, north_exchng
  end type

  type, bind(c) :: roms_cfg
    integer(c_int) :: nonlin_eos, salinity, lmd_mixing, uv_vis2, ts_dif2
    real(c_double) :: dt
    integer(c_int) :: ndtfast, nfast
    real(c_double) :: weight(ROMS_MAX_FAST, 2)   ! C weight[2][288] -> Fortran (288,2)
    real(c_double) :: g, rho0, rdrg, rdrg2, Zob, gamma2
    real(c_double) :: Akv_bak, Akt_bak(2)
    real(c_double) :: Tcoef, T0, Scoef, S0
    real(c_double) :: theta_s, theta_b, hc
    integer(c_int) :: obc                        ! OBC_WEST 1, OBC_EAST 2, OBC_SOUTH 4, OBC_NORTH 8
    real(c_double) :: ubind
    integer(c_int) :: curvgrid                   ! CURVGRID
    integer(c_int) :: uv_adv, uv_cor             ! UV_ADV, UV_COR
    integer(c_int) :: pot_tides                  ! TIDES pot_tides
    integer(c_int) :: bulk_frc                   ! BULK_FRC
    integer(c_int) :: adv_isoneutral             ! ADV_ISONEUTRAL (+SW_TRIADS, STABILIZE)
  end type

  type, bind(c) :: roms_tlev
    integer(c_int) :: iic, ntstart, forw_start, iif, nfast, kstp, knew, nstp, nrhs, nnew
  end type

  type, bind(c) :: roms_case
    integer(c_int) :: case_id, LLm, MMm, N, NT, salinity, nonlin_eos, lmd_mixing
    real(c_double) :: dt
    integer(c_int) :: ndtfast
    real(c_double) :: sizex, sizey
    integer(c_int) :: surf_flux
    integer(c_int) :: obc
    real(c_double) :: v_sponge
    integer(c_int) :: island
    integer(c_int) :: curvgrid
    integer(c_int) :: uv_adv, uv_cor
    integer(c_int) :: bulk_frc
    integer(c_int) :: adv_isoneutral
  end type

  ! LMD switch bits of lmd_mixing (ROMS_LMD_*)
  integer(c_int), parameter :: ROMS_LMD_MIXING = 1, ROMS_LMD_KPP = 2, ROMS_LMD_BKPP = 4, ROMS_LMD_RIMIX = 8, &
                               ROMS_LMD_CONVEC = 16, ROMS_LMD_NONLOCAL = 32, ROMS_LMD_DDMIX = 64
  integer(c_int), parameter :: ROMS_GPU_ABI = 16   ! ROMS_GPU_ABI_VERSION, include/roms_gpu.h
  integer(c_int), parameter :: ROMS_FRC_SURFACE = 1, ROMS_FRC_BRY = 2

  ! field ids (enum roms_field) used by the drivers below
  integer(c_int), parameter :: ROMS_ALL = -1
  integer(c_int), parameter :: ROMS_zeta = 22, ROMS_ubar = 23, ROMS_vbar = 24, ROMS_u = 25, ROMS_v = 26, &
                               ROMS_t = 27, ROMS_Hz = 32, ROMS_z_r = 35, ROMS_NFIELDS = 105

  interface
    integer(c_int) function roms_gpu_abi_version() bind(c)
      import :: c_int
    end function
    integer(c_int) function roms_gpu_init(dims, cfg, device, comm) bind(c)
      import :: c_int, c_ptr, roms_dims, roms_cfg
      type(roms_dims), intent(in) :: dims
      type(roms_cfg), intent(in) :: cfg
      integer(c_int), value :: device
      type(c_ptr), value :: comm
    end function
    integer(c_int) function roms_gpu_finalize() bind(c)
      import :: c_int
    end function
    type(c_ptr) function roms_gpu_last_error() bind(c)
      import :: c_ptr
    end function
    integer(c_long) function roms_gpu_field_size(id) bind(c)
      import :: c_int, c_long
      integer(c_int), value :: id
    end function
    integer(c_int) function roms_gpu_register(id, host, count) bind(c)
      import :: c_int, c_long, c_ptr
      integer(c_int), value :: id
      type(c_ptr), value :: host
      integer(c_long), value :: count
    end function
    integer(c_int) function roms_gpu_upload(id) bind(c)
      import :: c_int
      integer(c_int), value :: id
    end function
    integer(c_int) function roms_gpu_download(id) bind(c)
      import :: c_int
      integer(c_int), value :: id
    end function
    integer(c_int) function roms_gpu_copy_out(id, dst, count) bind(c)
      import :: c_int, c_long, c_ptr
      integer(c_int), value :: id
      type(c_ptr), value :: dst
      integer(c_long), value :: count
    end function
    integer(c_int) function roms_gpu_sync() bind(c)
      import :: c_int
    end function
    ! hot-path routines (one per reference subroutine)
    integer(c_int) function roms_gpu_rho_eos(tidx, t) bind(c)
      import :: c_int, roms_tlev
      integer(c_int), value :: tidx
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_lmd_vmix(tind, t) bind(c)
      import :: c_int, roms_tlev
      integer(c_int), value :: tind
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_set_huv(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_omega(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_prsgrd(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_pre_step3d(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_set_huv1(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_step3d_uv1(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_visc3d(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_step2d(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_step3d_uv2(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_step3d_t(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_t3dmix(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_set_depth(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_swr_frac(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(in) :: t
    end function
    ! after set_forces' set_pipe_frc (pipe_frc.F:33): pipe_idx(GLOBAL_2D_ARRAY) integer,
    ! pipe_flx(GLOBAL_2D_ARRAY), pipe_prf(npip,N), pipe_trc(npip,nt)
    integer(c_int) function roms_gpu_set_pipe_frc(npip, pipe_idx, pipe_flx, pipe_prf, pipe_trc) bind(c)
      import :: c_int, c_double
      integer(c_int), value :: npip
      integer(c_int), intent(in) :: pipe_idx(*)
      real(c_double), intent(in) :: pipe_flx(*), pipe_prf(*), pipe_trc(*)
    end function
    ! set_river_frc (river_frc.F:57-282): riv_uflx/riv_vflx as calc_river_flux
    ! leaves them, riv_vol(nriv), riv_trc(nriv,nt)
    integer(c_int) function roms_gpu_set_river_frc(nriv, riv_uflx, riv_vflx, riv_vol, riv_trc) bind(c)
      import :: c_int, c_double
      integer(c_int), value :: nriv
      real(c_double), intent(in) :: riv_uflx(*), riv_vflx(*), riv_vol(*), riv_trc(*)
    end function
    integer(c_int) function roms_gpu_step(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(inout) :: t
    end function
    integer(c_int) function roms_gpu_init_sequence(t) bind(c)
      import :: c_int, roms_tlev
      type(roms_tlev), intent(inout) :: t
    end function
    integer(c_int) function roms_gpu_init_case(c, device, t) bind(c)
      import :: c_int, roms_case, roms_tlev
      type(roms_case), intent(in) :: c
      integer(c_int), value :: device
      type(roms_tlev), intent(out) :: t
    end function
    integer(c_int) function roms_gpu_init_case_comm(c, np_xi, np_eta, comm, device, t) bind(c)
      import :: c_int, c_ptr, roms_case, roms_tlev
      type(roms_case), intent(in) :: c
      integer(c_int), value :: np_xi, np_eta, device
      type(c_ptr), value :: comm
      type(roms_tlev), intent(out) :: t
    end function
    integer(c_int) function roms_gpu_set_weights(ndtfast, weight) bind(c)
      import :: c_int, c_double, ROMS_MAX_FAST
      integer(c_int), value :: ndtfast
      real(c_double), intent(out) :: weight(ROMS_MAX_FAST, 2)
    end function
    integer(c_int) function roms_gpu_diag(t, norms) bind(c)
      import :: c_int, c_double, roms_tlev
      type(roms_tlev), intent(in) :: t
      real(c_double), intent(out) :: norms(4)
    end function
    ! partitioned netCDF restart/history files (basic_output.F, get_init.F);
    ! path: a NUL-terminated character(kind=c_char) array
    integer(c_int) function roms_gpu_wrt_rst(path, rec, total_rec, time, t) bind(c)
      import :: c_int, c_double, c_char, roms_tlev
      character(kind=c_char), intent(in) :: path(*)
      integer(c_int), value :: rec, total_rec
      real(c_double), value :: time
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_wrt_his(path, rec, total_rec, time, t, wrt_mask) bind(c)
      import :: c_int, c_double, c_char, roms_tlev
      character(kind=c_char), intent(in) :: path(*)
      integer(c_int), value :: rec, total_rec, wrt_mask
      real(c_double), value :: time
      type(roms_tlev), intent(in) :: t
    end function
    integer(c_int) function roms_gpu_io_wait() bind(c)
      import :: c_int
    end function
    integer(c_int) function roms_gpu_get_init(path, req_rec, tindx, t, start_time) bind(c)
      import :: c_int, c_double, c_char, roms_tlev
      character(kind=c_char), intent(in) :: path(*)
      integer(c_int), value :: req_rec, tindx
      type(roms_tlev), intent(inout) :: t
      real(c_double), intent(out) :: start_time
    end function
    ! set_frc_data / set_tides on the device (k_forcing.hip)
    integer(c_int) function roms_gpu_frc_record(field_id, slot, rec_time, data) bind(c)
      import :: c_int, c_double
      integer(c_int), value :: field_id, slot
      real(c_double), value :: rec_time
      real(c_double), intent(in) :: data(*)
    end function
    integer(c_int) function roms_gpu_frc_interp(modtime, kinds) bind(c)
      import :: c_int, c_double
      real(c_double), value :: modtime
      integer(c_int), value :: kinds
    end function
    ! the tidal arrays are c_loc(...) of (GLOBAL_2D_ARRAY, ntides) arrays, or c_null_ptr
    integer(c_int) function roms_gpu_frc_clock(start_time, on) bind(c)
      import :: c_int, c_double
      real(c_double), value :: start_time
      integer(c_int), value :: on
    end function
    integer(c_int) function roms_gpu_set_tide_data(ntides, ftide, pot_re, pot_im, ztide_re, ztide_im, &
                                                   utide_re, utide_im, vtide_re, vtide_im) bind(c)
      import :: c_int, c_double, c_ptr
      integer(c_int), value :: ntides
      real(c_double), intent(in) :: ftide(*)
      type(c_ptr), value :: pot_re, pot_im, ztide_re, ztide_im, utide_re, utide_im, vtide_re, vtide_im
    end function
    integer(c_int) function roms_gpu_set_tides(time) bind(c)
      import :: c_int, c_double
      real(c_double), value :: time
    end function
    integer(c_int) function roms_gpu_comm_unique_id(id128) bind(c)
      import :: c_int, c_char
      character(kind=c_char), intent(out) :: id128(128)
    end function
    integer(c_int) function roms_gpu_comm_create(id128, nranks, rank, device, comm) bind(c)
      import :: c_int, c_char, c_ptr
      character(kind=c_char), intent(in) :: id128(128)
      integer(c_int), value :: nranks, rank, device
      type(c_ptr), intent(out) :: comm
    end function
    ! host channel: allgather is c_funloc of a bind(c) function
    ! integer(c_int) function f(ctx, send, nbytes, recv) (MPI_Allgather of
    ! MPI_BYTE over the model's communicator; INTEGRATION.md)
    integer(c_int) function roms_gpu_comm_create_host(nranks, rank, device, allgather, ctx, comm) bind(c)
      import :: c_int, c_ptr, c_funptr
      integer(c_int), value :: nranks, rank, device
      type(c_funptr), value :: allgather
      type(c_ptr), value :: ctx
      type(c_ptr), intent(out) :: comm
    end function
    integer(c_int) function roms_gpu_comm_destroy(comm) bind(c)
      import :: c_int, c_ptr
      type(c_ptr), value :: comm
    end function
    ! 1: IPC peer writes, 0: RCCL send/recv (or one rank), -1: a wait timed out
    integer(c_int) function roms_gpu_halo_transport() bind(c)
      import :: c_int
    end function
  end interface

contains

  ! abort with the library's message (error_log%raise + abort_check analogue)
  subroutine roms_gpu_check(rc, what)
    integer(c_int), intent(in) :: rc
    character(*), intent(in) :: what
    character(kind=c_char), pointer :: msg(:)
    integer :: n
    if (rc == 0) return
    call c_f_pointer(roms_gpu_last_error(), msg, [1024])
    n = 0
    do while (n < 1024)
      if (msg(n + 1) == c_null_char) exit
      n = n + 1
    end do
    write(*, '(3a,i0,2a)') 'roms_gpu: ', what, ' failed (', rc, '): ', transfer(msg(1:n), repeat(' ', n))
    error stop 1
  end subroutine

end module roms_gpu_mod
