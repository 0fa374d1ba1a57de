! register_driver.F90 -- a Fortran host that owns its module arrays, the way
! the reference's main.F does after init_arrays (ocean_vars.F:68-116): the
! prognostic state is allocated with the reference's bounds, handed to the
! library with roms_gpu_register, uploaded, advanced with roms_gpu_step and
! downloaded back.  The initial state is the Filament benchmark's
! (tests/Filament: 64x64x32, dt=5 s, ndtfast=60), taken from the library's
! analytic case once and then re-initialised through roms_gpu_init with a
! roms_cfg built here (set_weights via roms_gpu_set_weights).  Prints the
! per-step diag norms (KE, KE2b, Cu_adv, Cu_w) like filament_driver.
program register_driver
  use iso_c_binding
  use roms_gpu_mod
  implicit none
  integer, parameter :: LLm = 64, MMm = 64, N = 32, NT = 1
  type fbuf
    real(c_double), allocatable :: a(:)
  end type
  type(fbuf), target :: f(0:ROMS_NFIELDS - 1)
  ! ocean_vars.F / tracers.F / grid-shaped module arrays (GLOBAL_2D_ARRAY = -1:Lm+2,-1:Mm+2)
  real(c_double), allocatable, target :: zeta(:,:,:), ubar(:,:,:), vbar(:,:,:)
  real(c_double), allocatable, target :: u(:,:,:,:), v(:,:,:,:), t(:,:,:,:,:), Hz(:,:,:), z_r(:,:,:)
  type(roms_case) :: c
  type(roms_dims) :: d
  type(roms_cfg) :: cfg
  type(roms_tlev) :: tl
  real(c_double) :: norms(4), zsum0
  integer(c_int) :: id
  integer(c_long) :: nel
  integer :: step, nsteps
  character(len=32) :: arg

  nsteps = 20
  if (command_argument_count() >= 1) then
    call get_command_argument(1, arg)
    read(arg, *) nsteps
  end if
  if (roms_gpu_abi_version() /= ROMS_GPU_ABI) error stop 'ABI version mismatch'

  ! 1. the analytic Filament state (ana_grid / ana_init + roms_init), copied out
  c%case_id = 0; c%LLm = LLm; c%MMm = MMm; c%N = N; c%NT = NT
  c%salinity = 0; c%nonlin_eos = 0; c%lmd_mixing = 0
  c%dt = 5.0d0; c%ndtfast = 60; c%sizex = 12.8d3; c%sizey = 3.2d3; c%surf_flux = 0
  c%obc = 0; c%v_sponge = 0.0d0; c%island = 0; c%curvgrid = 0; c%uv_adv = 1; c%uv_cor = 1
  call roms_gpu_check(roms_gpu_init_case(c, 0_c_int, tl), 'init_case')
  allocate(zeta(-1:LLm+2, -1:MMm+2, 4), ubar(-1:LLm+2, -1:MMm+2, 4), vbar(-1:LLm+2, -1:MMm+2, 4))
  allocate(u(-1:LLm+2, -1:MMm+2, N, 3), v(-1:LLm+2, -1:MMm+2, N, 3), t(-1:LLm+2, -1:MMm+2, N, 3, NT))
  allocate(Hz(-1:LLm+2, -1:MMm+2, N), z_r(-1:LLm+2, -1:MMm+2, N))
  do id = 0, ROMS_NFIELDS - 1
    nel = roms_gpu_field_size(id)
    allocate(f(id)%a(nel))
    call roms_gpu_check(roms_gpu_copy_out(id, c_loc(f(id)%a), nel), 'copy_out')
  end do
  call put(ROMS_zeta, zeta); call put(ROMS_ubar, ubar); call put(ROMS_vbar, vbar)
  call put(ROMS_Hz, Hz); call put(ROMS_z_r, z_r)
  u = reshape(f(ROMS_u)%a, shape(u)); v = reshape(f(ROMS_v)%a, shape(v)); t = reshape(f(ROMS_t)%a, shape(t))
  call roms_gpu_check(roms_gpu_finalize(), 'finalize')

  ! 2. a host-built configuration (param.F / cppdefs.opt / roms.in of tests/Filament)
  d%Lm = LLm; d%Mm = MMm; d%N = N; d%NT = NT; d%LLm = LLm; d%MMm = MMm
  d%np_xi = 1; d%np_eta = 1; d%inode = 0; d%jnode = 0; d%iSW_corn = 0; d%jSW_corn = 0
  d%ew_periodic = 1; d%ns_periodic = 1
  d%west_exchng = 0; d%east_exchng = 0; d%south_exchng = 0; d%north_exchng = 0
  cfg%nonlin_eos = 0; cfg%salinity = 0; cfg%lmd_mixing = 0; cfg%uv_vis2 = 1; cfg%ts_dif2 = 1
  cfg%dt = 5.0d0; cfg%ndtfast = 60
  cfg%nfast = roms_gpu_set_weights(cfg%ndtfast, cfg%weight)
  cfg%g = 9.81d0; cfg%rho0 = 1000.0d0; cfg%rdrg = 0.0d0; cfg%rdrg2 = 1.0d-3; cfg%Zob = 1.0d-2; cfg%gamma2 = 1.0d0
  cfg%Akv_bak = 0.0d0; cfg%Akt_bak = 0.0d0
  cfg%Tcoef = 0.2d0; cfg%T0 = 1.0d0; cfg%Scoef = 0.822d0; cfg%S0 = 1.0d0
  cfg%theta_s = 6.0d0; cfg%theta_b = 2.0d0; cfg%hc = 25.0d0
  cfg%obc = 0; cfg%ubind = 0.1d0; cfg%curvgrid = 0; cfg%uv_adv = 1; cfg%uv_cor = 1; cfg%pot_tides = 0
  call roms_gpu_check(roms_gpu_init(d, cfg, 0_c_int, c_null_ptr), 'init')

  ! 3. register the host arrays (module-shaped where the reference has them), upload
  do id = 0, ROMS_NFIELDS - 1
    select case (id)
    case (ROMS_zeta);  call reg(id, c_loc(zeta), size(zeta, kind=c_long))
    case (ROMS_ubar);  call reg(id, c_loc(ubar), size(ubar, kind=c_long))
    case (ROMS_vbar);  call reg(id, c_loc(vbar), size(vbar, kind=c_long))
    case (ROMS_u);     call reg(id, c_loc(u), size(u, kind=c_long))
    case (ROMS_v);     call reg(id, c_loc(v), size(v, kind=c_long))
    case (ROMS_t);     call reg(id, c_loc(t), size(t, kind=c_long))
    case (ROMS_Hz);    call reg(id, c_loc(Hz), size(Hz, kind=c_long))
    case (ROMS_z_r);   call reg(id, c_loc(z_r), size(z_r, kind=c_long))
    case default;      call reg(id, c_loc(f(id)%a), size(f(id)%a, kind=c_long))
    end select
  end do
  call roms_gpu_check(roms_gpu_upload(ROMS_ALL), 'upload')
  zsum0 = sum(zeta(1:LLm, 1:MMm, 1))

  ! 4. roms_init left iic=0 with every index at 1 (main.F:268-288)
  tl%iic = 0; tl%ntstart = 1; tl%forw_start = 1; tl%iif = 1; tl%nfast = cfg%nfast
  tl%kstp = 1; tl%knew = 1; tl%nstp = 1; tl%nrhs = 1; tl%nnew = 1
  call roms_gpu_check(roms_gpu_diag(tl, norms), 'diag')
  write(*, '(i6,4es24.16)') 0, norms
  do step = 1, nsteps
    call roms_gpu_check(roms_gpu_step(tl), 'step')
    call roms_gpu_check(roms_gpu_diag(tl, norms), 'diag')
    write(*, '(i6,4es24.16)') step, norms
  end do
  ! 5. the host arrays hold the new state after download (free surface moved)
  call roms_gpu_check(roms_gpu_download(ROMS_ALL), 'download')
  if (.not. (abs(sum(zeta(1:LLm, 1:MMm, tl%knew)) - zsum0) >= 0.0d0)) error stop 'non-finite zeta after download'
  write(*, '(a,i0,a,es24.16)') '# zeta(knew=', tl%knew, ') checksum ', sum(zeta(1:LLm, 1:MMm, tl%knew))
  call roms_gpu_check(roms_gpu_finalize(), 'finalize')

contains

  subroutine put(id, a)
    integer(c_int), intent(in) :: id
    real(c_double), intent(inout) :: a(..)
    select rank (a)
    rank (3)
      a = reshape(f(id)%a, shape(a))
    end select
  end subroutine

  subroutine reg(id, p, cnt)
    integer(c_int), intent(in) :: id
    type(c_ptr), intent(in) :: p
    integer(c_long), intent(in) :: cnt
    call roms_gpu_check(roms_gpu_register(id, p, cnt), 'register')
  end subroutine

end program register_driver
