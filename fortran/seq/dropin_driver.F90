! dropin_driver.F90 -- the reference's roms_step (src/main.F:374-479) kept as
! Fortran, calling the hot-path routines by their own names; the linked
! subroutines are the drop-ins of fortran/dropin/*.F, so every call lands in
! its per-routine C-ABI entry (roms_gpu_rho_eos, roms_gpu_set_huv, ...).
! Case: the Filament benchmark (tests/Filament: 64x64x32, dt = 5 s,
! ndtfast = 60, UV_VIS2 + TS_DIF2), initialised by the library's analytic
! case; prints the per-step diag norms in the ES23.16 columns of
! benchmark.result_* like filament_driver.
program dropin_driver
  use iso_c_binding
  use roms_gpu_mod
  use roms_gpu_glue
  use scalars
  use roms_step_seq
  implicit none
  type(roms_case) :: c
  type(roms_tlev) :: tl
  real(c_double) :: norms(4)
  integer :: step, nsteps
  character(len=32) :: arg

  nsteps = 20
  if (command_argument_count() >= 1) then
    call get_command_argument(1, arg)
    read(arg, *) nsteps
  end if
  c%case_id = 0; c%LLm = 64; c%MMm = 64; c%N = 32; c%NT = 1
  c%salinity = 0; c%nonlin_eos = 0; c%lmd_mixing = 0
  c%dt = 5.0d0; c%ndtfast = 60; c%sizex = 12.8d3; c%sizey = 3.2d3; c%surf_flux = 0
  c%obc = 0; c%v_sponge = 0.0d0; c%island = 0; c%curvgrid = 0
  c%uv_adv = 1; c%uv_cor = 1
  if (roms_gpu_abi_version() /= ROMS_GPU_ABI) error stop 'ABI version mismatch'
  ! ana_grid / ana_init / roms_init's set_depth, set_HUV, omega, rho_eos (main.F:205-230)
  call roms_gpu_check(roms_gpu_init_case(c, 0_c_int, tl), 'init_case')
  iic = tl%iic; ntstart = tl%ntstart; forw_start = tl%forw_start; nfast = tl%nfast
  kstp = tl%kstp; knew = tl%knew; iif = tl%iif; nstp = tl%nstp; nrhs = tl%nrhs; nnew = tl%nnew
  call roms_gpu_check(roms_gpu_diag(tl, norms), 'diag')
  write(*, '(i6,4es24.16)') 0, norms
  do step = 1, nsteps
    iic = ntstart + step - 1          ! main.F:68
    call roms_step
    call roms_gpu_tlev_now(tl)
    call roms_gpu_check(roms_gpu_diag(tl, norms), 'diag')
    write(*, '(i6,4es24.16)') step, norms
  end do
  call roms_gpu_check(roms_gpu_finalize(), 'finalize')

end program dropin_driver
