! filament_driver.F90 -- Fortran host over the C ABI: the reference's
! Filament benchmark (tests/Filament: 64x64x32, dt=5 s, ndtfast=60) on the
! GPU, printing the per-step diag norms (KE, KE2b, Cu_adv, Cu_w) in the
! ES23.16 columns of benchmark.result_* (diag.F code_check line).
program filament_driver
  use iso_c_binding
  use roms_gpu_mod
  implicit none
  type(roms_case) :: c
  type(roms_tlev) :: t
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
  c%uv_adv = 1; c%uv_cor = 1             ! tests/Filament/cppdefs.opt: UV_ADV, UV_COR
  if (roms_gpu_abi_version() /= ROMS_GPU_ABI) error stop 'ABI version mismatch'
  call roms_gpu_check(roms_gpu_init_case(c, 0_c_int, t), 'init_case')
  call roms_gpu_check(roms_gpu_diag(t, norms), 'diag')
  write(*, '(i6,4es24.16)') 0, norms
  do step = 1, nsteps
    call roms_gpu_check(roms_gpu_step(t), 'step')
    call roms_gpu_check(roms_gpu_diag(t, norms), 'diag')
    write(*, '(i6,4es24.16)') step, norms
  end do
  call roms_gpu_check(roms_gpu_finalize(), 'finalize')
end program filament_driver
