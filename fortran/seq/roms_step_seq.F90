! roms_step_seq.F90 -- the reference's roms_step (src/main.F:374-479) with the
! Filament switches (no LMD_MIXING, no forcing), kept as Fortran and calling
! the hot-path routines by their own names: the linked subroutines are the
! drop-ins of fortran/dropin/*.F, so every call lands in its per-routine
! C-ABI entry.  Shared by the single-rank driver (seq/dropin_driver.F90) and
! the MPI one (mpi/dropin_mpi_driver.F90).
module roms_step_seq
  use scalars
  implicit none
contains

  subroutine roms_step
    nstp = 1 + mod(iic - ntstart, 2)
    nrhs = nstp; nnew = 3
    call rho_eos(nrhs)
    call set_HUV
    call omega
    call prsgrd
    call pre_step3d(0)
    call set_HUV1(0)
    nrhs = 3; nnew = 3 - nstp
    call omega
    call rho_eos(nrhs)
    call prsgrd
    call step3d_uv1(0)
    call visc3d
    do iif = 1, nfast
      kstp = knew
      knew = kstp + 1
      if (knew > 4) knew = 1
      call step2d
    end do
    call step3d_uv2(0)
    call omega
    call step3d_t(0)
    call t3dmix
    call rho_eos(nnew)
  end subroutine roms_step
end module roms_step_seq
