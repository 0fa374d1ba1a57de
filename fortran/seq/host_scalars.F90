! host_scalars.F90 -- the time indices of the reference's module `scalars`
! (src/scalars.F:32-36: iic, kstp, knew, iif, nstp, nnew, nrhs; ntstart,
! nfast and forw_start beside them) for a host program that links the
! drop-ins outside a reference tree.  dropin/roms_gpu_glue.F reads them from
! here exactly as it reads them from `scalars` inside the reference build
! (fortran/refbuild/build_dropins.sh), so the drop-in sources are the same
! files in both builds.
module scalars
  implicit none
  integer :: iic = 0, kstp = 1, knew = 1, iif = 1, nstp = 1, nnew = 1, nrhs = 1
  integer :: ntstart = 1, nfast = 1, forw_start = 1
end module scalars
