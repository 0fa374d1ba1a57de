! mpi_f08_shim.f90 -- the few mpi_f08 names the reference's module files
! (param.F, hidden_mpi_vars.F) need to compile here: the image's MPICH ships
! an mpi.mod in gfortran format only, which amdflang cannot read.  Values
! follow /opt/conda/include/mpif.h.  Build-check use only (no MPI calls).
module mpi_f08
  implicit none
  type, bind(c) :: mpi_comm
    integer :: mpi_val
  end type
  type(mpi_comm), parameter :: MPI_COMM_WORLD = mpi_comm(1140850688)
  integer, parameter :: MPI_DOUBLE_PRECISION = 1275070495
  integer, parameter :: MPI_STATUS_SIZE = 5
end module mpi_f08
