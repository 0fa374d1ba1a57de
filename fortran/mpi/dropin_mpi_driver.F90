! dropin_mpi_driver.F90 -- the north_star's deployment, run: a Fortran + MPI
! host with one process per rank, the reference's bootstrap
! (src/main.F:26-28: MPI_Init, then mpi_setup's processor grid,
! src/mpi_setup.F:14-211) and its roms_step (main.F:374-479, module
! roms_step_seq) calling the hot-path routines by name; the linked routines
! are the drop-ins (fortran/dropin/*.F), so every call lands in its
! per-routine C-ABI entry on this rank's GPU.
!
! The library's communicator comes from roms_gpu_comm_create_host with a
! Fortran callback doing MPI_Allgather of bytes over MPI_COMM_WORLD: it
! carries the IPC handles of the halo buffers at init and the diag /
! area-volume gathers; every halo exchange is then a GPU-to-GPU peer write.
!
! Usage: mpiexec -n NP_XI*NP_ETA dropin_mpi_driver [nsteps [NP_XI NP_ETA [LLm MMm N]]]
! Case: the Filament benchmark physics (tests/Filament switches, dt = 5 s,
! ndtfast = 60) on the library's analytic grid; the default is BASELINE C1,
! 128x128x20 on a 2x2 processor grid.  Rank 0 prints the per-step diag norms
! in benchmark.result_*'s ES23.16 columns.
module mpi_channel
  use iso_c_binding
  implicit none
  include 'mpif.h'
contains
  ! roms_host_allgather_fn (include/roms_gpu.h): recv(r*nbytes+1 : ...) = rank r's send
  integer(c_int) function mpi_allgather_bytes(ctx, send, nbytes, recv) bind(c)
    type(c_ptr), value :: ctx, send, recv
    integer(c_long), value :: nbytes
    integer(c_int8_t), pointer :: s(:), r(:)
    integer :: ierr, np
    call MPI_Comm_size(MPI_COMM_WORLD, np, ierr)
    call c_f_pointer(send, s, [nbytes])
    call c_f_pointer(recv, r, [nbytes * np])
    call MPI_Allgather(s, int(nbytes), MPI_BYTE, r, int(nbytes), MPI_BYTE, MPI_COMM_WORLD, ierr)
    mpi_allgather_bytes = ierr
  end function mpi_allgather_bytes
end module mpi_channel

program dropin_mpi_driver
  use iso_c_binding
  use mpi_channel
  use roms_gpu_mod
  use roms_gpu_glue
  use scalars
  use roms_step_seq
  implicit none
  type(roms_case) :: c
  type(roms_tlev) :: tl
  type(c_ptr) :: comm
  real(c_double) :: norms(4)
  integer :: step, nsteps, ierr, mynode, nnodes, np_xi, np_eta, inode, jnode, ndev
  integer :: LLm, MMm, N
  character(len=32) :: arg
  character(len=16) :: trans

  call MPI_Init(ierr)                                 ! main.F:26
  call MPI_Comm_rank(MPI_COMM_WORLD, mynode, ierr)
  call MPI_Comm_size(MPI_COMM_WORLD, nnodes, ierr)
  nsteps = 20; np_xi = 2; np_eta = 2; LLm = 128; MMm = 128; N = 20
  if (command_argument_count() >= 1) then
    call get_command_argument(1, arg); read(arg, *) nsteps
  end if
  if (command_argument_count() >= 3) then
    call get_command_argument(2, arg); read(arg, *) np_xi
    call get_command_argument(3, arg); read(arg, *) np_eta
  end if
  if (command_argument_count() >= 6) then
    call get_command_argument(4, arg); read(arg, *) LLm
    call get_command_argument(5, arg); read(arg, *) MMm
    call get_command_argument(6, arg); read(arg, *) N
  end if
  ! mpi_setup.F:37-61: the processor grid must match the communicator
  if (nnodes /= np_xi * np_eta) then
    if (mynode == 0) write(*, '(a,i4,a,2i4)') 'dropin_mpi_driver: ', nnodes, ' ranks for a processor grid ', np_xi, np_eta
    call MPI_Abort(MPI_COMM_WORLD, 2, ierr)
  end if
  inode = mod(mynode, np_xi)
  jnode = mynode / np_xi
  if (roms_gpu_abi_version() /= ROMS_GPU_ABI) error stop 'ABI version mismatch'

  ! one GPU per rank; ranks beyond the node's devices share them round-robin
  ndev = 1
  arg = ''
  call get_environment_variable('ROMS_MPI_NDEV', arg)
  if (len_trim(arg) > 0) read(arg, *) ndev
  call roms_gpu_check(roms_gpu_comm_create_host(int(nnodes, c_int), int(mynode, c_int), int(mod(mynode, ndev), c_int), &
                                                c_funloc(mpi_allgather_bytes), c_null_ptr, comm), 'comm_create_host')

  c%case_id = 0; c%LLm = LLm; c%MMm = MMm; c%N = N; c%NT = 1
  c%salinity = 0; c%nonlin_eos = 0; c%lmd_mixing = 0
  c%dt = 5.0d0; c%ndtfast = 60; c%sizex = 100.0d0 * LLm; c%sizey = 25.0d0 * MMm; c%surf_flux = 0
  c%obc = 0; c%v_sponge = 0.0d0; c%island = 0; c%curvgrid = 0
  c%uv_adv = 1; c%uv_cor = 1
  ! ana_grid / ana_init / roms_init on this rank's subdomain (main.F:205-230)
  call roms_gpu_check(roms_gpu_init_case_comm(c, int(np_xi, c_int), int(np_eta, c_int), comm, &
                                              int(mod(mynode, ndev), c_int), tl), 'init_case_comm')
  iic = tl%iic; ntstart = tl%ntstart; forw_start = tl%forw_start; nfast = tl%nfast
  kstp = tl%kstp; knew = tl%knew; iif = tl%iif; nstp = tl%nstp; nrhs = tl%nrhs; nnew = tl%nnew
  select case (roms_gpu_halo_transport())
  case (1)
    trans = 'ipc'
  case (0)
    trans = 'rccl'
  case default
    trans = 'failed'
  end select
  if (mynode == 0) write(*, '(a,i3,a,i2,a,i2,a,a)') '# ranks', nnodes, ' grid', np_xi, ' x', np_eta, &
                                                    ' halo transport ', trim(trans)
  call roms_gpu_check(roms_gpu_diag(tl, norms), 'diag')   ! collective (diag.F:409-552)
  if (mynode == 0) write(*, '(i6,4es24.16)') 0, norms
  do step = 1, nsteps
    iic = ntstart + step - 1                     ! main.F:68
    call roms_step
    call roms_gpu_tlev_now(tl)
    call roms_gpu_check(roms_gpu_diag(tl, norms), 'diag')
    if (mynode == 0) write(*, '(i6,4es24.16)') step, norms
  end do
  call roms_gpu_check(roms_gpu_finalize(), 'finalize')
  call roms_gpu_check(roms_gpu_comm_destroy(comm), 'comm_destroy')
  call MPI_Finalize(ierr)
end program dropin_mpi_driver
