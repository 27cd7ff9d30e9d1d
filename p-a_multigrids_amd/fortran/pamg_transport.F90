! Fortran host of the multigrid hot path: the reference's mode-9 driver
! Semi_implicit_iterative (transport_tri_semi.F90:14-891, selected by
! main.F90:16,46-47) with every hot-path call replaced by libpamg through the
! iso_c_binding shim (module pamg). Setup, the time loop and the V-cycle
! control flow stay on the Fortran side at the reference's call sites; the
! fields stay resident on the GPU between calls.
!
! Run-time configuration (the reference hard-codes these, :99,:118,:135 and
! main.F90:46-47) comes from the namelist file given as the first argument
! (default pamg_run.nml):
!   &transport mesh_file='untitled8.msh', n_split=3, multi_levels=3, n_smooth=4,
!             solver=3, ntime=2, n_multigrid=2, device=0, dump='out.bin',
!             call_sites=1, vtk_interval=0 /
! call_sites=1 drives the fine-grained entry points exactly at the reference
! call sites; call_sites=0 calls pamg_run (the same sequence inside libpamg).
! vtk_interval > 0 writes Tracer_<itime>.vtu at the start of every vtk_interval-th
! step as the reference's get_vtu call site does (:301-311; main.F90:46 passes 1),
! through pamg_write_vtu (full precision, raw appended binary).
program pamg_transport
  use iso_c_binding
  use pamg
  use structures, only: MeshRec => Mesh
  use LinearSolvers, only: pamg_bind_handle, GSsolver_MeshSD
  use pamg_dump, only: write_dump
  implicit none

  character(len=512) :: mesh_file = 'untitled8.msh', dump = ''
  integer :: n_split = 1, multi_levels = 1, n_smooth = 4, solver = 3, ntime = 2, n_multigrid = 2
  integer :: device = 0, call_sites = 1, facade_sweeps = 0, vtk_interval = 0, vtk_io, cycle = 0
  character(len=64) :: vtu_name
  namelist /transport/ mesh_file, n_split, multi_levels, n_smooth, solver, ntime, n_multigrid, device, dump, &
       call_sites, facade_sweeps, vtk_interval, cycle

  character(len=512) :: cfg
  type(c_ptr) :: m = c_null_ptr, h = c_null_ptr
  type(pamg_params) :: p
  integer(c_int) :: U, rc
  real(c_double), allocatable :: X(:)
  integer(c_int), allocatable :: region(:), neig(:), fneig(:), dir(:)
  integer :: u_, itime, multigrid, ilevel, i
  integer(8) :: c0, c1, crate
  type(MeshRec), allocatable :: meshList(:)

  cfg = 'pamg_run.nml'
  if (command_argument_count() >= 1) call get_command_argument(1, cfg)
  open(10, file=trim(cfg), status='old', action='read')
  read(10, nml=transport)
  close(10)

  print *, '---------------------------------------------------------'
  print *, '|       Reading the .msh file     |'
  rc = pamg_msh_read(c_path(mesh_file), m)                       ! ReadMSH (:99)
  call pamg_check(rc, c_null_ptr, 'pamg_msh_read '//trim(mesh_file))
  call pamg_check(pamg_msh_size(m, U), c_null_ptr, 'pamg_msh_size')
  allocate(X(6*U), region(U), neig(3*U), fneig(3*U), dir(3*U))
  call pamg_check(pamg_msh_get(m, X, region, neig, fneig, dir), c_null_ptr, 'pamg_msh_get')
  call pamg_msh_free(m)

  if (multi_levels > n_split) then                          ! :120-123
    print *, 'error:: The number of multi_levels is higher than n_split'
    stop
  end if

  call pamg_default_params(p)
  p%n_split = n_split
  p%multi_levels = multi_levels
  p%n_smooth = n_smooth
  p%solver = solver
  p%device = device
  p%cycle = cycle                 ! 1: the corrected V-cycle (pamg.h), used by pamg_run (call_sites = 0)
  call pamg_check(pamg_create(p, h), c_null_ptr, 'pamg_create')
  call pamg_check(pamg_upload_mesh(h, U, X, region, neig, fneig, dir), h, 'pamg_upload_mesh')

  allocate(meshList(U))
  do u_ = 1, U
    meshList(u_)%X = reshape(X(6*(u_-1)+1:6*u_), [2, 3])
    meshList(u_)%Neig = neig(3*(u_-1)+1:3*u_)
    meshList(u_)%fNeig = fneig(3*(u_-1)+1:3*u_)
    meshList(u_)%Dir = dir(3*(u_-1)+1:3*u_) /= 0
    meshList(u_)%region_id = region(u_)
  end do
  call pamg_bind_handle(h, int(U), n_split, multi_levels)

  print *, '|   n_split =', n_split
  print *, '|   multigrid levels =', multi_levels
  print *, '|   totele_unst, totele_str, totele', U, 4**n_split, U * 4**n_split
  print *, '|   ntime = ', ntime
  print *, '|   dt    = ', p%dt
  print *, '---------------------------------------------------------'
  call system_clock(c0, crate)

  if (call_sites == 0) then
    call pamg_check(pamg_run(h, int(ntime, c_int), int(n_multigrid, c_int)), h, 'pamg_run')
  else
    vtk_io = vtk_interval                                   ! :132
    do itime = 1, ntime                                     ! :299
      if (vtk_interval > 0 .and. vtk_io <= itime) then      ! :301-311
        write(vtu_name, '(a,i0,a)') 'Tracer_', itime, '.vtu'
        call pamg_check(pamg_write_vtu(h, c_path(vtu_name), 0_c_int), h, 'pamg_write_vtu')
        vtk_io = vtk_io + vtk_interval
      end if
      call pamg_check(pamg_begin_timestep(h), h, 'begin_timestep')     ! :316-317
      do multigrid = 1, n_multigrid                         ! :319
        do ilevel = 1, multi_levels                         ! restriction leg :323-340
          call pamg_check(pamg_copy_to_nonlin(h, ilevel), h, 'copy')   ! :325-327
          call pamg_check(pamg_smoother(h, ilevel, 1_c_int), h, 'smoother')   ! :331
          call pamg_check(pamg_restrictor(h, ilevel), h, 'restrictor')        ! :336
          call pamg_check(pamg_get_residual(h, ilevel), h, 'get_residual')    ! :338
        end do
        ilevel = multi_levels                               ! coarsest level :344-359
        call pamg_check(pamg_copy_to_nonlin(h, ilevel), h, 'copy')
        do i = 1, 15
          call pamg_check(pamg_smoother(h, ilevel, 1_c_int), h, 'smoother')  ! :352
        end do
        do ilevel = multi_levels - 1, 1, -1                 ! prolongation leg :363-378
          call pamg_check(pamg_copy_to_nonlin(h, ilevel), h, 'copy')          ! :365-367
          call pamg_check(pamg_prolongator(h, ilevel), h, 'prolongator')      ! :370
          call pamg_check(pamg_smoother(h, ilevel, 1_c_int), h, 'smoother')   ! :376
        end do
      end do
      print *, 'semi', itime
    end do
  end if
  if (facade_sweeps > 0) call GSsolver_MeshSD(meshList, 1, facade_sweeps)
  call pamg_check(pamg_synchronize(h), h, 'synchronize')
  call system_clock(c1)
  print *, '----------------------------------------------------------'
  print *, '|        cpu_time for time_loop = ', real(c1 - c0, 8) / real(crate, 8), '|'
  print *, '----------------------------------------------------------'

  if (len_trim(dump) > 0) call write_dump(h, trim(dump), int(U), n_split, multi_levels)
  call pamg_check(pamg_destroy(h), c_null_ptr, 'pamg_destroy')

end program pamg_transport
