! A reference-shaped caller of the LinearSolvers facade: it builds meshList(:) of the
! reference's type(mesh) (module structures), binds it (pamg_bind_mesh), starts a time step
! (:316-317) and calls GSsolver_MeshSD(meshL, level, it) exactly as LinearSolvers.F90:719-733
! declares it, then reads the state back as the reference's type(fields) tracer(:).
!   facade_host <mesh.msh> <n_split> <multi_levels> <level> <it | -1 for the default> <out.bin>
! out.bin (stream, fp64): U, nsub, tnn_level, it_used, then tracer(level)%tnew, tnew_nonlin,
! tracer(level)%RHS and tracer(1)%source, each (3, nsub, U).
program facade_host
  use iso_c_binding
  use structures, only: Mesh, fields
  use LinearSolvers
  use pamg
  implicit none
  character(len=512) :: arg, mesh_file, out_file
  integer :: n_split, levels, level, it, k, lv, io
  type(c_ptr) :: m = c_null_ptr
  integer(c_int) :: U
  real(c_double), allocatable :: X(:)
  integer(c_int), allocatable :: region(:), neig(:), fneig(:), dir(:)
  type(mesh), allocatable :: meshList(:)
  type(fields), allocatable :: tracer(:)
  real, allocatable :: tnn(:,:,:)

  call get_command_argument(1, mesh_file)
  call get_command_argument(2, arg); read(arg, *) n_split
  call get_command_argument(3, arg); read(arg, *) levels
  call get_command_argument(4, arg); read(arg, *) level
  call get_command_argument(5, arg); read(arg, *) it
  call get_command_argument(6, out_file)

  ! the caller's meshList, as ReadMSH + getNeigDataMesh fill it (Msh2Tri.F90:132-548)
  call pamg_check(pamg_msh_read(c_path(mesh_file), m), c_null_ptr, 'pamg_msh_read')
  call pamg_check(pamg_msh_size(m, U), c_null_ptr, 'pamg_msh_size')
  allocate(X(6 * U), region(U), neig(3 * U), fneig(3 * U), dir(3 * U))
  call pamg_check(pamg_msh_get(m, X, region, neig, fneig, dir), c_null_ptr, 'pamg_msh_get')
  call pamg_msh_free(m)
  allocate(meshList(U))
  do k = 1, U
    meshList(k)%X = reshape(X(6 * (k - 1) + 1:6 * k), [2, 3])
    meshList(k)%Neig = neig(3 * (k - 1) + 1:3 * k)
    meshList(k)%fNeig = fneig(3 * (k - 1) + 1:3 * k)
    meshList(k)%Dir = dir(3 * (k - 1) + 1:3 * k) /= 0
    meshList(k)%region_id = region(k)
    meshList(k)%k_coef = 1.0
  end do

  call pamg_bind_mesh(meshList, n_split, levels)
  call pamg_check(pamg_begin_timestep(pamg_bound_handle()), pamg_bound_handle(), 'begin_timestep')
  if (it >= 0) then
    call GSsolver_MeshSD(meshList, level, it)
  else
    call GSsolver_MeshSD(meshList, level)      ! the reference's default, size(meshL)/2
    it = size(meshList) / 2
  end if
  call pamg_get_fields(tracer)
  call pamg_get_tnew_nonlin(tnn, lv)

  open(newunit=io, file=trim(out_file), access='stream', form='unformatted', status='replace')
  write(io) real(U, 8), real(size(tracer(level)%tnew, 2), 8), real(lv, 8), real(it, 8)
  write(io) real(tracer(level)%tnew, 8), real(tnn, 8), real(tracer(level)%RHS, 8), real(tracer(1)%source, 8)
  close(io)
  call pamg_check(pamg_destroy(pamg_bound_handle()), c_null_ptr, 'pamg_destroy')
  print *, 'facade_host: GSsolver_MeshSD(meshL,', level, ',', it, ') on', U, 'elements'
end program facade_host
