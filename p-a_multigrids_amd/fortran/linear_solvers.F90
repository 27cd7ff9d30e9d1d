! Drop-in facade of the reference's LinearSolvers.F90 smoothers.
!
! The reference's GSsolver_MeshCC / GSsolver_MeshSD / GSsolver_MeshMix
! (LinearSolvers.F90:632-671, 719-781, 788-848) take (meshL, level, it) with
! meshL(:) of type(mesh) from `use structures` (LinearSolvers.F90:2, Structures.F90:143-170)
! and iterate on Triangle%StencilCC/SD/UpUF fields that no compiled code ever populates
! (SURVEY.md 0.3; the module does not even compile: it uses the missing modules TriangleOps
! and MeshOps). The live multigrid path is the smoother of transport_tri_semi.F90:543-722.
!
! This facade keeps the entry points' names, argument types and meaning -- meshL(:) is the
! caller's own type(mesh) array from module structures (structures.F90, the reference's
! components), the level, an optional iteration count with the reference defaults
! (size(meshL)/2 for SD, size(meshL) for CC, 5*size(meshL) for Mix) -- and runs that many
! sweeps of the live smoother on the GPU: tnew_nonlin := tnew (:325-327), then `it` sweeps
! with the smoother's state semantics (tnew = the iterate before the last sweep, tnew_nonlin
! = the last, :550 vs :693). The device state is bound to meshL by pamg_bind_mesh (a handle
! built from meshL's X, Neig, fNeig, Dir, region_id) or pamg_bind_handle (an existing one);
! pamg_get_fields returns it as the reference's type(fields) tracer(:) arrays.
module LinearSolvers
  use iso_c_binding
  use structures, only: Mesh, fields
  use pamg
  implicit none
  private

  type(c_ptr), save :: bound = c_null_ptr
  integer, save :: bound_U = -1, bound_split = 0, bound_levels = 0

  public :: pamg_bind_mesh, pamg_bind_handle, pamg_bound_handle, pamg_get_fields, pamg_get_tnew_nonlin
  public :: GSsolver_MeshCC, GSsolver_MeshSD, GSsolver_MeshMix

contains

  ! a libpamg handle for the caller's meshList (the setup of transport_tri_semi.F90:178-288 on
  ! the device); the optional arguments override the reference's mode-9 defaults
  subroutine pamg_bind_mesh(meshL, n_split, multi_levels, n_smooth, solver, device, arith)
    type(mesh), intent(in), dimension(:) :: meshL
    integer, intent(in) :: n_split, multi_levels
    integer, optional, intent(in) :: n_smooth, solver, device, arith
    type(pamg_params), target :: p
    type(c_ptr) :: h
    integer(c_int) :: U
    real(c_double), allocatable :: X(:)
    integer(c_int), allocatable :: region(:), neig(:), fneig(:), dir(:)
    integer :: k
    U = int(size(meshL), c_int)
    allocate(X(6 * U), region(U), neig(3 * U), fneig(3 * U), dir(3 * U))
    do k = 1, U
      X(6 * (k - 1) + 1:6 * k) = reshape(meshL(k)%X, [6])
      region(k) = meshL(k)%region_id
      neig(3 * (k - 1) + 1:3 * k) = meshL(k)%Neig
      fneig(3 * (k - 1) + 1:3 * k) = meshL(k)%fNeig
      dir(3 * (k - 1) + 1:3 * k) = merge(1, 0, meshL(k)%Dir)
    end do
    call pamg_default_params(p)
    p%n_split = n_split
    p%multi_levels = multi_levels
    if (present(n_smooth)) p%n_smooth = n_smooth
    if (present(solver)) p%solver = solver
    if (present(device)) p%device = device
    if (present(arith)) p%arith = arith
    call pamg_check(pamg_create(p, h), c_null_ptr, 'pamg_create')
    call pamg_check(pamg_upload_mesh(h, U, X, region, neig, fneig, dir), h, 'pamg_upload_mesh')
    bound = h
    bound_U = U
    bound_split = n_split
    bound_levels = multi_levels
  end subroutine pamg_bind_mesh

  ! bind a handle the caller created and uploaded itself (U elements, n_split, multi_levels)
  subroutine pamg_bind_handle(h, U, n_split, multi_levels)
    type(c_ptr), intent(in) :: h
    integer, optional, intent(in) :: U, n_split, multi_levels
    bound = h
    bound_U = -1
    if (present(U)) bound_U = U
    if (present(n_split)) bound_split = n_split
    if (present(multi_levels)) bound_levels = multi_levels
  end subroutine pamg_bind_handle

  type(c_ptr) function pamg_bound_handle()
    pamg_bound_handle = bound
  end function pamg_bound_handle

  subroutine require_bound(n)
    integer, intent(in) :: n
    if (.not. c_associated(bound)) then
      print *, 'LinearSolvers facade: no libpamg handle bound (call pamg_bind_mesh)'
      error stop 1
    end if
    if (bound_U >= 0 .and. n /= bound_U) then
      print *, 'LinearSolvers facade: meshL has', n, 'elements, the bound handle', bound_U
      error stop 1
    end if
  end subroutine require_bound

  subroutine run_sweeps(n, level, iterations)
    integer, intent(in) :: n, level, iterations
    call require_bound(n)
    call pamg_check(pamg_copy_to_nonlin(bound, int(level, c_int)), bound, 'copy_to_nonlin')
    call pamg_check(pamg_sweep(bound, int(level, c_int), int(iterations, c_int)), bound, 'sweep')
  end subroutine run_sweeps

  ! LinearSolvers.F90:719-733 signature and default (it = size(meshL)/2)
  subroutine GSsolver_MeshSD(meshL, level, it)
    type(mesh), intent(inout), dimension(:) :: meshL
    integer, intent(in) :: level
    integer, optional, intent(in) :: it
    integer :: iteration
    iteration = size(meshL) / 2
    if (present(it)) iteration = it
    call run_sweeps(size(meshL), level, iteration)
  end subroutine GSsolver_MeshSD

  ! LinearSolvers.F90:632-643 signature and default (it = size(meshL))
  subroutine GSsolver_MeshCC(meshL, level, it)
    type(mesh), intent(inout), dimension(:) :: meshL
    integer, intent(in) :: level
    integer, optional, intent(in) :: it
    integer :: iteration
    iteration = size(meshL)
    if (present(it)) iteration = it
    call run_sweeps(size(meshL), level, iteration)
  end subroutine GSsolver_MeshCC

  ! LinearSolvers.F90:788-800 signature and default (it = 5*size(meshL))
  subroutine GSsolver_MeshMix(meshL, level, it)
    type(mesh), intent(inout), dimension(:) :: meshL
    integer, intent(in) :: level
    integer, optional, intent(in) :: it
    integer :: iteration
    iteration = size(meshL) * 5
    if (present(it)) iteration = it
    call run_sweeps(size(meshL), level, iteration)
  end subroutine GSsolver_MeshMix

  ! the device state as the reference's tracer(1:multi_levels) (Structures.F90:185-188,
  ! allocated (3, 4**(n_split-l+1), U) as transport_tri_semi.F90:178-187); source: level 1's
  ! cascaded source term s'
  subroutine pamg_get_fields(tracer)
    type(fields), intent(inout), allocatable :: tracer(:)
    integer :: l, nsub
    real(c_double), allocatable :: buf(:)
    call require_bound(bound_U)
    if (bound_U < 0 .or. bound_levels < 1) then
      print *, 'LinearSolvers facade: pamg_get_fields needs the handle bound by pamg_bind_mesh'
      error stop 1
    end if
    if (allocated(tracer)) deallocate(tracer)
    allocate(tracer(bound_levels))
    do l = 1, bound_levels
      nsub = 4**(bound_split - l + 1)
      allocate(buf(3 * nsub * bound_U))
      call get_one(PAMG_TNEW, l, buf)
      tracer(l)%tnew = reshape(buf, [3, nsub, bound_U])
      call get_one(PAMG_TOLD, l, buf)
      tracer(l)%told = reshape(buf, [3, nsub, bound_U])
      call get_one(PAMG_RHS, l, buf)
      tracer(l)%RHS = reshape(buf, [3, nsub, bound_U])
      call get_one(PAMG_RESIDUAL, l, buf)
      tracer(l)%residuale = reshape(buf, [3, nsub, bound_U])
      if (l == 1) then
        call get_one(PAMG_SOURCE, l, buf)
        tracer(l)%source = reshape(buf, [3, nsub, bound_U])
      end if
      deallocate(buf)
    end do
  end subroutine pamg_get_fields

  ! tnew_nonlin (transport_tri_semi.F90:85) of the level it currently holds
  subroutine pamg_get_tnew_nonlin(tnn, level)
    real, intent(inout), allocatable :: tnn(:,:,:)
    integer, intent(out) :: level
    real(c_double), allocatable :: buf(:)
    integer :: nsub
    level = pamg_tnn_level(bound)
    nsub = 4**(bound_split - level + 1)
    allocate(buf(3 * nsub * bound_U))
    call get_one(PAMG_TNEW_NONLIN, level, buf)
    tnn = reshape(buf, [3, nsub, bound_U])
  end subroutine pamg_get_tnew_nonlin

  subroutine get_one(what, level, buf)
    integer(c_int), intent(in) :: what
    integer, intent(in) :: level
    real(c_double), intent(inout) :: buf(:)
    call pamg_check(pamg_get_state(bound, int(level, c_int), what, buf), bound, 'pamg_get_state')
  end subroutine get_one

end module LinearSolvers
