! Signature-compatible facade of the reference's LinearSolvers.F90 smoothers.
!
! The reference's GSsolver_MeshCC / GSsolver_MeshSD / GSsolver_MeshMix
! (LinearSolvers.F90:632-671, 719-781, 788-848) take (meshL, level, it) and
! iterate on Triangle%StencilCC/SD/UpUF fields that no compiled code ever
! populates (SURVEY.md 0.3; the module does not even compile: it uses the
! missing modules TriangleOps and MeshOps). The live multigrid path is the
! smoother of transport_tri_semi.F90:543-722. This facade keeps the north
! star's entry-point names and argument meaning -- meshL(:), the level, an
! optional iteration count with the reference defaults (size(meshL)/2 for SD,
! size(meshL) for CC, 5*size(meshL) for Mix) -- and runs that many device
! sweeps of the live smoother on the libpamg handle bound with
! pamg_bind_handle. The per-element `Mesh` record carries the fields the hot
! path consumes (Structures.F90:143-170: X, Neig, fNeig, Dir, region_id).
module LinearSolvers
  use iso_c_binding
  use pamg
  implicit none
  private

  type, public :: Mesh
    double precision, dimension(2,3) :: X
    integer, dimension(3) :: Neig = 0, fNeig = 0
    logical, dimension(3) :: Dir = .false.
    integer :: region_id = 0
  end type Mesh

  type(c_ptr), save :: bound = c_null_ptr

  public :: pamg_bind_handle, GSsolver_MeshCC, GSsolver_MeshSD, GSsolver_MeshMix

contains

  subroutine pamg_bind_handle(h)
    type(c_ptr), intent(in) :: h
    bound = h
  end subroutine pamg_bind_handle

  subroutine run_sweeps(level, iterations)
    integer, intent(in) :: level, iterations
    if (.not. c_associated(bound)) then
      print *, 'LinearSolvers facade: no libpamg handle bound (call pamg_bind_handle)'
      error stop 1
    end if
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
    call run_sweeps(level, iteration)
  end subroutine GSsolver_MeshSD

  ! LinearSolvers.F90:632-643 signature and default (it = size(meshL))
  subroutine GSsolver_MeshCC(meshL, level, it)
    type(mesh), intent(inout), dimension(:) :: meshL
    integer, intent(in) :: level
    integer, optional, intent(in) :: it
    integer :: iteration
    iteration = size(meshL)
    if (present(it)) iteration = it
    call run_sweeps(level, iteration)
  end subroutine GSsolver_MeshCC

  ! LinearSolvers.F90:788-800 signature and default (it = 5*size(meshL))
  subroutine GSsolver_MeshMix(meshL, level, it)
    type(mesh), intent(inout), dimension(:) :: meshL
    integer, intent(in) :: level
    integer, optional, intent(in) :: it
    integer :: iteration
    iteration = size(meshL) * 5
    if (present(it)) iteration = it
    call run_sweeps(level, iteration)
  end subroutine GSsolver_MeshMix

end module LinearSolvers
