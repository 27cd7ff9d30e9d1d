! module structures -- the derived types of the reference's Structures.F90, as the drop-in
! boundary needs them: a reference caller (main.F90 -> Semi_implicit_iterative, or anything
! calling LinearSolvers' GSsolver_Mesh*) `use structures` and passes its own meshList(:) of
! type(Mesh) to the facade in linear_solvers.F90 unchanged.
!
! Every type keeps the reference's component names, types, ranks and allocatable
! attributes (Structures.F90:106-118 Triangle, :120-122 multigrid_scaling, :143-170 Mesh,
! :174-176 element_info, :180-182 pointer_Mesh, :185-188 fields, :196-201 sparse, :208-211
! m_CSR, :215-219 neig_data, :235-241 Kcoord), so code written against the reference's module
! compiles against this one. Default `real` follows the compiler flags exactly as in the
! reference: this module is built with -fdefault-real-8, the reference's fp64 parity build
! (oracle/build_ref.py); the HIP path computes in fp64 either way.
!
! Which components the GPU path reads (pamg_bind_mesh in linear_solvers.F90):
!   X(2,3)     vertex coordinates             -> pamg_upload_mesh X
!   Neig(3)    neighbour un_ele per face      -> neig (0 = domain boundary)
!   fNeig(3)   the neighbour's face index     -> fneig
!   Dir(3)     same-direction flag            -> dir (0 / 1)
!   region_id  physical region (4: IC = 1)    -> region
! The rest (stencils, overlaps, scaling) lives on the device in the layouts of DESIGN.md 3;
! the fields come back through pamg_get_fields as type(fields) arrays (3, nsub, U).
module structures
  implicit none
  private

  ! the orphaned structured-triangle record (LinearSolvers.F90's Tri(level)); never
  ! populated by compiled reference code (SURVEY.md 0.3)
  type, public :: Triangle
    double precision, allocatable, dimension(:,:,:) :: UpUF, UpResAux
    double precision, allocatable, dimension(:,:,:) :: DownUF, DownResAux
    double precision, allocatable, dimension(:,:,:) :: StencilCC, StencilSD, StencilMix
    double precision, dimension(2,3) :: X
    integer :: SizeUp, SizeDown
    logical :: Visited
  end type Triangle

  ! per-level shape-function scaling of one un_ele (semi_tri_det_nlx_multigrid)
  type, public :: multigrid_scaling
    real, allocatable :: detwei(:), nx(:,:,:), sdetwei(:,:)
  end type multigrid_scaling

  ! one unstructured element of the semi-structured mesh (ReadMSH / getNeigDataMesh)
  type, public :: Mesh
    double precision, dimension(2,3) :: X
    real, dimension(2) :: center
    real, dimension(3) :: dc_unele, dc_str_ele
    real :: str_area
    real, allocatable :: detwei(:)            ! (ngi)
    real, allocatable :: sdetwei(:,:)         ! (sngi, nface)
    real, allocatable :: snorm(:,:,:)         ! (sngi, ndim, nface)
    real, allocatable :: nx(:,:,:)            ! (ngi, ndim, nloc)
    integer :: method, v1, v2
    integer, dimension(3) :: Neig, fNeig
    integer, allocatable :: S_nodes(:,:)
    logical, dimension(3) :: Dir
    real :: k_coef
    real, allocatable :: t_overlap(:,:)       ! (2**n_split * nloc, nface)
    real, allocatable :: t_overlap_old(:,:)   ! (2**n_split * nloc, nface)
    real, allocatable :: u_overlap(:,:,:)     ! (ndim, 2**n_split * nloc, nface)
    real, allocatable :: u_ele(:,:,:)         ! (ndim, nloc, totele_str)
    integer :: region_id
    integer, allocatable :: s_ele(:,:)        ! (2**n_split, nface)
    type(Triangle), allocatable, dimension(:) :: Tri
    type(multigrid_scaling), allocatable, dimension(:) :: scaling_var
  end type Mesh

  ! per-level sub-element tables (loc_surf_ele_multigrid, get_str_neig_multigrid)
  type, public :: element_info
    integer, allocatable :: surf_ele(:,:), str_neig(:,:)
  end type element_info

  type, public :: pointer_Mesh
    type(Mesh), pointer :: ptr
  end type pointer_Mesh

  ! the multigrid state of one level, (nloc, 4**i_split, totele_unst) each
  type, public :: fields
    real, dimension(:,:,:), allocatable :: tnew, told, error
    real, allocatable :: residuale(:,:,:), RHS(:,:,:), source(:,:,:)
  end type fields

  ! the assembled CSR matrices of matrices.F90 (g_iloc row starts, g_jloc columns, val)
  type, public :: sparse
    integer, allocatable :: g_iloc(:)
    integer, allocatable :: g_jloc(:)
    double precision, allocatable :: val(:)
  end type sparse

  type, public :: m_CSR
    integer :: ele_id
    double precision, allocatable :: values(:,:)
  end type m_CSR

  type, public :: neig_data
    integer, dimension(3) :: Nside, Npos
    integer, allocatable :: Nnodes(:)
  end type neig_data

  type, public :: Kcoord
    double precision, dimension(2) :: Xc1, Xc2, Xc3, Xc4
    double precision :: k
  end type Kcoord

end module structures
