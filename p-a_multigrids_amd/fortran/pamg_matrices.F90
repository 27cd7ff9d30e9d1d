! Drop-in for the reference's matrices.F90 SpMV: csr_mul_array(sparse_matrix, array, result)
! (matrices.F90:172-193) over the reference's `type sparse` (Structures.F90:196-201),
! computed on the GPU by libpamg's csr kernel -- bitwise equal to the reference's routine
! (fp64: the reference's REAL built with -fdefault-real-8; tests/test_csr.py).
! `sparse` is module structures' (the reference's Structures.F90 type, structures.F90), so a
! caller's own type(sparse) matrices pass straight in; csr_mul_array_arrays takes the bare
! components. Each call uploads the matrix;
! a constant matrix used every step is uploaded once with csr_upload / csr_mul_array_gpu.
module pamg_matrices
  use iso_c_binding
  use pamg
  use structures, only: sparse
  implicit none
  private
  type(c_ptr), save :: h_csr = c_null_ptr

  ! the reference's type sparse (Structures.F90:196-201), from module structures
  public :: sparse

  type, public :: csr_gpu
    type(c_ptr) :: m = c_null_ptr
    integer :: nrows = 0
  end type csr_gpu

  public :: csr_mul_array, csr_mul_array_arrays, csr_upload, csr_mul_array_gpu, csr_release
  public :: pamg_bind_csr_handle

contains

  subroutine pamg_bind_csr_handle(h)
    type(c_ptr), intent(in) :: h
    h_csr = h
  end subroutine pamg_bind_csr_handle

  subroutine ensure_handle()
    type(pamg_params), target :: p
    if (c_associated(h_csr)) return
    call pamg_default_params(p)
    call pamg_check(pamg_create(p, h_csr), h_csr, 'create (pamg_matrices)')
  end subroutine ensure_handle

  subroutine csr_upload(g_iloc, g_jloc, val, a)
    integer, intent(in) :: g_iloc(:), g_jloc(:)
    doubleprecision, intent(in) :: val(:)
    type(csr_gpu), intent(out) :: a
    integer(c_int), allocatable :: j(:)
    call ensure_handle()
    j = int(g_jloc, c_int)
    a%nrows = size(g_iloc)
    call pamg_check(pamg_csr_create(h_csr, int(size(g_iloc), c_long), int(size(g_jloc), c_long), j, val, a%m), &
                    h_csr, 'csr_create')
  end subroutine csr_upload

  subroutine csr_mul_array_gpu(a, array, result)
    type(csr_gpu), intent(in) :: a
    doubleprecision, intent(in) :: array(:)
    doubleprecision, intent(inout) :: result(:)
    call pamg_check(pamg_csr_mul_array(h_csr, a%m, int(size(array), c_long), array, result), h_csr, 'csr_mul_array')
  end subroutine csr_mul_array_gpu

  subroutine csr_release(a)
    type(csr_gpu), intent(inout) :: a
    integer(c_int) :: rc
    rc = pamg_csr_free(a%m)
    a%m = c_null_ptr
  end subroutine csr_release

  subroutine csr_mul_array_arrays(g_iloc, g_jloc, val, array, result)
    integer, intent(in) :: g_iloc(:), g_jloc(:)
    doubleprecision, intent(in) :: val(:), array(:)
    doubleprecision, intent(inout) :: result(:)
    type(csr_gpu) :: a
    call csr_upload(g_iloc, g_jloc, val, a)
    call csr_mul_array_gpu(a, array, result)
    call csr_release(a)
  end subroutine csr_mul_array_arrays

  ! matrices.F90:172 signature
  subroutine csr_mul_array(sparse_matrix, array, result)
    type(sparse), intent(in) :: sparse_matrix
    real(8), allocatable, dimension(:), intent(in) :: array
    real(8), allocatable, intent(inout) :: result(:)
    call csr_mul_array_arrays(sparse_matrix%g_iloc, sparse_matrix%g_jloc, sparse_matrix%val, array, result)
  end subroutine csr_mul_array

end module pamg_matrices
