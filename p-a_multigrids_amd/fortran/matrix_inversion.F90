! Drop-in for the reference's local block solve: module matrix_inversion with
! FINDInv(matrix, inverse, n, errorflag) (matrix_inversion.F90:50-148, the same
! routine as matrices.F90:1618-1716), computed on the GPU by libpamg's
! pamg_block_inverse -- the reference's Gauss-Jordan without pivoting, its
! zero-pivot row repair and give-up rule, bitwise equal to it (fp64: the
! reference's REAL built with -fdefault-real-8). A call site keeps
! `use matrix_inversion` and `call FINDInv(...)` unchanged. The routine uses the
! handle bound with pamg_bind_inverse_handle, or creates one on device 0.
module matrix_inversion
  use iso_c_binding
  use pamg
  implicit none
  private
  type(c_ptr), save :: h_inv = c_null_ptr
  public :: FINDInv, FINDInv_batch, pamg_bind_inverse_handle

contains

  subroutine pamg_bind_inverse_handle(h)
    type(c_ptr), intent(in) :: h
    h_inv = h
  end subroutine pamg_bind_inverse_handle

  subroutine ensure_handle()
    type(pamg_params), target :: p
    if (c_associated(h_inv)) return
    call pamg_default_params(p)
    call pamg_check(pamg_create(p, h_inv), h_inv, 'create (matrix_inversion)')
  end subroutine ensure_handle

  ! matrix_inversion.F90:50 signature
  subroutine FINDInv(matrix, inverse, n, errorflag)
    integer, intent(in) :: n
    integer, intent(out) :: errorflag
    double precision, intent(in), dimension(n, n) :: matrix
    double precision, intent(out), dimension(n, n) :: inverse
    integer(c_int) :: err(1)
    call ensure_handle()
    call pamg_check(pamg_block_inverse(h_inv, int(n, c_int), 1_c_long, matrix, inverse, err), h_inv, 'block_inverse')
    errorflag = err(1)
    if (errorflag /= 0) print *, "Matrix is non - invertible"   ! :89, :99
  end subroutine FINDInv

  ! nb independent n x n blocks in one launch (the element blocks of a mesh)
  subroutine FINDInv_batch(matrices, inverses, n, nb, errorflags)
    integer, intent(in) :: n, nb
    double precision, intent(in), dimension(n, n, nb) :: matrices
    double precision, intent(out), dimension(n, n, nb) :: inverses
    integer, intent(out), dimension(nb) :: errorflags
    integer(c_int) :: err(nb)
    call ensure_handle()
    call pamg_check(pamg_block_inverse(h_inv, int(n, c_int), int(nb, c_long), matrices, inverses, err), h_inv, &
                    'block_inverse')
    errorflags = err
  end subroutine FINDInv_batch

end module matrix_inversion
