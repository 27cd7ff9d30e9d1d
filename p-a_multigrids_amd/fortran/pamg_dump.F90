! PAMGREC1 state dump of the Fortran host (same record names and layout as
! oracle/ref_hooks/pamg_ref_hooks.F90 and tests/pamg_records.py).
module pamg_dump
  use iso_c_binding
  use pamg
  implicit none
  private
  public :: write_dump
contains

  ! PAMGREC1 records, same names and layout as oracle/ref_hooks/pamg_ref_hooks.F90
  subroutine rec(u, name, a, dims)
    integer, intent(in) :: u
    character(len=*), intent(in) :: name
    real(8), intent(in) :: a(:)
    integer(8), intent(in) :: dims(:)
    write(u) 'PAMGREC1'
    write(u) int(len_trim(name), 4)
    write(u) trim(name)
    write(u) 1_4
    write(u) int(size(dims), 4)
    write(u) dims
    write(u) a
  end subroutine rec

  subroutine write_dump(h, fn, U, n_split, multi_levels)
    type(c_ptr), intent(in) :: h
    character(len=*), intent(in) :: fn
    integer, intent(in) :: U, n_split, multi_levels
    integer :: u_, l, nsub
    real(c_double), allocatable, target :: a(:), b(:)
    character(len=32) :: nm
    integer, parameter :: what(4) = [PAMG_TNEW, PAMG_TOLD, PAMG_RHS, PAMG_RESIDUAL]
    character(len=4), parameter :: names(4) = ['tnew', 'told', 'RHS ', 'res ']
    integer :: q
    open(newunit=u_, file=fn, access='stream', form='unformatted', status='replace')
    do l = 1, multi_levels
      nsub = 4**(n_split - l + 1)
      allocate(a(3*nsub*U))
      do q = 1, 4
        call pamg_check(pamg_get_state(h, int(l, c_int), int(what(q), c_int), a), h, 'get_state')
        write(nm, '(a,a,i0)') trim(names(q)), '_L', l
        call rec(u_, trim(nm), a, [3_8, int(nsub, 8), int(U, 8)])
      end do
      deallocate(a)
    end do
    ! at the end of the time loop tnew_nonlin holds level 1 (last smoother call, :376)
    allocate(a(3*4**n_split*U))
    call pamg_check(pamg_get_state(h, 1_c_int, int(PAMG_TNEW_NONLIN, c_int), a), h, 'get_state')
    call rec(u_, 'tnew_nonlin', a, [3_8, int(4**n_split, 8), int(U, 8)])
    deallocate(a)
    allocate(a(2**n_split*3*3*U), b(2**n_split*3*3*U))
    call pamg_check(pamg_get_overlap(h, a, b), h, 'get_overlap')
    call rec(u_, 't_overlap', a, [int(2**n_split*3, 8), 3_8, int(U, 8)])
    call rec(u_, 't_overlap_old', b, [int(2**n_split*3, 8), 3_8, int(U, 8)])
    close(u_)
  end subroutine write_dump

end module pamg_dump
