! ORACLE TEST INFRASTRUCTURE -- driver around the reference's own FINDInv
! (matrix_inversion.F90:50-148, compiled unmodified from /root/reference by
! oracle/build_ref.py with -fdefault-real-8). Reads findinv_in.bin
! (int32 n, int32 count, count n x n column-major matrices of default real) and
! writes findinv_out.bin (the count inverses, then the count errorflags, int32).
program findinv_driver
  use matrix_inversion, only: FINDInv
  implicit none
  integer(4) :: n, cnt, q, ierr
  real, allocatable :: a(:,:), inv(:,:), outv(:,:,:)
  integer(4), allocatable :: flags(:)
  open(10, file='findinv_in.bin', access='stream', form='unformatted', status='old')
  read(10) n, cnt
  allocate(a(n, n), inv(n, n), outv(n, n, cnt), flags(cnt))
  do q = 1, cnt
    read(10) a
    call FINDInv(a, inv, n, ierr)
    outv(:, :, q) = inv
    flags(q) = ierr
  end do
  close(10)
  open(11, file='findinv_out.bin', access='stream', form='unformatted', status='replace')
  write(11) outv, flags
  close(11)
end program findinv_driver
