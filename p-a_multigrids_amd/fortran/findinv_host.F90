! Host example of the FINDInv drop-in (module matrix_inversion): reads
! findinv_in.bin (int32 n, int32 count, count n x n column-major fp64 matrices),
! inverts each with `call FINDInv(a, inv, n, ierr)` exactly as a reference call
! site does, writes findinv_out.bin (the inverses, then the int32 errorflags).
program findinv_host
  use matrix_inversion, only: FINDInv
  implicit none
  integer(4) :: n, cnt, q, ierr
  double precision, allocatable :: a(:,:), inv(:,:), outv(:,:,:)
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
end program findinv_host
