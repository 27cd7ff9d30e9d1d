! ORACLE TEST INFRASTRUCTURE -- driver around the reference's own csr_mul_array
! (matrices.F90:172-193, compiled from /root/reference by oracle/build_ref.py with the
! rest of the Makefile's modules, -fdefault-real-8). Reads csr_in.bin (int32 nrows,
! nnz, n; nrows int32 g_iloc; nnz int32 g_jloc (1-based); nnz fp64 val; n fp64 array)
! and writes csr_out.bin (size(result) = nrows fp64 values after the call).
program csr_driver
  use Structures, only: sparse
  use matrices, only: csr_mul_array
  implicit none
  integer(4) :: nrows, nnz, n
  type(sparse) :: m
  real, allocatable :: array(:), result(:)
  open(10, file='csr_in.bin', access='stream', form='unformatted', status='old')
  read(10) nrows, nnz, n
  allocate(m%g_iloc(nrows), m%g_jloc(nnz), m%val(nnz), array(n), result(nrows))
  read(10) m%g_iloc, m%g_jloc, m%val, array
  close(10)
  result = -1.0
  call csr_mul_array(m, array, result)
  open(11, file='csr_out.bin', access='stream', form='unformatted', status='replace')
  write(11) result
  close(11)
end program csr_driver
