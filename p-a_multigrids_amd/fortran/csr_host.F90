! Host example of the csr_mul_array drop-in (module pamg_matrices): reads csr_in.bin
! (int32 nrows, nnz, n; nrows int32 g_iloc; nnz int32 g_jloc; nnz fp64 val; n fp64
! array), fills a `type(sparse)` and calls csr_mul_array(sparse_matrix, array, result)
! exactly as a reference call site does (transport_tri_semi_complete_implicit.F90:390),
! writes csr_out.bin (the nrows results).
program csr_host
  use pamg_matrices, only: sparse, csr_mul_array
  implicit none
  integer(4) :: nrows, nnz, n
  type(sparse) :: m
  real(8), allocatable :: array(:), result(:)
  open(10, file='csr_in.bin', access='stream', form='unformatted', status='old')
  read(10) nrows, nnz, n
  allocate(m%g_iloc(nrows), m%g_jloc(nnz), m%val(nnz), array(n), result(nrows))
  read(10) m%g_iloc, m%g_jloc, m%val, array
  close(10)
  result = -1.0d0
  call csr_mul_array(m, array, result)
  open(11, file='csr_out.bin', access='stream', form='unformatted', status='replace')
  write(11) result
  close(11)
end program csr_host
