! iso_c_binding interface of libpamg (include/pamg.h) for Fortran hosts.
!
! This is the thin shim the reference's Fortran driver binds: every hot-path
! entry replaces one call site of Semi_implicit_iterative
! (transport_tri_semi.F90:299-381) -- smoother :331/:352/:376, restrictor :336,
! get_residual :338, prolongator :370 -- and the arrays cross the boundary in
! the reference's own layout tracer(l)%x(3, 4**(n_split-l+1), U), fp64.
module pamg
  use iso_c_binding
  implicit none
  private

  integer(c_int), parameter, public :: PAMG_OK = 0
  integer(c_int), parameter, public :: PAMG_TNEW = 0, PAMG_TOLD = 1, PAMG_RHS = 2, PAMG_RESIDUAL = 3
  integer(c_int), parameter, public :: PAMG_TNEW_NONLIN = 4, PAMG_SOURCE = 5

  type, bind(C), public :: pamg_params
    integer(c_int) :: n_split, multi_levels, n_smooth, n_coarse, solver, device
    real(c_double) :: dt, k, omega, theta
    integer(c_int) :: halo_mode
    integer(c_int) :: fused
    integer(c_int) :: coarse_solver
    integer(c_int) :: arith
    integer(c_int) :: halo_exchange
    integer(c_int) :: cycle
    integer(c_int) :: op
    integer(c_int) :: reserved(1)
  end type pamg_params

  public :: pamg_default_params, pamg_msh_read, pamg_msh_size, pamg_msh_get, pamg_msh_free
  public :: pamg_create, pamg_upload_mesh, pamg_set_state, pamg_get_state, pamg_get_overlap
  public :: pamg_begin_timestep, pamg_copy_to_nonlin, pamg_smoother, pamg_sweep, pamg_restrictor
  public :: pamg_get_residual, pamg_prolongator, pamg_vcycle, pamg_run, pamg_synchronize
  public :: pamg_destroy, pamg_last_error, pamg_check, c_path, pamg_block_inverse, pamg_direct_solve
  public :: pamg_write_vtu, pamg_csr_create, pamg_csr_mul_array, pamg_csr_free, pamg_tnn_level

  interface
    subroutine pamg_default_params(p) bind(C, name='pamg_default_params')
      import :: pamg_params
      type(pamg_params), intent(out) :: p
    end subroutine
    integer(c_int) function pamg_msh_read(path, m) bind(C, name='pamg_msh_read')
      import :: c_int, c_char, c_ptr
      character(kind=c_char), intent(in) :: path(*)
      type(c_ptr), intent(out) :: m
    end function
    integer(c_int) function pamg_msh_size(m, U) bind(C, name='pamg_msh_size')
      import :: c_int, c_ptr
      type(c_ptr), value :: m
      integer(c_int), intent(out) :: U
    end function
    integer(c_int) function pamg_msh_get(m, X, region, neig, fneig, dir) bind(C, name='pamg_msh_get')
      import :: c_int, c_ptr, c_double
      type(c_ptr), value :: m
      real(c_double), intent(out) :: X(*)
      integer(c_int), intent(out) :: region(*), neig(*), fneig(*), dir(*)
    end function
    subroutine pamg_msh_free(m) bind(C, name='pamg_msh_free')
      import :: c_ptr
      type(c_ptr), value :: m
    end subroutine
    integer(c_int) function pamg_create(p, h) bind(C, name='pamg_create')
      import :: c_int, c_ptr, pamg_params
      type(pamg_params), intent(in) :: p
      type(c_ptr), intent(out) :: h
    end function
    integer(c_int) function pamg_upload_mesh(h, U, X, region, neig, fneig, dir) bind(C, name='pamg_upload_mesh')
      import :: c_int, c_ptr, c_double
      type(c_ptr), value :: h
      integer(c_int), value :: U
      real(c_double), intent(in) :: X(*)
      integer(c_int), intent(in) :: region(*), neig(*), fneig(*), dir(*)
    end function
    integer(c_int) function pamg_set_state(h, level, what, a) bind(C, name='pamg_set_state')
      import :: c_int, c_ptr, c_double
      type(c_ptr), value :: h
      integer(c_int), value :: level, what
      real(c_double), intent(in) :: a(*)
    end function
    integer(c_int) function pamg_get_state(h, level, what, a) bind(C, name='pamg_get_state')
      import :: c_int, c_ptr, c_double
      type(c_ptr), value :: h
      integer(c_int), value :: level, what
      real(c_double), intent(out) :: a(*)
    end function
    integer(c_int) function pamg_get_overlap(h, a, b) bind(C, name='pamg_get_overlap')
      import :: c_int, c_ptr, c_double
      type(c_ptr), value :: h
      real(c_double), intent(out) :: a(*), b(*)
    end function
    integer(c_int) function pamg_begin_timestep(h) bind(C, name='pamg_begin_timestep')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function pamg_copy_to_nonlin(h, level) bind(C, name='pamg_copy_to_nonlin')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: level
    end function
    integer(c_int) function pamg_smoother(h, level, n_calls) bind(C, name='pamg_smoother')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: level, n_calls
    end function
    integer(c_int) function pamg_sweep(h, level, n_sweeps) bind(C, name='pamg_sweep')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: level, n_sweeps
    end function
    integer(c_int) function pamg_restrictor(h, level) bind(C, name='pamg_restrictor')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: level
    end function
    integer(c_int) function pamg_get_residual(h, level) bind(C, name='pamg_get_residual')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: level
    end function
    integer(c_int) function pamg_prolongator(h, level) bind(C, name='pamg_prolongator')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: level
    end function
    integer(c_int) function pamg_vcycle(h, n) bind(C, name='pamg_vcycle')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: n
    end function
    integer(c_int) function pamg_run(h, ntime, n_multigrid) bind(C, name='pamg_run')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: ntime, n_multigrid
    end function
    integer(c_int) function pamg_tnn_level(h) bind(C, name='pamg_tnn_level')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function pamg_synchronize(h) bind(C, name='pamg_synchronize')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function pamg_block_inverse(h, n, nb, a, inv, errorflag) bind(C, name='pamg_block_inverse')
      import :: c_int, c_ptr, c_double, c_long
      type(c_ptr), value :: h
      integer(c_int), value :: n
      integer(c_long), value :: nb
      real(c_double), intent(in) :: a(*)
      real(c_double), intent(out) :: inv(*)
      integer(c_int), intent(out) :: errorflag(*)
    end function
    integer(c_int) function pamg_direct_solve(h, level) bind(C, name='pamg_direct_solve')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: level
    end function
    integer(c_int) function pamg_csr_create(h, nrows, nnz, g_jloc, val, m) bind(C, name='pamg_csr_create')
      import :: c_int, c_ptr, c_long, c_double
      type(c_ptr), value :: h
      integer(c_long), value :: nrows, nnz
      integer(c_int), intent(in) :: g_jloc(*)
      real(c_double), intent(in) :: val(*)
      type(c_ptr), intent(out) :: m
    end function
    integer(c_int) function pamg_csr_mul_array(h, m, n, array, result) bind(C, name='pamg_csr_mul_array')
      import :: c_int, c_ptr, c_long, c_double
      type(c_ptr), value :: h, m
      integer(c_long), value :: n
      real(c_double), intent(in) :: array(*)
      real(c_double), intent(inout) :: result(*)
    end function
    integer(c_int) function pamg_csr_free(m) bind(C, name='pamg_csr_free')
      import :: c_int, c_ptr
      type(c_ptr), value :: m
    end function
    integer(c_int) function pamg_write_vtu(h, path, ascii) bind(C, name='pamg_write_vtu')
      import :: c_int, c_ptr, c_char
      type(c_ptr), value :: h
      character(kind=c_char), intent(in) :: path(*)
      integer(c_int), value :: ascii
    end function
    integer(c_int) function pamg_destroy(h) bind(C, name='pamg_destroy')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function pamg_last_error(h, buf, n) bind(C, name='pamg_last_error')
      import :: c_int, c_ptr, c_char
      type(c_ptr), value :: h
      character(kind=c_char), intent(out) :: buf(*)
      integer(c_int), value :: n
    end function
  end interface

contains

  ! NUL-terminated copy of a Fortran string for char* arguments
  function c_path(s) result(c)
    character(len=*), intent(in) :: s
    character(kind=c_char) :: c(len_trim(s) + 1)
    integer :: i
    do i = 1, len_trim(s)
      c(i) = s(i:i)
    end do
    c(len_trim(s) + 1) = c_null_char
  end function c_path

  ! The reference stops on errors (transport_tri_semi.F90:120-123); so does the shim.
  subroutine pamg_check(rc, h, what)
    integer(c_int), intent(in) :: rc
    type(c_ptr), intent(in) :: h
    character(len=*), intent(in) :: what
    character(kind=c_char) :: buf(512)
    character(len=512) :: msg
    integer :: i, ios
    if (rc == PAMG_OK) return
    msg = ''
    if (c_associated(h)) then
      ios = pamg_last_error(h, buf, 512_c_int)
      do i = 1, 512
        if (buf(i) == c_null_char) exit
        msg(i:i) = buf(i)
      end do
    end if
    print '(a,a,a,i0,a,a)', 'pamg: ', what, ' failed, rc=', rc, ' ', trim(msg)
    error stop 1
  end subroutine pamg_check

end module pamg
