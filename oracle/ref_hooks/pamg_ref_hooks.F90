! ORACLE TEST INFRASTRUCTURE -- not product code.
!
! Hooks linked into the patched, instrumented build of the reference Fortran
! (oracle/build_ref.py). They give the reference's mode-9 driver
! (transport_tri_semi.F90:14-891) a run-time configuration instead of its
! hard-coded mesh path / n_split / ntime (transport_tri_semi.F90:99,118,135 and
! main.F90:46-47) and write the driver's state as binary records so that the
! build's HIP path can be compared at full fp64 precision (the reference's own
! VTU output is F12.10 text, get_vtk_files.F90:50-52, too coarse for parity).
!
! Record format ("PAMGREC1"), shared with tests/pamg_records.py:
!   8 bytes magic 'PAMGREC1' | int32 name_len | name | int32 dtype (1=f64, 2=i32)
!   | int32 ndim | int64 dims(ndim) | data in Fortran (column-major) order
module pamg_ref_hooks
  use Structures
  implicit none

  character(len=512) :: pamg_mesh = './test_sn2.msh'
  character(len=512) :: pamg_dump_prefix = ''
  integer :: pamg_nsplit = 1, pamg_ntime = 2, pamg_nmultigrid = 2
  integer :: pamg_solver = 3, pamg_levels = 1, pamg_nsmooth = 4
  integer :: pamg_vtk = 100000, pamg_dump_calls = 0
  integer :: pamg_call_counter = 0
  namelist /pamg_ref/ pamg_mesh, pamg_dump_prefix, pamg_nsplit, pamg_ntime, &
       pamg_nmultigrid, pamg_solver, pamg_levels, pamg_nsmooth, pamg_vtk, pamg_dump_calls

contains

  subroutine pamg_cfg_read()
    integer :: u, ios
    open(newunit=u, file='pamg_ref.nml', status='old', action='read', iostat=ios)
    if (ios /= 0) then
      print *, 'pamg_ref_hooks: pamg_ref.nml not found, using defaults'
      return
    end if
    read(u, nml=pamg_ref, iostat=ios)
    if (ios /= 0) then
      print *, 'pamg_ref_hooks: error reading namelist pamg_ref'
      stop 2
    end if
    close(u)
  end subroutine pamg_cfg_read

  subroutine rec_head(u, name, dtype, dims)
    integer, intent(in) :: u, dtype
    character(len=*), intent(in) :: name
    integer(8), intent(in) :: dims(:)
    write(u) 'PAMGREC1'
    write(u) int(len_trim(name), 4)
    write(u) trim(name)
    write(u) int(dtype, 4)
    write(u) int(size(dims), 4)
    write(u) dims
  end subroutine rec_head

  subroutine rec_f3(u, name, a)
    integer, intent(in) :: u
    character(len=*), intent(in) :: name
    real, intent(in) :: a(:,:,:)
    integer(8) :: d(3)
    d = shape(a, kind=8)
    call rec_head(u, name, 1, d)
    write(u) real(a, 8)
  end subroutine rec_f3

  subroutine rec_i2(u, name, a)
    integer, intent(in) :: u
    character(len=*), intent(in) :: name
    integer, intent(in) :: a(:,:)
    integer(8) :: d(2)
    d = shape(a, kind=8)
    call rec_head(u, name, 2, d)
    write(u) int(a, 4)
  end subroutine rec_i2

  subroutine rec_d(u, name, a, dims)
    integer, intent(in) :: u
    character(len=*), intent(in) :: name
    real(8), intent(in) :: a(:)
    integer(8), intent(in) :: dims(:)
    call rec_head(u, name, 1, dims)
    write(u) a
  end subroutine rec_d

  ! Full multigrid state: every level's tnew/told/RHS/residuale plus the
  ! driver's scratch tnew_nonlin (transport_tri_semi.F90:85, :325-327).
  subroutine write_state(u, tracer, tnew_nonlin, nlev)
    integer, intent(in) :: u, nlev
    type(fields), intent(in) :: tracer(:)
    real, intent(in) :: tnew_nonlin(:,:,:)
    integer :: l
    character(len=32) :: nm
    do l = 1, nlev
      write(nm, '(a,i0)') 'tnew_L', l
      call rec_f3(u, trim(nm), tracer(l)%tnew)
      write(nm, '(a,i0)') 'told_L', l
      call rec_f3(u, trim(nm), tracer(l)%told)
      write(nm, '(a,i0)') 'RHS_L', l
      call rec_f3(u, trim(nm), tracer(l)%RHS)
      write(nm, '(a,i0)') 'res_L', l
      call rec_f3(u, trim(nm), tracer(l)%residuale)
    end do
    call rec_f3(u, 'tnew_nonlin', tnew_nonlin)
  end subroutine write_state

  ! Per-call dump, first V-cycle of the first time step only.
  subroutine pamg_dump_call(tag, ilevel, itime, multigrid, tracer, tnew_nonlin, nlev)
    character(len=*), intent(in) :: tag
    integer, intent(in) :: ilevel, itime, multigrid, nlev
    type(fields), intent(in) :: tracer(:)
    real, intent(in) :: tnew_nonlin(:,:,:)
    integer :: u
    character(len=700) :: fn
    if (pamg_dump_calls == 0 .or. len_trim(pamg_dump_prefix) == 0) return
    if (itime /= 1 .or. multigrid /= 1) return
    pamg_call_counter = pamg_call_counter + 1
    write(fn, '(a,a,i3.3,a,a,a,i0,a)') trim(pamg_dump_prefix), '_call', pamg_call_counter, '_', &
         trim(tag), '_L', ilevel, '.bin'
    open(newunit=u, file=trim(fn), access='stream', form='unformatted', status='replace')
    call write_state(u, tracer, tnew_nonlin, nlev)
    close(u)
  end subroutine pamg_dump_call

  ! Final dump after the time loop (transport_tri_semi.F90:383): state,
  ! halo buffers t_overlap / t_overlap_old (splitting.F90:1210-1397) and the
  ! setup quantities the hot path consumes: mesh topology (Msh2Tri.F90:132-334,
  ! 454-548), per-level detwei / nx (ShapFun.F90:1661-1684) and the 3x3
  ! stencils of get_un_ele_mass_stiff_diffvol (ShapFun_unstruc.F90:304-335)
  ! reduced exactly as the smoother does (transport_tri_semi.F90:592-607).
  subroutine pamg_dump_final(tracer, tnew_nonlin, meshList, nlev, n_split, n, k, dt, ngi, nloc, ndim)
    use ShapFun_unstruc, only: get_un_ele_mass_stiff_diffvol
    type(fields), intent(in) :: tracer(:)
    real, intent(in) :: tnew_nonlin(:,:,:)
    type(Mesh), intent(in), target :: meshList(:)
    integer, intent(in) :: nlev, n_split, ngi, nloc, ndim
    real, intent(in) :: n(:,:), k, dt
    integer :: u, U_, e, l, i, j, d, slots
    character(len=700) :: fn
    character(len=32) :: nm
    real(8), allocatable :: buf(:)
    integer, allocatable :: ib(:,:)
    real, allocatable :: mass_stcl(:,:), stiff_stcl(:,:,:,:), diff_vol_stcl(:,:,:,:), ml_ele(:), nx(:,:,:)
    real, allocatable :: diff_vol1(:,:)
    real, pointer :: detwei(:)

    if (len_trim(pamg_dump_prefix) == 0) return
    U_ = size(meshList)
    fn = trim(pamg_dump_prefix)//'_final.bin'
    open(newunit=u, file=trim(fn), access='stream', form='unformatted', status='replace')
    call write_state(u, tracer, tnew_nonlin, nlev)

    slots = size(meshList(1)%t_overlap, 1)
    allocate(buf(slots*3*U_))
    do e = 1, U_
      buf((e-1)*slots*3+1:e*slots*3) = reshape(real(meshList(e)%t_overlap, 8), [slots*3])
    end do
    call rec_d(u, 't_overlap', buf, [int(slots,8), 3_8, int(U_,8)])
    do e = 1, U_
      buf((e-1)*slots*3+1:e*slots*3) = reshape(real(meshList(e)%t_overlap_old, 8), [slots*3])
    end do
    call rec_d(u, 't_overlap_old', buf, [int(slots,8), 3_8, int(U_,8)])
    deallocate(buf)

    allocate(buf(6*U_))
    do e = 1, U_
      buf((e-1)*6+1:e*6) = reshape(meshList(e)%X, [6])
    end do
    call rec_d(u, 'X', buf, [2_8, 3_8, int(U_,8)])
    deallocate(buf)
    allocate(ib(3, U_))
    do e = 1, U_
      ib(:, e) = meshList(e)%Neig
    end do
    call rec_i2(u, 'Neig', ib)
    do e = 1, U_
      ib(:, e) = meshList(e)%fNeig
    end do
    call rec_i2(u, 'fNeig', ib)
    do e = 1, U_
      do i = 1, 3
        ib(i, e) = merge(1, 0, meshList(e)%Dir(i))
      end do
    end do
    call rec_i2(u, 'Dir', ib)
    do e = 1, U_
      ib(:, e) = meshList(e)%region_id
    end do
    call rec_i2(u, 'region', ib)
    deallocate(ib)

    allocate(mass_stcl(nloc,nloc), stiff_stcl(nloc,ngi,ndim,nloc), diff_vol_stcl(ngi,ndim,nloc,nloc))
    allocate(ml_ele(nloc), nx(ngi,ndim,nloc), diff_vol1(nloc,nloc))
    allocate(buf(9*U_*3))
    do l = 1, nlev
      ! mass (3,3,U), diffusion (3,3,U), lumped mass (3,U), detwei (ngi,U), nx (ngi,ndim,nloc,U)
      do e = 1, U_
        detwei => meshList(e)%scaling_var(l)%detwei
        nx = meshList(e)%scaling_var(l)%nx
        call get_un_ele_mass_stiff_diffvol(mass_stcl, stiff_stcl, diff_vol_stcl, n, nx, detwei, k, &
             nloc, ngi, ndim, dt, ml_ele)
        diff_vol1 = 0.0
        do i = 1, nloc
          do d = 1, ndim
            do j = 1, nloc
              diff_vol1(i,j) = diff_vol1(i,j) + sum(diff_vol_stcl(:,d,i,j))
            end do
          end do
        end do
        buf((e-1)*9+1:e*9) = reshape(real(mass_stcl, 8), [9])
        buf(9*U_+(e-1)*9+1:9*U_+e*9) = reshape(real(diff_vol1, 8), [9])
        buf(18*U_+(e-1)*3+1:18*U_+e*3) = real(ml_ele, 8)
        buf(21*U_+(e-1)*3+1:21*U_+e*3) = real(detwei, 8)
      end do
      write(nm, '(a,i0)') 'mass_L', l
      call rec_d(u, trim(nm), buf(1:9*U_), [3_8, 3_8, int(U_,8)])
      write(nm, '(a,i0)') 'kdiff_L', l
      call rec_d(u, trim(nm), buf(9*U_+1:18*U_), [3_8, 3_8, int(U_,8)])
      write(nm, '(a,i0)') 'ml_L', l
      call rec_d(u, trim(nm), buf(18*U_+1:21*U_), [3_8, int(U_,8)])
      write(nm, '(a,i0)') 'detwei_L', l
      call rec_d(u, trim(nm), buf(21*U_+1:24*U_), [3_8, int(U_,8)])
    end do
    close(u)
  end subroutine pamg_dump_final

end module pamg_ref_hooks
