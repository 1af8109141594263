! abi_probe.f90 -- a Fortran host driving the C ABI as the reference's `run` would
! (ARTES.f90:121-267): build the device tables of a small isotropic atmosphere, run one
! imaging_mono batch, read back the detector.  Prints key=value lines for
! tests/test_fortran_binding.py.
program abi_probe
  use, intrinsic :: iso_c_binding
  use artes_amd_c
  implicit none
  integer, parameter :: nr = 4, nth = 1, nph = 1, nwl = 1, nx = 5, ny = 5
  real(c_double), target :: radial(nr + 1), theta(nth + 1), phi(nph), wl(nwl)
  real(c_double), target :: ksca(nr, nth, nph, nwl), kabs(nr, nth, nph, nwl)
  real(c_double), target :: scatter(nr, nth, nph, nwl, 16, 180)
  real(c_double) :: detector(nx, ny, 4, 4), totals(ARTES_NUM_TOTALS)
  integer(c_int64_t) :: counters(ARTES_NUM_COUNTERS), err(ARTES_NUM_ERR)
  type(artes_grid_desc) :: desc
  type(artes_run_params) :: prm
  type(c_ptr) :: grid
  integer(c_int32_t) :: rc
  integer :: i, npk
  real(c_double), parameter :: pi = 3.14159265358979323846_c_double
  character(len=32) :: arg

  npk = 100000
  if (command_argument_count() >= 1) then
     call get_command_argument(1, arg)
     read (arg, *) npk
  end if
  print '(a,i0)', 'abi_version=', artes_abi_version()
  print '(a,i0)', 'sizeof_desc=', c_sizeof(desc)
  print '(a,i0)', 'sizeof_params=', c_sizeof(prm)

  do i = 1, nr + 1
     radial(i) = 69911.e3_c_double + (i - 1) * 25.e3_c_double
  end do
  theta = [0._c_double, 180._c_double]
  phi = [0._c_double]
  wl = [0.7_c_double]
  ksca = 1._c_double / 100.e3_c_double
  kabs = 0._c_double
  scatter = 0._c_double
  scatter(:, :, :, :, 1, :) = 1._c_double / (4._c_double * pi)   ! isotropic P11

  desc = artes_grid_desc(nr, nth, nph, nwl, c_loc(radial), c_loc(theta), c_loc(phi), c_loc(wl), &
       c_loc(ksca), c_loc(kabs), c_loc(scatter), c_null_ptr, 0._c_double)

  ! invalid input: radial faces that do not increase -> -22, nothing allocated
  radial(2) = radial(1)
  rc = artes_grid_create(desc, 0, grid)
  print '(a,i0)', 'bad_grid_rc=', rc
  print '(a,a)', 'bad_grid_msg=', trim(artes_error_message())
  radial(2) = radial(1) + 25.e3_c_double

  ! a null grid handle -> -22
  rc = artes_run(c_null_ptr, prm, 0_c_int64_t, 1_c_int64_t, 1_c_int64_t, detector, totals, counters, err)
  print '(a,i0)', 'null_grid_rc=', rc

  print '(a,i0)', 'devices=', artes_device_count()
  rc = artes_grid_create(desc, 0, grid)
  print '(a,i0)', 'grid_rc=', rc
  if (rc /= 0) then
     print '(a,a)', 'grid_msg=', trim(artes_error_message())
     stop
  end if
  ! imaging_mono at theta = phi = 90 deg, the defaults of ARTES.f90:280-314
  prm = artes_run_params(0, nx, ny, 1, 1, 0, 0, artes_grid_cell_depth(grid, 0), &
       pi / 2, pi / 2, 1.3_c_double * radial(nr + 1), 1.3_c_double * radial(nr + 1), 1.e-5_c_double, 1.e-20_c_double, &
       0._c_double, 0._c_double, 0._c_double, 1, 1, 0, 0, 0._c_double)
  detector = 0; totals = 0; counters = 0; err = 0
  rc = artes_run(grid, prm, 0_c_int64_t, int(npk, c_int64_t), 20171015_c_int64_t, detector, totals, counters, err)
  print '(a,i0)', 'run_rc=', rc
  print '(a,es24.16)', 'detector_I=', sum(detector(:, :, 1, 1))
  print '(a,es24.16)', 'detector_Q=', sum(detector(:, :, 2, 1))
  print '(a,i0)', 'packets=', counters(4)
  print '(a,i0)', 'scatters=', counters(2)
  print '(a,i0)', 'errors=', sum(err)
  call artes_grid_destroy(grid)
end program abi_probe
