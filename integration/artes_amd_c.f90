! artes_amd_c.f90 -- the ISO_C_BINDING interface a maintainer of bgin/ARTES would add to
! call the MI355X transport engine (include/artes_amd.h) from the Fortran driver in place
! of the OpenMP packet loop of radiative_transfer (ARTES.f90:518-1006).
! Compiled and exercised by tests/test_fortran_binding.py (amdflang, ROCm 7.2).
module artes_amd_c
  use, intrinsic :: iso_c_binding
  implicit none

  integer(c_int32_t), parameter :: ARTES_NUM_TOTALS = 10, ARTES_NUM_COUNTERS = 8, ARTES_NUM_ERR = 64

  ! raw atmosphere.fits arrays (ARTES.f90:2067-2198), C order = the Fortran order reversed
  type, bind(C) :: artes_grid_desc
     integer(c_int32_t) :: nr, ntheta, nphi, nwav
     type(c_ptr) :: radial, theta_deg, phi_deg, wavelength_um
     type(c_ptr) :: kappa_sca, kappa_abs, scatter, temperature
     real(c_double) :: oblateness
  end type

  ! the globals radiative_transfer reads, per call
  type, bind(C) :: artes_run_params
     integer(c_int32_t) :: wl_index, nx, ny, photon_source, photon_scattering
     integer(c_int32_t) :: phase_far, stellar_direction, cell_depth
     real(c_double) :: det_theta, det_phi, x_max, y_max, fstop, photon_minimum
     real(c_double) :: surface_albedo, theta_star, phi_star
     integer(c_int32_t) :: photon_emission, thermal_weight, ring, packet_moments
     real(c_double) :: photon_bias
  end type

  interface
     integer(c_int32_t) function artes_abi_version() bind(C)
       import :: c_int32_t
     end function
     integer(c_int32_t) function artes_device_count() bind(C)
       import :: c_int32_t
     end function
     type(c_ptr) function artes_last_error() bind(C)
       import :: c_ptr
     end function
     integer(c_int32_t) function artes_grid_create(desc, device, grid) bind(C)
       import :: c_int32_t, c_ptr, artes_grid_desc
       type(artes_grid_desc), intent(in) :: desc
       integer(c_int32_t), value :: device
       type(c_ptr), intent(out) :: grid
     end function
     integer(c_int32_t) function artes_grid_cell_depth(grid, wl) bind(C)
       import :: c_int32_t, c_ptr
       type(c_ptr), value :: grid
       integer(c_int32_t), value :: wl
     end function
     integer(c_int32_t) function artes_run(grid, params, first, n, seed, detector, totals, counters, err) bind(C)
       import :: c_int32_t, c_int64_t, c_ptr, c_double, artes_run_params
       type(c_ptr), value :: grid
       type(artes_run_params), intent(in) :: params
       integer(c_int64_t), value :: first, n, seed        ! uint64 on the C side
       real(c_double), intent(inout) :: detector(*)       ! (nx,ny,4,4) = C [4][4][ny][nx]
       real(c_double), intent(inout) :: totals(*)         ! ARTES_NUM_TOTALS
       integer(c_int64_t), intent(inout) :: counters(*), err(*)
     end function
     subroutine artes_grid_destroy(grid) bind(C)
       import :: c_ptr
       type(c_ptr), value :: grid
     end subroutine
  end interface

contains

  ! the thread-local message behind artes_last_error as a Fortran string
  function artes_error_message() result(msg)
    character(len=256) :: msg
    character(kind=c_char), pointer :: p(:)
    integer :: i
    msg = ''
    call c_f_pointer(artes_last_error(), p, [256])
    do i = 1, 256
       if (p(i) == c_null_char) exit
       msg(i:i) = p(i)
    end do
  end function

end module artes_amd_c
