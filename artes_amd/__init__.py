"""artes_amd -- MI355X-native Monte Carlo polarized radiative transfer (drop-in for bgin/ARTES).

Layout:
  fitsio      minimal FITS reader/writer (atmosphere.fits, stokes.fits, error.fits)
  config      artes.in keyword system (ARTES.f90:4361-4500)
  opacity     isotropic / Henyey-Greenstein / Rayleigh generators (python/opacity*.py)
  atmosphere  atmosphere.in -> atmosphere.fits builder (python/atmosphere.py)
  synthetic   benchmark / parity atmospheres
  engine      ctypes binding of the HIP transport engine (include/artes_amd.h)
  driver      detector geometry, package energy, photometry, output writers
  runner      run modes (imaging_mono / spectrum / phase / imaging_broad) + CLI
  dist        one process per GPU, RCCL detector all-reduce
"""

__version__ = "0.1.0"
