import os

import numpy as np

from artes_amd import fitsio
from conftest import GOLDEN


def test_roundtrip_multi_hdu(tmp_path):
    a = np.arange(24, dtype=np.float64).reshape(2, 3, 4) * 1.5 - 7
    b = np.array([1.0, 2.0, 3.0])
    c = np.random.default_rng(0).normal(size=(5, 1, 2, 3))
    p = tmp_path / "x.fits"
    fitsio.write(p, [a, b, c], names=["", "B", "C"])
    hd = fitsio.read(p)
    assert len(hd) == 3
    np.testing.assert_array_equal(hd[0].data, a)
    np.testing.assert_array_equal(hd[1].data, b)
    np.testing.assert_array_equal(hd[2].data, c)
    assert hd[0].header["NAXIS1"] == 4 and hd[0].header["NAXIS3"] == 2     # FITS axis 1 = last numpy axis
    assert hd[1].header["XTENSION"] == "IMAGE" and hd[2].name == "C"
    assert os.path.getsize(p) % 2880 == 0


def test_reads_reference_outputs():
    d = os.path.join(GOLDEN, "reference_runs", "t_ray3d_ARTES_det_1e6")
    s = fitsio.read(os.path.join(d, "stokes.fits"))
    e = fitsio.read(os.path.join(d, "error.fits"))
    assert s[0].data.shape == (4, 25, 25) and s[0].header["BITPIX"] == -64
    assert e[0].data.shape == (5, 25, 25)
    assert np.all(np.isfinite(s[0].data))
    assert s[0].data[0].sum() > 0 and np.all(s[0].data[3] == 0)    # V = 0 for Rayleigh


def test_other_bitpix(tmp_path):
    a = np.arange(12, dtype=np.int32).reshape(3, 4)
    p = tmp_path / "i.fits"
    fitsio.write(p, [a], bitpix=32)
    np.testing.assert_array_equal(fitsio.read(p)[0].data, a)
