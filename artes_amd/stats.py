"""Monte-Carlo statistics used for parity checks (honest per-pixel variance, z-scores).

The reference reports sigma = sqrt(sum w^2 - (sum w)^2 / n_peels) per pixel
(``ARTES.f90:3490-3493``), treating every peel as independent.  A packet peels ~2.5
times and its peels land in the same 7300-km pixel, so that underestimates the error
by ~1.7-3x.  The engine also returns, per pixel and Stokes component, the
packet-level second moment M2 = sum_p X_p^2 (detector plane 3), from which the
variance of the pixel sum over N iid packets is N * Var(X) = M2 - S1^2 / N.
"""

from __future__ import annotations

import os
import re

import numpy as np

from . import fitsio


def pixel_sigma_raw(raw: np.ndarray, n_packets: int) -> np.ndarray:
    """Honest sigma of the per-pixel sums, raw weight units. raw: [4][4][ny][nx] -> [4][ny][nx]."""
    s1 = raw[0]
    m2 = raw[3]
    return np.sqrt(np.clip(m2 - s1 * s1 / float(n_packets), 0.0, None))


def per_packet_pixel_variance(raw: np.ndarray, n_packets: int) -> np.ndarray:
    """Var(X) of one packet's contribution to each pixel (raw units), [4][ny][nx]."""
    return pixel_sigma_raw(raw, n_packets) ** 2 / float(n_packets)


def total_sigma_raw(totals: np.ndarray, n_packets: int) -> np.ndarray:
    """Honest sigma of the integrated sums per Stokes (raw units) from totals[0:8]."""
    t1, t2 = totals[:4], totals[4:8]
    return np.sqrt(np.clip(t2 - t1 * t1 / float(n_packets), 0.0, None))


def total_sigma_scaled(totals: np.ndarray, n_packets: int, energy: float, n_other: int | None = None) -> np.ndarray:
    """Honest sigma of the integrated Stokes sums in energy units, for this run (n_other=None)
    or for a run of ``n_other`` packets of the same workload (its energy is energy*n/n_other)."""
    var1 = total_sigma_raw(totals, n_packets) ** 2 / float(n_packets)
    n2 = n_packets if n_other is None else n_other
    return np.sqrt(n2 * var1) * energy * n_packets / float(n2)


def read_photometry(path: str) -> np.ndarray:
    """Numbers of a photometry.dat data record (list-directed output may wrap lines)."""
    with open(path) as f:
        txt = f.read()
    body = txt.rsplit("]", 1)[1] if "]" in txt else txt
    nums = re.findall(r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eEdD][-+]?\d+)?", body)
    return np.array([float(x.replace("D", "E").replace("d", "e")) for x in nums])


def load_reference_run(path: str) -> dict:
    """A frozen reference output directory (tests/golden/reference_runs/<run>)."""
    stokes = fitsio.read(os.path.join(path, "stokes.fits"))[0].data.astype(np.float64)
    error = fitsio.read(os.path.join(path, "error.fits"))[0].data.astype(np.float64)
    ph = read_photometry(os.path.join(path, "photometry.dat"))
    return dict(stokes=stokes, error=error, photometry=ph)


def zscores(a: np.ndarray, sa: np.ndarray, b: np.ndarray, sb: np.ndarray, mask: np.ndarray | None = None):
    """z = (a - b) / sqrt(sa^2 + sb^2) over ``mask`` (default: pixels where sigma > 0)."""
    s = np.sqrt(sa * sa + sb * sb)
    m = (s > 0) if mask is None else (mask & (s > 0))
    return (a[m] - b[m]) / s[m]


def compare_to_reference(raw: np.ndarray, n_packets: int, energy: float, pixel_scale: float,
                         ref: dict, n_ref: int, stokes: int = 0) -> dict:
    """Per-pixel z-scores of this run against a frozen reference image (fits units).

    Both sigmas come from this run's packet-level variance, scaled to each side's packet
    count (same inputs, same estimator => same per-packet variance)."""
    unit = 1.0e-6 / (pixel_scale * pixel_scale)
    mine = raw[0, stokes] * energy * unit
    var1 = per_packet_pixel_variance(raw, n_packets)[stokes]
    sig_mine = np.sqrt(n_packets * var1) * energy * unit
    e_ref = energy * n_packets / float(n_ref)
    sig_ref = np.sqrt(n_ref * var1) * e_ref * unit
    refimg = ref["stokes"][stokes]
    z = zscores(mine, sig_mine, refimg, sig_ref, mask=(refimg != 0) | (mine != 0))
    return dict(rms_z=float(np.sqrt(np.mean(z * z))) if z.size else float("nan"),
                mean_z=float(np.mean(z)) if z.size else float("nan"),
                median_abs_z=float(np.median(np.abs(z))) if z.size else float("nan"),
                frac_gt4=float(np.mean(np.abs(z) > 4.0)) if z.size else float("nan"),
                max_abs_z=float(np.max(np.abs(z))) if z.size else float("nan"), n_pixels=int(z.size))


def records_agree(a: np.ndarray, b: np.ndarray, rtol: float = 1e-9) -> np.ndarray:
    """Per-packet agreement of two ``artes_run_trace`` record arrays ``[n][8]`` (GPU engine vs
    CPU oracle, same seeds): the same scatter count, crossing count and end state, the same
    peeled Stokes I to ``rtol``, and the same peeled -Q, U, V to ``rtol`` of the peeled I."""
    scale = np.abs(a[:, 0]) + np.abs(b[:, 0])
    ok = (np.isclose(a[:, 0], b[:, 0], rtol=rtol, atol=1e-300) & (a[:, 1] == b[:, 1]) & (a[:, 2] == b[:, 2])
          & (a[:, 3] == b[:, 3]))
    for k in (4, 5, 6):
        ok &= np.abs(a[:, k] - b[:, k]) <= rtol * scale + 1e-300
    return ok
