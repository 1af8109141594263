"""Generate tests/golden/molecular/self_luminous_100wl.npz (run in the build container only:
it reads the reference's dat/molecules tables, which do not travel to the GPU box).

BASELINE configs[4]: self-luminous thermal emission with P-T dependent molecular
opacities (opacityMolecules), 100 wavelengths.  The P-T profile is
pressureTemperatureSelfLuminous.py's default (Teff 800 K, kappa 1e-2 cm2/g, log g 3.4,
1e-3..1e2 bar, 20 levels); the per-layer opacities are artes_amd.gas.molecule_opacities
(the restatement of opacityMolecules.py:120-300) over the 100 table wavelengths from
1.0 micron.  Only the [layer][4][wavelength] opacity tables are stored; the H2 Rayleigh
scattering matrices are regenerated at test time (gas.rayleigh_matrix_table).

usage: python tools/make_molecular_fixture.py [dat_dir]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from artes_amd import gas  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "molecular", "self_luminous_100wl.npz")
NWAV = 100


def build(dat_dir: str):
    p, t = gas.pt_self_luminous(t_eff=800.0, kappa=1e-2, log_g=3.4, p_min=1e-3, p_max=1e2, levels=20)
    wl, _ = gas.read_grid_opacity(dat_dir, 1)
    i0 = int(np.searchsorted(wl, 1.0))
    # molecule_opacities keeps lambda >= min and stops after the first lambda > max
    ops = gas.molecule_opacities(p, t, dat_dir, wavelength_min=1.0, wavelength_max=float(wl[i0 + NWAV - 2]))
    layers = np.array(sorted(ops), dtype=np.int64)
    opacity = np.stack([ops[k][0] for k in layers])
    assert opacity.shape == (len(p), 4, NWAV), opacity.shape
    return dict(pressure=p, temperature=t, layers=layers, opacity=opacity)


if __name__ == "__main__":
    dat = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/dat/molecules"
    d = build(dat)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez(OUT, **d)
    print(OUT, {k: v.shape for k, v in d.items()}, d["opacity"][0, 0, [0, -1]])
