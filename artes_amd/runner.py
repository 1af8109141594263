"""Drop-in command line for ``./bin/ARTES`` and its run modes.

``python -m artes_amd <atmosphere> <photons> -o <output> [-k key=value]... [--seed S]``

Mirrors ``initialize`` / ``argument_input`` / ``argument_keywords`` / ``run`` /
``write_output`` of the reference (``ARTES.f90:121-516``, ``3472-3772``, ``4232-4309``):
the working directory must contain ``input/<atmosphere>/{artes.in,atmosphere.fits}``;
``-o`` wipes and recreates ``output/<name>/{input,output,plot}`` and copies the inputs;
each ``-k`` is applied after ``artes.in`` and appended to the copied ``artes.in``.
Outputs: ``output/<name>/{error.log,plot.dat}``, ``output/<name>/output/{stokes.fits,
error.fits,photometry.dat,normalization.dat,cell_depth.dat}`` (imaging_mono), plus
``spectrum.dat`` / ``phase.dat`` for the other modes (with ``optical_depth.dat`` in
``spectrum`` and ``imaging_broad``), ``luminosity.dat`` /
``cell_luminosity.fits`` for the planet source and ``flow_global.fits`` /
``flow_latitudinal.fits`` with ``output:flow_global`` / ``output:flow_latitudinal``.

The packet loop runs on the GPU engine (``artes_amd.engine``).  Under
``torchrun --nproc-per-node G`` every rank transports its shard on its own GPU and the
sums are all-reduced (``artes_amd.dist``); rank 0 writes the outputs.
Deliberate differences: the reference's clock-seeded RNG becomes ``--seed`` (default:
clock); the process exits with status 0 on the reference's fatal errors, as it does.
"""

from __future__ import annotations

import math
import os
import shutil
import sys
import time

import numpy as np

from . import atmosphere as atmos
from . import dist, driver
from .config import PI, ConfigError, RunConfig, read_artes_in, split_key_value


class Transport:
    """Packet-loop backend: the HIP engine on this rank's GPU."""

    def __init__(self, atm: dict, device: int, oblateness: float, tuning: dict | None = None):
        from .engine import Grid

        self.grid = Grid(atm, device=device, oblateness=oblateness)
        if tuning:   # engine:<key>=<value> keys (RunConfig.engine)
            self.grid.set_tuning(**tuning)

    def cell_depth(self, wl: int) -> int:
        return self.grid.cell_depth(wl)

    def thermal(self, wl: int, thermal_weight: bool, ring: bool):
        return self.grid.thermal(wl, thermal_weight, ring)

    def run(self, params, first: int, n: int, seed: int, flow_global: bool = False, flow_latitudinal: bool = False):
        return self.grid.run(params, first, n, seed, flow_global=flow_global, flow_latitudinal=flow_latitudinal)


def _usage() -> None:
    print("How to run ARTES:")
    print("./bin/ARTES [inputDirectory] [photons] -o [outputDirectory] -k [keyWord]=[value]")


def run(argv: list[str], root: str | None = None, transport_factory=None, stdout=sys.stdout) -> int:
    root = os.getcwd() if root is None else root
    seed = None
    args = []
    i = 0
    while i < len(argv):
        if argv[i] == "--seed" and i + 1 < len(argv):
            seed = int(argv[i + 1])
            i += 2
            continue
        args.append(argv[i])
        i += 1
    if len(args) <= 1:                                    # ARTES.f90:4242-4247
        _usage()
        return 0
    atm_name = args[0]
    packages = int(float(args[1].replace("d", "e").replace("D", "E")))
    atm_dir = os.path.join(root, "input", atm_name)
    input_file = os.path.join(atm_dir, "artes.in")
    if not os.path.isfile(input_file):                    # ARTES.f90:373-378
        print("Input file does not exist!", file=stdout)
        return 0
    r = dist.init()
    try:
        cfg = read_artes_in(input_file)
    except ConfigError as e:
        print(e, file=stdout)
        return 0

    # argument_keywords (ARTES.f90:4260-4309), in argv order
    output_name = ""
    j = 0
    while j < len(args):
        a = args[j]
        if a == "-o" and j + 1 < len(args):
            output_name = args[j + 1]
            if r.rank == 0:
                run_dir = os.path.join(root, "output", output_name)
                shutil.rmtree(run_dir, ignore_errors=True)
                for sub in ("", "input", "output", "plot"):
                    os.makedirs(os.path.join(run_dir, sub), exist_ok=True)
                for fname in ("artes.in", "atmosphere.in", "atmosphere.fits", "atmosphere.dat", "pressureTemperature.dat"):
                    src = os.path.join(atm_dir, fname)
                    if os.path.exists(src):
                        shutil.copy(src, os.path.join(run_dir, "input", fname))
            j += 2
            continue
        if a == "-k" and j + 1 < len(args):
            kw = args[j + 1]
            key, value = split_key_value(kw)
            try:
                cfg.apply(key, value)
            except ConfigError as e:
                print(e, file=stdout)
                return 0
            copied = os.path.join(root, "output", output_name, "input", "artes.in")
            if r.rank == 0 and os.path.exists(copied):
                with open(copied, "a") as f:
                    f.write("\n" + kw + "\n")
            j += 2
            continue
        j += 1

    run_dir = os.path.join(root, "output", output_name)
    out_dir = os.path.join(run_dir, "output")
    if r.rank == 0:
        os.makedirs(out_dir, exist_ok=True)
        open(os.path.join(run_dir, "error.log"), "a").close()

    atm = atmos.read_atmosphere_fits(os.path.join(atm_dir, "atmosphere.fits"))
    r_top = float(atm["radial"][-1])
    ntheta = atm["theta"].size - 1
    det = driver.detector_geometry(cfg, r_top)
    if seed is None:   # the reference's clock seed (ARTES.f90:4187), drawn once on rank 0
        seed = dist.broadcast_int(int(time.time() * 1e6) & 0x7FFFFFFFFFFFFFFF, r)
    device = dist.device_of(r)
    if transport_factory is None:
        transport = (Transport(atm, device=device, oblateness=cfg.oblateness, tuning=cfg.engine) if cfg.engine
                     else Transport(atm, device=device, oblateness=cfg.oblateness))
    else:
        transport = transport_factory(atm, device, cfg.oblateness)
    if r.rank == 0:
        driver.write_plot_dat(run_dir, cfg, float(atm["radial"][0]), ntheta, det.x_fov)
    wavelengths = np.asarray(atm["wavelength"], dtype=np.float64) * 1.0e-6
    t_start = time.time()
    err_total = np.zeros(64, dtype=np.uint64)
    call = [0]

    planet = cfg.photon_source == 2
    thermal = {}

    def source(wl: int):
        """(cell_depth, emissivity_total, cell_luminosity) of the wavelength: grid_initialize(2)."""
        if wl not in thermal:
            thermal[wl] = (transport.thermal(wl, cfg.thermal_weight, cfg.ring) if planet
                           else (transport.cell_depth(wl), None, None))
        return thermal[wl]

    def energy(wl: int, det_phi: float) -> float:
        return driver.package_energy(cfg, wavelengths[wl], r_top, packages, det_phi, emissivity_total=source(wl)[1])

    def write_source(wl: int, res, mono: bool):
        """normalization.dat (star) or luminosity.dat / cell_luminosity.fits (planet), ARTES.f90:3623-3685."""
        if planet:
            if mono:
                driver.write_cell_luminosity(out_dir, source(wl)[2])
            e_pack = source(wl)[1] / float(packages)
            driver.write_luminosity(out_dir, wavelengths[wl], float(res.totals[8]), float(res.totals[9]), e_pack)
        else:
            driver.write_normalization(out_dir, cfg, wavelengths[wl], r_top)

    flows = {"flow_global": True} if cfg.flow_global else {}
    if cfg.flow_theta:
        flows["flow_latitudinal"] = True

    def transport_call(wl: int, det_phi: float):
        params = driver.run_params(cfg, det, wl, det_phi=det_phi, cell_depth=source(wl)[0], packet_moments=False)
        base = call[0] * packages
        call[0] += 1
        res = dist.run_sharded(lambda first, n, s: transport.run(params, base + first, n, s, **flows), packages, seed, r)
        if r.rank == 0 and flows:
            # every write_output rewrites the flow files (ARTES.f90:3715-3768): the last call wins
            if cfg.flow_global:
                driver.write_flow_global(out_dir, res.flow_global, source(wl)[0])
            if cfg.flow_theta:
                if not planet:
                    print("artes_amd: output:flow_latitudinal with photon:source=star -- the reference normalises "
                          "by flux_exit, which only the planet source defines; written unnormalised", file=stdout)
                driver.write_flow_latitudinal(out_dir, res.flow_latitudinal, source(wl)[0],
                                              float(res.totals[9]) if planet else None)
        return res

    mode = cfg.mode
    if mode == "imaging_mono":
        wl = 0
        res = transport_call(wl, det.det_phi)
        err_total += res.err
        if r.rank == 0:
            E = energy(wl, det.det_phi)
            d = driver.scale_detector(res.det[:3], E)
            ph = driver.photometry(d)
            driver.write_stokes_outputs(out_dir, d, det.pixel_scale)
            driver.write_photometry(out_dir, wavelengths[wl], ph)
            write_source(wl, res, True)
            driver.write_cell_depth(out_dir, wavelengths[wl], source(wl)[0])
    elif mode == "spectrum":                              # ARTES.f90:132-166
        for wl in range(wavelengths.size):
            if r.rank == 0:   # grid_initialize(2) of the wavelength (ARTES.f90:2457-2491)
                driver.write_optical_depth(out_dir, wavelengths[wl], atm, wl)
            res = transport_call(wl, det.det_phi)
            err_total += res.err
            if r.rank == 0:
                E = energy(wl, det.det_phi)
                d = driver.scale_detector(res.det[:3], E)
                driver.write_spectrum_line(out_dir, wavelengths[wl], d)
                write_source(wl, res, False)
                driver.write_cell_depth(out_dir, wavelengths[wl], source(wl)[0])
    elif mode == "imaging_broad":                         # ARTES.f90:168-204
        # detector_thread is zeroed once (array_start at wl_count == 1, ARTES.f90:175-180) and
        # accumulates over the wavelengths; every radiative_transfer call rescales the running
        # sums by the CURRENT wavelength's package energy (959-975), so the last one wins, and
        # write_output runs once after the loop (199)
        acc = None
        E = 0.0
        for wl in range(wavelengths.size):
            if r.rank == 0:
                driver.write_optical_depth(out_dir, wavelengths[wl], atm, wl)
            res = transport_call(wl, det.det_phi)
            err_total += res.err
            acc = res.det[:3].copy() if acc is None else acc + res.det[:3]
            E = energy(wl, det.det_phi)
            # planet source: the reference's single write_output reads flux_emitted / flux_exit
            # after grid_finished(1) has deallocated them (2557-2565, undefined behaviour);
            # here luminosity.dat gets one line per wavelength instead
            if r.rank == 0 and planet:
                write_source(wl, res, False)
        if r.rank == 0:
            d = driver.scale_detector(acc, E)
            driver.write_stokes_outputs(out_dir, d, det.pixel_scale)
            if not planet:   # normalization.dat of the last wavelength (write_output, 3622-3652)
                write_source(wavelengths.size - 1, None, False)
    elif mode == "phase":                                 # ARTES.f90:206-250
        wl = 0
        for k, phi in enumerate(driver.phase_angles()):
            res = transport_call(wl, phi)
            err_total += res.err
            if r.rank == 0:
                E = energy(wl, phi)
                d = driver.scale_detector(res.det[:3], E)
                driver.write_phase_line(out_dir, phi, d)
                if planet or phi < PI / 180.0:
                    write_source(wl, res, False)
    else:
        print("No detector type (detector:type) selected", file=stdout)
        return 0
    if r.rank == 0:
        driver.write_error_log(os.path.join(run_dir, "error.log"), err_total)
        dt = time.time() - t_start
        print(f"artes_amd: {mode}, {packages} packets x {call[0]} call(s), {dt:.2f} s"
              + (" -- WARNING: check error log!" if err_total.sum() else ""), file=stdout)
    return 0


def main() -> int:
    return run(sys.argv[1:])
