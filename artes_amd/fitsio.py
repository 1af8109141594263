"""Minimal FITS image reader/writer (numpy only; no astropy / cfitsio).

ARTES reads ``atmosphere.fits`` through cfitsio by HDU *position* and the
NAXISn keywords only (``ARTES.f90:2067-2198``), and writes ``stokes.fits`` /
``error.fits`` as a single primary HDU with BITPIX = -64 (``ARTES.f90:3774-3806``).
The Python setup path writes its files with astropy (``atmosphere.py:449-460``,
``opacity*.py``).  This module implements exactly the subset those files use:

* a primary HDU followed by any number of ``XTENSION= 'IMAGE'`` HDUs,
* BITPIX in {8, 16, 32, 64, -32, -64}, big-endian, optional BSCALE/BZERO,
* 2880-byte blocks, 80-character cards.

Array convention: FITS axis 1 (fastest) is the *last* numpy axis, so a Fortran
array ``a(n1, n2, n3)`` round-trips as a C-order numpy array of shape
``(n3, n2, n1)`` -- the same convention astropy uses.
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

BLOCK = 2880
CARD = 80

_BITPIX_DTYPE = {8: ">u1", 16: ">i2", 32: ">i4", 64: ">i8", -32: ">f4", -64: ">f8"}


@dataclass
class HDU:
    data: np.ndarray | None
    header: dict = field(default_factory=dict)
    name: str = ""


class FITSError(ValueError):
    pass


def _parse_value(raw: str):
    raw = raw.strip()
    if not raw:
        return None
    if raw.startswith("'"):
        end = raw.find("'", 1)
        while end != -1 and end + 1 < len(raw) and raw[end + 1] == "'":
            end = raw.find("'", end + 2)
        return raw[1:end].replace("''", "'").rstrip()
    val = raw.split("/", 1)[0].strip()
    if val == "T":
        return True
    if val == "F":
        return False
    try:
        return int(val)
    except ValueError:
        pass
    try:
        return float(val.replace("D", "E").replace("d", "e"))
    except ValueError:
        return val


def _read_header(buf: memoryview, off: int):
    header: dict = {}
    order: list = []
    while True:
        if off + BLOCK > len(buf):
            raise FITSError("truncated FITS header")
        block = bytes(buf[off:off + BLOCK]).decode("ascii", errors="replace")
        off += BLOCK
        done = False
        for i in range(0, BLOCK, CARD):
            card = block[i:i + CARD]
            key = card[:8].strip()
            if key == "END":
                done = True
                break
            if not key or key in ("COMMENT", "HISTORY"):
                continue
            if card[8:10] == "= ":
                header[key] = _parse_value(card[10:])
                order.append(key)
        if done:
            return header, off


def read(path: str | os.PathLike) -> list[HDU]:
    """Read every HDU of a FITS file. Image data are returned as native-endian arrays."""
    with open(path, "rb") as f:
        raw = f.read()
    buf = memoryview(raw)
    off = 0
    hdus: list[HDU] = []
    while off < len(buf):
        if not bytes(buf[off:off + 8]).strip(b" \0"):
            break
        header, off = _read_header(buf, off)
        bitpix = int(header.get("BITPIX", 8))
        naxis = int(header.get("NAXIS", 0))
        shape_f = [int(header[f"NAXIS{i + 1}"]) for i in range(naxis)]
        nelem = int(np.prod(shape_f)) if naxis > 0 else 0
        pcount = int(header.get("PCOUNT", 0))
        gcount = int(header.get("GCOUNT", 1))
        nbytes = (abs(bitpix) // 8) * gcount * (pcount + nelem)
        data = None
        if nelem > 0:
            if bitpix not in _BITPIX_DTYPE:
                raise FITSError(f"unsupported BITPIX {bitpix}")
            arr = np.frombuffer(buf, dtype=_BITPIX_DTYPE[bitpix], count=nelem, offset=off)
            arr = arr.reshape(shape_f[::-1])
            bscale = header.get("BSCALE", 1.0)
            bzero = header.get("BZERO", 0.0)
            if bscale != 1.0 or bzero != 0.0:
                data = arr.astype(np.float64) * bscale + bzero
            else:
                data = arr.astype(arr.dtype.newbyteorder("="))
        off += nbytes + (-nbytes % BLOCK)
        hdus.append(HDU(data=data, header=header, name=str(header.get("EXTNAME", ""))))
    if not hdus:
        raise FITSError(f"{path}: no HDU found")
    return hdus


def _card(key: str, value, comment: str = "") -> str:
    if isinstance(value, bool):
        v = f"{'T' if value else 'F':>20}"
    elif isinstance(value, (int, np.integer)):
        v = f"{int(value):>20}"
    elif isinstance(value, (float, np.floating)):
        v = f"{float(value):>20.14G}"
    else:
        s = str(value).replace("'", "''")
        v = f"'{s:<8}'"
    card = f"{key:<8}= {v}"
    if comment:
        card += f" / {comment}"
    return card[:CARD].ljust(CARD)


def _hdu_bytes(data, primary: bool, name: str = "", bitpix: int = -64) -> bytes:
    if data is None:
        arr = None
        naxes: list[int] = []
    else:
        arr = np.ascontiguousarray(np.asarray(data, dtype=_BITPIX_DTYPE[bitpix]))
        naxes = list(arr.shape[::-1]) if arr.ndim > 0 else [1]
        if arr.ndim == 0:
            arr = arr.reshape(1)
    cards = []
    if primary:
        cards.append(_card("SIMPLE", True, "conforms to FITS standard"))
    else:
        cards.append(_card("XTENSION", "IMAGE", "Image extension"))
    cards.append(_card("BITPIX", bitpix, "array data type"))
    cards.append(_card("NAXIS", len(naxes), "number of array dimensions"))
    for i, n in enumerate(naxes):
        cards.append(_card(f"NAXIS{i + 1}", int(n)))
    if primary:
        cards.append(_card("EXTEND", True))
    else:
        cards.append(_card("PCOUNT", 0, "number of parameters"))
        cards.append(_card("GCOUNT", 1, "number of groups"))
    if name:
        cards.append(_card("EXTNAME", name, "extension name"))
    cards.append("END".ljust(CARD))
    head = "".join(cards)
    head += " " * (-len(head) % BLOCK)
    body = b"" if arr is None else arr.tobytes()
    body += b"\0" * (-len(body) % BLOCK)
    return head.encode("ascii") + body


def write(path: str | os.PathLike, arrays, names=None, bitpix: int = -64) -> None:
    """Write ``arrays`` as primary HDU + IMAGE extensions (BITPIX -64 by default)."""
    if isinstance(arrays, np.ndarray):
        arrays = [arrays]
    names = list(names) if names is not None else [""] * len(arrays)
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        for i, a in enumerate(arrays):
            f.write(_hdu_bytes(a, primary=(i == 0), name=names[i] if i > 0 else "", bitpix=bitpix))
    os.replace(tmp, path)
