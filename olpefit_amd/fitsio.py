"""Minimal FITS primary-HDU reader/writer (no astropy on the GPU box).

Covers what apf_step2.py needs from ``astropy.io.fits`` (apf_step2.py:160-161,
:176-179): the primary data array (BITPIX 8/16/32/64/-32/-64 with BSCALE/BZERO)
and case-insensitive header keywords (``itime``, ``coadds``, ``multisam``,
``sampmode``).  Data are returned with big-endian dtypes exactly like
``fits.open(f)[0].data`` (e.g. ``>f4`` for BITPIX -32); header values are parsed
into int/float/bool/str.
"""
from __future__ import annotations

import numpy as np

_BLOCK = 2880
_CARD = 80
_BITPIX = {8: ">u1", 16: ">i2", 32: ">i4", 64: ">i8", -32: ">f4", -64: ">f8"}


class Header(dict):
    """Case-insensitive keyword -> value mapping (FITS keywords are upper-case)."""

    def __getitem__(self, key):
        return dict.__getitem__(self, key.upper())

    def __contains__(self, key):
        return dict.__contains__(self, key.upper())

    def get(self, key, default=None):
        return dict.get(self, key.upper(), default)


def _parse_value(raw: str):
    s = raw.strip()
    if s.startswith("'"):
        end = s.find("'", 1)
        while end != -1 and end + 1 < len(s) and s[end + 1] == "'":
            end = s.find("'", end + 2)
        return s[1:end].replace("''", "'").rstrip()
    if "/" in s:
        s = s.split("/", 1)[0].strip()
    if s == "T":
        return True
    if s == "F":
        return False
    try:
        return int(s)
    except ValueError:
        pass
    try:
        return float(s.replace("D", "E"))
    except ValueError:
        return s


def read_header_bytes(buf: bytes):
    """Parse header cards from ``buf``.  Returns (Header, n_header_bytes)."""
    hdr = Header()
    off = 0
    while True:
        if off + _BLOCK > len(buf):
            raise ValueError("truncated FITS header (no END card)")
        block = buf[off:off + _BLOCK].decode("ascii", errors="replace")
        off += _BLOCK
        for k in range(0, _BLOCK, _CARD):
            card = block[k:k + _CARD]
            key = card[:8].strip()
            if key == "END":
                return hdr, off
            if card[8:10] == "= " and key:
                hdr[key.upper()] = _parse_value(card[10:])


def getdata_header(path: str):
    """Read the primary HDU: (data, header).  ``data`` mirrors ``fits.open(path)[0].data``."""
    with open(path, "rb") as f:
        buf = f.read()
    hdr, off = read_header_bytes(buf)
    if not hdr.get("SIMPLE", False):
        raise ValueError(f"{path}: not a FITS file (SIMPLE != T)")
    bitpix = int(hdr["BITPIX"])
    naxis = int(hdr.get("NAXIS", 0))
    if naxis == 0:
        return None, hdr
    shape = tuple(int(hdr[f"NAXIS{i}"]) for i in range(naxis, 0, -1))
    dt = np.dtype(_BITPIX[bitpix])
    count = int(np.prod(shape))
    data = np.frombuffer(buf, dtype=dt, count=count, offset=off).reshape(shape).copy()
    bscale = hdr.get("BSCALE", 1)
    bzero = hdr.get("BZERO", 0)
    if bscale != 1 or bzero != 0:
        if bitpix > 0:
            data = data.astype(np.float32 if bitpix <= 16 else np.float64)
        data = data * bscale + bzero
    return data, hdr


def _card(key: str, value, comment: str = "") -> str:
    if isinstance(value, bool):
        v = "T" if value else "F"
        s = f"{key:<8}= {v:>20}"
    elif isinstance(value, (int, np.integer)):
        s = f"{key:<8}= {int(value):>20d}"
    elif isinstance(value, (float, np.floating)):
        s = f"{key:<8}= {repr(float(value)).upper():>20}"
    else:
        v = "'" + str(value).replace("'", "''").ljust(8) + "'"
        s = f"{key:<8}= {v:<20}"
    if comment:
        s += " / " + comment
    return s[:_CARD].ljust(_CARD)


def write(path: str, data: np.ndarray, header: dict | None = None) -> None:
    """Write ``data`` (2-D) as a primary HDU with extra ``header`` keywords."""
    data = np.asarray(data)
    inv = {v: k for k, v in _BITPIX.items()}
    be = data.dtype.newbyteorder(">") if data.dtype.byteorder != ">" else data.dtype
    bitpix = inv.get(be.str)
    if bitpix is None:
        raise ValueError(f"unsupported dtype {data.dtype}")
    cards = [_card("SIMPLE", True), _card("BITPIX", bitpix), _card("NAXIS", data.ndim)]
    for i, n in enumerate(reversed(data.shape), start=1):
        cards.append(_card(f"NAXIS{i}", n))
    for k, v in (header or {}).items():
        cards.append(_card(k.upper(), v))
    cards.append("END".ljust(_CARD))
    text = "".join(cards)
    text += " " * ((-len(text)) % _BLOCK)
    raw = np.ascontiguousarray(data, dtype=be).tobytes()
    raw += b"\0" * ((-len(raw)) % _BLOCK)
    with open(path, "wb") as f:
        f.write(text.encode("ascii"))
        f.write(raw)
