"""The step1 -> step2 -> step3 file surface kept by the build.

* step-1 guess file ``<dir>/<frame>_initialguess`` (apf_step1.py:166-175), read with
  ``np.loadtxt`` (apf_step2.py:261-262)
* initial parameter vector (apf_step2.py:264-273; 3body/apf_step2_3body.py:255-265)
* step-2a warm start: last row of ``step2a.csv`` (apf_step2.py:248-256)
* chain files ``{rank}_finalarray_mpi.csv``: ``csv.writer`` rows, NaN first row,
  PS columns (apf_step2.py:278-279, :342-360), and ``{rank}_acceptance_rate.csv`` =
  ``str(total_accept / total_tries)`` (:362-365)
* output directory ``<dir>/<frame>_apf_results/`` where ``<frame>`` is
  ``basename.split('.')[-3]`` (apf_step2.py:164-173)
"""
from __future__ import annotations

import os

import numpy as np

SIGMA0 = (50 / 9.95) / 2.35   # apf_step2.py:242-245


def image_paths(image_path: str):
    """(directory, frame, output_directory) exactly as apf_step2.py:164-170 builds
    them (string concatenation on '/')."""
    d = image_path.split('/')
    directory = ''
    for i in range(len(d) - 1):
        directory = directory + str(d[i]) + '/'
    frame = d[-1].split('.')[-3]
    return directory, frame, directory + frame + '_apf_results/'


def read_guess(path: str):
    """apf_step2.py:262: ``np.loadtxt(open(fileguess, "rb"), delimiter=' ')``."""
    with open(path, "rb") as f:
        return np.loadtxt(f, delimiter=' ')


def initial_parameters(image, guess, nsrc: int = 2):
    """apf_step2.py:264-273 (2 sources) / 3body :255-265 (3 sources).  The chi^2 slot
    is 0; apf_step2.py:283-289 fills it with the initial chi^2."""
    sigma = SIGMA0
    if nsrc == 2:
        xcs, ycs, xcc, ycc = guess[0], guess[1], guess[2], guess[3]
        amps = image[int(ycs - 1), int(xcs - 1)]
        ampc = image[int(ycc - 1), int(xcc - 1)]
        box = image[int(guess[5]):int(guess[5]) + 10, int(guess[4]):int(guess[4]) + 10]
        bkgd = np.median(box)
        return np.array([xcs, ycs, xcc, ycc, 0., 0., amps, ampc, 0.2, bkgd, sigma, sigma,
                         sigma * 3, sigma * 3, 0., 0., 0.], dtype=np.float64)
    xca, yca, xcb, ycb, xcc, ycc = (guess[k] for k in range(6))
    ampa = image[int(yca - 0.5 + 1), int(xca - 0.5 + 1)]
    ampb = image[int(ycb - 0.5 + 1), int(xcb - 0.5 + 1)]
    ampc = image[int(ycc - 0.5 + 1), int(xcc - 0.5 + 1)]
    box = image[int(guess[7]):int(guess[7]) + 10, int(guess[6]):int(guess[6]) + 10]
    bkgd = np.median(box)
    return np.array([xca, yca, xcb, ycb, xcc, ycc, 0., 0., ampa, ampb, ampc, 0.2, bkgd,
                     sigma, sigma, sigma * 3, sigma * 3, 0., 0., 0.], dtype=np.float64)


def read_step2a(path: str):
    """apf_step2.py:253-256: ``genfromtxt(step2a.csv)[-1:][0]``."""
    a = np.genfromtxt(path, delimiter=',')
    return np.atleast_2d(a)[-1:][0]


def format_rows(chain, nan_row: bool = False) -> str:
    """CSV text ``csv.writer`` produces for ``writerows(rows)`` of float rows: ','
    separator, '\\r\\n' terminator, repr() floats, NaN as 'nan' (libolpe's native
    formatter, olpe_csv_format); ``nan_row`` prepends the reference's all-NaN row."""
    import ctypes as C
    from . import _lib
    from ._lib import check
    rows = np.ascontiguousarray(np.atleast_2d(np.asarray(chain, dtype=np.float64)))
    lib = _lib.load()
    pd = rows.ctypes.data_as(C.POINTER(C.c_double))
    n = C.c_size_t(0)
    check(lib.olpe_csv_format(pd, rows.shape[0], rows.shape[1], int(nan_row), None, 0,
                              C.byref(n)))
    buf = C.create_string_buffer(n.value)
    check(lib.olpe_csv_format(pd, rows.shape[0], rows.shape[1], int(nan_row), buf, n.value,
                              C.byref(n)))
    return buf.raw[:n.value].decode("ascii")


def write_chain_csvs(paths, chains, nan_row: bool = True, threads: int = 0) -> None:
    """Per-walker ``{rank}_finalarray_mpi.csv`` files (apf_step2.py:342-360): file i
    gets ``chains[i]`` [nrows, PS] after the reference's all-NaN seed row, formatted
    and written natively from a pool of threads (olpe_csv_write_chains)."""
    import ctypes as C
    from . import _lib
    from ._lib import check
    chains = np.ascontiguousarray(np.asarray(chains, dtype=np.float64))
    if chains.ndim != 3 or chains.shape[0] != len(paths):
        raise ValueError(f"chains must be [len(paths), nrows, ncols], got {chains.shape}")
    arr = (C.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
    check(_lib.load().olpe_csv_write_chains(arr, chains.ctypes.data_as(C.POINTER(C.c_double)),
                                            len(paths), chains.shape[1], chains.shape[2],
                                            int(nan_row), int(threads)))


def append_chain_csvs(paths, chains, nrows=None, threads: int = 0) -> np.ndarray:
    """Append rows [0, nrows) of ``chains[i]`` ([len(paths), rows, PS]) to file i --
    the streaming form of the reference's every-10-iterations rewrite
    (apf_step2.py:355-360) -- natively from a pool of threads
    (olpe_csv_append_chains).  Returns each file's size in bytes afterwards."""
    import ctypes as C
    from . import _lib
    from ._lib import check
    chains = np.ascontiguousarray(np.asarray(chains, dtype=np.float64))
    if chains.ndim != 3 or chains.shape[0] != len(paths):
        raise ValueError(f"chains must be [len(paths), nrows, ncols], got {chains.shape}")
    nrows = chains.shape[1] if nrows is None else int(nrows)
    sizes = np.zeros(len(paths), dtype=np.int64)
    arr = (C.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
    check(_lib.load().olpe_csv_append_chains(
        arr, chains.ctypes.data_as(C.POINTER(C.c_double)), len(paths), chains.shape[1], nrows,
        chains.shape[2], int(threads), sizes.ctypes.data_as(C.POINTER(C.c_longlong))))
    return sizes


NPY_HEADER = 128


def npy_header(rows: int, cols: int) -> bytes:
    """A fixed-size (128-byte) .npy v1.0 header for a C-order float64 [rows, cols]
    array, so that a chain file can grow in place: append rows, rewrite the header."""
    d = "{'descr': '<f8', 'fortran_order': False, 'shape': (%d, %d), }" % (rows, cols)
    body = d.encode("latin1")
    pad = NPY_HEADER - 10 - len(body) - 1
    if pad < 0:
        raise ValueError("chain too large for the fixed .npy header")
    return b"\x93NUMPY\x01\x00" + np.uint16(NPY_HEADER - 10).tobytes() + body + b" " * pad + b"\n"


def append_npy_chains(paths, chains, nrows, rows_before: int) -> None:
    """``{w}_chain.npy`` sidecars grown by one launch: rows [0, nrows) of chains[i] are
    appended after ``rows_before`` rows and the header rewritten (each file stays a
    valid .npy between launches)."""
    chains = np.asarray(chains, dtype=np.float64)
    cols = chains.shape[2]
    for i, path in enumerate(paths):
        mode = "r+b" if os.path.exists(path) else "w+b"
        with open(path, mode) as f:
            f.seek(NPY_HEADER + rows_before * cols * 8)
            f.truncate()
            f.write(np.ascontiguousarray(chains[i, :nrows]).tobytes())
            f.seek(0)
            f.write(npy_header(rows_before + nrows, cols))


def write_chain_csv(path: str, rows) -> None:
    """One ``{rank}_finalarray_mpi.csv``: ``rows`` must already hold the NaN seed row."""
    rows = np.atleast_2d(np.asarray(rows, dtype=np.float64))
    write_chain_csvs([path], rows[None], nan_row=False, threads=1)


def with_seed_row(chain):
    """Prepend the all-NaN row the reference starts ``total_parameters`` with
    (apf_step2.py:278-279)."""
    chain = np.asarray(chain, dtype=np.float64)
    return np.vstack([np.full((1, chain.shape[-1]), np.nan), chain.reshape(-1, chain.shape[-1])])


def acceptance_text(accepts, tries) -> str:
    """apf_step2.py:363-364: ``str(total_accept / total_tries)``."""
    with np.errstate(all="ignore"):
        return str(np.asarray(accepts, dtype=np.float64) / np.asarray(tries, dtype=np.float64))


def write_acceptance(path: str, accepts, tries) -> None:
    """Write to a temporary name and rename it over the file (as the native writer
    does), so a run killed mid-write leaves the previous complete file, never a
    truncated one (the writes run in the background after a checkpoint)."""
    tmp = path + ".tmp"
    try:
        with open(tmp, "w") as f:
            f.write(acceptance_text(accepts, tries))
        os.replace(tmp, path)
    except BaseException:
        # no '<path>.tmp' left behind by a failed write
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise


def write_acceptance_files(paths, accepts, tries, threads: int = 0) -> None:
    """write_acceptance for many walkers: accepts / tries [W][P].  The native writer
    (olpe_acceptance_write, threaded) takes the rows NumPy prints in fixed notation;
    the others (scientific notation, a never-tried parameter's NaN) go through
    str() here."""
    from . import _lib
    import ctypes as C
    acc = np.ascontiguousarray(accepts, dtype=np.float64)
    tr = np.ascontiguousarray(tries, dtype=np.float64)
    n, p = acc.shape
    if n == 0:
        return
    done = np.zeros(n, dtype=np.uint8)
    arr = (C.c_char_p * n)(*[os.fsencode(x) for x in paths])
    lib = _lib.load()
    _lib.check(lib.olpe_acceptance_write(arr, acc.ctypes.data_as(_lib._pd),
                                         tr.ctypes.data_as(_lib._pd), n, p, int(threads),
                                         done.ctypes.data_as(_lib._pu8)))
    for k in np.flatnonzero(done == 0):
        write_acceptance(paths[k], acc[k], tr[k])


def written_rows(count: int, burn_in: int) -> int:
    """Data rows on disk after ``count`` iterations: the reference appends a row every
    iteration with count >= burn_in but rewrites the file only when count % 10 == 0
    (apf_step2.py:342-360), so the file holds rows up to the last multiple of 10."""
    last = (count // 10) * 10
    first = max(burn_in, 1)          # count is incremented before the burn-in check
    return last - first + 1 if last >= first else 0
