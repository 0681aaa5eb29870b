"""Host-side mirror of the apf_step2 hot path, backed by libolpe.so on one GPU.

Reference functions and the method that replaces each (reference paths relative to
the reference checkout):

===============================================  =====================================
apf_step2.py                                     olpefit_amd
===============================================  =====================================
:176-210 saturation mask + sigma map              ``noise_model`` / ``Sampler.__init__``
:106-124 ``build_analytical_model(p)``            ``Sampler.build_analytical_model``
:134-137 ``chi_squared(data, model, err)``        ``Sampler.chi_squared`` (batched)
:300-333 Gibbs loop (proposal, accept_reject)     ``Sampler.run`` (fused HIP kernel)
:342-351 chain stacking after burn-in             ``Sampler.run(..., record_stride)``
global ``np.random`` (unseeded per rank)           ``Sampler.seed`` (per-walker seeds)
===============================================  =====================================

Nothing here computes the model on the CPU: every evaluation goes through the HIP
library, and constructing a Sampler without a GPU raises ``OlpeError``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import OlpeError, check

__all__ = ["OlpeError", "Sampler", "noise_model", "param_count", "SIGMA0"]

SIGMA0 = (50 / 9.95) / 2.35   # apf_step2.py:242-245


def param_count(nsrc: int) -> int:
    """Proposable parameters (16 for 2 sources, 19 for 3); the state adds chi^2."""
    if nsrc not in (2, 3):
        raise ValueError("nsrc must be 2 or 3")
    return 16 if nsrc == 2 else 19


def _dptr(a):
    return a.ctypes.data_as(_lib._pd) if a is not None else None


def noise_model(image, itime, coadds, multisam, sampmode):
    """apf_step2.py:176-210: (mask, pois2, readnoise2, satlevel, readnoise).

    ``mask`` = ``np.ma.masked_greater(image, 0.8*satlevel)``'s mask (:188) together with
    every pixel whose residual the reference's ``np.ma`` arithmetic drops in
    ``chi_squared`` (:134-137): ``np.ma.divide`` masks a non-finite quotient and a zero
    divisor, so a NaN or -inf data pixel, and a pixel whose ``err`` is NaN or 0, never
    enters chi^2 (+inf is already above the saturation level).  olpe_create applies the
    same rule to what it is given.
    ``pois2`` = ``np.sqrt(np.abs(image))**2`` in the image dtype (float32 for BITPIX
    -32, as the reference rounds it); ``readnoise2`` = ``readnoise**2``."""
    itime = float(itime) * 1000.
    coadds = float(coadds)
    multisam = float(multisam)
    if sampmode == 3:
        satlevel = coadds * 24000.0 * (1.0 - 0.1 * (multisam - 1.0) / (itime / 1000.))
    else:
        satlevel = coadds * 22000.0
    mask = np.ma.getmaskarray(np.ma.masked_greater(image, 0.8 * satlevel))
    if sampmode == 3.0:
        readnoise = (38.0 / np.sqrt(multisam)) * (np.sqrt(coadds))
    else:
        readnoise = 38 * (np.sqrt(coadds))
    rn = np.float64(readnoise)
    with np.errstate(invalid="ignore"):
        pois2 = np.sqrt(np.abs(image)) ** 2
        err = np.sqrt(rn * rn + pois2.astype(np.float64))          # :210
        mask = mask | ~np.isfinite(image) | ~np.isfinite(err) | (err == 0)
    return mask, pois2, float(rn * rn), satlevel, float(readnoise)


class Sampler:
    """One cutout + one walker ensemble on one GPU (one ``olpe_ctx``)."""

    def __init__(self, image, itime=1.0, coadds=1, multisam=1, sampmode=2, nsrc=2,
                 bkgd_mode=0, device=0, mask=None, pois2=None, readnoise2=None):
        lib = _lib.load()
        img = np.asarray(image)
        if img.ndim != 2:
            raise ValueError("image must be 2-D")
        if pois2 is None or readnoise2 is None or mask is None:
            m, p2, rn2, self.satlevel, self.readnoise = noise_model(img, itime, coadds,
                                                                    multisam, sampmode)
            mask = m if mask is None else mask
            pois2 = p2 if pois2 is None else pois2
            readnoise2 = rn2 if readnoise2 is None else readnoise2
        if img.dtype.kind == "f" and img.dtype.itemsize == 4:
            dt, npdt = _lib.DTYPE_F32, np.float32
        else:
            dt, npdt = _lib.DTYPE_F64, np.float64
        self._img = np.ascontiguousarray(img, dtype=npdt)
        self._pois2 = np.ascontiguousarray(pois2, dtype=npdt)
        self._mask = np.ascontiguousarray(mask, dtype=np.uint8)
        self.n = img.shape[1]
        self.nsrc = nsrc
        self.np_ = param_count(nsrc)
        self.ps = self.np_ + 1
        self.W = 0
        self.nranks = 1                 # until comm_init
        self._nrec = 0                  # rows per walker of the last launch
        ctx = C.c_void_p()
        check(lib.olpe_create(self._img.ctypes.data, dt, self._pois2.ctypes.data,
                              float(readnoise2), self._mask.ctypes.data_as(_lib._pu8),
                              img.shape[0], img.shape[1], nsrc, bkgd_mode, device,
                              C.byref(ctx)))
        self._ctx = ctx
        self._lib = lib

    # -- lifetime ---------------------------------------------------------------
    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.olpe_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_eval_mode(self, mode: str):
        check(self._lib.olpe_set_eval_mode(self._ctx, {"exact": _lib.EVAL_EXACT,
                                                       "fast": _lib.EVAL_FAST}[mode]))

    # -- model / chi^2 ----------------------------------------------------------
    def _vec(self, params):
        p = np.ascontiguousarray(params, dtype=np.float64)
        if p.shape[-1] == self.np_:
            p = np.concatenate([p, np.zeros(p.shape[:-1] + (1,))], axis=-1)
        if p.shape[-1] != self.ps:
            raise ValueError(f"parameter vectors must have {self.np_} or {self.ps} entries")
        return np.ascontiguousarray(p)

    def build_analytical_model(self, p):
        """apf_step2.py:106-124 (3body :106-125) -> (n, n) float64 model image."""
        p = self._vec(p).reshape(self.ps)
        out = np.empty((self.n, self.n))
        check(self._lib.olpe_model(self._ctx, _dptr(p), _dptr(out)))
        return out

    def chi_squared(self, params):
        """chi_squared(image_nanmask, build_analytical_model(p), err) for one vector
        (returns float) or a batch [W, PS] (returns [W])."""
        p = self._vec(params)
        single = p.ndim == 1
        p = p.reshape(-1, self.ps)
        out = np.empty(p.shape[0])
        check(self._lib.olpe_chi2_batch(self._ctx, _dptr(p), p.shape[0], _dptr(out)))
        return float(out[0]) if single else out

    # -- ensemble ---------------------------------------------------------------
    def seed(self, seeds):
        """np.random.seed(seeds[w]) for each walker w; allocates the ensemble."""
        s = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64) & 0xFFFFFFFF,
                                 dtype=np.uint32)
        check(self._lib.olpe_seed(self._ctx, s.ctypes.data_as(_lib._pu32), s.size))
        self.W = int(s.size)

    def set_state(self, state, tries=None, accepts=None):
        st = np.ascontiguousarray(np.broadcast_to(state, (self.W, self.ps)), dtype=np.float64)
        t = None if tries is None else np.ascontiguousarray(
            np.broadcast_to(tries, (self.W, self.np_)), dtype=np.float64)
        a = None if accepts is None else np.ascontiguousarray(
            np.broadcast_to(accepts, (self.W, self.np_)), dtype=np.float64)
        check(self._lib.olpe_state_set(self._ctx, _dptr(st), _dptr(t), _dptr(a)))

    def get_state(self):
        st = np.empty((self.W, self.ps))
        t = np.empty((self.W, self.np_))
        a = np.empty((self.W, self.np_))
        check(self._lib.olpe_state_get(self._ctx, _dptr(st), _dptr(t), _dptr(a)))
        return st, t, a

    def run_async(self, n_iters, burn_in=0, record_stride=0, accept_min=0):
        """Launch n_iters iterations (no host sync).  Returns rows recorded per walker."""
        nrec = C.c_longlong(0)
        check(self._lib.olpe_run(self._ctx, int(n_iters), int(burn_in), int(record_stride),
                                 int(accept_min), C.byref(nrec)))
        self._nrec = int(nrec.value)
        return self._nrec

    def run(self, n_iters, burn_in=0, record_stride=1, accept_min=0, read_chain=True):
        """Run n_iters Gibbs iterations of every walker.  Returns the recorded chain
        [W, nrec, PS] (or None)."""
        nrec = self.run_async(n_iters, burn_in, record_stride, accept_min)
        self.sync()
        if read_chain and nrec > 0:
            return self.chain()
        return None

    def chain(self):
        out = np.empty((self.W, self._nrec, self.ps))
        check(self._lib.olpe_chain_read(self._ctx, _dptr(out)))
        return out

    @property
    def count(self) -> int:
        c = C.c_longlong(0)
        check(self._lib.olpe_count(self._ctx, C.byref(c)))
        return int(c.value)

    def reset_count(self, count: int = 0):
        check(self._lib.olpe_count_reset(self._ctx, int(count)))

    def done_at(self):
        out = np.empty(self.W, dtype=np.int64)
        check(self._lib.olpe_done_at(self._ctx, out.ctypes.data_as(_lib._pll)))
        return out

    def rng_state(self):
        mt = np.empty((self.W, 625), dtype=np.uint32)
        g = np.empty((self.W, 2))
        check(self._lib.olpe_rng_get(self._ctx, mt.ctypes.data_as(_lib._pu32), _dptr(g)))
        return mt, g

    def set_rng_state(self, mt, g):
        mt = np.ascontiguousarray(mt, dtype=np.uint32)
        g = np.ascontiguousarray(g, dtype=np.float64)
        check(self._lib.olpe_rng_set(self._ctx, mt.ctypes.data_as(_lib._pu32), _dptr(g)))

    def rng_stream(self, kind: str, n: int):
        k = {"raw": 0, "rand": 1, "gauss": 2, "randint": 3}[kind]
        out = np.empty((self.W, n), dtype=np.uint32 if k == 0 else np.float64)
        check(self._lib.olpe_rng_stream(self._ctx, k, int(n), out.ctypes.data))
        return out

    def enable_trace(self, on: bool = True):
        check(self._lib.olpe_trace_enable(self._ctx, int(bool(on))))

    def trace(self, n_iters):
        out = np.empty((self.W, n_iters, 6))
        check(self._lib.olpe_trace_read(self._ctx, _dptr(out)))
        return out

    def sync(self):
        check(self._lib.olpe_sync(self._ctx))

    def last_kernel_ms(self) -> float:
        ms = C.c_double(0)
        check(self._lib.olpe_last_kernel_ms(self._ctx, C.byref(ms)))
        return float(ms.value)

    def kernel_times(self, n: int):
        """Durations (ms) of the last n sampler launches, oldest first (n <= 64)."""
        out = np.empty(int(n))
        check(self._lib.olpe_kernel_times(self._ctx, int(n), _dptr(out)))
        return out

    def unit_stats(self):
        """(waits, ns waited) of chunk hand-offs since the context was created."""
        out = np.zeros(2, dtype=np.int64)
        check(self._lib.olpe_unit_stats(self._ctx, out.ctypes.data_as(_lib._pll)))
        return int(out[0]), int(out[1])

    def last_units(self) -> int:
        """Chunks per walker of the last sampler launch."""
        v = C.c_int(0)
        check(self._lib.olpe_last_units(self._ctx, C.byref(v)))
        return v.value

    # -- devices ----------------------------------------------------------------
    @staticmethod
    def device_count() -> int:
        n = C.c_int(0)
        check(_lib.load().olpe_device_count(C.byref(n)))
        return n.value

    @staticmethod
    def device_pci_id(device: int) -> str:
        """PCI bus id of a HIP device: tells GPUs apart across processes."""
        buf = C.create_string_buffer(64)
        check(_lib.load().olpe_device_pci_id(int(device), buf, 64))
        return buf.value.decode()

    # -- multi-GPU --------------------------------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        check(_lib.load().olpe_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        check(self._lib.olpe_comm_init(self._ctx, buf, nranks, rank))
        self.nranks = nranks

    def comm_timeout(self, seconds: float):
        """Bound on a collective's wait for the other ranks (olpe_comm_timeout; 0 =
        none): past it the communicator is aborted and the call raises (OLPE_ECOMM)."""
        check(self._lib.olpe_comm_timeout(self._ctx, float(seconds)))

    def comm_info(self) -> tuple[int, int]:
        """RCCL's own (rank count, rank) of this context's communicator."""
        n, r = C.c_int(-1), C.c_int(-1)
        check(self._lib.olpe_comm_info(self._ctx, C.byref(n), C.byref(r)))
        return n.value, r.value

    def allgather_state(self):
        out = np.empty((self.nranks * self.W, self.ps))
        check(self._lib.olpe_comm_allgather_state(self._ctx, _dptr(out)))
        return out

    def allgather_chain(self, w0: int = 0, wn: int | None = None, out: bool = True):
        """Chain concatenation over RCCL: walkers [w0, w0 + wn) of the last launch's
        chain from every rank -> [nranks, wn, nrec, PS] (rank-major), or None with
        ``out=False`` (gathered into the device buffer only: timing the collective)."""
        wn = self.W - w0 if wn is None else wn
        nrec = C.c_longlong(0)
        buf = np.empty((self.nranks, wn, self._nrec, self.ps)) if out else None
        check(self._lib.olpe_comm_allgather_chain(self._ctx, int(w0), int(wn), _dptr(buf),
                                                  C.byref(nrec)))
        return buf

    def gather_limit(self, nbytes: int):
        """Byte limit of the chain gather's device receive buffer (0 = none)."""
        check(self._lib.olpe_comm_gather_limit(self._ctx, int(nbytes)))

    def allreduce_moments(self):
        """Posterior sums over every rank's walkers (olpe_comm_allreduce_moments; this
        context alone without comm_init): the olpe_moments_summary layout with the
        centre at the pooled mean -- see ``step3.summary_from_moments``."""
        out = np.empty(self.moments_len)
        check(self._lib.olpe_comm_allreduce_moments(self._ctx, _dptr(out)))
        return out

    def hold_handoff(self, on: bool = True):
        """Test hook (olpe_test_hold_handoff, include/olpe_test.h): chunked launches hold
        each first chunk's hand-off until a later chunk is waiting for one, so a hand-off
        wait happens by construction (olpe_unit_stats counts it)."""
        check(self._lib.olpe_test_hold_handoff(self._ctx, 1 if on else 0))

    def moments_fault(self, where: int):
        """Test hook (olpe_moments_fault, include/olpe_test.h): 1 = the summary's
        allocation fails, 2 = its launch fails after the uniformity check, 3 = the check
        words fail to reach the device (every collective), 4 = round 1's sums fail to come
        back, 0 = clear."""
        check(self._lib.olpe_moments_fault(self._ctx, int(where)))

    # -- whole-run moments ---------------------------------
    @property
    def moments_len(self) -> int:
        return 2 + 3 * self.ps + 2 * self.np_           # OLPE_MOMENTS_LEN(PS, P)

    def moments_accumulate(self):
        """Fold the last launch's recorded rows into every walker's running (mean, M2)
        (async, on the device; once per launch)."""
        check(self._lib.olpe_moments_accumulate(self._ctx))

    def moments_reset(self):
        check(self._lib.olpe_moments_reset(self._ctx))

    def moments(self):
        """(n rows per walker, mean [W, PS], M2 [W, PS])."""
        n = C.c_longlong(0)
        mean = np.empty((self.W, self.ps))
        m2 = np.empty((self.W, self.ps))
        check(self._lib.olpe_moments_get(self._ctx, C.byref(n), _dptr(mean), _dptr(m2)))
        return int(n.value), mean, m2

    def set_moments(self, n, mean=None, m2=None):
        mean = None if mean is None else np.ascontiguousarray(mean, dtype=np.float64)
        m2 = None if m2 is None else np.ascontiguousarray(m2, dtype=np.float64)
        check(self._lib.olpe_moments_set(self._ctx, int(n), _dptr(mean), _dptr(m2)))

    def moments_summary(self, centre=None):
        """Per-column sums over this context's walkers (olpe_moments_summary)."""
        out = np.empty(self.moments_len)
        c = None if centre is None else np.ascontiguousarray(centre, dtype=np.float64)
        check(self._lib.olpe_moments_summary(self._ctx, _dptr(c), _dptr(out)))
        return out
