"""A stand-in for olpefit_amd.core.Sampler that runs no kernel, for the CPU tests of
bench.py's rank launcher and its N > 1 reporting (bench.sampler_class reads
OLPE_BENCH_SAMPLER=bench_stub:StubSampler).

Each launch "takes" OLPE_STUB_MS milliseconds (a sleep), so the timed region, the
reported value and the exchange fields follow from known numbers.  OLPE_STUB_FAIL
injects the failures the tests pin:

* ``chain``  -- allgather_chain raises on every rank (the line carries comm_error);
* ``rank1``  -- rank 1 exits with status 5 right after it joins the host group
  (the launcher must report the failure and stop the other ranks).

OLPE_STUB_MS_PER_RANK adds that many milliseconds per rank index to each launch (a
slow GPU: the line's per_rank_kernel_ms spread); OLPE_STUB_NODES=k puts rank r on the
fake node r mod k (dist.node_id via OLPE_NODE_ID): identical nodes repeat PCI bus ids.
"""
import os
import time

import numpy as np


class StubError(RuntimeError):
    pass


class StubSampler:
    def __init__(self, image, itime=1.0, coadds=1, multisam=1, sampmode=2, nsrc=2,
                 bkgd_mode=0, device=0, **_):
        self.n = np.asarray(image).shape[1]
        self.nsrc = nsrc
        self.np_ = 16 if nsrc == 2 else 19
        self.ps = self.np_ + 1
        self.W = 0
        self.device = device
        rank = int(os.environ.get("RANK", "0"))
        self.ms = float(os.environ.get("OLPE_STUB_MS", "2")) + \
            rank * float(os.environ.get("OLPE_STUB_MS_PER_RANK", "0"))
        if os.environ.get("OLPE_STUB_NODES"):
            os.environ["OLPE_NODE_ID"] = f"node{rank % int(os.environ['OLPE_STUB_NODES'])}"
        self._nrec = 0
        self._rows = 0
        self._kms = []
        self.nranks = 1
        self.fail = os.environ.get("OLPE_STUB_FAIL", "")
        if self.fail == "rank1" and os.environ.get("RANK") == "1":
            os._exit(5)

    def close(self):
        if getattr(self, "_made_fault", False) and os.path.exists(self._fault_file()):
            os.remove(self._fault_file())

    @staticmethod
    def device_count():
        return int(os.environ.get("OLPE_STUB_NDEV", "8"))

    @staticmethod
    def device_pci_id(device):
        return f"0000:{0x10 + device:02x}:00.0"

    def chi_squared(self, p):
        return 4096.0

    def seed(self, seeds):
        self.seeds = np.asarray(seeds, dtype=np.uint32)
        self.W = self.seeds.size

    def set_state(self, state):
        self.state = np.array(np.broadcast_to(state, (self.W, self.ps)), dtype=np.float64)
        # every rank's walkers distinguishable after a gather: the seed in column 0
        self.state[:, 0] = self.seeds

    def get_state(self):
        t = np.full((self.W, self.np_), 10.0)
        return self.state.copy(), t, t * 0.5

    def set_eval_mode(self, mode):
        self.mode = mode

    def run_async(self, n_iters, burn_in=0, record_stride=0, accept_min=0):
        time.sleep(self.ms * 1e-3)
        self._kms.append(self.ms)
        self._nrec = n_iters // record_stride if record_stride else 0
        return self._nrec

    def moments_accumulate(self):
        self._rows += self._nrec

    def sync(self):
        pass

    def kernel_times(self, n):
        out = np.array(self._kms[-n:], dtype=np.float64)
        return out

    def last_units(self):
        return 1

    @staticmethod
    def clock_meter(pci):
        class Meter:               # (bench.SmiClock's interface: a fixed 2.05 GHz)
            def start(self):
                pass

            def stop(self):
                return 2.05, 3
        return Meter()

    def chain(self):
        return np.broadcast_to(self.state[:, None, :], (self.W, self._nrec, self.ps)).copy()

    # -- exchange ---------------------------------------------------------------
    @staticmethod
    def comm_unique_id():
        return b"s" * 128

    def comm_init(self, uid, nranks, rank):
        # RCCL prints a banner to stdout when a communicator is created (fd 1, not
        # sys.stdout): the bench must keep it off its one-line stdout
        # (through C stdio, buffered, as RCCL's printf is)
        import ctypes
        libc = ctypes.CDLL(None)
        libc.printf(b"RCCL version : stub banner\n")
        if uid != b"s" * 128:
            raise StubError("unique id not broadcast")
        self.nranks, self.rank = nranks, rank

    def comm_timeout(self, seconds):
        self.timeout = seconds

    def comm_info(self):
        # what ncclCommCount / ncclCommUserRank report for a communicator of nranks
        return self.nranks, self.rank

    def allgather_state(self):
        # what RCCL would return: every rank's walkers in rank order (seeds are global
        # indices + 1000, so rank r's block is the seeds [1000 + r W, 1000 + (r+1) W))
        out = np.tile(self.state, (self.nranks, 1))
        for r in range(self.nranks):
            out[r * self.W:(r + 1) * self.W, 0] = 1000 + r * self.W + np.arange(self.W)
        return out

    def allgather_chain(self, w0=0, wn=None, out=True):
        if self.fail == "chain":
            raise StubError("olpe_comm_allgather_chain: injected failure")
        wn = self.W - w0 if wn is None else wn
        if not out:
            return None
        return np.broadcast_to(self.chain()[w0:w0 + wn], (self.nranks, wn, self._nrec,
                                                          self.ps)).copy()

    # the fault drill (bench.fault_drill): a fault set on one rank fails the all-reduce on
    # every rank, as olpe_comm_proto.h makes it -- shared between the stub ranks through a
    # file (the drill puts a barrier between setting it and the calls)
    def _fault_file(self):
        import tempfile
        return os.path.join(tempfile.gettempdir(),
                            f"olpe_stub_fault_{os.environ.get('MASTER_PORT', 'x')}")

    def moments_fault(self, where):
        f = self._fault_file()
        if where:
            with open(f, "w") as fh:
                fh.write(f"{self.rank} {where}")
            self._made_fault = True
        elif os.path.exists(f):
            os.remove(f)

    def _check_fault(self):
        f = self._fault_file()
        if os.path.exists(f):
            who, where = map(int, open(f).read().split())
            e = StubError(f"moments all-reduce: fault {where} on rank {who}")
            e.code = -2 if who == getattr(self, "rank", 0) else -5
            raise e

    @property
    def moments_len(self):
        return 2 + 3 * self.ps + 2 * self.np_

    def allreduce_moments(self):
        self._check_fault()
        m = np.zeros(self.moments_len)
        M = self.nranks * self.W
        ps, np_ = self.ps, self.np_
        m[0], m[1] = self._rows, M
        m[2:2 + ps] = M * 1.0
        m[2 + ps:2 + 2 * ps] = self._rows * M * 1.0
        m[2 + 2 * ps:2 + 3 * ps] = M * 0.5
        m[2 + 3 * ps:2 + 3 * ps + np_] = M * 100.0
        m[2 + 3 * ps + np_:] = M * 40.0
        return m

    def moments_summary(self, centre=None):
        m = self.allreduce_moments() / self.nranks
        m[0] = self._rows
        m[1] = self.W
        if centre is not None:          # every walker's column means are 1.0 here
            m[2 + 2 * self.ps:2 + 3 * self.ps] = self.W * (1.0 - np.asarray(centre)) ** 2
        return m
